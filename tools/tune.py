"""A/B tuning of launch knobs on one GPU, interleaved in one process (guide §5.4 rule 24).

python tools/tune.py --config C3 --spp 64 --rounds 3 --var IZPI_SLOTS=1048576,2097152,8388608
Prints ms per frame (median, min) per variant and checks every variant's image is
bit-identical to the first (the knobs must never change results)."""
import argparse
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--bvh", default="gpu")
    ap.add_argument("--var", action="append", default=[], help="NAME=v1,v2,... (env knob)")
    a = ap.parse_args()
    import numpy as np
    from izpi_amd import configs
    from izpi_amd.renderer import GPURenderer
    cfg = configs.configs()[a.config]
    scene = cfg.build()
    r = GPURenderer(scene, cfg.width, cfg.height, a.spp, max_depth=cfg.max_depth, sampler=cfg.sampler, bvh=a.bvh)
    variants = [{}]
    for v in a.var:
        name, vals = v.split("=")
        variants = [dict(d, **{name: x}) for d in variants for x in vals.split(",")]
    times = {i: [] for i in range(len(variants))}
    ref = None
    ref_cnt = None
    r.render()  # warm
    for _ in range(a.rounds):
        for i, env in enumerate(variants):
            for k, val in env.items():
                os.environ[k] = val
            t = time.perf_counter()
            img = r.render()
            times[i].append((time.perf_counter() - t) * 1e3)
            st = r.stats
            cnt = tuple(st[k] for k in ("rays", "node_visits", "tri_tests", "sph_tests", "light_tri_tests"))
            if ref is None:
                ref = img.copy()
                ref_cnt = cnt
            elif img.tobytes() != ref.tobytes() or cnt != ref_cnt:
                print("RESULT MISMATCH for", env, cnt, ref_cnt, flush=True)
            for k in env:
                del os.environ[k]
            print("round", env, "%.1f ms" % times[i][-1], "trace %.1f shade %.1f launches %d" %
                  (st["kernel_ms"], st["shade_ms"], st["launches"]), flush=True)
    samples = cfg.width * cfg.height * a.spp
    for i, env in enumerate(variants):
        med = statistics.median(times[i])
        print("VARIANT", env, "median %.1f ms  min %.1f ms  %.1f Msamples/s" % (med, min(times[i]), samples / med / 1e3))


if __name__ == "__main__":
    main()
