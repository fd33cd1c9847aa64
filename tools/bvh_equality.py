"""Render each benchmark config on the reference tree (hitable.NewBVH4, rebuilt bit for
bit on the host) and on the GPU-built linear BVH4, and compare the canvases.

    python tools/bvh_equality.py [--configs C1,C2,C3,C4,C5] [--spp-cap N]

Prints one JSON line per config: differing pixels, max abs difference, RMSE, and both
render times. Used to back DESIGN.md's claim about the GPU builder (SURVEY.md §8(f)
row 4: "validate ... by equal-image checks on C1-C3").
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C2,C3,C4,C5")
    ap.add_argument("--spp-cap", type=int, default=512)
    args = ap.parse_args()
    import numpy as np
    from izpi_amd import _native as N
    from izpi_amd import configs
    from izpi_amd.renderer import GPURenderer
    for name in args.configs.split(","):
        cfg = configs.configs()[name]
        spp = min(cfg.spp, args.spp_cap)
        scene = cfg.build()
        post = N.POST_SPECTRAL if cfg.sampler == N.SAMPLER_SPECTRAL else N.POST_NONE
        out = {"config": name, "width": cfg.width, "height": cfg.height, "spp": spp}
        imgs = {}
        for bvh in ("reference", "gpu"):
            r = GPURenderer(scene, cfg.width, cfg.height, spp, sampler=cfg.sampler, bvh=bvh)
            t = time.perf_counter()
            imgs[bvh] = r.render(post=post)
            out[bvh + "_s"] = round(time.perf_counter() - t, 3)
            out[bvh + "_nodes_per_ray"] = round(r.stats["node_visits"] / max(r.stats["rays"], 1), 3)
            out[bvh + "_rays"] = int(r.stats["rays"])
            r.close()
        a, b = imgs["reference"], imgs["gpu"]
        diff = np.abs(a - b)
        px = (a.view(np.uint64) != b.view(np.uint64)).any(-1)
        out["differing_pixels"] = int(px.sum())
        out["max_abs_diff"] = float(np.nanmax(diff)) if diff.size else 0.0
        out["rmse"] = float(np.sqrt(np.nanmean((a - b) ** 2)))
        out["bitwise_equal"] = bool(a.tobytes() == b.tobytes())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
