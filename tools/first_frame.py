"""One-shot frame cost: a fresh renderer's first Render() against its second, with the
device memory in use after each (what leader.go:155-158 sees: one frame per process).

    python tools/first_frame.py [--config C3] [--frames 2]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C3")
    p.add_argument("--frames", type=int, default=2)
    p.add_argument("--spp", type=int, default=None)
    p.add_argument("--stats", action="store_true", help="print every counter of the last frame")
    p.add_argument("--slots", type=int, default=0, help="tuning: wavefront slots (0 = library sizing)")
    p.add_argument("--chunk-units", type=int, default=0, help="tuning: per-sample result units per chunk")
    a = p.parse_args()
    import torch
    from izpi_amd import _native as N
    from izpi_amd import configs
    from izpi_amd.renderer import GPURenderer
    cfg = configs.configs()[a.config]
    spp = a.spp or cfg.spp
    scene = cfg.build()
    free0, total = torch.cuda.mem_get_info(0)  # (also initialises torch's HIP context outside the timed frames)
    tune = N.tuning(slots=a.slots, chunk_units=a.chunk_units) if (a.slots or a.chunk_units) else None
    t0 = time.perf_counter()
    r = GPURenderer(scene, cfg.width, cfg.height, spp, max_depth=cfg.max_depth, sampler=cfg.sampler, device=0, bvh="gpu",
                    tuning=tune)
    setup = time.perf_counter() - t0
    out = {"config": a.config, "spp": spp, "setup_s": setup, "frames": []}
    for i in range(a.frames):
        t = time.perf_counter()
        r.render()
        dt = time.perf_counter() - t
        free, _ = torch.cuda.mem_get_info(0)
        out["frames"].append({"wall_ms": dt * 1e3, "device_ms": r.stats["total_ms"], "trace_ms": r.stats["kernel_ms"],
                              "shade_ms": r.stats["shade_ms"], "tail_ms": r.stats["tail_ms"],
                              "rays": r.stats["rays"], "parks": r.stats["parks"], "hbm_used_gb": (free0 - free) / 1e9,
                              "alloc_ms": r.stats["alloc_ms"], "slots": r.stats["slots"], "chunk_spp": r.stats["chunk_spp"],
                              "workspace_gb": r.stats["workspace_bytes"] / 1e9})
        print(json.dumps(out["frames"][-1]), flush=True)
    if a.stats:
        print(json.dumps({"stats": r.stats}), flush=True)
    r.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
