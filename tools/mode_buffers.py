"""Which workspace buffer's pages set k_shade's time? One C3 renderer: frames,
then each buffer in turn re-allocated on other pages (izpi_gpu_debug_realloc) and frames
again; a buffer whose re-allocation moves shade_ms carries the mode.

    python tools/mode_buffers.py --spp 128 --cycles 3
"""
import argparse, json, sys
sys.path.insert(0, ".")
from izpi_amd import configs
from izpi_amd import _native as N
from izpi_amd.renderer import GPURenderer

NAMES = ["samples", "recs", "pool", "ring", "running", "state", "spill"]
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--spp", type=int, default=128)
ap.add_argument("--cycles", type=int, default=3)
ap.add_argument("--buffers", default="samples,recs,pool,state")
a = ap.parse_args()
cfg = configs.configs()[a.config]
r = GPURenderer(cfg.build(), cfg.width, cfg.height, a.spp, max_depth=cfg.max_depth, sampler=cfg.sampler, device=0, bvh="gpu")
L = N.lib()


def frame(tag):
    r.render()
    st = r.stats
    print(json.dumps({"after": tag, "trace_ms": round(st["kernel_ms"], 3), "shade_ms": round(st["shade_ms"], 3),
                      "device_ms": round(st["total_ms"], 3)}), flush=True)


frame("start")
frame("start")
for c in range(a.cycles):
    for name in a.buffers.split(","):
        assert L.izpi_gpu_debug_realloc(r.ctx, 1 << NAMES.index(name)) == 0
        frame("realloc %s (cycle %d)" % (name, c))
r.close()
