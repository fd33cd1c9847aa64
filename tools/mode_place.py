"""Does a short probe kernel predict the shading-time mode of a workspace?
One renderer; per cycle the record array (or the state, or both) is re-allocated on other
pages (izpi_gpu_debug_realloc), then izpi_gpu_debug_place_probe times a streamed state
read-modify-write mixed with random record writes over `--probe-gb` GB of state, then a
frame is rendered. One JSON line per cycle: probe ms against shade ms.

    python tools/mode_place.py --spp 128 --cycles 8 --probe-gb 4 --realloc recs
"""
import argparse, ctypes, json, sys
sys.path.insert(0, ".")
from izpi_amd import configs
from izpi_amd import _native as N
from izpi_amd.renderer import GPURenderer

NAMES = ["samples", "recs", "pool", "ring", "running", "state", "spill"]
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--spp", type=int, default=128)
ap.add_argument("--cycles", type=int, default=8)
ap.add_argument("--probe-gb", default="4", help="comma-separated list of state sizes to probe over")
ap.add_argument("--realloc", default="recs", help="comma-separated buffers re-allocated per cycle")
a = ap.parse_args()
cfg = configs.configs()[a.config]
r = GPURenderer(cfg.build(), cfg.width, cfg.height, a.spp, max_depth=cfg.max_depth, sampler=cfg.sampler, device=0, bvh="gpu")
L = N.lib()
mask = sum(1 << NAMES.index(n) for n in a.realloc.split(","))
sizes = [float(x) for x in a.probe_gb.split(",")]
r.render()
for c in range(a.cycles + 1):
    if c:
        assert L.izpi_gpu_debug_realloc(r.ctx, mask) == 0
    probe = {}
    for gb in sizes:
        ms = ctypes.c_float()
        assert L.izpi_gpu_debug_place_probe(r.ctx, gb, ctypes.byref(ms)) == 0
        probe[str(gb)] = round(ms.value, 3)
    r.render()
    st = r.stats
    print(json.dumps({"cycle": c, "realloc": a.realloc if c else "none", "probe_ms": probe,
                      "trace_ms": round(st["kernel_ms"], 3), "shade_ms": round(st["shade_ms"], 3),
                      "device_ms": round(st["total_ms"], 3)}), flush=True)
r.close()
