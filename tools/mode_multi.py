"""Shading-time modes across WORKSPACES of one process: several renderers of the
same scene and request, each with its own workspace allocation, alive together or one after
another; if their k_shade times differ inside one process, the mode follows the allocation's
pages rather than the process.

    python tools/mode_multi.py --config C3 --spp 128 --renderers 3 --frames 2
"""
import argparse, hashlib, json, sys
sys.path.insert(0, ".")
from izpi_amd import configs
from izpi_amd import _native as N
from izpi_amd.renderer import GPURenderer

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--spp", type=int, default=128)
ap.add_argument("--renderers", type=int, default=3)
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--variant", default=None, help="a library built by tools/variants.py build NAME")
a = ap.parse_args()
if a.variant:
    from pathlib import Path
    N.LIB_PATH = Path(__file__).resolve().parents[1] / "izpi_amd" / "_lib" / "variants" / a.variant / "libizpi_gpu.so"
cfg = configs.configs()[a.config]
scene = cfg.build()
rs = []
for k in range(a.renderers):
    rs.append(GPURenderer(scene, cfg.width, cfg.height, a.spp, max_depth=cfg.max_depth, sampler=cfg.sampler, device=0, bvh="gpu"))
post = N.POST_SPECTRAL if cfg.sampler == N.SAMPLER_SPECTRAL else N.POST_NONE
for rnd in range(a.rounds):
    for k, r in enumerate(rs):
        for f in range(a.frames):
            img = r.render(post=post)
            st = r.stats
            print(json.dumps({"variant": a.variant or "base", "round": rnd, "renderer": k, "frame": f, "trace_ms": round(st["kernel_ms"], 3),
                              "shade_ms": round(st["shade_ms"], 3), "device_ms": round(st["total_ms"], 3),
                              "alloc_ms": round(st.get("alloc_ms", 0.0), 1),
                              "workspace_gb": round(st["workspace_bytes"] / 1e9, 1), "slots": st["slots"],
                              "digest": hashlib.sha1(img.tobytes()).hexdigest()[:12]}), flush=True)
for r in rs:
    r.close()
