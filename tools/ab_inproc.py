"""A/B of izpi_render_tuning settings inside ONE process (a process keeps its
shading-time mode, so settings compared in one process share it): the settings take turns,
one frame each, for --rounds rounds; one JSON line per frame.

    python tools/ab_inproc.py --config C4 --spp 128 --rounds 3 base flags=256
"""
import argparse, hashlib, json, sys
sys.path.insert(0, ".")
from izpi_amd import configs
from izpi_amd import _native as N
from izpi_amd.renderer import GPURenderer

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--spp", type=int, default=0)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--acc", default="forward", choices=["forward", "recursive"])
ap.add_argument("--quantized", action="store_true", help="the GPU tree with IZPI_SCENE_QUANTIZED_BVH")
ap.add_argument("settings", nargs="+", help="'base' or comma-separated field=value of izpi_render_tuning")
a = ap.parse_args()
cfg = configs.configs()[a.config]
spp = a.spp or cfg.spp
tunes = {}
accs = {}
for s in a.settings:  # 'base', 'acc=recursive', or tuning fields (optionally with acc=...)
    kv = dict(x.split("=") for x in s.split(",")) if s != "base" else {}
    accs[s] = {"forward": N.ACC_FORWARD, "recursive": N.ACC_RECURSIVE}[kv.pop("acc", a.acc)]
    tunes[s] = N.tuning(**{k: int(v) for k, v in kv.items()}) if kv else None
r = GPURenderer(cfg.build(), cfg.width, cfg.height, spp, max_depth=cfg.max_depth, sampler=cfg.sampler, device=0, bvh="gpu",
                bvh_quantized=a.quantized,
                accumulation=N.ACC_FORWARD if a.acc == "forward" else N.ACC_RECURSIVE)
post = N.POST_SPECTRAL if cfg.sampler == N.SAMPLER_SPECTRAL else N.POST_NONE
for rnd in range(a.rounds + 1):  # round 0 warms up every setting
    for s, t in tunes.items():
        r.tuning = t
        r.accumulation = accs[s]
        img = r.render(post=post)
        st = r.stats
        if rnd:
            print(json.dumps({"config": a.config, "spp": spp, "setting": s, "round": rnd, "trace_ms": round(st["kernel_ms"], 3),
                              "shade_ms": round(st["shade_ms"], 3), "node_visits": st["node_visits"], "quantized": a.quantized, "tail_ms": round(st["tail_ms"], 3),
                              "device_ms": round(st["total_ms"], 3), "workspace_gb": round(st["workspace_bytes"] / 1e9, 1),
                              "digest": hashlib.sha1(img.tobytes()).hexdigest()[:16]}), flush=True)
r.close()
