"""Where a fresh renderer's first frame spends its host time (IZPI_TUNE_PASS_LOG's IZPI_HOST
line: sizing, allocation, setup, issue, completion), against its second and third frames.

    python tools/first_frame_host.py [--spp 512] [--acc forward]
"""
import argparse, json, re, subprocess, sys
sys.path.insert(0, ".")

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=512)
ap.add_argument("--acc", default="forward")
ap.add_argument("--child", action="store_true")
a = ap.parse_args()
if not a.child:  # the renderer in a child process, its stderr parsed here
    out = subprocess.run([sys.executable, __file__, "--child", "--spp", str(a.spp), "--acc", a.acc],
                         capture_output=True, text=True)
    keys = ("tiles", "tracer", "meminfo", "sized", "allocated", "launched", "issued", "done")
    frames = [dict(zip(keys, map(float, m))) for m in
              re.findall(r"IZPI_HOST " + " ".join(k + r" (\S+)" for k in keys), out.stderr)]
    for line in out.stdout.splitlines():
        d = json.loads(line)
        d["host"] = frames[d["frame"]] if d["frame"] < len(frames) else None
        print(json.dumps(d))
    sys.exit(out.returncode)
import time
import torch
from izpi_amd import configs
from izpi_amd import _native as N
from izpi_amd.renderer import GPURenderer
torch.zeros(1, device="cuda:0")
cfg = configs.configs()["C3"]
t0 = time.perf_counter()
r = GPURenderer(cfg.build(), cfg.width, cfg.height, a.spp, device=0, bvh="gpu",
                accumulation=N.ACC_FORWARD if a.acc == "forward" else N.ACC_RECURSIVE,
                tuning=N.tuning(flags=N.TUNE_PASS_LOG))
setup = time.perf_counter() - t0
canvas = torch.zeros((cfg.height, cfg.width, 4), dtype=torch.float64, device="cuda:0")
for f in range(3):
    t = time.perf_counter()
    r.render_device(canvas.data_ptr())
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) * 1e3
    st = r.stats
    print(json.dumps({"frame": f, "wall_ms": round(wall, 3), "device_ms": round(st["total_ms"], 3),
                      "trace_ms": round(st["kernel_ms"], 3), "shade_ms": round(st["shade_ms"], 3),
                      "alloc_ms": round(st["alloc_ms"], 3), "setup_s": round(setup, 3)}), flush=True)
r.close()
