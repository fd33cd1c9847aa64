"""Shading-time modes inside ONE process: C3 frames at 128 spp before and after
events that could change the memory system's state (a 100-GB fill, idling, a second
renderer's allocation), with rocm-smi's clock readout sampled during a longer render. If k_shade's
time moves within the process, the mode is a clock / power state, not page placement."""
import json, subprocess, sys, time
sys.path.insert(0, ".")
import torch
from izpi_amd import configs
from izpi_amd import _native as N
from izpi_amd.renderer import GPURenderer

cfg = configs.configs()["C3"]
r = GPURenderer(cfg.build(), cfg.width, cfg.height, 128, max_depth=cfg.max_depth, sampler=cfg.sampler, device=0, bvh="gpu")


def frames(tag, k=2):
    for i in range(k):
        r.render(post=N.POST_NONE)
        st = r.stats
        print(json.dumps({"event": tag, "frame": i, "trace_ms": round(st["kernel_ms"], 2), "shade_ms": round(st["shade_ms"], 2),
                          "device_ms": round(st["total_ms"], 2)}), flush=True)


def clocks(tag):
    p = subprocess.Popen(["rocm-smi", "--showclocks"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    frames(tag + "+smi", 6)
    out = p.communicate(timeout=60)[0]
    print(tag, "clocks:", " | ".join(l.strip() for l in out.splitlines() if "clock level" in l.lower() or "clk" in l.lower()), flush=True)


frames("start")
clocks("start")
x = torch.empty(int(100e9) // 8, dtype=torch.float64, device="cuda")
x.fill_(1.0); torch.cuda.synchronize()
frames("after 100 GB fill, held")
del x; torch.cuda.synchronize()
frames("after fill freed")
time.sleep(5)
frames("after 5 s idle")
y = torch.empty(int(4e9) // 8, dtype=torch.float64, device="cuda")
t0 = time.time()
while time.time() - t0 < 3:
    y.mul_(1.0000001)
torch.cuda.synchronize()
frames("after 3 s of streaming")
clocks("end")
r.close()
