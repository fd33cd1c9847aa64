"""How fast fresh VRAM is handed out right after another process freed a large workspace:
allocate CHUNKS x GB device buffers one at a time (hipMalloc through torch), timing each,
optionally after a pause. Prints one JSON line.

    python tools/alloc_probe.py [--chunks 8] [--gb 16] [--pause 0]
"""
import argparse
import json
import time


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--chunks", type=int, default=8)
    p.add_argument("--gb", type=float, default=16.0)
    p.add_argument("--pause", type=float, default=0.0)
    a = p.parse_args()
    import torch
    torch.cuda.init()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if a.pause:
        time.sleep(a.pause)
    bufs, ms = [], []
    for _ in range(a.chunks):
        t = time.perf_counter()
        bufs.append(torch.empty(int(a.gb * 1e9), dtype=torch.uint8, device="cuda"))
        torch.cuda.synchronize()
        ms.append(round((time.perf_counter() - t) * 1e3, 1))
    print(json.dumps({"gb_per_chunk": a.gb, "pause_s": a.pause, "alloc_ms": ms, "total_ms": round(sum(ms), 1),
                      "since_start_s": round(time.perf_counter() - t0, 2)}), flush=True)


if __name__ == "__main__":
    main()
