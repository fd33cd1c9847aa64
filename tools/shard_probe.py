"""Per-rank render time of a W-way tile shard on ONE GPU (strong-scaling probe).

python tools/shard_probe.py --config C3 --worlds 1,2,4,8
For each W, renders every rank's tiles (packed layout, device memory) and prints ms,
passes and the implied efficiency T(1) / (W * max rank time), i.e. the scaling the
multi-GPU bench would see without the gather, split into the share imbalance
(max / mean rank time) and the per-share overhead (W * mean / T(1))."""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--bvh", default="gpu")
    ap.add_argument("--pass-log", action="store_true", help="per-pass trace/shade times and queue lengths on stderr")
    ap.add_argument("--tail-paths", type=int, default=0, help="tuning: k_tail takes over at <= this many paths")
    ap.add_argument("--variant", default=None, help="a library built by tools/variants.py build NAME")
    ap.add_argument("--acc", default="forward", choices=["forward", "recursive"])
    ap.add_argument("--ranks", default="", help="comma list of the ranks to render (default all)")
    ap.add_argument("--share-slots", default="", help="comma list: tuning slot caps tried for the shares of W > 1 (the W = 1 frame keeps the default)")
    ap.add_argument("--share-tunes", default="", help="semicolon list of 'field=value,...' tunings tried for the shares of W > 1")
    ap.add_argument("--split", type=int, default=1, help="deal sub-tiles: each tile cut into split x split before dealing (W > 1)")
    a = ap.parse_args()
    import torch
    from izpi_amd import _native as N
    if a.variant:
        N.LIB_PATH = Path(__file__).resolve().parents[1] / "izpi_amd" / "_lib" / "variants" / a.variant / "libizpi_gpu.so"
    from izpi_amd import configs, sharding
    from izpi_amd.renderer import GPURenderer, common_tiles
    cfg = configs.configs()[a.config]
    spp = a.spp or cfg.spp
    tune = {}
    if a.pass_log:
        tune["flags"] = [N.TUNE_PASS_LOG]
    if a.tail_paths:
        tune["tail_paths"] = a.tail_paths
    r = GPURenderer(cfg.build(), cfg.width, cfg.height, spp, max_depth=cfg.max_depth, sampler=cfg.sampler, bvh=a.bvh,
                    tuning=N.tuning(**tune) if tune else None,
                    accumulation=N.ACC_FORWARD if a.acc == "forward" else N.ACC_RECURSIVE)
    all_tiles = common_tiles(cfg.width, cfg.height)
    import numpy as np
    def split_tiles(tl, k):
        out = []
        for x0, y0, x1, y1 in np.asarray(tl).reshape(-1, 4):
            w, h = (x1 - x0 + 1) // k, (y1 - y0 + 1) // k
            for j in range(k):
                for i in range(k):
                    out.append((x0 + i * w, y0 + j * h, x0 + i * w + w - 1, y0 + j * h + h - 1))
        return np.asarray(out, np.uint32)
    deal_tiles = split_tiles(all_tiles, a.split) if a.split > 1 else all_tiles
    t1 = None
    base_tuning = r.tuning
    runs = [(int(x), None) for x in a.worlds.split(",")]
    if a.share_slots:
        runs = [(w, sl) for w, _ in runs for sl in ([None] if w == 1 else [None] + [int(v) for v in a.share_slots.split(",")])]
    if a.share_tunes:
        runs = [(w, sl) for w, _ in runs for sl in ([None] if w == 1 else [None] + a.share_tunes.split(";"))]
    for w, sl in runs:
        r.tuning = base_tuning
        if isinstance(sl, str):
            kv = {k: int(v) for k, v in (x.split("=") for x in sl.split(","))}
            r.tuning = N.tuning(**dict(tune, **kv))
        elif sl:
            r.tuning = N.tuning(**dict(tune, slots=sl))
        worst, times = 0.0, []
        for rank in ([int(x) for x in a.ranks.split(",")] if a.ranks and w > 1 else range(w)):
            src = deal_tiles if w > 1 else all_tiles
            mine = sharding.shard_tiles(src, rank, w)
            buf = torch.zeros(sharding.packed_len(src, w), dtype=torch.float64, device="cuda")
            r.render_device(buf.data_ptr(), tiles=mine, layout=N.OUT_PACKED)  # warm
            torch.cuda.synchronize()
            t = time.perf_counter()
            st = r.render_device(buf.data_ptr(), tiles=mine, layout=N.OUT_PACKED)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) * 1e3
            worst = max(worst, ms)
            times.append(ms)
            print("W=%d%s rank=%d tiles=%d %.1f ms (trace %.1f shade %.1f tail %.1f, %d passes)" %
                  (w, (" " + sl if isinstance(sl, str) else " slots=%d" % sl) if sl else "", rank, len(mine), ms, st["kernel_ms"], st["shade_ms"], st["tail_ms"], st["launches"]), flush=True)
        if t1 is None:
            t1 = worst
        mean = sum(times) / len(times)
        print("W=%d%s implied efficiency %.3f (imbalance max/mean %.3f, overhead W*mean/T1 %.3f)" %
              (w, (" " + sl if isinstance(sl, str) else " slots=%d" % sl) if sl else "", t1 / (w * worst), worst / mean, w * mean / t1), flush=True)


if __name__ == "__main__":
    main()
