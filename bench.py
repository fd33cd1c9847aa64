"""Benchmark: Msamples/s (pixels x spp) of the izpi path-tracing inner loop on MI355X.

Workload (BASELINE.json metric "Msamples/sec at 1024x1024/512spp"): config C3 — the
Cornell box with the synthetic ~817k-triangle dragon, Colour sampler, maxDepth 50,
1024x1024 pixels x 512 spp = 536,870,912 samples per frame.

One step = one full frame through the hot path (BVH4 traversal, shading, light pdfs,
ordered per-pixel accumulation) with the scene already resident in HBM. Timing: barrier
+ synchronize on both sides of the K timed steps, max over ranks.

GPUs (strong scaling: the frame is fixed, its 32x32 tiles are dealt tile % N):
  * under torchrun (WORLD_SIZE set): one process per GPU, each renders its share and the
    library's own RCCL communicator gathers the shares to rank 0 (izpi_gpu_render_rank);
    gloo carries only the launcher's barrier, the communicator id and the max of times;
  * `--gpus N` without torchrun: ONE process drives N GPUs through izpi_gpu_multi_render
    (a host thread and stream per GPU, xGMI peer copies to GPU 0).
  Both forms do the gather inside the timed step.

The JSON line also carries
  roofline:     the dominant kernel k_trace2 against HBM peak. `achieved` = L2 memory-side
                traffic per frame, measured by rocprofv3 PMC passes (FETCH_SIZE x2 +
                WRITE_SIZE; the x2 is MI355X_MICROARCH.md's gfx950 correction, checked for
                k_trace2's access shapes by tools/fetch_calib) over a one-frame child run of
                this same revision, divided by k_trace2's HIP-event time per frame in the timed
                run. Those counters include Infinity-Cache hits, so `frac` is the L2-miss
                fabric rate against HBM peak (`levels.l2_miss_fabric_frac`); `levels` puts the
                same bytes against the Infinity Cache's measured random-gather rate
                (`mall_frac`) and SURVEY.md §8(d)'s algorithmic bytes (128 B per node visit,
                72 B per triangle test, 32 B per sphere test, counted exactly by the kernel)
                against the L2's rate (`l2_frac`), and names the nearest ceiling. TCC hit
                rates come from a third PMC pass.
  cpu_baseline: the CPU oracle (deterministic restatement of the Go hot path) on a
                bounded sample of the same frame on the CPUs this process may use (rank 0,
                N=1), with the host's CPU model and core counts.
"""
import argparse
import csv
import json
import math
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md, L2 (per XCD): 34.5 TB/s aggregate over the 8 XCDs
# MI355X_MICROARCH.md, "Indexed rows: gather into LDS": uniformly random rows served by the
# Infinity Cache read at 8.6 TB/s chip-wide from a 38 MB table and 7.4-7.9 TB/s from a 151 MB
# one; C3's BVH + triangles are 136 MB, so the 151-MB figure (mid-range) is the ceiling
MALL_GATHER_GBS = 7650.0
PMC_PASSES = {"fetch": ["FETCH_SIZE"], "write": ["WRITE_SIZE"], "tcc": ["TCC_HIT_sum", "TCC_MISS_sum"],
              "sq": ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                     "SQ_ACTIVE_INST_FLAT", "SQ_WAIT_INST_ANY"]}
# global loads / stores are FLAT-encoded on gfx950: SQ_ACTIVE_INST_VMEM reads 0 for them and
# SQ_ACTIVE_INST_FLAT equals SQ_INSTS_FLAT (one issue cycle per instruction), calibrated on
# known kernels in profiles/r5b/fetch_calib_sq.jsonl (tools/fetch_calib.py)
KERNELS = {"k_trace2": "k_trace2<", "k_shade": "k_shade<"}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None, help="GPUs (default: WORLD_SIZE under torchrun, else 1)")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", default="C3")
    p.add_argument("--spp", type=int, default=None, help="override spp (debug only; the metric uses 512)")
    p.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC passes (roofline traffic)")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--dry-run", action="store_true",
                   help="launcher plumbing only (rank setup, tile shares, barriers, max of times): no GPU work")
    p.add_argument("--scene", default=None, help="render a transport.Scene file (.pbtxt/.izpi) at the config's size")
    p.add_argument("--bvh", default="gpu", choices=["reference", "gpu"],
                   help="gpu (default): the GPU linear BVH4 builder, checked at N=1 against a frame on the "
                        "reference tree; reference: hitable.NewBVH4's tree rebuilt bit for bit on the host")
    p.add_argument("--bvh-leaf-max", type=int, default=None, help="primitives per leaf of the GPU-built tree")
    p.add_argument("--no-reference-check", action="store_true",
                   help="skip the reference-tree frame (timing and image comparison) of --bvh gpu")
    p.add_argument("--obj", default=None, help="C3 with this OBJ mesh (e.g. the Stanford dragon) instead of the "
                                               "synthetic one")
    p.add_argument("--accumulation", default="forward", choices=["forward", "recursive"],
                   help="forward (default): IZPI_ACC_FORWARD, checked at N=1 against frames of the bitwise "
                        "recursion in the same run (pixel RMSE < 1e-6, same NaN / Inf pixels, else the recursion's "
                        "figures are reported); recursive: IZPI_ACC_RECURSIVE, bit-identical to the oracle")
    return p.parse_args(argv)


# ---------------------------------------------------------------- host facts
def host_cpus():
    """CPUs this process may use (affinity, capped by a cgroup CPU quota), and the host's."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except Exception:
        pass
    usable = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"usable": usable, "affinity": aff, "cgroup_cpus": quota, "host_threads": os.cpu_count(), "model": model}


# ---------------------------------------------------------------- scene/config
def load_config(args):
    from izpi_amd import configs
    cfg = configs.configs()[args.config]
    t0 = time.time()
    scene = None if (args.scene or args.obj) else cfg.build()
    if args.scene:  # leader.go:43-112: file scene, SPECTRAL scenes use the spectral sampler
        from izpi_amd import ingest
        scene = ingest.ProtoScene.from_file(args.scene)
        cfg = configs.Config("%s (%s)" % (cfg.name, Path(args.scene).name), cfg.width, cfg.height, cfg.spp,
                             scene.sampler, None, cfg.max_depth)
    elif args.obj:
        scene = configs.cornell_obj(args.obj, cfg.width / cfg.height)
        cfg = configs.Config("%s (mesh %s)" % (cfg.name, Path(args.obj).name), cfg.width, cfg.height, cfg.spp,
                             cfg.sampler, None, cfg.max_depth)
    return cfg, scene, time.time() - t0


STAT_KEYS = ("node_visits", "tri_tests", "sph_tests", "light_tri_tests", "light_sph_tests", "rays", "kernel_ms",
             "shade_ms", "total_ms", "launches", "samples", "node_steps", "prim_steps", "leaf_shortcuts", "tail_ms",
             "tail_node_visits", "tail_tri_tests", "tail_sph_tests", "parks")


def add_stats(agg, st):
    for k in STAT_KEYS:
        agg[k] += float(st[k]) if st else 0.0


# ---------------------------------------------------------------- PMC passes
def pmc_children(args, timeout=240):
    """rocprofv3 --pmc passes over a one-frame child of this bench (same workload,
    single GPU): per-kernel counter sums and dispatch counts."""
    out = {}
    base = [sys.executable, str(ROOT / "bench.py"), "--pmc-child", "--config", args.config, "--steps", "1",
            "--warmup", "0", "--bvh", args.bvh, "--accumulation", args.accumulation]
    if args.spp:
        base += ["--spp", str(args.spp)]
    if args.scene:
        base += ["--scene", args.scene]
    if args.obj:
        base += ["--obj", args.obj]
    if args.bvh_leaf_max:
        base += ["--bvh-leaf-max", str(args.bvh_leaf_max)]
    env = dict(os.environ, TMPDIR="/tmp")
    for name, counters in PMC_PASSES.items():
        d = tempfile.mkdtemp(prefix="izpi_pmc_", dir="/tmp")
        cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", "run", "--", *base]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=env)
        except Exception as e:  # missing profiler, timeout: report, no traffic figure
            out["error"] = "%s pass: %s" % (name, e)
            return out
        if r.returncode != 0:
            out["error"] = "%s pass: rc %d: %s" % (name, r.returncode, r.stderr[-400:])
            return out
        for f in Path(d).rglob("*counter_collection.csv"):
            for row in csv.DictReader(open(f)):
                for short, pat in KERNELS.items():
                    if pat in row["Kernel_Name"]:
                        e = out.setdefault(short, {"dispatches": set()})
                        e[row["Counter_Name"]] = e.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                        e["dispatches"].add((name, row["Dispatch_Id"]))
    for short in KERNELS:
        if short in out:
            out[short]["dispatches"] = len([x for x in out[short]["dispatches"] if x[0] == "fetch"])
    return out


def traffic_summary(pmc):
    """Bytes per frame and TCC hit rates per kernel from the PMC passes. FETCH_SIZE and
    WRITE_SIZE are in KB; gfx950 reports half of the bytes of wide reads, so FETCH_SIZE is
    doubled (MI355X_MICROARCH.md, HBM section). Both count L2 memory-side requests
    (Infinity-Cache hits included), an upper bound of the HBM bytes."""
    out = {}
    for short in KERNELS:
        e = pmc.get(short)
        if not e or "FETCH_SIZE" not in e or "WRITE_SIZE" not in e:
            continue
        fb = 2.0 * 1024.0 * e["FETCH_SIZE"]
        wb = 1024.0 * e["WRITE_SIZE"]
        hit, miss = e.get("TCC_HIT_sum"), e.get("TCC_MISS_sum")
        out[short] = {"fetch_bytes_per_frame": fb, "write_bytes_per_frame": wb, "bytes_per_frame": fb + wb,
                      "dispatches": e["dispatches"],
                      "tcc_hit_rate": hit / (hit + miss) if hit is not None and miss and hit + miss > 0 else None}
        wc = e.get("SQ_WAVE_CYCLES")
        if wc:  # what the kernel's waves spend their cycles on, measured in this run
            out[short]["wave_cycles"] = {
                "waiting": e.get("SQ_WAIT_ANY", 0.0) / wc, "issuing_any": e.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
                "issuing_valu": e.get("SQ_ACTIVE_INST_VALU", 0.0) / wc,
                "issuing_flat": e.get("SQ_ACTIVE_INST_FLAT", 0.0) / wc,
                "waiting_to_issue": e.get("SQ_WAIT_INST_ANY", 0.0) / wc}
    return out


# ---------------------------------------------------------------- CPU baseline
def cpu_baseline(cfg, scene, budget_s, spp, bvh, leaf_max):
    """Oracle render of a bounded sample of the same frame (tiles spread over the frame,
    full spp when it fits the budget), timed on the CPUs this process may use, on the tree
    the GPU figure uses (like for like) and on izpi's own NewBVH4 tree; half the budget each."""
    import ctypes as C
    import numpy as np
    from izpi_amd import _native as N
    from izpi_amd.renderer import GPU_BVH_METHOD, common_tiles
    from oracle import oracle as O
    cpus = host_cpus()
    threads = cpus["usable"]
    tiles = common_tiles(cfg.width, cfg.height)
    px_per_tile = int((tiles[0, 2] - tiles[0, 0] + 1) * (tiles[0, 3] - tiles[0, 1] + 1))

    def measure(o, budget):
        def run(ts, s):
            req = N.RenderReq(width=cfg.width, height=cfg.height, spp=s, max_depth=cfg.max_depth, sampler=cfg.sampler,
                              seed=12345)
            t = np.ascontiguousarray(ts, np.uint32)
            req.num_tiles = len(t)
            req.tiles = t.ctypes.data_as(C.POINTER(C.c_uint32))
            _, st = o.render(req, threads=threads)
            return st
        # calibrate on one tile per thread at 2 spp, then size the sample for the budget
        st = run(tiles[:threads], 2)
        rate = st["samples"] / max(st["seconds"], 1e-6)
        want_samples = rate * budget
        s = spp
        ntiles = int(want_samples // (px_per_tile * s))
        if ntiles < threads:
            ntiles = threads
            s = max(1, int(want_samples // (px_per_tile * ntiles)))
        ntiles = min(ntiles, len(tiles))
        stride = max(1, len(tiles) // ntiles)
        st = run(tiles[::stride][:ntiles], s)
        return st["samples"] / st["seconds"] / 1e6, "%d evenly spread tiles (%d px) x %d spp = %d samples, %.1f s" % (
            ntiles, ntiles * px_per_tile, s, st["samples"], st["seconds"])

    o = O.OracleScene(scene, aspect_override=cfg.width / cfg.height)
    ref_value, ref_sample = measure(o, budget_s / 2)
    value, sample, tree = ref_value, ref_sample, "izpi's own NewBVH4 tree"
    if bvh == "gpu":  # the GPU-built tree, restated on the CPU node for node (oracle.lbvh4)
        nodes, order = O.lbvh4(o.prim_boxes(), leaf_max, GPU_BVH_METHOD)
        o.set_bvh(nodes, order)
        value, sample = measure(o, budget_s / 2)
        tree = "the GPU-built PLOC tree (the tree of `value`)"
    o.close()
    res = {"value": value, "unit": "Msamples/s", "cores": threads, "kind": "port",
           "sample": "%s: %s on %d threads of the CPU oracle (C++ restatement of the Go hot path, per-sample RNG "
                     "streams) on %s; on izpi's own tree: %s" % (cfg.name, sample, threads, tree, ref_sample),
           "tree": "gpu" if bvh == "gpu" else "reference", "value_reference_tree": ref_value,
           "cpu_model": cpus["model"], "host_threads": cpus["host_threads"], "affinity_cpus": cpus["affinity"],
           "cgroup_cpus": cpus["cgroup_cpus"]}
    if cpus["host_threads"] and cpus["host_threads"] > threads:
        # the box gives this process `threads` CPUs of a larger host: linear extrapolation to
        # every hardware thread of the host (an upper bound: SMT siblings add less than a core)
        res["extrapolated_all_host_threads"] = value * cpus["host_threads"] / threads
    return res


# ---------------------------------------------------------------- launcher plumbing
def dist_setup(world, rank):
    """gloo group for the launcher's barrier / id broadcast / max of times (CPU only)."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def dry_run(args, world, rank, mode):
    """The launcher without GPU work: share dealing over the frame (izpi_host_share_tiles),
    barriers and the max of per-rank times; prints the JSON skeleton on rank 0."""
    import numpy as np
    from izpi_amd import configs, sharding
    from izpi_amd.renderer import common_tiles
    cfg = configs.configs()[args.config]
    tiles = common_tiles(cfg.width, cfg.height)
    n = world if mode == "ranks" else (args.gpus or 1)
    dist = dist_setup(world, rank) if mode == "ranks" else None
    mine = [sharding.shard_tiles(tiles, r, n) for r in range(n)] if mode != "ranks" else \
        [sharding.shard_tiles(tiles, rank, n)]
    t0 = time.perf_counter()
    covered = sum(len(m) for m in mine)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        dist.barrier()
        tc = torch.tensor([covered, elapsed], dtype=torch.float64)
        dist.all_reduce(tc[:1], op=dist.ReduceOp.SUM)
        e = tc[1:].clone()
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        covered, elapsed = int(tc[0].item()), float(e.item())
    if rank == 0:
        line = {"metric": "Msamples/sec (pixels x spp) at 1024x1024/512spp", "value": None, "unit": "Msamples/s",
                "n_gpus": n, "steps": args.steps, "warmup": args.warmup, "dry_run": True, "mode": mode,
                "config": {"workload": cfg.name, "parallelism": "tiles%d" % n},
                "tiles": int(len(tiles)), "tiles_covered": covered,
                "max_share_tiles": int(max(len(sharding.shard_tiles(tiles, r, n)) for r in range(n)))}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


# ---------------------------------------------------------------- main
def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if env_world is not None and world > 1:
        mode = "ranks"
        if args.gpus is not None and args.gpus != world:
            sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d (one rank per GPU)" % (args.gpus, world))
        n_gpus = world
    else:
        world, rank = 1, 0
        n_gpus = args.gpus or 1
        mode = "threads" if n_gpus > 1 else "single"
    if args.dry_run:
        return dry_run(args, world, rank, mode)

    import numpy as np
    import torch
    from izpi_amd import build
    dist = dist_setup(world, rank) if mode == "ranks" else None
    # one rank (re)builds the library when its sources are newer, the others wait for it
    if dist is None or rank == 0:
        build.build_gpu(verbose=False)
    if dist is not None:
        dist.barrier()
    from izpi_amd import _native as N
    from izpi_amd.renderer import GPURenderer, MultiGPURenderer
    cfg, scene, scene_s = load_config(args)
    spp = args.spp or cfg.spp
    post = N.POST_SPECTRAL if cfg.sampler == N.SAMPLER_SPECTRAL else N.POST_NONE
    if mode != "threads":
        torch.cuda.set_device(local)
    # torch's own HIP context starts lazily with its first tensor: start it here, so that
    # detail.first_frame_ms is the renderer's first frame (what leader.go:155-158 sees)
    for d in ([local] if mode != "threads" else range(n_gpus)):
        torch.zeros(1, device="cuda:%d" % d)

    def sync_all():
        if mode == "threads":
            for d in range(n_gpus):
                torch.cuda.synchronize(d)
        else:
            torch.cuda.synchronize()

    acc_main = N.ACC_FORWARD if args.accumulation == "forward" else N.ACC_RECURSIVE

    def timed(bvh, steps, warmup, keep=False, reuse=None, acc=None, retree=True, host_canvas=False):
        """warmup untimed + `steps` timed frames; returns (elapsed, per-step stats sums of
        this process's device(s), canvas, info). keep: leave the (single-GPU) renderer open
        and return it as info["renderer"]; reuse: such a renderer, whose context and render
        buffers take the scene again with the `bvh` tree when `retree` (one workspace per
        process: the driver clears every byte a process touched before handing it to the next
        one). acc: the accumulation mode (N.ACC_*, default the run's). host_canvas: each step
        returns the canvas to host memory as izpi_gpu_render does for the Go shim."""
        acc = acc_main if acc is None else acc
        ts = time.time()
        if reuse is not None:
            r = reuse
            r.accumulation = acc
            if retree:
                r.use_tree(scene, bvh, bvh_leaf_max=args.bvh_leaf_max)
            canvas_holder = {}

            def step():
                if host_canvas:
                    canvas_holder["c"] = r.render(post=post)
                    return [r.stats]
                canvas, st = r.render_distributed(rank, world, post=post)
                canvas_holder["c"] = canvas
                return [st]
        elif mode == "threads":
            r = MultiGPURenderer(scene, cfg.width, cfg.height, spp, list(range(n_gpus)), max_depth=cfg.max_depth,
                                 sampler=cfg.sampler, bvh=bvh, bvh_leaf_max=args.bvh_leaf_max, accumulation=acc)

            def step():
                r.render(post=post, to_host=False)
                return r.stats
        else:
            r = GPURenderer(scene, cfg.width, cfg.height, spp, max_depth=cfg.max_depth, sampler=cfg.sampler,
                            device=local, bvh=bvh, bvh_leaf_max=args.bvh_leaf_max, accumulation=acc)
            if mode == "ranks":
                cid = bytearray(N.COMM_ID_BYTES)
                if rank == 0:
                    import ctypes as C
                    buf = (C.c_uint8 * N.COMM_ID_BYTES)()
                    if N.lib().izpi_gpu_comm_id(buf) != 0:
                        raise RuntimeError("izpi_gpu_comm_id failed")
                    cid = bytearray(bytes(buf))
                obj = [bytes(cid)]
                dist.broadcast_object_list(obj, src=0)
                r.comm_init(world, rank, obj[0])
            canvas_holder = {}

            def step():  # Render(): spectral configs include FireflyRejection + XYZToRGB (renderer.go:215-219)
                canvas, st = r.render_distributed(rank, world, post=post)
                canvas_holder["c"] = canvas
                return [st]
        # render.New's part (renderer.go:73-104): the workspace, sized and first touched, outside
        # Render (izpi times Render alone, renderer.go:170,213); a reused renderer keeps its own
        if reuse is None:
            r.prepare(post=post)
        setup = time.time() - ts
        first_ms = first_alloc_ms = first_dev = None
        for i in range(warmup):
            t = time.perf_counter()
            sts = step()
            sync_all()
            print("bench: warmup frame %d: %.1f ms" % (i, (time.perf_counter() - t) * 1e3), file=sys.stderr, flush=True)
            if i == 0:
                first_ms = (time.perf_counter() - t) * 1e3
                # host time of the workspace allocation inside that frame (hipMalloc of fresh
                # VRAM: its cost depends on what the box's driver must clear first)
                first_alloc_ms = max((x or {}).get("alloc_ms", 0.0) for x in sts)
                first_dev = {k: max((x or {}).get(k, 0.0) for x in sts) for k in ("total_ms", "kernel_ms", "shade_ms", "tail_ms")}
        if dist is not None:
            dist.barrier()
        sync_all()
        t1 = time.perf_counter()
        agg = {k: 0.0 for k in STAT_KEYS}
        for k in range(steps):
            for st in step():
                add_stats(agg, st)
            if rank == 0 and (k + 1) % max(1, steps // 4) == 0:  # progress (long frames: C5 takes ~2 min)
                print("bench: %d of %d timed frames issued" % (k + 1, steps), file=sys.stderr, flush=True)
        sync_all()
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t1
        if dist is not None:
            e = torch.tensor([elapsed], dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            elapsed = float(e.item())
        last = r.stats[0] if mode == "threads" else r.stats
        info = {"triangles": int(r.host.desc.num_tris), "nodes": int(r.host.desc.num_nodes),
                "leaf_max": getattr(r, "bvh_leaf_max", None),
                "build_ms": r.bvh_build_ms if bvh == "gpu" else r.host.build_ms, "setup_s": setup,
                "first_frame_ms": first_ms, "first_frame_alloc_ms": first_alloc_ms, "first_frame_device": first_dev, "workspace_gb": (last or {}).get("workspace_bytes", 0) / 1e9,
                "scene_gb": (last or {}).get("scene_bytes", 0) / 1e9, "slots": (last or {}).get("slots"),
                "rec_dense": (last or {}).get("rec_dense"), "pool_blocks": (last or {}).get("pool_blocks"),
                "chunk_spp": (last or {}).get("chunk_spp")}
        img = None
        if mode == "threads":  # one more frame, to the host, for the image summary
            img = r.render(post=post)
        elif rank == 0:
            c = canvas_holder.get("c")
            img = None if c is None else c if isinstance(c, np.ndarray) else c.cpu().numpy()
        if keep and mode == "single":
            info["renderer"] = r
        elif reuse is None:  # (a reused renderer stays open: its owner closes it)
            r.close()
        return elapsed, agg, img, info

    if args.pmc_child:  # one frame under rocprofv3 --pmc (the parent reads the counters)
        elapsed, agg, img, info = timed(args.bvh, 1, 0)
        print(json.dumps({"pmc_child": True, "ms": elapsed * 1e3}), flush=True)
        return

    want_checks = mode == "single" and not args.no_reference_check
    elapsed, agg, img, info = timed(args.bvh, args.steps, args.warmup, keep=want_checks)
    kept = info.pop("renderer", None)
    samples_per_step = cfg.width * cfg.height * spp
    value = samples_per_step * args.steps / elapsed / 1e6
    ref_check = acc_check = host_check = None
    rsteps = min(args.steps, 3)
    if want_checks:
        # izpi_gpu_render's form: the canvas back in host memory, as the Go shim's Render
        # returns it (renderer.go:26-28); the timed frames above leave it in device memory
        h_elapsed, h_agg, _, _ = timed(args.bvh, rsteps, 0, reuse=kept, retree=False, host_canvas=True)
        host_check = {"value": round(samples_per_step * rsteps / h_elapsed / 1e6, 3),
                      "ms_per_step": round(h_elapsed / rsteps * 1e3, 3), "steps": rsteps}
    if want_checks and acc_main == N.ACC_FORWARD:
        # The same frame through the recursion (IZPI_ACC_RECURSIVE, bit-identical to the CPU
        # oracle), on the same tree and context: the forward form only counts if it is within
        # north_star's tolerance of it (pixel RMSE < 1e-6) with NaN / Inf on the same pixels.
        a_elapsed, a_agg, a_img, a_info = timed(args.bvh, rsteps, 1, reuse=kept, acc=N.ACC_RECURSIVE, retree=False)
        fin = np.isfinite(img) & np.isfinite(a_img)
        rmse = float(np.sqrt(np.mean((img[fin] - a_img[fin]) ** 2))) if fin.any() else 0.0
        rel = np.abs(img[fin] - a_img[fin]) / np.maximum(np.abs(a_img[fin]), 1e-300)
        same_special = bool(np.array_equal(np.isnan(img), np.isnan(a_img)) and
                            np.array_equal(np.isinf(img) & (img > 0), np.isinf(a_img) & (a_img > 0)) and
                            np.array_equal(np.isinf(img) & (img < 0), np.isinf(a_img) & (a_img < 0)))
        a_value = samples_per_step * rsteps / a_elapsed / 1e6
        counters_equal = all(a_agg[k] / rsteps == agg[k] / args.steps for k in
                             ("rays", "node_visits", "tri_tests", "sph_tests", "light_tri_tests", "light_sph_tests"))
        acc_check = {"accumulation": "recursive", "value": round(a_value, 3),
                     "ms_per_step": round(a_elapsed / rsteps * 1e3, 3), "steps": rsteps,
                     "image_rmse": rmse, "image_max_rel_err": float(rel.max()) if rel.size else 0.0,
                     "image_bitwise_equal": img.tobytes() == a_img.tobytes(),
                     "nan_inf_positions_equal": same_special, "counters_equal": bool(counters_equal),
                     "trace_ms_per_step": a_agg["kernel_ms"] / rsteps, "shade_ms_per_step": a_agg["shade_ms"] / rsteps,
                     "first_frame_ms": a_info["first_frame_ms"], "hbm_workspace_gb": round(a_info["workspace_gb"], 2)}
        if not (rmse < 1e-6 and same_special and counters_equal):
            print("WARNING: forward accumulation differs from the recursion beyond north_star's tolerance (rmse %g); "
                  "reporting the recursion" % rmse, file=sys.stderr)
            elapsed, agg, img = a_elapsed * args.steps / rsteps, a_agg, a_img
            for k in agg:
                agg[k] *= args.steps / rsteps
            value = a_value
            args.accumulation = "recursive"
            acc_main = N.ACC_RECURSIVE
    if want_checks and args.bvh == "gpu":
        # The same frame on hitable.NewBVH4's own tree (rebuilt bit for bit on the host):
        # the GPU-built tree only counts if its image is the reference tree's image. Same
        # context, render buffers and accumulation as the timed frames.
        r_elapsed, r_agg, r_img, r_info = timed("reference", rsteps, 1, reuse=kept)
        equal = img.tobytes() == r_img.tobytes()
        rmse = float(np.sqrt(np.mean((img - r_img) ** 2)))
        ref_value = samples_per_step * rsteps / r_elapsed / 1e6
        ref_check = {"value": round(ref_value, 3), "ms_per_step": round(r_elapsed / rsteps * 1e3, 3),
                     "steps": rsteps, "image_bitwise_equal": equal, "image_rmse": rmse,
                     "node_visits_per_ray": r_agg["node_visits"] / max(r_agg["rays"], 1),
                     "trace_ms_per_step": r_agg["kernel_ms"] / rsteps,
                     "shade_ms_per_step": r_agg["shade_ms"] / rsteps, "bvh_build_ms": r_info["build_ms"]}
        if not rmse < 1e-6:  # north-star tolerance: fall back to the reference tree's numbers
            print("WARNING: GPU-built BVH image differs from the reference tree's (rmse %g); reporting the "
                  "reference tree" % rmse, file=sys.stderr)
            elapsed, agg, img, info = r_elapsed * args.steps / rsteps, r_agg, r_img, r_info
            for k in agg:
                agg[k] *= args.steps / rsteps
            value = ref_value
            args.bvh = "reference"
    if kept is not None:
        kept.close()

    # dominant kernel: k_trace2 (the traversals k_tail runs at the end of the frame are counted apart)
    steps = args.steps
    trace_ms_frame = agg["kernel_ms"] / steps / (n_gpus if mode == "threads" else 1)
    trace_bytes = (128.0 * (agg["node_visits"] - agg["tail_node_visits"]) + 72.0 * (agg["tri_tests"] - agg["tail_tri_tests"])
                   + 32.0 * (agg["sph_tests"] - agg["tail_sph_tests"]))
    alg_frame = trace_bytes / steps / (n_gpus if mode == "threads" else 1)
    achieved_alg = alg_frame / (trace_ms_frame * 1e-3) / 1e9 if trace_ms_frame > 0 else 0.0
    launches = max(agg["launches"] / steps, 1.0)
    if rank != 0:
        dist.destroy_process_group()
        return
    pmc = traffic_summary(pmc_children(args)) if (mode == "single" and not args.no_pmc) else {}
    roof = {"bound": "hbm", "kernel": "k_trace2", "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "achieved": None, "frac": None, "traffic": None,
            "achieved_algorithmic": round(achieved_alg, 2),
            "algorithmic_bytes_per_launch": alg_frame / launches,
            "avg_launch_ms": trace_ms_frame / launches, "launches_per_frame": launches}
    if "k_trace2" in pmc:
        t = pmc["k_trace2"]
        roof["traffic"] = t["bytes_per_frame"] / max(t["dispatches"], 1)  # L2 memory-side bytes per launch
        roof["achieved"] = round(t["bytes_per_frame"] / (trace_ms_frame * 1e-3) / 1e9, 2)
        roof["frac"] = round(roof["achieved"] / HBM_PEAK_GBS, 5)
        # What `frac` measures, level by level: FETCH_SIZE / WRITE_SIZE count the
        # L2's memory-side requests, Infinity-Cache hits included, so `achieved` is the L2-miss
        # fabric rate, an upper bound of the HBM rate. The same bytes against the measured
        # Infinity-Cache random-gather rate, and the algorithmic bytes against the L2's rate:
        roof["levels"] = {
            "l2_miss_fabric_frac": roof["frac"],
            "mall_frac": round(roof["achieved"] / MALL_GATHER_GBS, 5),
            "l2_frac": round(achieved_alg / L2_PEAK_GBS, 5),
            "mall_gather_gbs": MALL_GATHER_GBS, "l2_gbs": L2_PEAK_GBS,
            # FETCH_SIZE x 2 = 128 B per line requested past L2, checked for this kernel's access
            # shapes (16-B streams, 128-B nodes, 80-B records, 48-B runs, 32-B partial reads) by
            # tools/fetch_calib (profiles/r4a/fetch_calib.jsonl)
            "fetch_correction": "x2, calibrated",
        }
        lv = {k: roof["levels"][k] for k in ("l2_miss_fabric_frac", "mall_frac", "l2_frac")}
        roof["levels"]["nearest_ceiling"] = max(lv, key=lv.get)
        rays_frame = agg["rays"] / steps  # sampler rays (k_tail's few included)
        if rays_frame > 0:
            roof["bytes_per_ray_past_l2"] = {"fetch": round(t["fetch_bytes_per_frame"] / rays_frame, 2),
                                             "write": round(t["write_bytes_per_frame"] / rays_frame, 2)}
        roof["traffic_per_frame"] = t["bytes_per_frame"]
        roof["fetch_per_frame"] = t["fetch_bytes_per_frame"]
        roof["write_per_frame"] = t["write_bytes_per_frame"]
        roof["tcc_hit_rate"] = t["tcc_hit_rate"]
        roof["pmc_dispatches"] = t["dispatches"]
        if "wave_cycles" in t:  # SQ counters of the same workload: fractions of k_trace2's wave cycles
            roof["wave_cycles"] = {k: round(v, 4) for k, v in t["wave_cycles"].items()}
        if "k_shade" in pmc:
            s = pmc["k_shade"]
            roof["k_shade"] = {"bytes_per_frame": s["bytes_per_frame"], "fetch_per_frame": s["fetch_bytes_per_frame"],
                               "write_per_frame": s["write_bytes_per_frame"], "tcc_hit_rate": s["tcc_hit_rate"],
                               "achieved": round(s["bytes_per_frame"] / (agg["shade_ms"] / steps * 1e-3) / 1e9, 2)}
            if "wave_cycles" in s:
                roof["k_shade"]["wave_cycles"] = {k: round(v, 4) for k, v in s["wave_cycles"].items()}
    elif pmc.get("error"):
        roof["pmc_error"] = pmc["error"]
    cpu = None
    if mode == "single" and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, scene, args.cpu_seconds, spp, args.bvh, info.get("leaf_max"))
        # like for like: the GPU and the CPU oracle on the same tree
        cpu["gpu_speedup"] = value / cpu["value"]
        if ref_check and cpu.get("value_reference_tree"):
            cpu["gpu_speedup_reference_tree"] = ref_check["value"] / cpu["value_reference_tree"]
        if cpu.get("extrapolated_all_host_threads"):
            cpu["gpu_speedup_vs_extrapolated"] = value / cpu["extrapolated_all_host_threads"]
    line = {
        "metric": "Msamples/sec (pixels x spp) at 1024x1024/512spp",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        # a fresh renderer's first frame, workspace allocation included: what izpi's leader
        # sees, which renders one frame per process (leader.go:155-158, renderer.go:170,213)
        "first_frame_msamples": round(samples_per_step / (info["first_frame_ms"] * 1e-3) / 1e6, 3)
        if info.get("first_frame_ms") else None,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic Cornell box + 817k-triangle displaced cube-sphere dragon)",
        "config": {"workload": cfg.name, "width": cfg.width, "height": cfg.height, "spp": spp,
                   "max_depth": cfg.max_depth, "triangles": info["triangles"],
                   "bvh4_nodes": info["nodes"], "bvh": args.bvh, "bvh_leaf_max": info["leaf_max"],
                   "accumulation": args.accumulation, "parallelism": "tiles%d" % n_gpus, "mode": mode,
                   "samples_per_step": samples_per_step},
        "roofline": roof,
        "cpu_baseline": cpu,
        "detail": {
            "first_frame_ms": info["first_frame_ms"],
            "first_frame_alloc_ms": info["first_frame_alloc_ms"],
            # the first frame's device times (render call, k_trace2, k_shade, k_tail), against
            # rank0_*_ms_per_step below: what the extra host time of the first frame is not
            "first_frame_device_ms": info["first_frame_device"],
            "setup_s": round(info["setup_s"], 3),
            "hbm_workspace_gb": round(info["workspace_gb"], 2),
            "hbm_scene_gb": round(info["scene_gb"], 3),
            "slots": info["slots"], "rec_dense": info["rec_dense"], "pool_blocks": info["pool_blocks"],
            "chunk_spp": info["chunk_spp"],
            "rank0_trace_ms_per_step": agg["kernel_ms"] / steps,
            "rank0_shade_ms_per_step": agg["shade_ms"] / steps,
            "rank0_tail_ms_per_step": agg["tail_ms"] / steps,
            "rank0_render_ms_per_step": agg["total_ms"] / steps,
            "rank0_rays_per_step": agg["rays"] / steps,
            "rank0_parks_per_step": agg["parks"] / steps,
            "rank0_node_visits_per_ray": agg["node_visits"] / max(agg["rays"], 1),
            "rank0_tri_tests_per_ray": agg["tri_tests"] / max(agg["rays"], 1),
            # k_trace2 SIMD efficiency: useful lane-steps / (64 x wave-level steps)
            "rank0_node_step_lane_util": (agg["node_visits"] - agg["tail_node_visits"] - agg["leaf_shortcuts"]) /
                                         max(64 * agg["node_steps"], 1),
            "rank0_prim_step_lane_util": (agg["tri_tests"] + agg["sph_tests"] - agg["tail_tri_tests"] - agg["tail_sph_tests"]) /
                                         max(64 * agg["prim_steps"], 1),
            "rank0_leaf_shortcut_frac": agg["leaf_shortcuts"] / max(agg["node_visits"], 1),
            "scene_gen_s": round(scene_s, 2),
            "bvh_build_ms": info["build_ms"],
            "reference_tree": ref_check,
            "accumulation_check": acc_check,
            "host_canvas": host_check,
            "image_mean_rgb": [float(x) for x in img[1:, :, :3].mean(axis=(0, 1))] if img is not None else None,
        },
    }
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
