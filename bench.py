"""Benchmark: Msamples/s (pixels x spp) of the izpi path-tracing inner loop on MI355X.

Workload (BASELINE.json metric "Msamples/sec at 1024x1024/512spp"): config C3 — the
Cornell box with the synthetic ~817k-triangle dragon, Colour sampler, maxDepth 50,
1024x1024 pixels x 512 spp = 536,870,912 samples per frame.

One step = one full frame through the hot path (BVH4 traversal, shading, light pdfs,
ordered per-pixel accumulation) with the scene already resident in HBM. With N GPUs
(one process each, torchrun) the frame's 32x32 tiles are dealt round-robin to ranks
and the packed tiles are gathered to rank 0 over RCCL inside the timed step
(strong scaling: total work fixed). Timing: barrier + synchronize on both sides of
the K timed steps, max over ranks.

The JSON line also carries
  roofline:     achieved algorithmic GB/s of the dominant kernel (k_trace) — node,
                triangle and sphere bytes of SURVEY.md §8(d) counted exactly by the
                kernel (== oracle counts) over its HIP-event time — against 8 TB/s.
  cpu_baseline: the CPU oracle (deterministic restatement of the Go hot path) on a
                bounded sample of the same frame on this host's cores (rank 0, N=1).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", default="C3")
    p.add_argument("--spp", type=int, default=None, help="override spp (debug only; the metric uses 512)")
    p.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--scene", default=None, help="render a transport.Scene file (.pbtxt/.izpi) at the config's size")
    p.add_argument("--bvh", default="gpu", choices=["reference", "gpu"],
                   help="gpu (default): the GPU linear BVH4 builder, checked at N=1 against a frame on the "
                        "reference tree; reference: hitable.NewBVH4's tree rebuilt bit for bit on the host")
    p.add_argument("--bvh-leaf-max", type=int, default=None, help="primitives per leaf of the GPU-built tree")
    p.add_argument("--no-reference-check", action="store_true",
                   help="skip the reference-tree frame (timing and image comparison) of --bvh gpu")
    p.add_argument("--obj", default=None, help="C3 with this OBJ mesh (e.g. the Stanford dragon) instead of the "
                                               "synthetic one")
    return p.parse_args()


def pmc_traffic(config):
    """HBM bytes per k_trace launch from the committed rocprofv3 PMC pass, if any
    (keyed "<config>/<bvh>", e.g. "C3/gpu")."""
    f = ROOT / "profiles" / "pmc_summary.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        return d.get(config, {}).get("hbm_bytes_per_trace_launch")
    except Exception:
        return None


def cpu_baseline(cfg, scene, budget_s, spp):
    """Oracle render of a bounded sample of the same frame (centre tiles, full spp when
    it fits the budget), timed on this host's cores."""
    import numpy as np
    from izpi_amd import _native as N
    from izpi_amd.renderer import common_tiles
    from oracle import oracle as O
    threads = max(1, min(16, os.cpu_count() or 1))
    o = O.OracleScene(scene, aspect_override=cfg.width / cfg.height)
    tiles = common_tiles(cfg.width, cfg.height)
    # calibrate on one tile at 2 spp, then size the sample for the budget
    def run(ts, s):
        req = N.RenderReq(width=cfg.width, height=cfg.height, spp=s, max_depth=cfg.max_depth, sampler=cfg.sampler,
                          seed=12345)
        t = np.ascontiguousarray(ts, np.uint32)
        req.num_tiles = len(t)
        req.tiles = t.ctypes.data_as(__import__("ctypes").POINTER(__import__("ctypes").c_uint32))
        _, st = o.render(req, threads=threads)
        return st
    st = run(tiles[:threads], 2)
    rate = st["samples"] / max(st["seconds"], 1e-6)
    px_per_tile = int((tiles[0, 2] - tiles[0, 0] + 1) * (tiles[0, 3] - tiles[0, 1] + 1))
    want_samples = rate * budget_s
    s = spp
    ntiles = int(want_samples // (px_per_tile * s))
    if ntiles < threads:
        ntiles = threads
        s = max(1, int(want_samples // (px_per_tile * ntiles)))
    ntiles = min(ntiles, len(tiles))
    stride = max(1, len(tiles) // ntiles)
    st = run(tiles[::stride][:ntiles], s)  # tiles spread over the whole frame
    o.close()
    return {"value": st["samples"] / st["seconds"] / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "%s: %d evenly spread tiles (%d px) x %d spp = %d samples, %.1f s on %d threads of the CPU oracle "
                      "(C++ restatement of the Go hot path, per-sample RNG streams)"
                      % (cfg.name, ntiles, ntiles * px_per_tile, s, st["samples"], st["seconds"], threads)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    from izpi_amd import build
    build.build_gpu(verbose=False)
    from izpi_amd import configs
    from izpi_amd.renderer import GPURenderer

    cfg = configs.configs()[args.config]
    spp = args.spp or cfg.spp
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
    scene_s = time.time() - t0
    from izpi_amd import _native as N
    post = N.POST_SPECTRAL if cfg.sampler == N.SAMPLER_SPECTRAL else N.POST_NONE
    keys = ("node_visits", "tri_tests", "sph_tests", "light_tri_tests", "light_sph_tests", "rays", "kernel_ms",
            "shade_ms", "total_ms", "launches", "samples", "node_steps", "prim_steps", "leaf_shortcuts", "tail_ms",
            "tail_node_visits", "tail_tri_tests", "tail_sph_tests")

    def timed(bvh):
        """W untimed + K timed frames on tree `bvh`; returns (elapsed, stats sums, canvas, renderer info)."""
        ts = time.time()
        r = GPURenderer(scene, cfg.width, cfg.height, spp, max_depth=cfg.max_depth, sampler=cfg.sampler, device=local,
                        bvh=bvh, bvh_leaf_max=args.bvh_leaf_max)
        setup = time.time() - ts

        def step():  # Render(): spectral configs include FireflyRejection + XYZToRGB (renderer.go:215-219)
            return r.render_distributed(rank, world, post=post)

        for _ in range(args.warmup):
            step()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        agg = {k: 0.0 for k in keys}
        canvas = None
        for _ in range(args.steps):
            canvas, st = step()
            for k in agg:
                agg[k] += float(st[k]) if st else 0.0
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t1
        if world > 1:
            e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            elapsed = float(e.item())
        info = {"triangles": int(r.host.desc.num_tris), "nodes": int(r.host.desc.num_nodes),
                "build_ms": r.bvh_build_ms if bvh == "gpu" else r.host.build_ms, "setup_s": setup}
        img = canvas.cpu().numpy() if canvas is not None else None
        r.close()
        return elapsed, agg, img, info

    elapsed, agg, img, info = timed(args.bvh)
    setup_s = info["setup_s"]  # host scene (+ reference BVH) build and upload of the timed renderer
    samples_per_step = cfg.width * cfg.height * spp
    value = samples_per_step * args.steps / elapsed / 1e6
    ref_check = None
    if world == 1 and args.bvh == "gpu" and not args.no_reference_check:
        # The same frame on hitable.NewBVH4's own tree (rebuilt bit for bit on the host):
        # the GPU-built tree only counts if its image is the reference tree's image.
        import numpy as np
        r_elapsed, r_agg, r_img, r_info = timed("reference")
        equal = img.tobytes() == r_img.tobytes()
        rmse = float(np.sqrt(np.mean((img - r_img) ** 2)))
        ref_value = samples_per_step * args.steps / r_elapsed / 1e6
        ref_check = {"value": round(ref_value, 3), "ms_per_step": round(r_elapsed / args.steps * 1e3, 3),
                     "image_bitwise_equal": equal, "image_rmse": rmse,
                     "node_visits_per_ray": r_agg["node_visits"] / max(r_agg["rays"], 1),
                     "trace_ms_per_step": r_agg["kernel_ms"] / args.steps,
                     "shade_ms_per_step": r_agg["shade_ms"] / args.steps, "bvh_build_ms": r_info["build_ms"]}
        if not rmse < 1e-6:  # north-star tolerance: fall back to the reference tree's numbers
            print("WARNING: GPU-built BVH image differs from the reference tree's (rmse %g); reporting the "
                  "reference tree" % rmse, file=sys.stderr)
            elapsed, agg, img, info, value = r_elapsed, r_agg, r_img, r_info, ref_value
            args.bvh = "reference"

    # roofline of the dominant kernel on this rank: algorithmic bytes / k_trace2 time
    # (the traversals k_tail runs at the end of the frame are counted apart)
    trace_bytes = (128.0 * (agg["node_visits"] - agg["tail_node_visits"]) + 72.0 * (agg["tri_tests"] - agg["tail_tri_tests"])
                   + 32.0 * (agg["sph_tests"] - agg["tail_sph_tests"]))
    achieved = trace_bytes / (agg["kernel_ms"] * 1e-3) / 1e9 if agg["kernel_ms"] > 0 else 0.0
    launches = max(agg["launches"], 1.0)
    traffic = pmc_traffic("%s/%s" % (args.config, args.bvh))
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, scene, args.cpu_seconds, spp)
    line = {
        "metric": "Msamples/sec (pixels x spp) at 1024x1024/512spp",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic Cornell box + 817k-triangle displaced cube-sphere dragon)",
        "config": {"workload": cfg.name, "width": cfg.width, "height": cfg.height, "spp": spp,
                   "max_depth": cfg.max_depth, "triangles": info["triangles"],
                   "bvh4_nodes": info["nodes"], "bvh": args.bvh, "parallelism": "tiles%d" % world,
                   "samples_per_step": samples_per_step},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": traffic,
                     "kernel": "k_trace2", "algorithmic_bytes_per_launch": trace_bytes / launches,
                     "avg_launch_ms": agg["kernel_ms"] / launches, "launches": int(agg["launches"])},
        "cpu_baseline": cpu,
        "detail": {
            "rank0_trace_ms_per_step": agg["kernel_ms"] / args.steps,
            "rank0_shade_ms_per_step": agg["shade_ms"] / args.steps,
            "rank0_tail_ms_per_step": agg["tail_ms"] / args.steps,
            "rank0_render_ms_per_step": agg["total_ms"] / args.steps,
            "rank0_rays_per_step": agg["rays"] / args.steps,
            "rank0_node_visits_per_ray": agg["node_visits"] / max(agg["rays"], 1),
            "rank0_tri_tests_per_ray": agg["tri_tests"] / max(agg["rays"], 1),
            # k_trace2 SIMD efficiency: useful lane-steps / (64 x wave-level steps)
            "rank0_node_step_lane_util": (agg["node_visits"] - agg["tail_node_visits"] - agg["leaf_shortcuts"]) /
                                         max(64 * agg["node_steps"], 1),
            "rank0_prim_step_lane_util": (agg["tri_tests"] + agg["sph_tests"] - agg["tail_tri_tests"] - agg["tail_sph_tests"]) /
                                         max(64 * agg["prim_steps"], 1),
            "rank0_leaf_shortcut_frac": agg["leaf_shortcuts"] / max(agg["node_visits"], 1),
            "scene_gen_s": round(scene_s, 2),
            "setup_s": round(setup_s, 2),
            "bvh_build_ms": info["build_ms"],
            "reference_tree": ref_check,
            "image_mean_rgb": [float(x) for x in img[1:, :, :3].mean(axis=(0, 1))] if img is not None else None,
        },
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
