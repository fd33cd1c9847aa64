"""GPU parity of IZPI_ACC_FORWARD (the forward-throughput accumulation, include/izpi_gpu.h).

Two checks per case:
* the kernels' forward mode == the oracle's restatement of it (ColourSampler::SampleForward,
  SpectralSampler::SampleSpectralForward) bit for bit, counters equal;
* the kernels' forward mode against the oracle's recursion (colour.go:33-65,
  sampler/spectral.go:47-80): pixel RMSE < 1e-6 (north_star), NaN / Inf at the same pixels,
  counters equal (tests/test_forward_accumulation.py gives the argument).
At BASELINE.json's sizes: every config's full frame (C3 at 2 spp, the others at 1 spp) and
the frames' centre tiles at their full spp.
"""
import ctypes as C

import numpy as np
import pytest

from izpi_amd import _native as N
from izpi_amd import configs
from izpi_amd.renderer import GPURenderer, MultiGPURenderer, common_tiles
from oracle import oracle as O
from tests.test_forward_accumulation import CASES, assert_within_tolerance, scene_case

pytestmark = pytest.mark.gpu


def oracle_both(scene, W, H, spp, sampler, tiles=None, o=None, threads=16):
    """The oracle's (recursive, forward) canvases and stats."""
    own = o is None
    if own:
        o = O.OracleScene(scene, aspect_override=W / H)
    out = []
    for acc in (N.ACC_RECURSIVE, N.ACC_FORWARD):
        req = N.RenderReq(width=W, height=H, spp=spp, max_depth=50, sampler=sampler, seed=12345,
                          abi_version=N.IZPI_ABI_VERSION, accumulation=acc)
        keep = None
        if tiles is not None:
            keep = np.ascontiguousarray(tiles, np.uint32)
            req.num_tiles = len(keep)
            req.tiles = keep.ctypes.data_as(C.POINTER(C.c_uint32))
        canvas, st = o.render(req, threads=threads)
        out.append((canvas.reshape(H, W, 4), st))
    if own:
        o.close()
    return out


def assert_bitwise(img, ref, stats, ref_stats):
    """Bit-identical canvases (a NaN matches a NaN: payloads are the platform's), equal counters."""
    a, b = img.view(np.uint64), ref.view(np.uint64)
    bad = np.argwhere((a != b) & ~(np.isnan(img) & np.isnan(ref)))
    assert len(bad) == 0, "not bit-identical: %d values differ, first %s" % (len(bad), bad[:5].tolist())
    for k in ("rays", "node_visits", "tri_tests", "sph_tests", "light_tri_tests", "light_sph_tests", "samples"):
        assert stats[k] == ref_stats[k], (k, stats[k], ref_stats[k])


def check_forward(img, stats, ora):
    (rec, rs), (fwd, fs) = ora
    assert stats["rec_dense"] == 0 and stats["pool_blocks"] == 0, stats  # no unwinding records
    assert_bitwise(img, fwd, stats, fs)           # == the oracle's forward form, bit for bit
    return assert_within_tolerance(img, rec, stats, rs)  # == the recursion within north_star's bound


@pytest.mark.parametrize("which", CASES)
def test_forward_small_scenes(gpu, which):
    scene, W, H, spp, sampler = scene_case(which)
    r = GPURenderer(scene, W, H, spp, sampler=sampler, accumulation=N.ACC_FORWARD)
    img = r.render()
    check_forward(img, r.stats, oracle_both(scene, W, H, spp, sampler))
    # the same renderer, back to the recursion: bit-identical to the oracle's
    r.accumulation = N.ACC_RECURSIVE
    img2 = r.render()
    assert r.stats["pool_blocks"] >= 0
    (rec, rs), _ = oracle_both(scene, W, H, spp, sampler)
    assert_bitwise(img2, rec, r.stats, rs)
    r.close()


@pytest.mark.parametrize("tune", [{"flags": N.TUNE_NO_TAIL}, {"slots": 3000}, {"chunk_units": 3000}])
def test_forward_launch_variants(gpu, tune):
    """k_tail or none, few slots (many refills), several chunks of per-sample results."""
    for which in ("glass_spectral", "pbr"):
        scene, W, H, spp, sampler = scene_case(which)
        r = GPURenderer(scene, W, H, spp, sampler=sampler, accumulation=N.ACC_FORWARD, tuning=N.tuning(**tune))
        img = r.render()
        check_forward(img, r.stats, oracle_both(scene, W, H, spp, sampler))
        r.close()


def test_forward_full_size_c3_frame(gpu):
    """BASELINE.json's C3 frame (1024x1024, 817k-triangle dragon) at 2 spp, forward mode."""
    cfg = configs.configs()["C3"]
    scene = cfg.build()
    r = GPURenderer(scene, cfg.width, cfg.height, 2, accumulation=N.ACC_FORWARD)
    img = r.render()
    check_forward(img, r.stats, oracle_both(scene, cfg.width, cfg.height, 2, N.SAMPLER_COLOUR))
    r.close()


@pytest.mark.parametrize("name", ["C1", "C2", "C4", "C5"])
def test_forward_full_size_frames(gpu, name):
    """C1 at its full 16 spp; C2, C4 and C5 as full frames at 1 spp (C5 with the Spectral
    post-processing on both sides)."""
    cfg = configs.configs()[name]
    scene = cfg.build()
    spp = cfg.spp if name == "C1" else 1
    r = GPURenderer(scene, cfg.width, cfg.height, spp, sampler=cfg.sampler, accumulation=N.ACC_FORWARD)
    if cfg.sampler == N.SAMPLER_SPECTRAL:
        img = r.render_spectral_rgb()
        o = O.OracleScene(scene, aspect_override=cfg.width / cfg.height)
        ora = oracle_both(scene, cfg.width, cfg.height, spp, cfg.sampler, o=o)
        ora = [(O.xyz_to_rgb(O.firefly(c.reshape(-1), cfg.width, cfg.height), cfg.width, cfg.height,
                             r.exposure).reshape(cfg.height, cfg.width, 4), st) for c, st in ora]
        o.close()
    else:
        img = r.render()
        ora = oracle_both(scene, cfg.width, cfg.height, spp, cfg.sampler)
    check_forward(img, r.stats, ora)
    r.close()


@pytest.mark.parametrize("name,ntiles,tune", [
    ("C3", 4, None),
    ("C2", 4, None),
    ("C4", 2, None),
    ("C5", 1, {"chunk_units": 1 << 20}),  # 5 chunks of per-sample results, as C5's full frame
])
@pytest.mark.timeout(600)
def test_forward_full_spp_centre_tiles(gpu, name, ntiles, tune):
    """Each config's first tiles in spiral order (the centre) at its FULL spp."""
    cfg = configs.configs()[name]
    scene = cfg.build()
    tiles = common_tiles(cfg.width, cfg.height)[:ntiles]
    r = GPURenderer(scene, cfg.width, cfg.height, cfg.spp, sampler=cfg.sampler, accumulation=N.ACC_FORWARD,
                    tuning=N.tuning(**tune) if tune else None)
    img = r.render(tiles=tiles)
    rmse = check_forward(img, r.stats, oracle_both(scene, cfg.width, cfg.height, cfg.spp, cfg.sampler, tiles=tiles))
    print("%s forward vs recursion: rmse %.3g" % (name, rmse))
    r.close()


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_forward_multi_gpu(gpu, devices):
    """The multi-context fan-out in forward mode: the canvas equals one context's."""
    scene, W, H, spp, sampler = scene_case("glass_spectral")
    m = MultiGPURenderer(scene, W, H, spp, devices, sampler=sampler, bvh="reference", accumulation=N.ACC_FORWARD)
    img = m.render()
    m.close()
    r = GPURenderer(scene, W, H, spp, sampler=sampler, accumulation=N.ACC_FORWARD)
    one = r.render()
    r.close()
    assert img.tobytes() == one.tobytes()


def test_forward_request_checks(gpu):
    """An unknown accumulation mode is refused; an ABI-2 request (abi_version 2: the field
    lies past its end) renders the recursion whatever the bytes there hold."""
    scene = configs.cornell_rgb()
    r = GPURenderer(scene, 24, 24, 2)
    req = r.request()
    req.accumulation = 7
    st = N.RenderStats()
    canvas = np.zeros((24, 24, 4))
    rc = N.lib().izpi_gpu_render(r.ctx, C.byref(req), canvas.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st))
    assert rc == N.IZPI_ERR_INVALID
    req.abi_version = 2
    req.accumulation = N.ACC_FORWARD
    assert N.lib().izpi_gpu_render(r.ctx, C.byref(req), canvas.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)) == 0
    assert st.rec_dense > 0  # the recursion's records
    (rec, _), _ = oracle_both(scene, 24, 24, 2, N.SAMPLER_COLOUR)
    assert canvas.tobytes() == rec.tobytes()
    r.close()


@pytest.mark.parametrize("acc", [N.ACC_FORWARD, N.ACC_RECURSIVE])
def test_prepare_allocates_ahead_of_the_first_frame(gpu, acc):
    """izpi_gpu_prepare sizes and allocates the workspace (render.New's part): the first
    frame after it allocates nothing and renders the same canvas as an unprepared renderer."""
    scene, W, H, spp, sampler = scene_case("pbr")
    r = GPURenderer(scene, W, H, spp, sampler=sampler, accumulation=acc)
    r.prepare()
    img = r.render()
    assert r.stats["alloc_ms"] < 0.5, r.stats["alloc_ms"]  # no allocation left for the frame
    r.close()
    q = GPURenderer(scene, W, H, spp, sampler=sampler, accumulation=acc)
    assert q.render().tobytes() == img.tobytes()
    q.close()


@pytest.mark.parametrize("max_depth", [0, 1, 3])
def test_forward_max_depth(gpu, max_depth):
    """Blue at maxDepth (colour.go:34-36) and the background SPD at depth 0
    (sampler/spectral.go:48-51) in forward mode: a path that starts and ends in k_refill's
    start (maxDepth 0) writes its sample there and leaves a dead entry."""
    for scene, sampler in ((configs.cornell_rgb(), N.SAMPLER_COLOUR), (configs.cornell_glass_spectral(), N.SAMPLER_SPECTRAL)):
        r = GPURenderer(scene, 24, 24, 4, max_depth=max_depth, sampler=sampler, accumulation=N.ACC_FORWARD,
                        tuning=N.tuning(slots=300))  # (few slots: most units start in k_refill)
        img = r.render()
        o = O.OracleScene(scene, aspect_override=1.0)
        out = []
        for acc in (N.ACC_RECURSIVE, N.ACC_FORWARD):
            req = N.RenderReq(width=24, height=24, spp=4, max_depth=max_depth, sampler=sampler, seed=12345,
                              abi_version=N.IZPI_ABI_VERSION, accumulation=acc)
            c, st = o.render(req, threads=8)
            out.append((c.reshape(24, 24, 4), st))
        o.close()
        check_forward(img, r.stats, out)
        r.close()


def test_forward_tiles_packed_and_shares(gpu):
    """A tile subset, packed into device memory and unpacked, and the eighth-shares of a
    frame (izpi_host_share_tiles' deal) in forward mode: each equals the oracle's forward
    form on the same tiles, and the shares assemble into the whole frame's canvas."""
    import torch
    from izpi_amd import sharding
    scene, W, H, spp, sampler = scene_case("glass_rgb_beer")
    W = H = 96
    r = GPURenderer(scene, W, H, spp, sampler=sampler, accumulation=N.ACC_FORWARD)
    whole = r.render()
    tiles = common_tiles(W, H)
    canvas = torch.zeros((H, W, 4), dtype=torch.float64, device="cuda:0")
    for rank in range(8):
        mine = sharding.shard_tiles(tiles, rank, 8)
        packed = torch.zeros(r.output_doubles(mine, N.OUT_PACKED), dtype=torch.float64, device="cuda:0")
        r.render_device(packed.data_ptr(), tiles=mine, layout=N.OUT_PACKED)
        r.unpack(mine, packed.data_ptr(), canvas.data_ptr())
    torch.cuda.synchronize()
    assert canvas.cpu().numpy().tobytes() == whole.tobytes()
    sub = tiles[1::3]
    img = r.render(tiles=sub)
    check_forward(img, r.stats, oracle_both(scene, W, H, spp, sampler, tiles=sub))
    r.close()


@pytest.mark.parametrize("name", ["C4", "C3"])
def test_forward_queue_refilled_while_units_remain(gpu, name, capfd):
    """Forward mode: after every shading pass k_refill fills the queue back to its slots
    while units remain (its new entries start 64-aligned, behind at most 63 dead entries,
    and end at the slot count), so no pass runs short of paths."""
    tu = N.tuning(flags=N.TUNE_PASS_LOG, slots=600000)
    cfg = configs.configs()[name]
    scene = cfg.build() if name == "C4" else configs.cornell_dragon(1.0, n=60)
    W, H, spp = (192, 108, 64) if name == "C4" else (128, 128, 64)
    r = GPURenderer(scene, W, H, spp, tuning=tu, accumulation=N.ACC_FORWARD)
    r.render()
    units = W * H * spp
    log = capfd.readouterr().err
    batches = [l.split() for l in log.splitlines() if l.startswith("IZPI_BATCH")]
    assert batches, log[-2000:]
    slots = r.stats["slots"]
    assert slots == 600000
    for b in batches:
        queue, head = int(b[2]), int(b[4])
        if head < units:  # units remain: the queue is full
            assert queue == slots, (b, slots)
    assert r.stats["launches"] <= 2 * (r.stats["rays"] // slots) + 48, r.stats
    r.close()


def test_forward_render_rank_world1(gpu):
    """The bench's multi-GPU form (izpi_gpu_render_rank: the rank's share, one ncclGather,
    rank 0 assembles and post-processes) in forward mode at world size 1: the spectral
    glass scene with Render's spectral post == one context's izpi_gpu_render, bit for bit."""
    import torch
    scene, W, H, spp, sampler = scene_case("glass_spectral")
    r = GPURenderer(scene, W, H, spp, sampler=sampler, accumulation=N.ACC_FORWARD)
    cid = (C.c_uint8 * N.COMM_ID_BYTES)()
    assert N.lib().izpi_gpu_comm_id(cid) == 0
    r.comm_init(1, 0, bytes(cid))
    canvas = torch.zeros((H, W, 4), dtype=torch.float64, device="cuda:0")
    r.render_rank(canvas.data_ptr(), post=N.POST_SPECTRAL)
    torch.cuda.synchronize()
    one = r.render(post=N.POST_SPECTRAL)
    assert canvas.cpu().numpy().tobytes() == one.tobytes()
    r.close()
