"""GPU parity: the gfx950 kernels (through the C ABI) against the CPU oracle.

The contract: same per-sample RNG streams, same flattened BVH4,
same Go-math restatement, no FMA contraction on either side -> the GPU canvas must be
BIT-IDENTICAL to the oracle's (the north-star tolerance, pixel RMSE < 1e-6, is the
fallback bound asserted alongside). Traversal/shading counters must match exactly.
"""
import ctypes as C
import struct

import numpy as np
import pytest

from izpi_amd import _native as N
from izpi_amd import configs
from izpi_amd.renderer import GPURenderer, common_tiles
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-6  # north_star: pixel RMSE < 1e-6 vs reference


def oracle_canvas(scene, W, H, spp, sampler, max_depth=50, tiles=None, seed=12345, bg=None, threads=16):
    o = O.OracleScene(scene, aspect_override=W / H)
    req = N.RenderReq(width=W, height=H, spp=spp, max_depth=max_depth, sampler=sampler, seed=seed)
    keep = []
    if tiles is not None:
        t = np.ascontiguousarray(tiles, np.uint32)
        keep.append(t)
        req.num_tiles = len(t)
        req.tiles = t.ctypes.data_as(C.POINTER(C.c_uint32))
    if bg is not None:
        wl, val = (np.ascontiguousarray(x, np.float64) for x in bg)
        keep += [wl, val]
        req.num_bg_spd = len(wl)
        req.bg_spd_wavelengths = wl.ctypes.data_as(C.POINTER(C.c_double))
        req.bg_spd_values = val.ctypes.data_as(C.POINTER(C.c_double))
    canvas, stats = o.render(req, threads=threads)
    return canvas.reshape(H, W, 4), stats


def assert_parity(gpu_img, ora_img, gstats=None, ostats=None):
    assert gpu_img.shape == ora_img.shape
    diff = np.abs(gpu_img - ora_img)
    rmse = float(np.sqrt(np.mean((gpu_img - ora_img) ** 2)))
    assert rmse < RMSE_TOL, rmse
    same = gpu_img.tobytes() == ora_img.tobytes()
    if not same:
        bad = np.argwhere(gpu_img.view(np.uint64) != ora_img.view(np.uint64))
        raise AssertionError("not bit-identical: %d values differ, first %s, max abs %g" %
                             (len(bad), bad[:5].tolist(), float(diff.max())))
    if gstats is not None:
        for k in ("rays", "node_visits", "tri_tests", "sph_tests", "light_tri_tests", "light_sph_tests", "samples"):
            assert gstats[k] == ostats[k], (k, gstats[k], ostats[k])


def test_gomath_device_bitwise(gpu):
    from tests.test_gomath import OPS, inputs, pow_fifth_inputs, pow_square_inputs
    r = GPURenderer(configs.cornell_rgb(), 8, 8, 1)
    L = N.lib()
    for name, op in list(OPS.items()) + [("pow2", OPS["pow"]), ("pow5", OPS["pow"])]:
        x, y = (pow_square_inputs() if name == "pow2" else pow_fifth_inputs() if name == "pow5"
                else inputs(name, n=20000, seed=3))
        x = np.ascontiguousarray(x, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        out = np.zeros_like(x)
        rc = L.izpi_gpu_gomath(r.ctx, op, O.dptr(x), O.dptr(y), len(x), O.dptr(out))
        assert rc == 0
        ref = np.array([O.gomath(op, float(a), float(b)) for a, b in zip(x, y)])
        mism = np.flatnonzero(out.view(np.uint64) != ref.view(np.uint64))
        assert mism.size == 0, (name, x[mism[:3]], y[mism[:3]], out[mism[:3]], ref[mism[:3]])
    # sincos_nonneg (ops 11, 12): the shared-reduction Sin / Cos of the random directions
    x = np.ascontiguousarray(6.283185307179586 * np.random.default_rng(9).uniform(0, 1, 20000), np.float64)
    x[:9] = np.arange(9) * (np.pi / 4)
    x[9] = 0.0
    y = np.zeros_like(x)
    for op, ref_op in ((11, OPS["sin"]), (12, OPS["cos"])):
        out = np.zeros_like(x)
        assert L.izpi_gpu_gomath(r.ctx, op, O.dptr(x), O.dptr(y), len(x), O.dptr(out)) == 0
        ref = np.array([O.gomath(ref_op, float(a), 0.0) for a in x])
        mism = np.flatnonzero(out.view(np.uint64) != ref.view(np.uint64))
        assert mism.size == 0, (op, x[mism[:3]], out[mism[:3]], ref[mism[:3]])
    # sdiv's shared reciprocal (op 13: sdiv((a, 0, 0), b).x) against the oracle's a / b, in
    # and out of its 2^+-300 window: zeros, subnormals, huge, inf, NaN on either side
    rng = np.random.default_rng(13)
    sp = [0.0, -0.0, 5e-324, -5e-324, 2.2250738585072014e-308, 1e-300, 1e-200, 1e-90, 2.0 ** -300, 2.0 ** -301,
          2.0 ** 300, 2.0 ** 301, 1e90, 1e200, 1.7976931348623157e308, float("inf"), float("-inf"), float("nan"), 1.0, -3.0]
    gx, gy = np.meshgrid(sp, sp)
    x = np.concatenate([rng.uniform(-1, 1, 20000) * 10.0 ** rng.integers(-120, 120, 20000), gx.ravel()])
    y = np.concatenate([rng.uniform(-1, 1, 20000) * 10.0 ** rng.integers(-120, 120, 20000), gy.ravel()])
    x, y = np.ascontiguousarray(x, np.float64), np.ascontiguousarray(y, np.float64)
    out = np.zeros_like(x)
    assert L.izpi_gpu_gomath(r.ctx, 13, O.dptr(x), O.dptr(y), len(x), O.dptr(out)) == 0
    ref = np.array([O.gomath(OPS["div"], float(a), float(b)) for a, b in zip(x, y)])
    # (NaN payloads are the platform's: a NaN quotient must be a NaN on both sides)
    mism = np.flatnonzero((out.view(np.uint64) != ref.view(np.uint64)) & ~(np.isnan(out) & np.isnan(ref)))
    assert mism.size == 0, ("sdiv", x[mism[:3]], y[mism[:3]], out[mism[:3]], ref[mism[:3]])
    # inside the window every quotient takes the shared-reciprocal path: bitwise with '/'
    # on the device itself (op 9) as well
    out9 = np.zeros_like(x)
    assert L.izpi_gpu_gomath(r.ctx, 9, O.dptr(x), O.dptr(y), len(x), O.dptr(out9)) == 0
    mism = np.flatnonzero((out.view(np.uint64) != out9.view(np.uint64)) & ~(np.isnan(out) & np.isnan(out9)))
    assert mism.size == 0, ("sdiv vs /", x[mism[:3]], y[mism[:3]], out[mism[:3]], out9[mism[:3]])
    r.close()


def test_ray_aabb4_kats_device(gpu):
    import json
    from pathlib import Path
    kats = json.loads((Path(__file__).parent / "golden" / "reference_kats.json").read_text())["ray_aabb4"]
    boxes, rays, exp = [], [], []
    for c in kats:
        f = lambda v: [float("inf") if x == "inf" else float(x) for x in v]
        boxes.append(f(c["min_x"]) + f(c["min_y"]) + f(c["min_z"]) + f(c["max_x"]) + f(c["max_y"]) + f(c["max_z"]))
        rays.append(f(c["org"]) + f(c["invdir"]) + [float(c["tmax"])])
        exp.append(c["expected"])
    # + the 1000 formulaic cases of bvh4_simd_test.go:200-268, expected from the oracle
    from tests.test_oracle_kats import formula_cases
    fb, fr = formula_cases()
    boxes = np.concatenate([np.array(boxes, np.float32), fb])
    rays = np.concatenate([np.array(rays, np.float32), fr])
    want = np.array(exp + [O.lib().oracle_ray_aabb4(b.ctypes.data_as(C.POINTER(C.c_float)),
                                                    r.ctypes.data_as(C.POINTER(C.c_float))) for b, r in zip(fb, fr)],
                    np.uint8)
    r = GPURenderer(configs.cornell_rgb(), 8, 8, 1)
    out = np.zeros(len(boxes), np.uint8)
    rc = N.lib().izpi_gpu_ray_aabb4(r.ctx, boxes.ctypes.data_as(C.POINTER(C.c_float)),
                                    rays.ctypes.data_as(C.POINTER(C.c_float)), len(boxes),
                                    out.ctypes.data_as(C.POINTER(C.c_uint8)))
    assert rc == 0
    np.testing.assert_array_equal(out, want)
    r.close()


def random_rays(n, seed=5, box=100.0):
    rng = np.random.default_rng(seed)
    o = np.column_stack([rng.uniform(1, box - 1, n), rng.uniform(1, box - 1, n), rng.uniform(-50, box - 1, n)])
    d = rng.normal(size=(n, 3))
    rays = np.zeros((n, 8))
    rays[:, :3], rays[:, 3:6], rays[:, 6], rays[:, 7] = o, d, 0.001, np.finfo(np.float64).max
    return rays


@pytest.mark.parametrize("which", ["box", "dragon", "glass", "pbr"])
def test_trace_closest_hit_bitwise(gpu, which):
    scene = {"box": configs.cornell_rgb, "dragon": lambda: configs.cornell_dragon(1.0, n=40),
             "glass": configs.cornell_glass_spectral, "pbr": configs.cornell_pbr}[which]()
    r = GPURenderer(scene, 16, 16, 1, sampler=N.SAMPLER_SPECTRAL if which == "glass" else N.SAMPLER_COLOUR)
    o = O.OracleScene(scene, aspect_override=1.0)
    rays = random_rays(20000)
    got = (N.Hit * len(rays))()
    assert N.lib().izpi_gpu_trace(r.ctx, rays.ctypes.data_as(C.POINTER(C.c_double)), len(rays), got) == 0
    want = o.trace(rays)
    for i in range(len(rays)):
        g, w = got[i], want[i]
        assert g.hit == w.hit, i
        if w.hit:
            assert g.prim_ref == w.prim_ref, i
            assert bytes(g)[:72] == bytes(w)[:72], (i, g.t, w.t, list(g.normal), list(w.normal))
    r.close()


def test_render_c1_bitwise(gpu):
    cfg = configs.configs()["C1"]
    scene = cfg.build()
    r = GPURenderer(scene, cfg.width, cfg.height, cfg.spp, sampler=cfg.sampler)
    img = r.render()
    ref, ostats = oracle_canvas(scene, cfg.width, cfg.height, cfg.spp, cfg.sampler)
    assert_parity(img, ref, r.stats, ostats)
    assert np.all(img[0] == 0.0)  # row 0 never written (rgb.go:41, A9)
    r.close()


def test_render_dragon_small_bitwise(gpu):
    scene = configs.cornell_dragon(1.0, n=60)
    r = GPURenderer(scene, 64, 64, 8)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 64, 64, 8, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


@pytest.mark.parametrize("tail", ["default", "none"])
def test_render_spectral_glass_bitwise(gpu, tail):
    """Dielectric spheres: path-length rays, sphere tests; with and without k_tail."""
    tu = N.tuning(flags=N.TUNE_NO_TAIL) if tail == "none" else None
    scene = configs.cornell_glass_spectral()
    r = GPURenderer(scene, 48, 48, 8, sampler=N.SAMPLER_SPECTRAL, tuning=tu)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 8, N.SAMPLER_SPECTRAL)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def test_render_pbr_bitwise(gpu):
    scene = configs.cornell_pbr(1.5, res=64)
    r = GPURenderer(scene, 60, 40, 8)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 60, 40, 8, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def test_max_depth_quirks(gpu):
    # depth >= maxDepth returns blue (colour.go:34-36); maxDepth 0 -> every sample blue
    scene = configs.cornell_rgb()
    for md in (0, 1, 3):
        r = GPURenderer(scene, 40, 40, 4, max_depth=md)
        img = r.render()
        ref, ostats = oracle_canvas(scene, 40, 40, 4, N.SAMPLER_COLOUR, max_depth=md)
        assert_parity(img, ref, r.stats, ostats)
        r.close()


def test_tiles_packed_and_unpack(gpu):
    import torch
    scene = configs.cornell_rgb()
    W = H = 96
    r = GPURenderer(scene, W, H, 4)
    tiles = common_tiles(W, H)
    sub = tiles[1::2]
    ref, _ = oracle_canvas(scene, W, H, 4, N.SAMPLER_COLOUR, tiles=sub)
    img = r.render(tiles=sub)
    assert_parity(img, ref)
    packed = torch.zeros(r.output_doubles(sub, N.OUT_PACKED), dtype=torch.float64, device="cuda:0")
    r.render_device(packed.data_ptr(), tiles=sub, layout=N.OUT_PACKED)
    canvas = torch.zeros((H, W, 4), dtype=torch.float64, device="cuda:0")
    r.unpack(sub, packed.data_ptr(), canvas.data_ptr())
    torch.cuda.synchronize()
    assert_parity(canvas.cpu().numpy(), ref)
    r.close()


@pytest.mark.parametrize("name", ["C4", "C3"])
def test_queue_keeps_every_slot_while_units_remain(gpu, name, capfd):
    """While work units remain, every finished path's record slot starts a new unit, so the
    queue stays at its first-fill length. (Round 2 regression: a block-iteration with no
    finished path marked its block "units exhausted" for the rest of the pass; on C4 the
    queue of 42M entries collapsed to one iteration per block and the frame took 3304
    passes instead of ~100. Images were still bit-exact, only slower.)"""
    # several shading iterations per block, units >> slots
    tu = N.tuning(flags=N.TUNE_PASS_LOG, slots=600000)
    cfg = configs.configs()[name]
    scene = cfg.build() if name == "C4" else configs.cornell_dragon(1.0, n=60)
    W, H, spp = (192, 108, 64) if name == "C4" else (128, 128, 64)
    r = GPURenderer(scene, W, H, spp, tuning=tu)
    r.render()
    units = W * H * spp
    log = capfd.readouterr().err
    batches = [l.split() for l in log.splitlines() if l.startswith("IZPI_BATCH")]
    assert batches, log[-2000:]
    slots = r.stats["slots"]
    assert slots == 600000
    for b in batches:
        queue, head = int(b[2]), int(b[4])
        if head < units:  # units remain: no slot may have been dropped
            assert queue == slots, (b, slots)
    assert r.stats["launches"] <= 2 * (r.stats["rays"] // slots) + 48, r.stats
    r.close()


@pytest.mark.parametrize("tune", [{"prim_weight": 1},
                                  {"prim_weight": 100000}, {"slots": 3000, "chunk_units": 5000},
                                  {"flags": N.TUNE_NO_LEAF_SHORTCUT}, {"trace_chunk": 1, "refill_min": 1},
                                  {"flags": N.TUNE_NO_DIST},
                                  {"flags": N.TUNE_NO_TAIL}, {"flags": N.TUNE_NO_TAIL, "slots": 3000},
                                  {"tail_paths": 100},
                                  {"flags": N.TUNE_GENERAL_TRACE}, {"flags": N.TUNE_NO_RAY_LDS},
                                  {"trace_chunk": 16, "refill_min": 64},
                                  {"rec_dense": 1, "pool_div": 100000},
                                  {"rec_dense": 2, "pool_div": 100000, "flags": N.TUNE_NO_TAIL},
                                  {"rec_dense": 50}])
def test_kernel_variants_bitwise(gpu, tune):
    """Traversal step weights, tiny slot/chunk counts, the sequential-leaf and
    sphere-capable instances, the pass loop without the k_tail finish, and the unwinding
    records' split (dense levels + overflow blocks: a 4096-block pool far below the demand
    parks slots, all-dense needs no pool) are launch knobs only: results and counters
    must not move."""
    scene = configs.cornell_dragon(1.0, n=60)
    r = GPURenderer(scene, 64, 64, 4, tuning=N.tuning(**tune))
    img = r.render()
    ref, ostats = oracle_canvas(scene, 64, 64, 4, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    if tune.get("pool_div") == 100000:
        assert r.stats["pool_blocks"] == 4096 and r.stats["parks"] > 0, r.stats  # the park path ran
    r.close()


@pytest.mark.parametrize("flags", [0, N.TUNE_NO_LDS_BVH, N.TUNE_NO_PRIM_LDS, N.TUNE_NO_RAY_LDS])
@pytest.mark.parametrize("which", ["cornell", "glass", "pbr"])
def test_small_scene_lds_bvh_bitwise(gpu, which, flags):
    """A scene whose whole BVH4 (inner nodes, leaf records, primitives) fits in 4 KB is
    traversed from every block's LDS copy (C1, C2, C4, C5), its rays kept in LDS too (with
    IZPI_TUNE_NO_RAY_LDS re-read from global memory by the primitive tests); with
    IZPI_TUNE_NO_LDS_BVH from global memory. Its primitives' shading records (GShade, triangle UVs and tangent frames,
    sphere records) are read from the shading blocks' LDS copy, or with
    IZPI_TUNE_NO_PRIM_LDS from global memory. All equal the oracle bit for bit, counters
    included (bvh4.go:49-164, triangle.go:223-264, sphere.go:71-92)."""
    scene, sampler = {"cornell": (configs.cornell_rgb(), N.SAMPLER_COLOUR),
                      "glass": (configs.cornell_glass_spectral(), N.SAMPLER_SPECTRAL),
                      "pbr": (configs.cornell_pbr(1.0, res=64), N.SAMPLER_COLOUR)}[which]
    r = GPURenderer(scene, 48, 48, 4, sampler=sampler, tuning=N.tuning(flags=flags) if flags else None)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 4, sampler)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


@pytest.mark.parametrize("tune", [{"rec_dense": 1, "pool_div": 100000},
                                  {"rec_dense": 3, "pool_div": 100000, "flags": N.TUNE_NO_TAIL}])
def test_record_pool_spectral_glass_bitwise(gpu, tune):
    """Overflow records under the spectral sampler with dielectrics: path-length rays,
    parked slots and 32-B records."""
    scene = configs.cornell_glass_spectral()
    r = GPURenderer(scene, 48, 48, 8, sampler=N.SAMPLER_SPECTRAL, tuning=N.tuning(**tune))
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 8, N.SAMPLER_SPECTRAL)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


@pytest.mark.parametrize("tune", [{}, {"rec_dense": 1, "pool_div": 100000},
                                  {"rec_dense": 2, "pool_div": 100000, "flags": N.TUNE_NO_TAIL}, {"slots": 3000}])
def test_deferred_unwinding_specular_colour_bitwise(gpu, tune):
    """Colour shading with specular materials (Metal, PBR) queues the unwindings that read
    records and runs them block-wide (fin_flush), frees their overflow blocks only then,
    and unwinds the others in place: with parked slots, without k_tail and
    with few slots (many flushes of partly filled queues), equal to the oracle bit for bit."""
    scene = configs.cornell_pbr(1.0, res=64)
    r = GPURenderer(scene, 48, 48, 8, tuning=N.tuning(**tune) if tune else None)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 8, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    if tune.get("pool_div") == 100000:
        assert r.stats["pool_blocks"] == 4096, r.stats
    r.close()


def test_slow_slab_path_bitwise(gpu):
    """The NaN-free packed slab (slab4_fast) and the scalar twin give the same image."""
    scene = configs.cornell_dragon(1.0, n=60)
    r = GPURenderer(scene, 64, 64, 4, tuning=N.tuning(flags=N.TUNE_SCALAR_SLAB))
    img = r.render()
    ref, ostats = oracle_canvas(scene, 64, 64, 4, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def test_axis_aligned_rays_trace_bitwise(gpu):
    """Rays with zero direction components (infinite f32 inverses) take the scalar-twin
    slab path; origins on slab planes give 0*inf = NaN there (A14)."""
    scene = configs.cornell_dragon(1.0, n=40)
    o = O.OracleScene(scene, aspect_override=1.0)
    r = GPURenderer(scene, 8, 8, 1)
    rng = np.random.default_rng(7)
    rays = []
    for i in range(4096):
        org = rng.uniform(-10, 110, 3)
        if i % 3 == 0:
            org = np.round(org)  # lands on box planes (x = 0, 100 ...) exactly
        d = np.zeros(3)
        d[i % 3] = 1.0 if (i // 3) % 2 else -1.0
        if i % 5 == 0:
            d[(i + 1) % 3] = rng.uniform(-1, 1)
        rays.append(list(org) + list(d) + [0.001, 1e300])
    rays = np.ascontiguousarray(rays, np.float64)
    got = (N.Hit * len(rays))()
    assert N.lib().izpi_gpu_trace(r.ctx, rays.ctypes.data_as(C.POINTER(C.c_double)), len(rays), got) == 0
    want = o.trace(rays)
    nhit = 0
    for i in range(len(rays)):
        g, w = got[i], want[i]
        assert g.hit == w.hit, i
        if w.hit:
            nhit += 1
            assert g.prim_ref == w.prim_ref, i
            assert bytes(g)[:72] == bytes(w)[:72], i
    assert nhit > 1000
    r.close()


def test_full_size_c3_frame_low_spp_bitwise(gpu):
    """BASELINE.json's full C3 frame (1024x1024, 817k-triangle dragon) at 2 spp: every
    pixel bit-identical to the oracle, counters equal."""
    cfg = configs.configs()["C3"]
    scene = cfg.build()
    r = GPURenderer(scene, cfg.width, cfg.height, 2)
    img = r.render()
    ref, ostats = oracle_canvas(scene, cfg.width, cfg.height, 2, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def test_full_size_c3_tiles_full_spp_bitwise(gpu):
    """Four centre tiles of the C3 frame at the metric's full 512 spp."""
    cfg = configs.configs()["C3"]
    scene = cfg.build()
    tiles = common_tiles(cfg.width, cfg.height)[:4]  # spiral order starts at the centre
    r = GPURenderer(scene, cfg.width, cfg.height, cfg.spp)
    img = r.render(tiles=tiles)
    ref, ostats = oracle_canvas(scene, cfg.width, cfg.height, cfg.spp, N.SAMPLER_COLOUR, tiles=tiles)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


@pytest.mark.parametrize("name,ntiles,tune", [
    ("C2", 4, None),
    ("C4", 2, None),
    # C5 in 5 chunks of per-sample results (the multi-chunk path C5's full frame takes)
    ("C5", 1, {"chunk_units": 1 << 20}),
])
@pytest.mark.timeout(400)
def test_full_spp_centre_tiles_bitwise(gpu, name, ntiles, tune):
    """BASELINE.json's configs at their FULL spp (C2 256, C4 1024, C5 4096) on the frame's
    first tiles in spiral order (the centre, where the dragon / glass is), against the oracle
    (render/rgb.go:12-57, render/spectral.go:71-106): bit-identical canvases, equal counters."""
    cfg = configs.configs()[name]
    scene = cfg.build()
    tiles = common_tiles(cfg.width, cfg.height)[:ntiles]
    r = GPURenderer(scene, cfg.width, cfg.height, cfg.spp, sampler=cfg.sampler,
                    tuning=N.tuning(**tune) if tune else None)
    img = r.render(tiles=tiles)
    if tune and "chunk_units" in tune:
        assert r.stats["chunk_spp"] < cfg.spp, r.stats  # several chunks ran
    ref, ostats = oracle_canvas(scene, cfg.width, cfg.height, cfg.spp, cfg.sampler, tiles=tiles)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def test_spectral_post_kernel_bitwise(gpu):
    """FireflyRejection + XYZToRGB (firefly_rejection.go, rgb_image.go) on a synthetic XYZ
    canvas with fireflies, zeros, negative and NaN luminance, edges and corners."""
    import torch
    W, H = 67, 45
    rng = np.random.default_rng(3)
    xyz = rng.uniform(0.0, 1.0, (H, W, 4))
    spikes = rng.random((H, W)) < 0.05
    xyz[spikes, :3] *= 50.0
    xyz[rng.random((H, W)) < 0.05, 1] = 0.0
    xyz[rng.random((H, W)) < 0.02, 1] = -0.3
    xyz[5, 7, 1] = np.nan
    xyz[0, :, :] = 0.0  # the row the reference never writes (A9)
    r = GPURenderer(configs.cornell_rgb(), W, H, 1)
    for exposure in (1.0, 0.7):
        want = O.xyz_to_rgb(O.firefly(xyz.reshape(-1), W, H), W, H, exposure).reshape(H, W, 4)
        src = torch.from_numpy(xyz.copy()).cuda()
        dst = torch.empty_like(src)
        assert N.lib().izpi_gpu_spectral_post(r.ctx, C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), W, H,
                                              C.c_double(exposure)) == 0
        got = dst.cpu().numpy()
        assert got.tobytes() == want.tobytes()
    r.close()


def test_render_spectral_rgb_bitwise(gpu):
    """Render() for the Spectral sampler: XYZ render + FireflyRejection + XYZToRGB."""
    scene = configs.cornell_glass_spectral()
    r = GPURenderer(scene, 48, 48, 8, sampler=N.SAMPLER_SPECTRAL)
    img = r.render_spectral_rgb()
    ref, _ = oracle_canvas(scene, 48, 48, 8, N.SAMPLER_SPECTRAL)
    want = O.xyz_to_rgb(O.firefly(ref.reshape(-1), 48, 48), 48, 48, r.exposure).reshape(48, 48, 4)
    assert_parity(img, want)
    r.close()


@pytest.mark.parametrize("name", ["C2", "C4", "C5"])
def test_full_size_frames_one_spp_bitwise(gpu, name):
    """BASELINE.json's other configurations at their full image sizes (1 spp): the
    Cornell box (C2), the PBR box with image textures and normal maps (C4) and the
    spectral glass scene with dielectric spheres and path-length rays (C5, including
    FireflyRejection + XYZToRGB). Every pixel bit-identical, counters equal."""
    cfg = configs.configs()[name]
    scene = cfg.build()
    r = GPURenderer(scene, cfg.width, cfg.height, 1, sampler=cfg.sampler)
    if cfg.sampler == N.SAMPLER_SPECTRAL:
        img = r.render_spectral_rgb()
        stats = r.stats
        ref, ostats = oracle_canvas(scene, cfg.width, cfg.height, 1, cfg.sampler)
        ref = O.xyz_to_rgb(O.firefly(ref.reshape(-1), cfg.width, cfg.height), cfg.width, cfg.height,
                           r.exposure).reshape(cfg.height, cfg.width, 4)
    else:
        img = r.render()
        stats = r.stats
        ref, ostats = oracle_canvas(scene, cfg.width, cfg.height, 1, cfg.sampler)
    assert_parity(img, ref, stats, ostats)
    r.close()


def test_ingested_pbtxt_scene_bitwise(gpu):
    """The reference's example .pbtxt through the C++ ingestion renders the same image as
    the C5 restatement, on the GPU, bit for bit (and as the oracle does)."""
    from pathlib import Path
    from izpi_amd import ingest
    path = Path(__file__).resolve().parents[1] / "izpi_amd" / "data" / "scenes" / \
        "cornell_box_transparent_pyramid_spectral.pbtxt"
    scene = ingest.ProtoScene.from_file(path)
    r = GPURenderer(scene, 40, 40, 4, sampler=scene.sampler)
    img = r.render()
    ref, ostats = oracle_canvas(configs.cornell_glass_spectral(1.0), 40, 40, 4, N.SAMPLER_SPECTRAL)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def test_ingested_obj_mesh_bitwise(gpu):
    """A Wavefront OBJ mesh streamed into a transport scene (wavefront.go transforms +
    GroupToTransportTrianglesWithMaterial, as scenes/spectral.go:639-657 does for the dragon)."""
    from pathlib import Path
    from izpi_amd import ingest
    from tests.test_ingest import _BOX_RGB
    cube = ingest.WavefrontObj.from_file(Path(__file__).resolve().parent / "golden" / "wavefront" / "cube.obj")
    cube.scale(30.0, 30.0, 30.0)
    cube.rotate(0.0, -ingest.go_radians(60), 0.0)
    cube.translate(50.0, 25.1, 60.0)
    scene = ingest.ProtoScene(_BOX_RGB.encode())
    scene.add_triangles(cube.group_to_transport_triangles(0, without_uvs=True), "White")
    r = GPURenderer(scene, 48, 48, 8)
    img = r.render()
    ref, ostats = oracle_canvas(scene, 48, 48, 8, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    r.close()


def test_postprocess_kernel_bitwise(gpu):
    """izpi_gpu_postprocess == the oracle's postprocess.Pipeline restatement, including
    NaN / negative / infinite inputs; the render flag applies Gamma, Clamp(1.0)."""
    import torch
    W, H = 100, 40  # a common.Tiles size (render part)
    rng = np.random.default_rng(11)
    c = rng.uniform(-0.5, 3.0, (H, W, 4))
    c[0, 0, :3] = [np.nan, np.inf, -0.0]
    r = GPURenderer(configs.cornell_rgb(), W, H, 2)
    for filters in ([(N.FILTER_GAMMA, 0.0), (N.FILTER_CLAMP, 1.0)], [(N.FILTER_CLAMP, 0.3)], [(N.FILTER_GAMMA, 0.0)]):
        d = torch.from_numpy(c.copy()).cuda()
        r.postprocess(d.data_ptr(), filters)
        torch.cuda.synchronize()
        ref = O.postprocess(c.ravel(), W, H, filters).reshape(H, W, 4)
        assert d.cpu().numpy().tobytes() == ref.tobytes(), filters
    img = r.render(post=N.POST_GAMMA_CLAMP)
    raw, _ = oracle_canvas(configs.cornell_rgb(), W, H, 2, N.SAMPLER_COLOUR)
    ref = O.postprocess(raw.ravel(), W, H, [(1, 0.0), (2, 1.0)]).reshape(H, W, 4)
    assert img.tobytes() == ref.tobytes()
    r.close()


@pytest.mark.parametrize("method", [N.BVH_PLOC, N.BVH_LBVH, N.BVH_PLOC_SAH])
@pytest.mark.parametrize("which", ["cornell", "dragon", "glass", "degenerate", "tiny"])
def test_gpu_bvh4_builder_equals_oracle_restatement(gpu, which, method):
    """izpi_gpu_build_bvh4 (Morton sort + Karras tree + refit + collapse on the GPU) ==
    the oracle's sequential restatement, node for node and in leaf order."""
    from izpi_amd.scene import HostScene
    from tests.test_bvh_build import check_tree
    if which == "degenerate":
        boxes = np.tile([1.0, 1.0, 1.0, 2.0, 2.0, 2.0], (1000, 1))
    elif which == "tiny":
        boxes = np.array([[0, 0, 0, 1, 1, 1], [2, 2, 2, 3, 3, 3], [5, 0, 0, 6, 1, 1]], np.float64)
    else:
        scene = {"cornell": configs.cornell_rgb(), "dragon": configs.cornell_dragon(1.0, n=80),
                 "glass": configs.cornell_glass_spectral()}[which]
        boxes = HostScene(scene, 1.0, skip_bvh=True).prim_boxes()
    r = GPURenderer(configs.cornell_rgb(), 8, 8, 1)
    nodes, order, ms = r.build_bvh4(boxes, 3, method)
    ref_nodes, ref_order = O.lbvh4(boxes, 3, method)
    assert order.tolist() == ref_order.tolist()
    assert nodes.tobytes() == ref_nodes.tobytes()
    check_tree(nodes, order, boxes, leaf_max=3)
    again, order2, _ = r.build_bvh4(boxes, 3, method)  # deterministic
    assert again.tobytes() == nodes.tobytes() and (order2 == order).all()
    r.close()


@pytest.mark.timeout(300)
def test_headline_tree_full_size_equals_oracle_restatement(gpu):
    """The tree BASELINE.json's headline figure runs on: C3's 817,464-triangle mesh built on
    the GPU (PLOC + SAH collapse, 3 primitives per leaf, as bench.py builds it) == the
    oracle's restatement (oracle_lbvh4), node for node and in leaf order, in BVH4Node's
    format (bvh4.go:23-39, 714-792)."""
    from izpi_amd.renderer import GPU_BVH_METHOD, gpu_leaf_max
    from izpi_amd.scene import HostScene
    from tests.test_bvh_build import check_tree
    cfg = configs.configs()["C3"]
    host = HostScene(cfg.build(), cfg.width / cfg.height, skip_bvh=True)
    boxes = host.prim_boxes()
    assert len(boxes) == 817464
    leaf = gpu_leaf_max(host.desc)
    r = GPURenderer(configs.cornell_rgb(), 8, 8, 1)
    nodes, order, _ = r.build_bvh4(boxes, leaf, GPU_BVH_METHOD)
    r.close()
    ref_nodes, ref_order = O.lbvh4(boxes, leaf, GPU_BVH_METHOD)
    assert np.array_equal(order, ref_order)
    assert nodes.tobytes() == ref_nodes.tobytes()
    check_tree(nodes, order, boxes, leaf_max=leaf)


@pytest.mark.parametrize("acc", [N.ACC_RECURSIVE, N.ACC_FORWARD])
@pytest.mark.timeout(400)
def test_headline_tree_c3_centre_tiles_full_spp_bitwise(gpu, acc):
    """C3's four centre tiles at the metric's 512 spp on the GPU-built headline tree (the
    tree of bench.py's `value`), against the oracle traversing the same tree: bit-identical,
    counters equal, in both accumulation modes."""
    cfg = configs.configs()["C3"]
    scene = cfg.build()
    tiles = common_tiles(cfg.width, cfg.height)[:4]
    r = GPURenderer(scene, cfg.width, cfg.height, cfg.spp, bvh="gpu", accumulation=acc)
    img = r.render(tiles=tiles)
    o = O.OracleScene(scene, aspect_override=cfg.width / cfg.height)
    o.set_bvh(r.bvh_nodes(), r.host._bvh_keep[1])
    req = N.RenderReq(width=cfg.width, height=cfg.height, spp=cfg.spp, max_depth=50, sampler=N.SAMPLER_COLOUR,
                      seed=12345, abi_version=N.IZPI_ABI_VERSION, accumulation=acc)
    t = np.ascontiguousarray(tiles, np.uint32)
    req.num_tiles = len(t)
    req.tiles = t.ctypes.data_as(C.POINTER(C.c_uint32))
    ref, ostats = o.render(req, threads=16)
    assert_parity(img, ref.reshape(cfg.height, cfg.width, 4), r.stats, ostats)
    o.close()
    r.close()


@pytest.mark.parametrize("which", ["C1", "C2", "C3", "C4", "C5"])
def test_quantized_nodes_equal_exact_boxes_image(gpu, which):
    """IZPI_SCENE_QUANTIZED_BVH on each config's GPU-built tree: the 64-B nodes (k_trace2's Q
    instance) and the decoded 128-B records (IZPI_TUNE_NO_QNODES, and the other instances)
    give the same canvas and counters; against the exact boxes the canvas is the same
    (bitwise here: the decoded boxes only add visits) with at least as many node visits."""
    cfg = configs.configs()[which]
    scene = cfg.build()
    W, H = (cfg.width, cfg.height) if which != "C5" else (512, 512)
    spp = 1
    imgs, stats = [], []
    for quant, tune in ((True, None), (True, N.tuning(flags=N.TUNE_NO_QNODES)), (False, None)):
        r = GPURenderer(scene, W, H, spp, sampler=cfg.sampler, bvh="gpu", bvh_quantized=quant, tuning=tune)
        imgs.append(r.render())
        stats.append(r.stats)
        r.close()
    assert imgs[0].tobytes() == imgs[1].tobytes()
    for k in ("rays", "node_visits", "tri_tests", "sph_tests", "light_tri_tests", "light_sph_tests"):
        assert stats[0][k] == stats[1][k], k
    assert imgs[0].tobytes() == imgs[2].tobytes()
    assert stats[0]["node_visits"] >= stats[2]["node_visits"] and stats[0]["rays"] == stats[2]["rays"]


def test_quantized_trace_component_bitwise(gpu):
    """izpi_gpu_trace (closest hit records) on the quantised GPU-built dragon tree == the
    oracle's trace over oracle.quantize_bvh4's boxes, including rays along the axes."""
    scene = configs.cornell_dragon(1.0, n=60)
    r = GPURenderer(scene, 8, 8, 1, bvh="gpu", bvh_quantized=True)
    o = O.OracleScene(scene, aspect_override=1.0)
    qnodes, applied = O.quantize_bvh4(r.bvh_nodes())
    assert applied
    o.set_bvh(qnodes, r.host._bvh_keep[1])
    rng = np.random.default_rng(5)
    n = 4096
    rays = np.zeros((n, 8))
    rays[:, 0:3] = rng.uniform([5, 5, -50], [95, 95, 95], (n, 3))
    d = rng.normal(size=(n, 3))
    d[:256] = 0.0
    d[np.arange(256), np.arange(256) % 3] = np.where(np.arange(256) % 2, 1.0, -1.0)
    rays[:, 3:6] = d
    rays[:, 6] = 0.001
    rays[:, 7] = np.where(rng.random(n) < 0.3, rng.uniform(1, 80, n), 1.7976931348623157e308)
    got = (N.Hit * n)()
    assert N.lib().izpi_gpu_trace(r.ctx, O.dptr(rays), n, got) == 0
    want = o.trace(rays)
    nhit = 0
    for i in range(n):
        g, w = got[i], want[i]
        assert g.hit == w.hit, i
        if w.hit:
            nhit += 1
            assert g.prim_ref == w.prim_ref, i
            assert bytes(g)[:72] == bytes(w)[:72], (i, g.t, w.t)
    assert nhit > n // 2
    o.close()
    r.close()


@pytest.mark.parametrize("quantized", [True, False])
@pytest.mark.parametrize("which", ["dragon", "glass"])
def test_render_on_gpu_built_bvh_bitwise(gpu, which, quantized):
    """The kernels on the GPU-built tree (exact boxes, or quantised 64-B nodes) == the oracle
    traversing the same tree (with oracle.quantize_bvh4's decoded boxes), bit for bit,
    counters included, and == the reference-tree image within the north-star bound."""
    if which == "dragon":
        scene, W, H, spp, sampler = configs.cornell_dragon(1.0, n=80), 64, 64, 8, N.SAMPLER_COLOUR
    else:
        scene, W, H, spp, sampler = configs.cornell_glass_spectral(), 48, 48, 8, N.SAMPLER_SPECTRAL
    r = GPURenderer(scene, W, H, spp, sampler=sampler, bvh="gpu", bvh_quantized=quantized)
    img = r.render()
    o = O.OracleScene(scene, aspect_override=W / H)
    nodes = r.bvh_nodes()
    if quantized:
        nodes, applied = O.quantize_bvh4(nodes)
        assert applied
    o.set_bvh(nodes, r.host._bvh_keep[1])
    req = N.RenderReq(width=W, height=H, spp=spp, max_depth=50, sampler=sampler, seed=12345)
    ref, ostats = o.render(req, threads=16)
    assert_parity(img, ref.reshape(H, W, 4), r.stats, ostats)
    base, _ = oracle_canvas(scene, W, H, spp, sampler)
    rmse = float(np.sqrt(np.mean((img - base) ** 2)))
    assert rmse < RMSE_TOL, rmse
    r.close()


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_gpu_render_bitwise(gpu, devices):
    """izpi_gpu_multi_render (one call, one context per device, shares gathered to device
    0) == the oracle, for 1-3 contexts (several contexts on this box's one GPU exercise
    the share dealing, the padded gather and the assembly)."""
    from izpi_amd.renderer import MultiGPURenderer
    scene = configs.cornell_dragon(1.0, n=40)
    r = MultiGPURenderer(scene, 64, 64, 4, devices, bvh="reference")
    img = r.render()
    ref, ostats = oracle_canvas(scene, 64, 64, 4, N.SAMPLER_COLOUR)
    assert_parity(img, ref)
    for k in ("rays", "node_visits", "tri_tests", "light_tri_tests", "samples"):
        assert sum(st[k] for st in r.stats) == ostats[k], k
    assert len(r.stats) == len(devices)
    r.close()


def test_multi_gpu_spectral_post_bitwise(gpu):
    """Render's spectral post (FireflyRejection + XYZToRGB) runs on the ASSEMBLED frame:
    two shares must give the single-device canvas, including the firefly halo across
    share boundaries."""
    from izpi_amd.renderer import MultiGPURenderer
    scene = configs.cornell_glass_spectral()
    one = GPURenderer(scene, 64, 64, 4, sampler=N.SAMPLER_SPECTRAL, bvh="gpu")
    want = one.render(post=N.POST_SPECTRAL | N.POST_GAMMA_CLAMP)
    one.close()
    r = MultiGPURenderer(scene, 64, 64, 4, [0, 0], sampler=N.SAMPLER_SPECTRAL, bvh="gpu")
    got = r.render(post=N.POST_SPECTRAL | N.POST_GAMMA_CLAMP)
    r.close()
    assert got.tobytes() == want.tobytes()


def test_render_rank_rccl_world1_bitwise(gpu):
    """The one-process-per-GPU form through the library's RCCL communicator (comm id,
    ncclCommInitRank, ncclGather to rank 0) at world size 1 == the oracle."""
    import ctypes as C
    import torch
    scene = configs.cornell_rgb()
    r = GPURenderer(scene, 64, 64, 4)
    cid = (C.c_uint8 * N.COMM_ID_BYTES)()
    assert N.lib().izpi_gpu_comm_id(cid) == 0
    r.comm_init(1, 0, bytes(cid))
    canvas = torch.zeros((64, 64, 4), dtype=torch.float64, device="cuda:0")
    r.render_rank(canvas.data_ptr())
    torch.cuda.synchronize()
    ref, ostats = oracle_canvas(scene, 64, 64, 4, N.SAMPLER_COLOUR)
    assert_parity(canvas.cpu().numpy(), ref, r.stats, ostats)
    r.close()


def test_render_rank_failures_return_without_hanging(gpu):
    """izpi_gpu_render_rank's failure paths at world size 1 (every collective still runs:
    the agreement steps and the gather) return the failing status, then the context renders
    normally again (render/remote.go:40-55 only logs a failed remote tile; here the caller
    gets the status)."""
    import ctypes as C
    import torch
    scene = configs.cornell_rgb()
    r = GPURenderer(scene, 64, 64, 4)
    L = N.lib()
    cid = (C.c_uint8 * N.COMM_ID_BYTES)()
    assert L.izpi_gpu_comm_id(cid) == 0
    r.comm_init(1, 0, bytes(cid))
    canvas = torch.zeros((64, 64, 4), dtype=torch.float64, device="cuda:0")
    req = r.request()
    st = N.RenderStats()
    # rank 0 without an output canvas: fails its local checks, before rendering
    assert L.izpi_gpu_render_rank(r.ctx, C.byref(req), None, C.byref(st)) == N.IZPI_ERR_INVALID
    for where, want in ((1, N.IZPI_ERR_DEVICE), (2, N.IZPI_ERR_DEVICE)):
        assert L.izpi_gpu_debug_fault(r.ctx, where) == 0
        rc = L.izpi_gpu_render_rank(r.ctx, C.byref(req), C.c_void_p(canvas.data_ptr()), C.byref(st))
        assert rc == want, (where, rc, L.izpi_gpu_last_error(r.ctx))
        assert b"inject" in L.izpi_gpu_last_error(r.ctx)
    assert L.izpi_gpu_debug_fault(r.ctx, 0) == 0
    r.render_rank(canvas.data_ptr())
    torch.cuda.synchronize()
    ref, _ = oracle_canvas(scene, 64, 64, 4, N.SAMPLER_COLOUR)
    assert_parity(canvas.cpu().numpy(), ref)
    r.close()


def test_render_rank_stalled_peer_hits_the_deadline(gpu):
    """A rank whose collective never completes (izpi_gpu_debug_fault 3 stalls this rank's
    stream before the gather, as a dead peer leaves it): with tuning.peer_timeout_ms the call
    polls the stream and ncclCommGetAsyncError, aborts the communicator past the deadline
    and returns IZPI_ERR_PEER instead of hanging; after a new izpi_gpu_comm_init the context
    renders bit-exact again."""
    import ctypes as C
    import time
    import torch
    scene = configs.cornell_rgb()
    r = GPURenderer(scene, 64, 64, 4)
    L = N.lib()
    cid = (C.c_uint8 * N.COMM_ID_BYTES)()
    assert L.izpi_gpu_comm_id(cid) == 0
    r.comm_init(1, 0, bytes(cid))
    canvas = torch.zeros((64, 64, 4), dtype=torch.float64, device="cuda:0")
    req = r.request()
    tu = N.tuning(peer_timeout_ms=300)
    req.tuning = C.pointer(tu)
    st = N.RenderStats()
    assert L.izpi_gpu_debug_fault(r.ctx, 3) == 0
    t0 = time.time()
    rc = L.izpi_gpu_render_rank(r.ctx, C.byref(req), C.c_void_p(canvas.data_ptr()), C.byref(st))
    dt = time.time() - t0
    assert rc == N.IZPI_ERR_PEER, (rc, L.izpi_gpu_last_error(r.ctx))
    assert b"no answer from the other ranks within 300 ms" in L.izpi_gpu_last_error(r.ctx)
    assert dt < 5.0, dt  # the deadline, not the stall's own bound (~7 s), ended the wait
    assert L.izpi_gpu_debug_fault(r.ctx, 0) == 0
    # the communicator is gone: the next call says so at once
    assert L.izpi_gpu_render_rank(r.ctx, C.byref(req), C.c_void_p(canvas.data_ptr()), C.byref(st)) == N.IZPI_ERR_INVALID
    assert L.izpi_gpu_comm_id(cid) == 0
    r.comm_init(1, 0, bytes(cid))
    assert L.izpi_gpu_render_rank(r.ctx, C.byref(req), C.c_void_p(canvas.data_ptr()), C.byref(st)) == 0
    torch.cuda.synchronize()
    ref, _ = oracle_canvas(scene, 64, 64, 4, N.SAMPLER_COLOUR)
    assert_parity(canvas.cpu().numpy(), ref)
    r.close()


def test_render_rank_failed_stream_aborts_the_communicator(gpu):
    """A rank whose stream fails in a collective step (izpi_gpu_debug_fault 4: the polls of
    the step see a HIP error, as after a sticky device fault) cannot join the remaining
    collectives: it aborts the communicator, so that peers blocked in them see the abort
    instead of waiting forever (peer_timeout_ms 0, the default), and returns IZPI_ERR_PEER;
    the communicator is gone, and after a new izpi_gpu_comm_init the context renders
    bit-exact again."""
    import ctypes as C
    import torch
    scene = configs.cornell_rgb()
    r = GPURenderer(scene, 64, 64, 4)
    L = N.lib()
    cid = (C.c_uint8 * N.COMM_ID_BYTES)()
    assert L.izpi_gpu_comm_id(cid) == 0
    r.comm_init(1, 0, bytes(cid))
    canvas = torch.zeros((64, 64, 4), dtype=torch.float64, device="cuda:0")
    req = r.request()
    st = N.RenderStats()
    assert L.izpi_gpu_debug_fault(r.ctx, 5) == N.IZPI_ERR_INVALID
    assert L.izpi_gpu_debug_fault(r.ctx, 4) == 0
    rc = L.izpi_gpu_render_rank(r.ctx, C.byref(req), C.c_void_p(canvas.data_ptr()), C.byref(st))
    assert rc == N.IZPI_ERR_PEER, (rc, L.izpi_gpu_last_error(r.ctx))
    assert b"this rank's stream failed" in L.izpi_gpu_last_error(r.ctx)
    assert b"communicator aborted" in L.izpi_gpu_last_error(r.ctx)
    assert L.izpi_gpu_debug_fault(r.ctx, 0) == 0
    assert L.izpi_gpu_render_rank(r.ctx, C.byref(req), C.c_void_p(canvas.data_ptr()), C.byref(st)) == N.IZPI_ERR_INVALID
    assert L.izpi_gpu_comm_id(cid) == 0
    r.comm_init(1, 0, bytes(cid))
    assert L.izpi_gpu_render_rank(r.ctx, C.byref(req), C.c_void_p(canvas.data_ptr()), C.byref(st)) == 0
    torch.cuda.synchronize()
    ref, _ = oracle_canvas(scene, 64, 64, 4, N.SAMPLER_COLOUR)
    assert_parity(canvas.cpu().numpy(), ref)
    r.close()


def test_abi1_request_tuning_prefix_is_honoured(gpu):
    """An ABI-1 request (abi_version 0: the field was padding) has its tuning pointer in the
    same place, and ABI 1's izpi_render_tuning ended at tail_paths: those fields are read
    (here a 2000-path cap), the later ones keep their defaults, and the image is the
    oracle's."""
    import ctypes as C
    scene = configs.cornell_rgb()
    r = GPURenderer(scene, 32, 32, 4)
    L = N.lib()
    req = r.request()
    tu = N.tuning(slots=2000, peer_timeout_ms=1)  # peer_timeout_ms lies past the ABI-1 struct
    req.tuning = C.pointer(tu)
    req.abi_version = 0
    canvas = np.zeros((32, 32, 4))
    st = N.RenderStats()
    assert L.izpi_gpu_render(r.ctx, C.byref(req), canvas.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)) == 0
    assert st.slots == 2000
    ref, _ = oracle_canvas(scene, 32, 32, 4, N.SAMPLER_COLOUR)
    assert_parity(canvas, ref)
    r.close()


def test_abi1_request_ignores_the_fields_past_its_tuning(gpu):
    """The ABI-1 truncation where it shows: peer_timeout_ms lies past ABI 1's tuning struct,
    and only izpi_gpu_render_rank reads it. With this rank's stream stalled before the gather
    (izpi_gpu_debug_fault 3, bounded at ~7 s), an ABI-3 request with a 300-ms deadline
    returns IZPI_ERR_PEER (test_render_rank_stalled_peer_hits_the_deadline); the same
    request marked ABI 1 must not see the deadline: it waits the stall out and succeeds."""
    import ctypes as C
    import time
    import torch
    scene = configs.cornell_rgb()
    r = GPURenderer(scene, 64, 64, 4)
    L = N.lib()
    cid = (C.c_uint8 * N.COMM_ID_BYTES)()
    assert L.izpi_gpu_comm_id(cid) == 0
    r.comm_init(1, 0, bytes(cid))
    canvas = torch.zeros((64, 64, 4), dtype=torch.float64, device="cuda:0")
    req = r.request()
    tu = N.tuning(peer_timeout_ms=300)
    req.tuning = C.pointer(tu)
    req.abi_version = 0
    st = N.RenderStats()
    assert L.izpi_gpu_debug_fault(r.ctx, 3) == 0
    t0 = time.time()
    rc = L.izpi_gpu_render_rank(r.ctx, C.byref(req), C.c_void_p(canvas.data_ptr()), C.byref(st))
    dt = time.time() - t0
    assert L.izpi_gpu_debug_fault(r.ctx, 0) == 0
    assert rc == 0, (rc, L.izpi_gpu_last_error(r.ctx))
    assert dt > 1.0, dt  # it waited for the stall, not 300 ms
    torch.cuda.synchronize()
    ref, _ = oracle_canvas(scene, 64, 64, 4, N.SAMPLER_COLOUR)
    assert_parity(canvas.cpu().numpy(), ref)
    r.close()


def test_multi_render_device_failure_is_reported(gpu):
    """izpi_gpu_multi_render with one failing device (a render fault injected on context 1,
    then a context without a scene): the call returns that device's status and names it,
    every device thread is joined, and the next frame renders bit-exact."""
    from izpi_amd.renderer import MultiGPURenderer
    L = N.lib()
    scene = configs.cornell_rgb()
    r = MultiGPURenderer(scene, 64, 64, 4, [0, 0], bvh="reference")
    ctx1 = L.izpi_gpu_multi_context(r.m, 1)
    assert L.izpi_gpu_debug_fault(ctx1, 2) == 0
    with pytest.raises(RuntimeError, match=r"status 5\): device 1: injected"):
        r.render()
    assert L.izpi_gpu_debug_fault(ctx1, 0) == 0
    img = r.render()
    ref, _ = oracle_canvas(scene, 64, 64, 4, N.SAMPLER_COLOUR)
    assert_parity(img, ref)
    r.close()
    # a device whose scene upload never happened
    m = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    assert L.izpi_gpu_multi_open(devs, 2, C.byref(m)) == 0
    one = GPURenderer(scene, 64, 64, 4)
    assert L.izpi_gpu_upload_scene(L.izpi_gpu_multi_context(m, 0), C.byref(one.host.desc)) == 0
    req = one.request()
    canvas = np.zeros((64, 64, 4))
    rc = L.izpi_gpu_multi_render(m, C.byref(req), canvas.ctypes.data_as(C.c_void_p), None)
    assert rc == N.IZPI_ERR_NO_SCENE, rc
    assert b"device 1" in L.izpi_gpu_multi_last_error(m)
    L.izpi_gpu_multi_close(m)
    one.close()


def test_cli_renders_like_the_python_host(gpu, tmp_path):
    """izpi-render (C++ host, C ABI only) == GPURenderer on the same scene file, bit for bit:
    the spectral example with Render's post-processing, and an OBJ mesh streamed into the
    RGB box through the dragon transforms."""
    import json
    import subprocess
    from pathlib import Path
    from izpi_amd import ingest
    root = Path(__file__).resolve().parents[1]
    cli = root / "izpi_amd" / "_lib" / "izpi-render"
    example = root / "izpi_amd" / "data" / "scenes" / "cornell_box_transparent_pyramid_spectral.pbtxt"
    raw = tmp_path / "c.f64"
    out = subprocess.run([str(cli), "--scene", str(example), "--x", "40", "--y", "40", "--samples", "4",
                          "--raw", str(raw)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["sampler"] == "spectral" and line["bvh"] == "gpu" and line["quantized"] == 0
    assert line["accumulation"] == "forward"
    s = ingest.ProtoScene.from_file(example)
    r = GPURenderer(s, 40, 40, 4, sampler=s.sampler, bvh="gpu", accumulation=N.ACC_FORWARD)
    img = r.render(post=N.POST_SPECTRAL)
    r.close()
    assert np.fromfile(raw, np.float64).tobytes() == img.tobytes()
    box = tmp_path / "box.pbtxt"
    box.write_text(configs.cornell_rgb_pbtxt(1.0))
    cube = root / "tests" / "golden" / "wavefront" / "cube.obj"
    out = subprocess.run([str(cli), "--scene", str(box), "--obj", str(cube), "--x", "40", "--y", "40", "--samples", "4",
                          "--bvh", "reference", "--png-pipeline", "--raw", str(raw)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    sc = configs.cornell_obj(cube)
    r = GPURenderer(sc, 40, 40, 4, accumulation=N.ACC_FORWARD)
    img = r.render(post=N.POST_GAMMA_CLAMP)
    r.close()
    assert np.fromfile(raw, np.float64).tobytes() == img.tobytes()
    import torch
    if torch.cuda.device_count() >= 2:  # --gpus: the multi-GPU entry points (izpi_gpu_multi_*)
        out = subprocess.run([str(cli), "--scene", str(example), "--x", "40", "--y", "40", "--samples", "4", "--gpus", "2",
                              "--raw", str(raw)], capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr


@pytest.mark.parametrize("table", ["duplicates", "unsorted", "single"])
def test_spectral_table_lookups_bitwise(gpu, table):
    """Tabulated SPD lookups (spectral_constant.go:88-106, spectral.go:151-181): the device
    bisects non-decreasing tables and scans the others; both must pick the reference's
    first matching interval. Tables with repeated wavelengths (0/0 at the tie), out of
    order, and with one entry, in the light, the glass index and a background SPD."""
    from izpi_amd.scene import Scene
    tabs = configs.spectral_tables()
    wl = list(tabs["cie_wavelengths"])
    light = list(tabs["light_sources"]["cie_f1_daylight_fluorescent"])
    if table == "duplicates":
        wl_l = wl[:10] + [wl[10]] * 3 + wl[13:]
        ref = ([380, 500, 500, 500, 620, 750], [1.55, 1.5, 1.52, 1.49, 1.47, 1.45])
        bg = (np.array([380.0, 450, 450, 600, 780]), np.array([0.1, 0.2, 0.3, 0.05, 0.4]))
    elif table == "unsorted":
        wl_l = wl[:20] + [wl[25], wl[21], wl[22], wl[23], wl[24], wl[20]] + wl[26:]
        ref = ([380, 620, 500, 560, 750], [1.55, 1.47, 1.5, 1.48, 1.45])
        bg = (np.array([380.0, 600, 450, 780]), np.array([0.1, 0.2, 0.3, 0.4]))
    else:
        wl_l = wl
        ref = ([550], [1.5])
        bg = (np.array([550.0]), np.array([0.25]))
    s = Scene("spd_tables")
    mats = {"Green": s.lambert(spectral=s.spectral_gaussian(0.9, 540, 40)),
            "Red": s.lambert(spectral=s.spectral_tabulated([400, 600, 600, 700], [0.1, 0.8, 0.6, 0.9])),
            "White": s.lambert(spectral=s.spectral_neutral(0.73)),
            "light": s.diffuse_light(spectral=s.spectral_spd(wl_l, light))}
    glass = s.dielectric(spectral_refidx=s.spectral_tabulated(*ref), spectral_absorb=s.spectral_neutral(0.01))
    configs.add_box(s, mats)
    s.add_sphere((50, 30, 50), 15, glass)
    s.set_camera((50, 50, -120), (50, 50, 50), (0, 1, 0), 35, 1.0, 0, 10, 0, 1, 1.0)
    r = GPURenderer(s, 40, 40, 8, sampler=N.SAMPLER_SPECTRAL, spectral_background=bg)
    img = r.render()
    ref_img, ostats = oracle_canvas(s, 40, 40, 8, N.SAMPLER_SPECTRAL, bg=bg)
    assert_parity(img, ref_img, r.stats, ostats)
    r.close()


def test_spectral_tabulated_lookup_device_bitwise(gpu):
    """SpectralConstant.Value of tabulated SPDs on the device (spectral_constant.go:88-106)
    against the oracle's linear scan, bit for bit: near-uniform tables (the interval is
    guessed from lambda, then checked), a table with a jittered grid, one with a repeated
    wavelength and an unsorted one (bisection / scan); lambdas on every grid point, one ulp
    either side, random ones and out-of-range ones."""
    import ctypes as C
    from izpi_amd.scene import Scene
    tabs = configs.spectral_tables()
    cie = np.asarray(tabs["cie_wavelengths"], np.float64)
    rng = np.random.default_rng(3)
    tables = [
        (cie, rng.random(len(cie))),                                   # uniform 5 nm (the CIE grid)
        (np.arange(380.0, 781.0, 10.0), rng.random(41)),                # uniform 10 nm
        (np.arange(400.0, 701.0, 20.0) + rng.uniform(-6, 6, 16), rng.random(16)),  # jittered grid
        (np.array([380.0, 430, 480, 480, 530, 580, 630, 680, 730, 780]), rng.random(10)),  # a tie
        (np.array([380.0, 500, 450, 600, 780]), rng.random(5)),           # unsorted
        (np.array([380.0, 780.0]), np.array([0.25, 0.75])),              # two entries
    ]
    tables[2] = (np.sort(tables[2][0]), tables[2][1])
    s = Scene("tabs")
    ids = [s.spectral_tabulated(wl, vl, proto_float=False) for wl, vl in tables]
    mats = {k: s.lambert(spectral=s.spectral_neutral(0.5)) for k in ("Green", "Red", "White")}
    mats["light"] = s.diffuse_light(spectral=s.spectral_neutral(4.0))
    configs.add_box(s, mats)
    s.set_camera((50, 50, -120), (50, 50, 50), (0, 1, 0), 35, 1.0, 0, 10, 0, 1, 1.0)
    r = GPURenderer(s, 8, 8, 1, sampler=N.SAMPLER_SPECTRAL)
    L = N.lib()
    for tid, (wl, vl) in zip(ids, tables):
        wl = np.ascontiguousarray(wl, np.float64)
        vl = np.ascontiguousarray(vl, np.float64)
        lams = np.ascontiguousarray(np.concatenate([wl, np.nextafter(wl, 0), np.nextafter(wl, 1e4),
                                                    rng.uniform(wl.min() - 5, wl.max() + 5, 5000),
                                                    [300.0, 900.0, float(wl[0]), float(wl[-1])]]))
        ids_arr = np.full(len(lams), float(tid))
        out = np.zeros_like(lams)
        assert L.izpi_gpu_gomath(r.ctx, 37, O.dptr(lams), O.dptr(ids_arr), len(lams), O.dptr(out)) == 0
        ref = np.array([O.lib().oracle_spd_tabulated_value(O.dptr(wl), O.dptr(vl), len(wl), float(x)) for x in lams])
        assert out.tobytes() == ref.tobytes(), (tid, np.flatnonzero(out != ref)[:10])
    r.close()


def test_spectral_sampling_device_bitwise(gpu):
    """SampleWavelength and GetCIEValues on the device (bisected over the CIE tables)
    equal the oracle's linear scans, including randoms that land on the running sums'
    entries and wavelengths on the table's grid points and ends."""
    r = GPURenderer(configs.cornell_rgb(), 8, 8, 1)
    L = N.lib()
    rng = np.random.default_rng(11)
    tabs = configs.spectral_tables()
    wl = np.asarray(tabs["cie_wavelengths"], np.float64)
    y = np.asarray(tabs["cie_y"], np.float64)
    rand = [rng.random(20000), np.array([0.0, 0.5, np.nextafter(1.0, 0.0)])]
    cum = np.cumsum(y)  # sequential float64 sums, the reference's running `current`
    integ = float(tabs["cie_y_integral"])
    rand.append(np.concatenate([cum / integ, np.nextafter(cum / integ, 0), np.nextafter(cum / integ, 2)]))
    rand = np.ascontiguousarray(np.concatenate(rand).clip(0, np.nextafter(1.0, 0.0)))
    lams = np.ascontiguousarray(np.concatenate([rng.uniform(370, 790, 20000), wl, np.nextafter(wl, 0),
                                                np.nextafter(wl, 1e4), [379.0, 380.0, 780.0, 800.0]]))
    def dev(op, x):
        out = np.zeros_like(x)
        assert L.izpi_gpu_gomath(r.ctx, op, O.dptr(x), None, len(x), O.dptr(out)) == 0
        return out
    lam, pdf = dev(32, rand), dev(33, rand)
    l_ref, p_ref = np.zeros_like(rand), np.zeros_like(rand)
    a, b = C.c_double(), C.c_double()
    for k, v in enumerate(rand):
        O.lib().oracle_sample_wavelength(float(v), C.byref(a), C.byref(b))
        l_ref[k], p_ref[k] = a.value, b.value
    assert lam.tobytes() == l_ref.tobytes() and pdf.tobytes() == p_ref.tobytes()
    xyz = np.stack([dev(op, lams) for op in (34, 35, 36)], 1)
    ref = np.zeros((len(lams), 3))
    o3 = (C.c_double * 3)()
    for k, v in enumerate(lams):
        O.lib().oracle_cie_values(float(v), o3)
        ref[k] = list(o3)
    assert xyz.tobytes() == ref.tobytes()
    r.close()


def test_progress_is_monotone_and_completes(gpu):
    """izpi_gpu_progress polled from another thread while a frame renders (the per-tile
    progress of renderer.go:119-121): never decreasing, bounded by the request's samples,
    equal to them once the call returns; the frame stays bit-exact."""
    import threading
    scene = configs.cornell_dragon(1.0, n=60)
    r = GPURenderer(scene, 96, 96, 32, tuning=N.tuning(slots=20000))
    seen, stop = [], threading.Event()

    def poll():
        while not stop.is_set():
            seen.append(r.progress())

    th = threading.Thread(target=poll)
    th.start()
    try:
        img = r.render()
    finally:
        stop.set()
        th.join()
    total = 96 * 96 * 32
    assert r.progress() == (total, total)
    done = [d for d, t in seen if t == total]
    assert done == sorted(done) and all(0 <= d <= total for d in done)
    assert any(0 < d < total for d in done), seen[:5]
    ref, ostats = oracle_canvas(scene, 96, 96, 32, N.SAMPLER_COLOUR)
    assert_parity(img, ref, r.stats, ostats)
    r.close()
