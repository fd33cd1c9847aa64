"""IZPI_ACC_FORWARD: the forward-throughput accumulation against the recursion.

The recursive samplers (colour.go:33-65, sampler/spectral.go:47-80) return
``emitted + att * (L * s) / p`` per non-specular bounce and ``att * L`` per specular one,
unwound from the deepest bounce. Every scattering material emits 0 (non_emitter.go:12-23,
dielectric.go:219-221), so the sample is the product of the bounces' factors times the
terminal radiance; the forward form carries that product from the camera on
(T = (T * att) * (s / p), T = T * att) and multiplies once at the end. Same rays, same
random draws, same counters; only the rounding differs.

NaN and Inf positions: an IEEE product or quotient is NaN / Inf / 0 / finite according to
two flags of its operands (holds a zero, holds an infinity; a quotient inverts the
divisor's), OR-ed over every factor in any order. The recursion and the forward product
multiply the same factors, so they agree on NaN / Inf / zero wherever no finite
intermediate overflows or underflows (the factors here are ratios of order one).

These CPU tests check the oracle's two forms against each other (the GPU tests check the
kernels' forward mode against the oracle's, bit for bit, in test_gpu_forward.py): pixel
RMSE < 1e-6 (north_star), NaN / Inf at the same pixels, equal counters.
"""
import ctypes as C

import numpy as np
import pytest

from izpi_amd import _native as N
from izpi_amd import configs
from oracle import oracle as O

RMSE_TOL = 1e-6  # north_star: pixel RMSE < 1e-6


def oracle_pair(scene, W, H, spp, sampler, max_depth=50, tiles=None, threads=8):
    """The oracle's recursive and forward canvases of one request, and their stats."""
    o = O.OracleScene(scene, aspect_override=W / H)
    out = []
    for acc in (N.ACC_RECURSIVE, N.ACC_FORWARD):
        req = N.RenderReq(width=W, height=H, spp=spp, max_depth=max_depth, sampler=sampler, seed=12345,
                          abi_version=N.IZPI_ABI_VERSION, accumulation=acc)
        keep = None
        if tiles is not None:
            keep = np.ascontiguousarray(tiles, np.uint32)
            req.num_tiles = len(keep)
            req.tiles = keep.ctypes.data_as(C.POINTER(C.c_uint32))
        canvas, st = o.render(req, threads=threads)
        out.append((canvas.reshape(H, W, 4), st))
    o.close()
    return out


def assert_within_tolerance(img, ref, stats=None, ref_stats=None):
    """north_star's contract between two accumulation orders: same NaN / Inf pixels, RMSE
    < 1e-6 over the finite ones, every counter equal."""
    assert img.shape == ref.shape
    assert np.array_equal(np.isnan(img), np.isnan(ref)), "NaN positions differ"
    assert np.array_equal(np.isposinf(img), np.isposinf(ref)), "+Inf positions differ"
    assert np.array_equal(np.isneginf(img), np.isneginf(ref)), "-Inf positions differ"
    fin = np.isfinite(img)
    rmse = float(np.sqrt(np.mean((img[fin] - ref[fin]) ** 2))) if fin.any() else 0.0
    assert rmse < RMSE_TOL, rmse
    if stats is not None:
        for k in ("rays", "node_visits", "tri_tests", "sph_tests", "light_tri_tests", "light_sph_tests", "samples"):
            assert stats[k] == ref_stats[k], (k, stats[k], ref_stats[k])
    return rmse


def special_scene(sampler):
    """Surfaces whose attenuation is infinite or negative (samples of Inf, NaN, signed
    zeros: the spectral path has no DeNAN, A8), glass, and an open box."""
    from izpi_amd.scene import Scene
    s = Scene("special")
    if sampler == N.SAMPLER_COLOUR:
        mats = configs.rgb_box_materials(s)
        configs.add_box(s, mats)
        s.add_sphere((35, 20, 45), 18, s.metal((0.9, float("inf"), -0.4), 0.05))
        s.add_sphere((70, 15, 30), 12, s.lambert(albedo=s.constant((float("inf"), 0.5, -0.7))))
        s.add_sphere((55, 60, 40), 10, s.dielectric(ref_idx=1.5, absorb=(0.12, 0.05, 0.02)))
    else:
        tabs = configs.spectral_tables()
        mats = {
            "Green": s.lambert(spectral=s.spectral_gaussian(0.9, 540, 40)),
            "Red": s.lambert(spectral=s.spectral_gaussian(float("inf"), 640, 40)),
            "light": s.diffuse_light(spectral=s.spectral_spd(tabs["cie_wavelengths"],
                                                              tabs["light_sources"]["cie_f1_daylight_fluorescent"])),
            "White": s.pbr(s.constant((0.7, 0.7, 0.7)), spectral=s.spectral_gaussian(-0.8, 560, 80)),
        }
        configs.add_box(s, mats)
        s.add_sphere((70, 15, 30), 12, s.dielectric(spectral_refidx=s.spectral_tabulated(configs._REFIDX_WL, configs._REFIDX_V)))
    configs.cornell_camera(s, 1.0)
    return s


def scene_case(which):
    """(scene, W, H, spp, sampler) of the forward-accumulation cases."""
    from tests.test_gpu_parity_materials import rgb_glass_box, spectral_pbr_box
    if which == "cornell":
        return configs.cornell_rgb(), 40, 40, 8, N.SAMPLER_COLOUR
    if which == "dragon":
        return configs.cornell_dragon(1.0, n=24), 32, 32, 8, N.SAMPLER_COLOUR
    if which == "pbr":
        return configs.cornell_pbr(1.5, res=64), 30, 20, 8, N.SAMPLER_COLOUR
    if which == "glass_spectral":
        return configs.cornell_glass_spectral(), 32, 32, 8, N.SAMPLER_SPECTRAL
    if which == "glass_rgb_beer":  # Beer-Lambert path-length rays (dielectric.go:118-153)
        return rgb_glass_box(True), 32, 32, 8, N.SAMPLER_COLOUR
    if which == "pbr_spectral":
        return spectral_pbr_box(True), 32, 32, 8, N.SAMPLER_SPECTRAL
    if which == "special_rgb":
        return special_scene(N.SAMPLER_COLOUR), 32, 32, 8, N.SAMPLER_COLOUR
    if which == "special_spectral":
        return special_scene(N.SAMPLER_SPECTRAL), 32, 32, 8, N.SAMPLER_SPECTRAL
    raise ValueError(which)


CASES = ["cornell", "dragon", "pbr", "glass_spectral", "glass_rgb_beer", "pbr_spectral", "special_rgb",
         "special_spectral"]


@pytest.mark.parametrize("which", CASES)
def test_oracle_forward_matches_recursion(which):
    scene, W, H, spp, sampler = scene_case(which)
    (rec, rs), (fwd, fs) = oracle_pair(scene, W, H, spp, sampler)
    assert_within_tolerance(fwd, rec, fs, rs)
    if which == "special_spectral":  # the case exercises non-finite samples
        assert (~np.isfinite(rec)).any()


@pytest.mark.parametrize("max_depth", [0, 1, 3])
def test_oracle_forward_max_depth(max_depth):
    """Blue at maxDepth (colour.go:34-36) and the background SPD (sampler/spectral.go:48-51)."""
    for scene, sampler in ((configs.cornell_rgb(), N.SAMPLER_COLOUR), (configs.cornell_glass_spectral(), N.SAMPLER_SPECTRAL)):
        (rec, rs), (fwd, fs) = oracle_pair(scene, 24, 24, 4, sampler, max_depth=max_depth)
        assert_within_tolerance(fwd, rec, fs, rs)
        if max_depth == 0:
            assert fwd.tobytes() == rec.tobytes()  # no bounce: T = 1 exactly


def test_class_algebra_of_special_values():
    """The NaN / Inf / zero class of a chain of IEEE products and quotients does not depend
    on the order it is evaluated in (the argument behind identical NaN / Inf positions):
    exhaustive over factor classes, recursive order (deepest first) against forward order."""
    import itertools
    vals = {"zero": 0.0, "fin": 0.75, "inf": np.inf, "nan": np.nan}

    def cls(x):
        return "nan" if np.isnan(x) else "inf" if np.isinf(x) else "zero" if x == 0 else "fin"

    with np.errstate(all="ignore"):
        for n in (1, 2, 3):
            for combo in itertools.product(vals, repeat=3 * n + 1):  # per level: att, s, p; then E
                levels = [tuple(vals[c] for c in combo[3 * k:3 * k + 3]) for k in range(n)]
                E = vals[combo[-1]]
                L = np.float64(E)
                for att, s, p in reversed(levels):  # colour.go:53-57, deepest level first
                    L = np.float64(0.0) + (np.float64(att) * (L * np.float64(s))) / np.float64(p)
                T = np.float64(1.0)
                for att, s, p in levels:  # the forward form
                    T = (T * np.float64(att)) * (np.float64(s) / np.float64(p))
                assert cls(T * np.float64(E)) == cls(L), (levels, E)
