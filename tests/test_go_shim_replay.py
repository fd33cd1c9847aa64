"""The Go shim's exact C call sequence (integration/go/render/gpu/renderer_gpu.go:101-283,
replayed by integration/c/go_shim_replay.c) on proto.Marshal-form wire bytes of a scene
file: parse_binary -> set_image -> scene_to_input -> build_scene_ex(SKIP_BVH) ->
build_bvh4 -> set_bvh -> upload -> render with Render's post flags. The canvas must equal
the Python host's (GPURenderer on the same scene, GPU tree, same post) bit for bit, on one
context and through izpi_gpu_multi_* with two."""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from izpi_amd import _native as N
from izpi_amd import build, configs, ingest
from izpi_amd.renderer import GPURenderer, gpu_leaf_max
from oracle import oracle as O

ROOT = Path(__file__).resolve().parents[1]
EXAMPLE = ROOT / "izpi_amd" / "data" / "scenes" / "cornell_box_transparent_pyramid_spectral.pbtxt"


def test_replay_binary_links_and_reports_usage():
    out = subprocess.run([str(build.REPLAY)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 1 and "usage" in out.stderr


def _replay(tmp_path, text, png, devices, extra=()):
    izpi = tmp_path / "scene.izpi"
    izpi.write_bytes(ingest.ProtoScene(text.encode()).to_wire())
    raw = tmp_path / "canvas.f64"
    cmd = [str(build.REPLAY), str(izpi), "40", "40", "4", str(raw)]
    if png:
        cmd.append("--png-pipeline")
    if devices:
        cmd += ["--devices", ",".join(map(str, devices))]
    cmd += list(extra)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    data = np.fromfile(raw, np.float64)
    return json.loads(out.stdout.strip().splitlines()[-1]), (data if extra else data.reshape(40, 40, 4)), izpi


@pytest.mark.gpu
@pytest.mark.parametrize("which,png,devices", [("spectral", False, None), ("spectral", True, [0, 0]),
                                               ("rgb", True, None), ("rgb", False, [0, 0, 0])])
def test_go_shim_call_sequence_bitwise(gpu, tmp_path, which, png, devices):
    text = EXAMPLE.read_text() if which == "spectral" else configs.cornell_rgb_pbtxt(1.0)
    info, got, izpi = _replay(tmp_path, text, png, devices)
    assert info["sampler"] == ("spectral" if which == "spectral" else "colour")
    s = ingest.ProtoScene.from_file(izpi)
    post = (N.POST_SPECTRAL if which == "spectral" else N.POST_NONE) | (N.POST_GAMMA_CLAMP if png else 0)
    r = GPURenderer(s, 40, 40, 4, sampler=s.sampler, bvh="gpu", accumulation=N.ACC_FORWARD)
    want = r.render(post=post)
    leaf_max, exposure = gpu_leaf_max(r.host.desc), r.exposure
    r.close()
    assert got.tobytes() == want.tobytes()
    # and the CPU oracle on the same (GPU-built) tree, with Render's post-processing
    assert got.tobytes() == _oracle_frame(s, 40, 40, 4, leaf_max, exposure, png).tobytes()


def _oracle_frame(s, W, H, spp, leaf_max, exposure, png, bg=None):
    """The oracle's Render() of scene s as the shim renders it by default: on the PLOC +
    surface-area tree (O.lbvh4 restates the GPU builder node for node), forward
    accumulation; the sampler, then FireflyRejection +
    XYZToRGB for the Spectral sampler (renderer.go:215-219), then Gamma + Clamp(1) for the
    png pipeline."""
    o = O.OracleScene(s, aspect_override=W / H)
    nodes, order = O.lbvh4(o.prim_boxes(), leaf_max, N.BVH_PLOC_SAH)
    o.set_bvh(nodes, order)
    req = N.RenderReq(width=W, height=H, spp=spp, max_depth=50, sampler=s.sampler, seed=12345,
                      abi_version=N.IZPI_ABI_VERSION, accumulation=N.ACC_FORWARD)
    keep = []
    if bg is not None:
        wl, val = (np.ascontiguousarray(x, np.float64) for x in bg)
        keep += [wl, val]
        req.num_bg_spd = len(wl)
        req.bg_spd_wavelengths = O.dptr(wl)
        req.bg_spd_values = O.dptr(val)
    canvas, _ = o.render(req, threads=8)
    o.close()
    canvas = canvas.reshape(-1)
    if s.sampler == N.SAMPLER_SPECTRAL:
        canvas = O.xyz_to_rgb(O.firefly(canvas, W, H), W, H, exposure)
    if png:
        canvas = O.postprocess(canvas, W, H, [(N.FILTER_GAMMA, 0.0), (N.FILTER_CLAMP, 1.0)])
    return np.asarray(canvas).reshape(H, W, 4)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_go_shim_spectral_black_background_bitwise(gpu, tmp_path, devices):
    """Leader mode passes colours.SpectralBlack (75 zeros, leader.go:142) as the spectral
    background: the shim holds it in C.malloc memory (cgo pointer rules) and the render
    equals the Python host's with the same background."""
    info, got, izpi = _replay(tmp_path, EXAMPLE.read_text(), False, devices, ["--bg-spd"])
    assert info["bg_spd"] == 75
    got = got.reshape(40, 40, 4)
    s = ingest.ProtoScene.from_file(izpi)
    wl = 380.0 + 5.0 * np.arange(75)
    r = GPURenderer(s, 40, 40, 4, sampler=s.sampler, bvh="gpu", spectral_background=(wl, np.zeros(75)),
                    accumulation=N.ACC_FORWARD)
    want = r.render(post=N.POST_SPECTRAL)
    leaf_max, exposure = gpu_leaf_max(r.host.desc), r.exposure
    r.close()
    assert got.tobytes() == want.tobytes()
    assert got.tobytes() == _oracle_frame(s, 40, 40, 4, leaf_max, exposure, False, bg=(wl, np.zeros(75))).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["spectral", "rgb"])
def test_go_shim_render_tiles_bitwise(gpu, tmp_path, which):
    """RenderTiles (the worker's RenderTile, worker/render.go:17-75): the frame's first
    tiles packed row by row from y0, alpha 1, no post-processing, equal to the same pixels
    of the Python host's whole-frame canvas (row H - y, rgb.go:41)."""
    from izpi_amd.renderer import common_tiles
    text = EXAMPLE.read_text() if which == "spectral" else configs.cornell_rgb_pbtxt(1.0)
    info, got, izpi = _replay(tmp_path, text, False, None, ["--tiles", "3"])
    assert info["tiles"] == 3
    s = ingest.ProtoScene.from_file(izpi)
    r = GPURenderer(s, 40, 40, 4, sampler=s.sampler, bvh="gpu", accumulation=N.ACC_FORWARD)
    canvas = r.render()  # raw XYZ / RGB, no post
    r.close()
    want = []
    for x0, y0, x1, y1 in common_tiles(40, 40)[:3]:
        for y in range(y0, y1 + 1):
            row = 40 - y
            want.append(canvas[row, x0:x1 + 1] if row < 40 else np.full((x1 - x0 + 1, 4), np.nan))
    want = np.concatenate(want).reshape(-1)
    known = ~np.isnan(want)  # sample row 0 lands on canvas row H, which the canvas drops (A9)
    assert got.size == want.size
    assert got[known].tobytes() == want[known].tobytes()
    assert np.all(got.reshape(-1, 4)[:, 3] == 1.0)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_go_shim_reference_bvh_bitwise(gpu, tmp_path, devices):
    """Options.BVH = BVHReference, Options.Accumulation = AccumulationRecursive: the shim
    keeps the host's NewBVH4 tree (no SKIP_BVH flag, no GPU build; replay --ref-bvh
    --recursive), and the canvas equals the Python host's on the reference tree and the
    oracle's own render (the recursion) bit for bit."""
    text = configs.cornell_rgb_pbtxt(1.0)
    info, got, izpi = _replay(tmp_path, text, False, devices, ["--ref-bvh", "--recursive"])
    assert info["ref_bvh"] == 1 and info["recursive"] == 1
    got = got.reshape(40, 40, 4)
    s = ingest.ProtoScene.from_file(izpi)
    r = GPURenderer(s, 40, 40, 4, sampler=s.sampler, bvh="reference")
    want = r.render()
    r.close()
    assert got.tobytes() == want.tobytes()
    o = O.OracleScene(s, aspect_override=1.0)
    req = N.RenderReq(width=40, height=40, spp=4, max_depth=50, sampler=s.sampler, seed=12345)
    canvas, _ = o.render(req, threads=8)
    o.close()
    assert got.tobytes() == np.asarray(canvas).reshape(40, 40, 4).tobytes()
