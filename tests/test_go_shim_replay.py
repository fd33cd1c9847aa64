"""The Go shim's exact C call sequence (integration/go/render/gpu/renderer_gpu.go:90-235,
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
from izpi_amd.renderer import GPURenderer

ROOT = Path(__file__).resolve().parents[1]
EXAMPLE = ROOT / "izpi_amd" / "data" / "scenes" / "cornell_box_transparent_pyramid_spectral.pbtxt"


def test_replay_binary_links_and_reports_usage():
    out = subprocess.run([str(build.REPLAY)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 1 and "usage" in out.stderr


def _replay(tmp_path, text, png, devices):
    izpi = tmp_path / "scene.izpi"
    izpi.write_bytes(ingest.ProtoScene(text.encode()).to_wire())
    raw = tmp_path / "canvas.f64"
    cmd = [str(build.REPLAY), str(izpi), "40", "40", "4", str(raw)]
    if png:
        cmd.append("--png-pipeline")
    if devices:
        cmd += ["--devices", ",".join(map(str, devices))]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout.strip().splitlines()[-1]), np.fromfile(raw, np.float64).reshape(40, 40, 4), izpi


@pytest.mark.gpu
@pytest.mark.parametrize("which,png,devices", [("spectral", False, None), ("spectral", True, [0, 0]),
                                               ("rgb", True, None), ("rgb", False, [0, 0, 0])])
def test_go_shim_call_sequence_bitwise(gpu, tmp_path, which, png, devices):
    text = EXAMPLE.read_text() if which == "spectral" else configs.cornell_rgb_pbtxt(1.0)
    info, got, izpi = _replay(tmp_path, text, png, devices)
    assert info["sampler"] == ("spectral" if which == "spectral" else "colour")
    s = ingest.ProtoScene.from_file(izpi)
    post = (N.POST_SPECTRAL if which == "spectral" else N.POST_NONE) | (N.POST_GAMMA_CLAMP if png else 0)
    r = GPURenderer(s, 40, 40, 4, sampler=s.sampler, bvh="gpu")
    want = r.render(post=post)
    r.close()
    assert got.tobytes() == want.tobytes()
