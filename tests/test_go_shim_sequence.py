"""The C replay issues the Go shim's library calls in the same order, in every branch
(tests/go_shim_sequence.py): one context or izpi_gpu_multi_*, GPU-built or host BVH,
Render or RenderTiles. The mutations prove the check bites."""
import pytest

from tests import go_shim_sequence as S

GO = S.SHIM.read_text()
CR = S.REPLAY.read_text()


def test_replay_issues_the_shims_calls_in_every_branch():
    assert S.check(GO, CR) == []
    # the walk covers the whole frame: the scenario with every option on
    full = S.c_sequence(CR, {"multi": True, "gpu_bvh": True, "tiles": False})
    assert full == ["izpi_scene_parse_binary", ("per item", "izpi_scene_set_image"), "izpi_scene_to_input",
                    "izpi_host_build_scene_ex", "izpi_gpu_multi_open", "izpi_gpu_multi_context",
                    "izpi_host_scene_prim_boxes", "izpi_gpu_build_bvh4", "izpi_host_scene_set_bvh",
                    "izpi_gpu_multi_upload_scene", "izpi_gpu_multi_prepare", "izpi_gpu_multi_render", "izpi_gpu_multi_close",
                    "izpi_host_scene_free", "izpi_scene_free"]
    one = S.go_sequence(GO, {"multi": False, "gpu_bvh": False, "tiles": True})
    assert one == ["izpi_scene_parse_binary", ("per item", "izpi_scene_set_image"), "izpi_scene_to_input",
                   "izpi_host_build_scene_ex", "izpi_gpu_open", "izpi_gpu_upload_scene", "izpi_gpu_prepare", "izpi_gpu_output_bytes",
                   "izpi_gpu_render", "izpi_gpu_close", "izpi_host_scene_free", "izpi_scene_free"]


def _swap_lines(src, a, b):
    """src with the (single) lines containing a and b exchanged."""
    lines = src.split("\n")
    ia = [i for i, l in enumerate(lines) if a in l]
    ib = [i for i, l in enumerate(lines) if b in l]
    assert len(ia) == 1 and len(ib) == 1, (a, b)
    lines[ia[0]], lines[ib[0]] = lines[ib[0]], lines[ia[0]]
    return "\n".join(lines)


REPLAY_MUTATIONS = [
    # two calls swapped
    lambda s: _swap_lines(s, "if (izpi_host_scene_prim_boxes(", "if (izpi_host_scene_set_bvh("),
    # the host-BVH branch builds on the GPU anyway
    lambda s: s.replace("if (!ref_bvh) {", "if (1) {", 1),
    # one context's close for a multi renderer
    lambda s: s.replace("if (m) izpi_gpu_multi_close(m);", "if (m) izpi_gpu_close(ctx);", 1),
    # a multi renderer uploads through device 0's context only
    lambda s: s.replace("if (izpi_gpu_multi_upload_scene(m, izpi_host_scene_desc(host)))",
                        "if (izpi_gpu_upload_scene(ctx, izpi_host_scene_desc(host)))", 1),
    # RenderTiles without sizing its output
    lambda s: s.replace("nout = (size_t)(izpi_gpu_output_bytes(&tr) / sizeof(double));", "nout = 0;", 1),
    # the image textures set after the scene conversion
    lambda s: _swap_lines(s, "if (izpi_scene_set_image(", "if (izpi_scene_to_input("),
]


def _fails(go, c):
    try:
        return S.check(go, c) != []
    except KeyError:  # an undecided condition around library calls fails the check too
        return True


@pytest.mark.parametrize("k", range(len(REPLAY_MUTATIONS)))
def test_check_rejects_replay_mutations(k):
    mutated = REPLAY_MUTATIONS[k](CR)
    assert mutated != CR
    assert _fails(GO, mutated)


GO_MUTATIONS = [
    ("\t\tC.izpi_host_scene_free(r.host)\n\t\tr.host = nil\n\t}\n\tif r.ps != nil {\n\t\tC.izpi_scene_free(r.ps)",
     "\t\tC.izpi_scene_free(r.ps)\n\t\tr.host = nil\n\t}\n\tif r.ps != nil {\n\t\tC.izpi_host_scene_free(r.host)"),
    ("\tif opt.BVH == BVHGPU {\n\t\tdesc", "\tif opt.BVH != BVHGPU {\n\t\tdesc"),
    ("packed := make([]float64, int(C.izpi_gpu_output_bytes(&req))/8)", "packed := make([]float64, 1<<20)"),
]


@pytest.mark.parametrize("old,new", GO_MUTATIONS)
def test_check_rejects_shim_mutations(old, new):
    assert old in GO, old
    assert _fails(GO.replace(old, new, 1), CR)


def test_undecided_branch_fails_loudly():
    """A new branch around library calls needs an entry in the condition tables."""
    mutated = CR.replace("if (ntiles > 0) {", "if (ntiles > 0 && W > 0) {", 1)
    with pytest.raises(KeyError):
        S.check(GO, mutated)
