"""The Go shim against the C headers, with no Go toolchain (tests/go_shim_check.py): every
C function, constant, type and struct field renderer_gpu.go names exists in include/, and
every argument and field assignment has the exact type cgo would demand. The mutations
below prove the check bites."""
import re

import pytest

from tests import go_shim_check as G

SRC = G.SHIM.read_text()


def test_shim_compiles_against_headers():
    ok, err, code = G.check(SRC)
    assert ok, err
    # the translation covers the whole C surface the shim uses
    called = set(re.findall(r"\bC\.(izpi_\w+)\(", SRC))
    for fn in called:
        assert "&%s" % fn in code or "sizeof(%s)" % fn in code, fn
    assert len(called) >= 25
    for field in ("abi_version", "width", "height", "spp", "max_depth", "out_layout", "seed", "exposure",
                  "background", "sampler", "num_bg_spd", "bg_spd_wavelengths", "bg_spd_values", "post",
                  "num_tiles", "tiles"):
        assert ").%s" % field in code, field


@pytest.mark.parametrize("old,new", [
    ("C.uint32_t(opt.SizeX)", "C.int(opt.SizeX)"),                       # wrong integer type for a field
    ("r.req.num_bg_spd = 75", "r.req.num_bg_spds = 75"),                 # misspelt field
    ("&numNodes, (*C.uint32_t)(unsafe.Pointer(&order[0])), &ms)", "&numNodes, (*C.uint32_t)(unsafe.Pointer(&order[0])))"),  # arity
    ("C.IZPI_POST_SPECTRAL", "C.IZPI_POST_SPECTRA"),                    # unknown constant
    ("(*C.double)(unsafe.Pointer(&boxes[0]))", "(*C.float)(unsafe.Pointer(&boxes[0]))"),  # pointer type
    ("st[i].rays", "st[i].ray"),                                          # field read
    ("C.izpi_gpu_progress(r.ctx, &d, &t)", "C.izpi_gpu_progress(r.ctx, &d, &d, &t)"),
])
def test_check_rejects_mutations(old, new):
    assert old in SRC, old
    ok, err, _ = G.check(SRC.replace(old, new, 1))
    assert not ok, "mutation %r -> %r passed the check" % (old, new)


def test_render_logs_ray_count_like_the_reference():
    """renderer.go:213 logs `Rendering completed in %v using %v rays`; the shim's Render
    passes stats in both forms and logs the same line with their ray sum."""
    body = SRC[SRC.index("func (r *Renderer) Render("):SRC.index("func (r *Renderer) NumRays(")]
    assert 'log.Infof("Rendering completed in %v using %v rays", time.Since(startTime), r.numRays)' in body
    assert "C.izpi_gpu_multi_render(r.m, &req, (*C.double)(unsafe.Pointer(&pix[0])), &st[0])" in body
    assert "C.izpi_gpu_render(r.ctx, &req, (*C.double)(unsafe.Pointer(&pix[0])), &st[0])" in body
    assert "r.numRays += uint64(st[i].rays)" in body
