"""The C ABI library: loads on a CPU-only host, exports every symbol include/*.h
declares, and its struct layouts agree with the ctypes mirror (and so with the Go
layout documented in INTEGRATION.md). No compute calls here (no GPU)."""
import re
import subprocess
from pathlib import Path

import pytest

from izpi_amd import _native as N

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        txt = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(izpi_[a-z_0-9]+)\s*\(", txt, re.M))
    return names


def test_every_declared_symbol_is_exported():
    L = N.lib()
    decl = declared_functions()
    assert len(decl) >= 15
    missing = [n for n in sorted(decl) if not hasattr(L, n)]
    assert not missing, missing
    assert set(N.EXPORTS) == decl


def test_dynamic_symbol_table():
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(r"\bT %s$" % name, out, re.M), name


def test_struct_layouts_match():
    import ctypes as C
    L = N.lib()
    for i, cls in enumerate(N.ABI_STRUCTS):
        assert L.izpi_abi_struct_size(i) == C.sizeof(cls), cls.__name__
    assert C.sizeof(N.BVH4Node) == 128  # == hitable.BVH4Node (bvh4.go:23-39)


def test_open_without_gpu_fails_cleanly():
    import ctypes as C
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except Exception:
        pass
    ctx = C.c_void_p()
    assert N.lib().izpi_gpu_open(0, C.byref(ctx)) == N.IZPI_ERR_HIP
    assert not ctx.value


def test_product_does_not_import_oracle():
    for f in (ROOT / "izpi_amd").rglob("*.py"):
        assert not re.search(r"^\s*(from|import)\s+oracle\b", f.read_text(), re.M), f
    for f in (ROOT / "izpi_amd" / "csrc").glob("*"):
        assert "oracle/" not in f.read_text() and "liboracle" not in f.read_text(), f


def test_no_fma_contraction_in_device_code(tmp_path):
    """-ffp-contract=off must reach the device: a*b+c stays two roundings (A21)."""
    src = tmp_path / "probe.hip"
    src.write_text("#include <hip/hip_runtime.h>\n__global__ void k(const double* a, double* o)"
                   "{ int i = threadIdx.x; o[i] = a[i] * a[i+1] + a[i+2]; }\n")
    from izpi_amd import build
    asm = tmp_path / "probe.s"
    subprocess.run([build.HIPCC, "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "--cuda-device-only", "-S",
                    "-o", str(asm), str(src)], check=True)
    text = asm.read_text()
    assert "v_mul_f64" in text and "v_add_f64" in text
    assert "v_fma_f64" not in text and "v_fmac_f64" not in text
