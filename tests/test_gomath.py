"""Go `math` restatements (oracle/go_math_ref.h vs izpi_amd/csrc/gomath.h).

The hot path calls math.Sin/Cos (vec3.go:122-137), Pow (material.go:42,
spectral_constant.go:71, pbr.go:124), Exp (dielectric.go:110,170-172), Atan2/Asin
(sphere.go:30-31), Tan (camera.go:33). Both restatements must agree bit for bit with
each other (and the device build, tests/test_gpu_parity.py); their accuracy against
the platform libm pins the transcribed Cephes/FreeBSD constants.
"""
import math
import struct

import numpy as np
import pytest

from izpi_amd import _native as N
from oracle import oracle as O

OPS = {"sin": 0, "cos": 1, "tan": 2, "exp": 3, "log": 4, "pow": 5, "atan2": 6, "asin": 7, "sqrt": 8, "div": 9, "atan": 10}


def ulp_diff(a, b):
    ia = struct.unpack("<q", struct.pack("<d", a))[0]
    ib = struct.unpack("<q", struct.pack("<d", b))[0]
    if ia < 0:
        ia = -(2 ** 63) - ia
    if ib < 0:
        ib = -(2 ** 63) - ib
    return abs(ia - ib)


def inputs(op, n=4000, seed=1):
    rng = np.random.default_rng(seed)
    if op in ("sin", "cos"):
        x = np.concatenate([rng.uniform(0, 2 * math.pi, n), rng.uniform(-50, 50, n // 4), [0.0, -0.0, math.pi / 4, 1e-300]])
        return x, np.zeros_like(x)
    if op == "tan":
        x = np.concatenate([rng.uniform(-1.5, 1.5, n), [0.0, 0.3490658503988659]])
        return x, np.zeros_like(x)
    if op == "exp":
        x = np.concatenate([rng.uniform(-745, 709, n // 2), rng.uniform(-5, 5, n // 2), [0.0, -0.5, 1e-10, -1e-10]])
        return x, np.zeros_like(x)
    if op == "log":
        x = np.concatenate([np.exp(rng.uniform(-700, 700, n)), [1.0, 0.5, 2.0]])
        return x, np.zeros_like(x)
    if op == "pow":
        x = np.concatenate([rng.uniform(0, 1, n // 2), rng.uniform(-3, 3, n // 2)])
        y = np.concatenate([np.full(n // 4, 5.0), np.full(n // 4, 2.0), rng.uniform(-3, 3, n // 2)])
        x = np.where(y != np.round(y), np.abs(x), x)
        # Go's special cases (pow.go): +-0, +-Inf, NaN, negative bases with integer exponents
        sx = [float("-inf"), float("inf"), -0.0, 0.0, -2.0, -0.5, 0.5, 1.0, -1.0, float("nan")]
        sy = [-3.0, -2.0, 2.0, 3.0, 0.5, -0.5, 2.5, float("inf"), float("-inf"), float("nan"), 1.0, 0.0]
        gx, gy = np.meshgrid(sx, sy)
        return np.concatenate([x, gx.ravel()]), np.concatenate([y, gy.ravel()])
    if op == "atan2":
        return rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)
    if op in ("asin",):
        x = np.concatenate([rng.uniform(-1, 1, n), [1.0, -1.0, 0.7, 0.69999]])
        return x, np.zeros_like(x)
    if op == "atan":
        x = np.concatenate([rng.uniform(-10, 10, n), [0.66, 2.414213562373095, 2.5]])
        return x, np.zeros_like(x)
    if op == "sqrt":
        x = np.concatenate([rng.uniform(0, 1e6, n), np.exp(rng.uniform(-700, 700, n // 2))])
        return x, np.zeros_like(x)
    if op == "div":
        return rng.uniform(-1e3, 1e3, n), rng.uniform(-1e3, 1e3, n) + 1e-3
    raise KeyError(op)


REF = {"sin": math.sin, "cos": math.cos, "tan": math.tan, "exp": math.exp, "log": math.log,
       "pow": lambda x, y: math.pow(x, y), "atan2": math.atan2, "asin": math.asin, "sqrt": math.sqrt,
       "div": lambda x, y: x / y, "atan": math.atan}
MAX_ULP = {"sin": 2, "cos": 2, "tan": 4, "exp": 1, "log": 1, "pow": 2, "atan2": 2, "asin": 2, "sqrt": 0, "div": 0, "atan": 2}


@pytest.mark.parametrize("op", sorted(OPS))
def test_product_header_matches_oracle_bitwise(op):
    L = N.lib()
    x, y = inputs(op)
    for a, b in zip(x, y):
        p = L.izpi_host_gomath(OPS[op], float(a), float(b))
        o = O.gomath(OPS[op], float(a), float(b))
        assert struct.pack("<d", p) == struct.pack("<d", o), (op, a, b, p, o)


@pytest.mark.parametrize("op", sorted(OPS))
def test_accuracy_against_libm(op):
    x, y = inputs(op, n=2000, seed=7)
    worst = 0
    for a, b in zip(x, y):
        if not (math.isfinite(a) and math.isfinite(b)) or (op == "pow" and (a == 0.0 or (a < 0 and b != round(b)))):
            continue  # special cases: checked against Go's table in test_pow_special_cases
        o = O.gomath(OPS[op], float(a), float(b))
        r = REF[op](float(a), float(b)) if op in ("pow", "atan2", "div") else REF[op](float(a))
        worst = max(worst, ulp_diff(o, r))
    assert worst <= MAX_ULP[op], (op, worst)


def pow_square_inputs():
    """x across the whole exponent range (subnormals, the 2^-511 edge of pow's x*x shortcut,
    huge values whose square overflows) with y = 2."""
    rng = np.random.default_rng(5)
    k = np.arange(-1074, 1024)
    x = np.ldexp(rng.uniform(1, 2, k.size), k) * np.where(rng.random(k.size) < 0.5, -1, 1)
    edge = np.ldexp(1.0, -511)
    x = np.concatenate([x, [edge, np.nextafter(edge, 0), np.nextafter(edge, 1), -edge, 5e-324, -5e-324, 1e-160, 1e154,
                            1.4e154, 0.0, -0.0, float("inf"), float("-inf"), float("nan")]])
    return x, np.full_like(x, 2.0)


def pow_fifth_inputs():
    """x across the whole exponent range (the 2^-204 / 2^204 edges of pow's x^5 shortcut,
    subnormal and overflowing fifth powers, the signed zeros) with y = 5."""
    rng = np.random.default_rng(7)
    k = np.arange(-1074, 1024)
    x = np.ldexp(rng.uniform(1, 2, k.size), k) * np.where(rng.random(k.size) < 0.5, -1, 1)
    lo, hi = np.ldexp(1.0, -204), np.ldexp(1.0, 204)
    u = rng.uniform(0, 1, 4000)  # PBR's 1 - cos(theta)
    x = np.concatenate([x, u, 1 - u, [lo, np.nextafter(lo, 0), np.nextafter(lo, 1), -lo, hi, np.nextafter(hi, 0),
                                       np.nextafter(hi, 1e308), -hi, 5e-324, 0.0, -0.0, 1.0, -1.0,
                                       float("inf"), float("-inf"), float("nan")]])
    return x, np.full_like(x, 5.0)


def test_pow_fifth_shortcut_bitwise():
    """gomath.h's Pow(x, 5) shortcut equals the oracle's restatement of pow.go's loop."""
    L = N.lib()
    for a, b in zip(*pow_fifth_inputs()):
        p = L.izpi_host_gomath(OPS["pow"], float(a), float(b))
        o = O.gomath(OPS["pow"], float(a), float(b))
        assert struct.pack("<d", p) == struct.pack("<d", o), (a, p, o)


def test_pow_square_shortcut_bitwise():
    """gomath.h's Pow(x, 2) shortcut (x * x outside the subnormal-square range) equals the
    oracle's restatement of pow.go's loop on every binade."""
    L = N.lib()
    for a, b in zip(*pow_square_inputs()):
        p = L.izpi_host_gomath(OPS["pow"], float(a), float(b))
        o = O.gomath(OPS["pow"], float(a), float(b))
        assert struct.pack("<d", p) == struct.pack("<d", o), (a, p, o)


def test_special_values():
    assert O.gomath(OPS["sin"], -0.0) == 0.0 and math.copysign(1, O.gomath(OPS["sin"], -0.0)) < 0
    assert math.isnan(O.gomath(OPS["cos"], float("inf")))
    assert O.gomath(OPS["exp"], float("-inf")) == 0.0
    assert O.gomath(OPS["pow"], 0.0, 5.0) == 0.0
    assert O.gomath(OPS["pow"], 2.0, 0.5) == math.sqrt(2.0)
    assert O.gomath(OPS["atan2"], 0.0, -1.0) == math.pi
    # Payne-Hanek range (|x| >= 2^29) is outside the restatement: NaN by design
    assert math.isnan(O.gomath(OPS["sin"], 2.0 ** 30))


def test_pow_special_cases():
    """pow.go's special-case table (the branches the GPU build writes out without recursion)."""
    inf, nan = float("inf"), float("nan")
    P = lambda x, y: O.gomath(OPS["pow"], x, y)
    H = lambda x, y: N.lib().izpi_host_gomath(OPS["pow"], x, y)
    cases = [((-inf, -3.0), -0.0), ((-inf, -2.0), 0.0), ((-inf, 3.0), -inf), ((-inf, 2.0), inf),
             ((-inf, 0.5), inf), ((-inf, -0.5), 0.0), ((-0.0, -3.0), -inf), ((-0.0, -2.0), inf), ((0.0, -1.0), inf),
             ((-0.0, 3.0), -0.0), ((-0.0, 2.0), 0.0), ((inf, -1.0), 0.0), ((inf, 2.0), inf), ((-1.0, inf), 1.0),
             ((0.5, inf), 0.0), ((2.0, -inf), 0.0), ((-2.0, 3.0), -8.0), ((-8.0, 1.0 / 3.0), nan), ((nan, 0.0), 1.0)]
    for (x, y), want in cases:
        for f in (P, H):
            got = f(x, y)
            if math.isnan(want):
                assert math.isnan(got), (x, y, got)
            else:
                assert got == want and math.copysign(1, got) == math.copysign(1, want), (x, y, got, want)


def test_sincos_shared_reduction_bitwise():
    """gomath.h's sincos_nonneg (one sin.go reduction and both polynomials, used for the
    random directions' phi = 2 Pi r, vec3.go:119-138) returns the oracle's Sin and Cos bit
    for bit for phi in [0, 2 Pi), at the octant boundaries and at +0."""
    rng = np.random.default_rng(5)
    r = np.concatenate([rng.uniform(0, 1, 20000), np.arange(0, 1, 1 / 64.0), [0.0, 5e-324, 1e-300, 0.9999999999999999]])
    phi = 6.283185307179586 * r
    octants = np.arange(9) * (math.pi / 4)
    phi = np.concatenate([phi, octants, np.nextafter(octants, 0), np.nextafter(octants, 10), [0.0]])
    phi = phi[phi >= 0]
    L = N.lib()
    for a in phi:
        a = float(a)
        assert struct.pack("<d", L.izpi_host_gomath(11, a, 0.0)) == struct.pack("<d", O.gomath(OPS["sin"], a, 0.0)), a
        assert struct.pack("<d", L.izpi_host_gomath(12, a, 0.0)) == struct.pack("<d", O.gomath(OPS["cos"], a, 0.0)), a
