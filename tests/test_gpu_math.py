"""Device math of the product (csrc/mcpt_device.hpp) against the CPU
specification, bit for bit: IEEE float/double division and sqrt, the fixed
sin/cos (float) and pow / x^5 (double) sequences, the TEA-16/Park-Miller RNG."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "hip"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def probe():
    import torch  # noqa: F401  (single HIP runtime)
    import build_probe
    L = C.CDLL(build_probe.build())
    fp = C.POINTER(C.c_float)
    L.math_probe.argtypes = [C.c_int, C.c_int, fp, fp, fp, fp, C.POINTER(C.c_uint32)]

    def run(op, a, b):
        a = np.ascontiguousarray(a, np.float32); b = np.ascontiguousarray(b, np.float32)
        n = a.size
        o0 = np.zeros(n, np.float32); o1 = np.zeros(n, np.float32); u = np.zeros(2 * n, np.uint32)
        rc = L.math_probe(op, n, a.ctypes.data_as(fp), b.ctypes.data_as(fp), o0.ctypes.data_as(fp),
                          o1.ctypes.data_as(fp), u.ctypes.data_as(C.POINTER(C.c_uint32)))
        assert rc == 0
        return o0, o1, u
    return run


def _inputs(n=200000, seed=0):
    r = np.random.default_rng(seed)
    a = np.concatenate([r.uniform(-10, 10, n // 2), r.standard_normal(n // 4) * 1e-3,
                        np.exp(r.uniform(-80, 80, n - n // 2 - n // 4))]).astype(np.float32)
    b = np.concatenate([r.uniform(-10, 10, n // 2), r.uniform(0.5, 2, n // 4),
                        np.exp(r.uniform(-40, 40, n - n // 2 - n // 4))]).astype(np.float32)
    return a, b


def test_float_div_rcp_sqrt_exact(probe):
    a, b = _inputs()
    with np.errstate(all="ignore"):
        o, _, _ = probe(0, a, b)
        assert np.array_equal(o.view(np.uint32), (a / b).view(np.uint32))
        o, _, _ = probe(1, a, b)
        assert np.array_equal(o.view(np.uint32), (np.float32(1) / a).view(np.uint32))
        aa = np.abs(a)
        o, _, _ = probe(2, aa, b)
        assert np.array_equal(o.view(np.uint32), np.sqrt(aa).view(np.uint32))
        o, _, _ = probe(8, a, b)
        ref = (a - b) * (np.float32(1) / (b - np.float32(0.5)))
        assert np.array_equal(o.view(np.uint32), ref.view(np.uint32))


def test_shared_div_formulas_exact(probe):
    """ops 12 / 13: the two recip_shared variants (IEEE double 1/d; v_rcp_f64 +
    two Newton steps) give IEEE f32 a / d bit for bit (tests/test_div_shared.py)."""
    from test_div_shared import same_bits, shared_cases
    a, d = shared_cases(400_000, seed=11)
    with np.errstate(all="ignore"):
        ref = a / d
    for op in (12, 13):
        o, _, _ = probe(op, a, d)
        assert same_bits(o, ref), op


def test_double_div_exact(probe):
    a, b = _inputs()
    _, _, u = probe(5, a, b)
    got = u.view(np.uint64)
    with np.errstate(all="ignore"):
        ref = (a.astype(np.float64) / b.astype(np.float64)).view(np.uint64)
    assert np.array_equal(got, ref)


def test_sincos_pow_match_spec(probe, oracle_mod):
    L = oracle_mod.lib()
    r = np.random.default_rng(1)
    phi = (np.float32(2 * 3.14159265359) * r.random(20000, dtype=np.float32)).astype(np.float32)
    s, c, _ = probe(3, phi, phi)
    rs = np.array([L.orc_sinf(float(x)) for x in phi], np.float32)
    rc = np.array([L.orc_cosf(float(x)) for x in phi], np.float32)
    assert np.array_equal(s, rs) and np.array_equal(c, rc)
    x = r.random(20000, dtype=np.float32)
    y = (1.0 / (r.integers(1, 2000, 20000) + 1)).astype(np.float32)
    y[:5000] = 5.0
    o, _, _ = probe(4, x, y)
    ref = np.array([L.orc_powf(float(a), float(b)) for a, b in zip(x, y)], np.float32)
    assert np.array_equal(o, ref)
    o5, _, _ = probe(11, x, x)
    ref5 = np.array([L.orc_pow5f(float(a)) for a in x], np.float32)
    assert np.array_equal(o5, ref5)


def test_rng_matches_spec(probe, oracle_mod):
    L = oracle_mod.lib()
    keys = np.random.default_rng(2).integers(0, 2**32, 2000, dtype=np.uint64).astype(np.uint32)
    samples = np.arange(2000, dtype=np.uint32)
    o, _, u = probe(6, keys.view(np.float32), samples.view(np.float32))
    for i in range(0, 2000, 7):
        sd = L.orc_rng_init(i, int(keys[i]), int(samples[i]))
        assert sd == u[2 * i]
        st = C.c_uint32(sd)
        assert L.orc_rng_next(C.byref(st)) == o[i]
        assert st.value == u[2 * i + 1]
