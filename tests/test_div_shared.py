"""The same-denominator division identity the kernel may use for the Cramer
quotients (CUTracer.cu:54-92) and normalize (Utils.hpp:27-34): for f32 a, d,
RN_f32(a * r) == a / d (IEEE) when r = RN_f64(1 / d).  Checked here with numpy on
random bit patterns, ordinary ranges, near-midpoint quotients and the IEEE
specials (csrc/mcpt_device.hpp recip_shared / div_shared; the device formulas
themselves are checked in tests/test_gpu_math.py)."""
import numpy as np


def shared_cases(n=1_000_000, seed=7):
    r = np.random.default_rng(seed)
    u = r.integers(0, 2**32, (2, n), dtype=np.uint64).astype(np.uint32)
    a1, b1 = u[0].view(np.float32), u[1].view(np.float32)
    a2 = r.uniform(-10, 10, n).astype(np.float32)
    b2 = r.uniform(-10, 10, n).astype(np.float32)
    # quotients next to f32 rounding midpoints: a = RN(d * m), m a 25-bit odd significand
    b3 = r.integers(1, 2**12, n).astype(np.float32)
    m = (r.integers(2**24, 2**25, n) | 1).astype(np.float64) * 2.0**-24
    a3 = (b3.astype(np.float64) * m).astype(np.float32)
    sp = np.array([0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 3.4e38, 1.17e-38, 1.0], np.float32)
    A, B = np.meshgrid(sp, sp)
    return (np.concatenate([a1, a2, a3, A.ravel()]), np.concatenate([b1, b2, b3, B.ravel()]))


def same_bits(x, y):
    return np.array_equal(x.view(np.uint32), y.view(np.uint32)) or bool(
        np.all((x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y))))


def test_shared_reciprocal_division_is_ieee():
    a, d = shared_cases()
    with np.errstate(all="ignore"):
        ref = a / d
        got = (a.astype(np.float64) * (np.float64(1) / d.astype(np.float64))).astype(np.float32)
    assert same_bits(got, ref)
