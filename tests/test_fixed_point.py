"""The exact stream-power limbs (csrc/ofdm_device.hpp fx_accum): the float32 path of the complex64
kernels must give the same two limbs as the double path for every float32 share p in [0, 2^24).
Restated here in NumPy with the kernels' operations (power-of-two products, floor, subtraction,
round-half-even), float32 against float64."""

import numpy as np


def limbs_f64(p32: np.ndarray):
    a = p32.astype(np.float64) * 256.0
    hi = np.floor(a)
    return hi.astype(np.uint64), np.rint((a - hi) * 4294967296.0).astype(np.uint64)


def limbs_f32(p32: np.ndarray):
    a = (p32 * np.float32(256.0)).astype(np.float32)
    hi = np.floor(a).astype(np.float32)
    fr = ((a - hi).astype(np.float32) * np.float32(4294967296.0)).astype(np.float32)
    return hi.astype(np.uint64), np.rint(fr).astype(np.uint64)


def test_float32_limbs_equal_double_limbs():
    rng = np.random.default_rng(7)
    # shares across the whole range: tiny (bits below 2^-40), around the limb boundary, large
    e = rng.uniform(-60.0, 23.9, size=400_000)
    p = (2.0 ** e * rng.uniform(1.0, 2.0, size=e.size)).astype(np.float32)
    p = np.concatenate([p, np.float32([0.0, 2.0 ** -41, 2.0 ** -40, 1.5 * 2.0 ** -41, 2.0 ** -17,
                                       1.0 - 2.0 ** -24, 1.0, 2.0 ** 24 - 2.0])])
    h64, l64 = limbs_f64(p)
    h32, l32 = limbs_f32(p)
    assert np.array_equal(h64, h32)
    assert np.array_equal(l64, l32)
    # the value the limbs carry is p rounded to 2^-40
    v = h64.astype(np.float64) * 2.0 ** -8 + l64.astype(np.float64) * 2.0 ** -40
    assert np.all(np.abs(v - p.astype(np.float64)) <= 2.0 ** -41 * (1 + 1e-12) + np.abs(p) * 2.0 ** -52)


def normalize(l0: np.ndarray, l1: np.ndarray):
    """fx_normalize: carry limb 0's bits above 2^32 into limb 1."""
    return l0 & np.uint64(0xFFFFFFFF), l1 + (l0 >> np.uint64(32))


def test_double_share_whose_fraction_rounds_to_2_32_carries():
    """A complex128 share whose fraction lies within 2^-41 of 1 rounds to exactly 2^32 units of
    2^-40: fx_accum converts it through 64 bits (a 32-bit conversion of 2^32 is undefined and
    the hardware clamps it to 2^32 - 1) and fx_normalize carries it into limb 1."""
    p = np.array([(4096.0 + 1.0 - 2.0 ** -40) / 256.0, (1.0 - 2.0 ** -45) / 256.0, 2.0 ** 23 - 2.0 ** -33])
    hi, lo = limbs_f64(p)
    assert lo[0] == 2 ** 32 and lo[1] == 2 ** 32
    l0, l1 = normalize(lo, hi)
    v = l1.astype(np.float64) * 2.0 ** -8 + l0.astype(np.float64) * 2.0 ** -40
    assert np.all(np.abs(v - p) <= 2.0 ** -41)
    assert l1[0] == 4097 and l0[0] == 0
