"""The throughput-mode stream definition restated in the oracle (oracle/philox_streams.py).

CPU-only: Philox4x32-10 against the Random123 known-answer vectors, the MWC64X step against
its defining recurrence, and the statistical and structural properties of the lane streams
that the GPU parity tests (test_gpu_philox_parity.py) then hold the fused kernels to.
"""

import numpy as np
import pytest
from scipy.stats import norm

import philox_streams as P


@pytest.mark.parametrize("ctr,key,want", [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
])
def test_philox4x32_10_known_answers(ctr, key, want):
    """Random123 kat_vectors, philox4x32 with 10 rounds."""
    got = P.philox4x32_10(*[np.array([c], np.uint64) for c in ctr], *key)
    assert tuple(int(g[0]) for g in got) == want


def test_mwc64x_recurrence():
    """MWC64X: output x ^ c, then A*x + c split into (carry, x); seeded c = (P1 >> 1) | 1."""
    p0, p1 = 0x89ABCDEF, 0xFFFFFFFF
    g = P.Mwc64x([p0], [p1])
    x, c = p0, (p1 >> 1) | 1
    for _ in range(50):
        assert int(g.next()[0]) == x ^ c
        v = 4294883355 * x + c
        x, c = v & 0xFFFFFFFF, v >> 32
        assert c < 4294883355


def test_lane_payload_words():
    """payload = (P2, P3, m0, m1) of the lane's Philox block and generator."""
    seed, s, N = 0x1234_5678_9ABC, np.array([3, 2**33 + 5]), 256
    lanes = P.lane_generators(seed, s, N)
    tps = N // 16
    lane = tps + 7  # symbol 2**33 + 5, lane 7
    p = P.philox4x32_10(np.array([7], np.uint64), np.array([5], np.uint64), np.array([2], np.uint64),
                        np.array([P.K_LANE], np.uint64), seed & 0xFFFFFFFF, seed >> 32)
    g = P.Mwc64x(p[0], p[1])
    want = [int(p[2][0]), int(p[3][0]), int(g.next()[0]), int(g.next()[0])]
    assert [int(w) for w in lanes.payload[lane]] == want
    assert int(lanes.next()[lane]) == int(g.next()[0])


def test_lane_streams_depend_only_on_seed_and_symbol():
    a = P.lane_generators(7, np.arange(10, 20), 1024)
    b = P.lane_generators(7, np.arange(15, 20), 1024)
    assert np.array_equal(a.payload[5 * 64:], b.payload)
    wa, wb = a.next(), b.next()
    assert np.array_equal(wa[5 * 64:], wb)
    c = P.lane_generators(8, np.arange(10, 20), 1024)
    assert not np.array_equal(c.payload, a.payload)


@pytest.mark.parametrize("N,b", [(1024, 6), (64, 2), (16, 4), (4096, 8)])
def test_payload_bits_uniform(N, b):
    S = max(1, 200_000 // N)
    idx = P.tx_indices(P.lane_generators(3, np.arange(S), N), S, N, b)
    assert idx.shape == (S, N) and idx.min() >= 0 and idx.max() < 2 ** b
    counts = np.bincount(idx.ravel(), minlength=2 ** b)
    exp = idx.size / 2 ** b
    assert np.all(np.abs(counts - exp) < 6 * np.sqrt(exp))


@pytest.mark.parametrize("phi", [0.0, np.pi / 7, np.pi / 4, 0.3])
def test_phase_table_projection_tails(phi):
    """Noise = Rayleigh radius x one of 64 phase points: the projection on any direction phi has
    the Gaussian tail P(> d sigma) = (1/64) sum_j exp(-d^2 / (2 cos^2(theta_j - phi))) to the
    trapezoid rule's accuracy on that smooth periodic integrand."""
    th = 2 * np.pi * (np.arange(P.NOISE_PHASES) + 0.5) / P.NOISE_PHASES - phi
    c = np.cos(th)
    c = c[c > 0]
    for d, tol in ((1.0, 3e-6), (2.0, 1e-8), (3.0, 1e-9), (3.7, 1e-10), (4.5, 1e-10)):
        p = np.exp(-d * d / (2 * c * c)).sum() / P.NOISE_PHASES
        assert abs(p / norm.sf(d) - 1) < tol, (d, p, norm.sf(d))


def test_radius_words():
    """radius^2 sigma^2 2 ln2 (32 - log2(w | 1)) = -2 sigma^2 ln u, u = (w | 1) 2^-32 (stream
    version 3: the radius takes the whole word; u runs over the odd multiples of 2^-32, the
    midpoints of 2^31 equiprobable cells); the largest radius is 6.660 sigma (words 0 and 1), the
    next 6.493 sigma (words 2 and 3); zero for the words whose float32 rounds to 2^32
    (w >= 0xFFFFFF80: 2^-25 of the words)."""
    w = np.array([0, 1, 2, 0x1F8, 0xFFFFFFFF, 1 << 20], np.uint32)
    n = P.noise_from_words(w, np.zeros(len(w), np.int64), 1.0)
    u = (w | 1).astype(np.float64) / 2.0 ** 32
    u[4] = 1.0  # float32(0xFFFFFFFF) rounds to 2^32
    assert np.allclose(np.abs(n), np.sqrt(-2 * np.log(u)), rtol=1e-6)
    assert abs(np.abs(n[0]) - 6.6604) < 1e-3 and np.abs(n[1]) == np.abs(n[0])
    assert abs(np.abs(n[2]) - 6.4934) < 1e-3
    assert np.abs(n[4]) == 0.0


def _radius_sf_on_words(x: float) -> float:
    """P(radius > x sigma) over the 2^32 radius words of stream version 3, counted exactly: the
    radius falls with float32(w | 1), so it exceeds x for the words below the first w whose float32
    value reaches 2^32 exp(-x^2 / 2) (binary search on the monotone map)."""
    t = 2.0 ** 32 * np.exp(-x * x / 2)
    lo, hi = 0, 2 ** 32  # invariant: f(lo - 1) < t <= f(hi), f(w) = float32(w | 1)
    f = lambda v: float(np.float32(np.uint32(v) | np.uint32(1)))
    if f(0) >= t:
        return 0.0
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if f(mid) < t:
            lo = mid
        else:
            hi = mid
    # words 0..lo have f < t (lo is the last such word); the radius at f exactly t equals x
    return (lo + 1) / 2.0 ** 32


@pytest.mark.parametrize("x", [1.0, 3.0, 4.5, 5.0, 5.65, 6.0, 6.3, 6.5, 6.55])
def test_radius_tail_is_rayleigh_to_6_5_sigma(x):
    """Stream version 3's radius is the Rayleigh quantile at the midpoints of 2^31 equiprobable cells
    of u: P(radius > x) = exp(-x^2 / 2) to within one cell (2^-31) plus the float32 rounding of u
    (relative 2^-24) for every x, exact at each cell boundary, the deepest at 6.555 sigma (P = 2^-31);
    version 2 had nothing left beyond 5.65 sigma."""
    want = np.exp(-x * x / 2)
    got = _radius_sf_on_words(x)
    assert abs(got - want) <= 2.0 ** -31 + 2.0 ** -23 * want, (x, got, want)


def test_component_tail_to_6_2_sigma():
    """The component tail the deep-BER checks rest on: P(Re n > d sigma) = (1/64) sum_j P(radius >
    d / cos theta_j) over the phase points with cos > 0, from the exact word counts, against the
    Gaussian Q(d): within 2^-33 absolute at every depth to 6.2 sigma (measured: < 0.15 x 2^-32), so
    within 1e-3 relative to d = 5.5 (BER ~1e-8 at 64-QAM) -- where version 2's truncated radius had
    lost the whole tail beyond 5.65 sigma."""
    th = 2 * np.pi * (np.arange(P.NOISE_PHASES) + 0.5) / P.NOISE_PHASES
    c = np.cos(th)
    c = c[c > 0]
    for d in (3.0, 4.0, 5.0, 5.5, 5.8, 6.0, 6.2):
        p = sum(_radius_sf_on_words(d / cj) for cj in c) / P.NOISE_PHASES
        assert abs(p - norm.sf(d)) <= 2.0 ** -33, (d, p, norm.sf(d))
        if d <= 5.5:
            assert abs(p / norm.sf(d) - 1) < 1e-3, (d, p, norm.sf(d))


def test_phase_words_are_their_own():
    """Version 3 layout: the lane's outputs after the payload are (q0, w0, w1, w2, w3, q1, w4, ...);
    noise sample n's phase is byte n & 3 of its q, low six bits."""
    g = P.lane_generators(11, np.arange(3), 256)
    h = P.lane_generators(11, np.arange(3), 256)
    for n in range(9):
        w, ph = g.noise_draw()
        if n % 4 == 0:
            q = h.next()
        assert np.array_equal(w, h.next())
        assert np.array_equal(ph, (q >> np.uint32(8 * (n % 4))) & np.uint32(63))


def test_noise_is_complex_gaussian():
    S, N, sigma = 1000, 1024, 0.3
    g = P.lane_generators(5, np.arange(S), N)
    n = P.lane_noise(g, S, N, sigma).ravel()
    for comp in (n.real, n.imag, (n * np.exp(-0.4j)).real):
        assert abs(comp.mean()) < 5 * sigma / np.sqrt(n.size)
        assert abs(comp.var() / sigma ** 2 - 1) < 0.01
        k = np.mean((comp / sigma) ** 4)
        assert abs(k - 3) < 0.05
        # tails P(|n| > d sigma) within 4.5 binomial standard errors (z-scores printed)
        for d in (1.0, 2.0, 3.0, 4.0):
            q = 2 * norm.sf(d)
            z = (np.mean(np.abs(comp) > d * sigma) - q) / np.sqrt(q * (1 - q) / comp.size)
            print(f"d {d}: z {z:+.2f}")
            assert abs(z) < 4.5, (d, z)
    assert abs(np.corrcoef(n.real, n.imag)[0, 1]) < 0.01
    # neighbouring time samples are uncorrelated
    assert abs(np.corrcoef(n.real[:-1], n.real[1:])[0, 1]) < 0.01


def test_oracle_link_noise_free_is_error_free():
    r = P.run_philox(2, 32, 1024, 64, np.array([0.8, 0.3j, 0.1]), 2, "MMSE", 30.0, noise_on=False)
    assert r.bit_errors == 0 and r.symbol_errors == 0


def test_noise_table_entries_are_robust():
    """The phase table's float32 cos / sin are the same whether a double cos is evaluated as the
    kernels do (cospi((2j + 1) / 64)) or as the oracle does (cos(pi (2j + 1) / 64)): every exact
    value lies far (> 1e-12 relative) from a float32 rounding midpoint, so any double evaluation
    within a few ulp rounds to the same float32 -- the premise of restating the receivers' noise
    bit for bit from their radii (philox_streams.noise_from_words(radius_fn=...))."""
    th = np.pi * (2.0 * np.arange(P.NOISE_PHASES, dtype=np.longdouble) + 1.0) / P.NOISE_PHASES
    for v in (np.cos(th), np.sin(th)):
        f = v.astype(np.float32)
        for g in (np.nextafter(f, np.float32(np.inf)), np.nextafter(f, np.float32(-np.inf))):
            mid = (f.astype(np.longdouble) + g.astype(np.longdouble)) / 2
            assert np.all(np.abs(v - mid) > 1e-12 * np.abs(v))
    # the oracle's table entries are those float32 values times float32(sigma sqrt(2 ln 2))
    t = P.noise_table(0.37)
    sc = np.float32(0.37 * P.SQRT_2LN2)
    assert np.array_equal(t.real, (sc * np.cos(th.astype(np.float64)).astype(np.float32)).astype(np.float64))


def test_noise_from_given_radii():
    """With the GPU's radii supplied, the noise is radius x table entry (exact in float64) and its
    bound is the product rounding alone; the float64 radius stays within its own bound of it."""
    w = np.random.default_rng(3).integers(0, 2 ** 32, size=20000, dtype=np.uint64).astype(np.uint32)
    sig = 0.21
    ph = np.random.default_rng(4).integers(0, P.NOISE_PHASES, size=w.size)
    n64, b64 = P.noise_from_words(w, ph, sig, with_bound=True)
    rad = lambda ws: np.sqrt(32.0 - np.log2((ws | P.RADIUS_OR).astype(np.float32).astype(np.float64))).astype(np.float32)
    n32, b32 = P.noise_from_words(w, ph, sig, with_bound=True, radius_fn=rad, product_rel=2.0 ** -53)
    assert np.all(np.abs(n32 - n64) <= b64)
    assert np.all(b32 <= 2.0 ** -52 * np.abs(n32) + 1e-300)
