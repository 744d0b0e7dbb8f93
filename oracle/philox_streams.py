"""Throughput-mode ("philox") streams and link restated on the CPU -- TEST INFRASTRUCTURE ONLY.

The reference draws its payload bits from PCG64 and its noise from NumPy's legacy normal
generator; ``ofdm_oracle.reference_streams`` reproduces those exactly.  The build's
throughput mode instead generates bits and noise inside the fused kernels from a
counter-based definition (``ofdm-based-systems_amd/csrc/ofdm_device.hpp``, section
"throughput-mode streams"), so that a run needs no host data and does not depend on how
symbols are batched or sharded.  This module restates that definition in NumPy and runs
the link through the oracle's arithmetic (``ofdm_oracle``: modulate, channel, equalise,
nearest-point decision -- the functions pinned to the reference's golden vectors), so the
fused throughput kernels are checked against the oracle on identical bits and noise.

Like ``ofdm_oracle`` it is the CHECKER: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.

Definition (stream version 3; one OFDM symbol s of N subcarriers, E = min(16, N) elements
per lane, TPS = N / E lanes; lane t owns subcarrier / time sample k = t + i*TPS for i < E):

* lane block: words P0..P3 of one Philox4x32-10 block, key = (seed mod 2^32, seed >> 32),
  counter = (t, s mod 2^32, s >> 32, 0x1A7E5EED);
* lane generator: MWC64X (D. B. Thomas: multiply-with-carry, base 2^32, A = 4294883355;
  output x ^ c, then (c, x) <- hi / lo of A*x + c) seeded with x = P0, c = (P1 >> 1) | 1;
  its outputs are m0, m1, ...;
* payload: the 128 bits (P2, P3, m0, m1); element i takes the low b bits of byte i (byte i =
  bits 8*(i & 3).. of word i >> 2); with adaptive bit loading b = b_k of its subcarrier
  (b_k = 0: the subcarrier is unused and carries 0+0j);
* noise: the generator continues into the lane's noise samples n = 0, 1, ... (element i is
  sample i, added to the kept time sample k): before samples n = 0, 4, 8, ... the lane draws a
  phase word q, then every sample draws its radius word w (outputs m2 = q, m3..m6 = w for samples
  0..3, m7 = the next q, ...).  Sample n is radius sqrt(32 - log2(float32(w | 1))) (i.e.
  sqrt(-2 ln u) / sqrt(2 ln 2) with u = (w | 1) 2^-32) times table entry j = (q >> 8 (n & 3)) & 63,
  where entry j is float32(sigma sqrt(2 ln 2)) * float32(cos, sin)(2 pi (j + 1/2) / 64) in float32.
  (float32 arithmetic on the GPU, with the hardware log2 / sqrt; here the radius argument follows
  the same float32 rounding of the word and the rest is evaluated in float64.)  u runs over the
  odd multiples of 2^-32 (words 2k and 2k + 1 share u = (2k + 1) 2^-32): the radius is the
  Rayleigh quantile at the midpoints of 2^31 equiprobable cells, so P(radius > x) is exact at every
  cell boundary -- the deepest at 6.555 sigma (P = 2^-31; its cell's mass sits at 6.660 sigma) --
  and within one cell (2^-31) between them.
  (Stream version 2 took the phase from bits 3..8 of the radius word, which truncated the radius
  at 5.65 sigma.)
* zero padding: after the elements' noise the lane's samples continue with the received tail
  samples N + k it owns (k = t + i*TPS < cp, in order of i): tail sample i is noise sample E + i.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

import ofdm_oracle as O  # oracle/ is on the path of its callers (tests, smoke, bench)

PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85
K_LANE = 0x1A7E5EED
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Philox4x32-10 (Salmon et al., SC'11; Random123 reference): 10 rounds of
    (hi(M0 c0) ^ c3 ^ k1 ... ) bijections keyed by the Weyl sequence k += W."""
    c = [np.asarray(v, dtype=np.uint64) & MASK32 for v in (c0, c1, c2, c3)]
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = PHILOX_M0 * c[0]
        p1 = PHILOX_M1 * c[2]
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ np.uint64(k0)) & MASK32, p1 & MASK32,
             ((p0 >> np.uint64(32)) ^ c[3] ^ np.uint64(k1)) & MASK32, p0 & MASK32]
        k0 = (k0 + PHILOX_W0) & 0xFFFFFFFF
        k1 = (k1 + PHILOX_W1) & 0xFFFFFFFF
    return [v.astype(np.uint32) for v in c]


MWC_A = np.uint64(4294883355)
NOISE_PHASES = 64
RADIUS_OR = np.uint32(1)  # u = (w | 1) 2^-32: word 0 joins word 1, u > 0
SQRT_2LN2 = 1.1774100225154747

# Deviations of a point beyond this many standard deviations of z_stat_bound's model are not
# expected (the largest of 1e6 Gaussian deviations is ~5 of them; the model's own uncertainty --
# the receiver's transform taken as no worse than the transmitter's measured one -- is covered by
# the margin).
STAT_K = 16.0


class Mwc64x:
    """MWC64X (D. B. Thomas): output x ^ c, then (c, x) <- hi / lo of A*x + c.  Vectorised
    over lanes; seeded with x = P0, c = (P1 >> 1) | 1 (never a fixed point, c < A)."""

    def __init__(self, p0, p1):
        self.x = np.asarray(p0, np.uint64) & MASK32
        self.c = ((np.asarray(p1, np.uint64) & MASK32) >> np.uint64(1)) | np.uint64(1)

    def next(self) -> np.ndarray:
        r = (self.x ^ self.c).astype(np.uint32)
        v = MWC_A * self.x + self.c  # < 2^64: no wrap
        self.x, self.c = v & MASK32, v >> np.uint64(32)
        return r


class LaneStream:
    """The lane block of every (symbol, lane): payload words and the continuing generator."""

    def __init__(self, p0, p1, p2, p3):
        self.gen = Mwc64x(p0, p1)
        self.payload = np.stack([p2, p3, self.gen.next(), self.gen.next()], axis=1).astype(np.uint32)
        self.n = 0      # next noise sample of every lane
        self.q = None   # its phase word

    def next(self) -> np.ndarray:
        return self.gen.next()

    def noise_draw(self):
        """(radius word, phase index) of every lane's next noise sample n: the phase word q is
        drawn before samples n = 0 mod 4, the radius word w by every sample; phase = byte n & 3 of q,
        low six bits."""
        if self.n % 4 == 0:
            self.q = self.gen.next()
        w = self.gen.next()
        ph = (self.q >> np.uint32(8 * (self.n % 4))) & np.uint32(NOISE_PHASES - 1)
        self.n += 1
        return w, ph


def geometry(N: int):
    E = min(16, N)
    return E, N // E


def lane_generators(seed: int, s: np.ndarray, N: int) -> LaneStream:
    """One lane block per (symbol, lane), lanes in row-major (s, t) order."""
    E, tps = geometry(N)
    s = np.asarray(s, dtype=np.int64)
    ss = np.repeat(s, tps).astype(np.uint64)
    t = np.tile(np.arange(tps, dtype=np.uint64), len(s))
    p = philox4x32_10(t, ss & MASK32, ss >> np.uint64(32), np.full_like(t, K_LANE),
                      seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return LaneStream(*p)


def noise_table(sigma: float) -> np.ndarray:
    """The 64 phase points times sigma sqrt(2 ln 2), float32 components (as built in LDS)."""
    sc = np.float32(sigma * SQRT_2LN2)
    th = np.pi * (2.0 * np.arange(NOISE_PHASES) + 1.0) / NOISE_PHASES
    re = sc * np.cos(th).astype(np.float32)
    im = sc * np.sin(th).astype(np.float32)
    return re.astype(np.float64) + 1j * im.astype(np.float64)


def noise_from_words(w: np.ndarray, ph: np.ndarray, sigma: float, with_bound: bool = False, radius_fn=None,
                     product_rel: float = 2.0 ** -24):
    """Complex normal of each noise sample: radius from its 32-bit radius word w (u = (w | 1) 2^-32),
    phase = table entry ph (0..63, from the lane's phase word).

    radius_fn: None -> the radius sqrt(32 - log2(f)) in float64 from the word's float32 value f;
    otherwise a function mapping the words to the float32 radii the GPU's hardware log2 / sqrt
    give (libofdm_hip's ofdm_noise_radius: the receivers' own noise_radius on these words).

    with_bound: also return a bound on |GPU noise - this value| per word.
    * float64 radius: the GPU evaluates log2 and sqrt with the float32 hardware instructions: log2
      within 2 ulp of its float32 result (<= 2^-18 absolute for arguments < 2^32), the subtraction
      from 32 and the square root within 1 ulp, the product with the table entry within 1/2 ulp per
      component.  With A = 32 - log2(f) and dA = 2^-18 + 2^-23 A, the radius error is at most
      dA / (sqrt(A) + sqrt(max(A - dA, 0))) (<= sqrt(dA)) + 2^-23 r.
    * the GPU's radii: the float32 radius times the float32 table entry is exact in float64, as it
      is in the complex128 receivers' fused multiply-add (product_rel 2^-53); the complex64
      receivers round it once (product_rel 2^-24).  The table is the GPU's bit for bit when sigma is (float32 entries
      of the same double sigma, tests/test_oracle_philox.py::test_noise_table_entries_are_robust)."""
    w = np.asarray(w, np.uint32)
    e = noise_table(sigma)[np.asarray(ph, np.int64)]
    if radius_fn is not None:
        r = np.asarray(radius_fn(w), np.float32).astype(np.float64)
        n = r * e
        return (n, product_rel * np.abs(n)) if with_bound else n
    f = (w | RADIUS_OR).astype(np.float32)  # round to nearest even, as v_cvt_f32_u32
    A = 32.0 - np.log2(f.astype(np.float64))
    r = np.sqrt(A)
    n = r * e
    if not with_bound:
        return n
    dA = 2.0 ** -18 + 2.0 ** -23 * A
    dr = dA / np.maximum(np.sqrt(A) + np.sqrt(np.maximum(A - dA, 0.0)), np.sqrt(dA)) + 2.0 ** -23 * r
    return n, dr * np.abs(e) + 2.0 ** -23 * np.abs(n)


def _lane_to_row(v: np.ndarray, S: int, N: int) -> np.ndarray:
    """(S*TPS, E) lane-major values -> (S, N) in subcarrier / time-sample order."""
    E, tps = geometry(N)
    return v.reshape(S, tps, E).transpose(0, 2, 1).reshape(S, N)


def tx_indices(gen: LaneStream, S: int, N: int, b) -> np.ndarray:
    """Constellation indices (S, N) from the payload words of every lane; b is the bits per
    subcarrier, one value or one per subcarrier (adaptive loading)."""
    E, _ = geometry(N)
    words = gen.payload  # (lanes, 4)
    i = np.arange(E)
    byte = (words[:, i >> 2] >> (8 * (i & 3)).astype(np.uint32)) & np.uint32(0xFF)
    mask = (np.int64(1) << np.broadcast_to(np.asarray(b, np.int64), (N,))) - 1
    return _lane_to_row(byte.astype(np.int64), S, N) & mask[None, :]


def lane_noise(gen: LaneStream, S: int, N: int, sigma: float, with_bound: bool = False, radius_fn=None,
               product_rel: float = 2.0 ** -24):
    """Complex noise (S, N) at the kept time samples, noise samples 0 .. E-1 of every lane
    (with_bound: and the (S, N) bound of noise_from_words)."""
    E, _ = geometry(N)
    parts = [noise_from_words(*gen.noise_draw(), sigma, with_bound, radius_fn, product_rel) for _ in range(E)]
    if not with_bound:
        return _lane_to_row(np.stack(parts, axis=1), S, N)
    return (_lane_to_row(np.stack([p[0] for p in parts], axis=1), S, N),
            _lane_to_row(np.stack([p[1] for p in parts], axis=1), S, N))


@dataclass
class PhiloxLink:
    bit_errors: int
    symbol_errors: int
    power_sum: float
    x_power_sum: float
    x_peak: float
    idx: np.ndarray        # (S, N) tx constellation indices
    y: np.ndarray          # stored channel samples before noise: (S, N) kept, or (S, N+cp) with ZP
    # (bit_lo, bit_hi, sym_lo, sym_hi): the error counts of every decision consistent with the
    # GPU's deviation from this restatement (decision_bracket), when run_philox(precision=...)
    bracket: Optional[tuple] = None
    # the same for the per-point statistical deviation scale (run_philox(stat_sigma=...))
    stat_bracket: Optional[tuple] = None


def run_philox(seed: int, S: int, N: int, M: int, h_raw: np.ndarray, cp: int, eq: str, snr_db: float,
               noise_on: bool = True, modulator: str = "OFDM", prefix: str = "CP",
               scheme: str = "QAM", orders=None, precision: Optional[str] = None, radius_fn=None,
               power_sum: Optional[float] = None, stat_sigma: Optional[float] = None,
               stat_k: float = STAT_K) -> PhiloxLink:
    """Global OFDM symbols [0, S) of a throughput-mode run, through the oracle arithmetic.

    modulator "OFDM" | "SC" (modulation/models.py:58-91), prefix "CP" | "ZP"
    (prefix/models.py:29-101), scheme "QAM" | "PSK".  With zero padding every lane's noise
    samples continue, after its elements', with the received tail samples N + k it owns
    (k = t + i*TPS < cp, in order of i).

    orders: per-subcarrier QAM orders (CAPACITY_BASED bit loading, 0 = unused; M is then
    ignored).  As in the reference's decode (constellation/adaptive.py:259-263) a trailing
    partial byte of the whole run's bit stream is not compared; symbol errors count every
    used subcarrier.

    precision "f32" | "f64": also return the decision bracket of a GPU run in that arithmetic
    (PhiloxLink.bracket, see decision_bracket).

    radius_fn: the GPU's noise radii of a word array (noise_from_words); power_sum: the GPU run's
    whole-stream sum |y|^2 (its exact fixed-point value), from which sigma is computed as the
    receivers compute it -- together they make the receivers' noise the restatement's bit for bit
    in complex128 (the decision bracket then only covers FFT / FIR / equaliser rounding).

    stat_sigma: the measured per-sample standard deviation of the GPU's transmitted samples from
    this restatement's (same seed, its transmitter alone; a float, or a function of this
    restatement's stored samples returning it): also return PhiloxLink.stat_bracket,
    the decision bracket for a per-point deviation of stat_k standard deviations of the model in
    z_stat_bound (complex64: the rigorous 2-norm bound of z_error_bound assigns every subcarrier
    the worst case of the whole transform, c log2(N) u sqrt(N) rms).
    """
    E, tps = geometry(N)
    gen = lane_generators(seed, np.arange(S), N)
    want_bound = precision is not None and noise_on
    prel = 2.0 ** -53 if precision == "f64" else 2.0 ** -24
    if orders is not None:
        orders = np.asarray(orders, np.int64)
        bk = np.array([int(np.log2(o)) if o > 0 else 0 for o in orders], np.int64)
        idx = tx_indices(gen, S, N, bk)
        make = O.psk_lut if scheme == "PSK" else O.qam_lut
        luts = {int(o): make(int(o)) for o in np.unique(orders) if o > 0}
        X = np.zeros((S, N), np.complex128)
        for o, lt in luts.items():
            cols = orders == o
            X[:, cols] = lt[idx[:, cols]]
    else:
        b = int(np.log2(M))
        lut = O.qam_lut(M) if scheme == "QAM" else O.psk_lut(M)
        idx = tx_indices(gen, S, N, b)
        X = lut[idx]
    s_t = np.fft.ifft(X, axis=1, norm="ortho") if modulator == "OFDM" else X
    if prefix == "ZP":
        x = np.concatenate([s_t, np.zeros((S, cp), np.complex128)], axis=1)
    else:
        x = O.add_cp(s_t, cp)                          # (S, N+cp) incl. prefix
    px = float(np.sum(np.abs(x) ** 2))
    mx = float(np.max(np.abs(x) ** 2))
    y = O.channel_conv(x.ravel(), np.asarray(h_raw, np.complex128)).reshape(S, N + cp)
    py = float(np.sum(np.abs(y) ** 2))
    if prefix == "ZP":
        yk, tail = y[:, :N].copy(), y[:, N:].copy()
    else:
        yk, tail = y[:, cp:].copy(), None
    rxs = yk.copy()
    # per received sample: the bound on the GPU's noise deviation (zero padding: a guard-tail sample's
    # own bound adds onto the bound of the sample it is overlap-added to, before the per-symbol sums)
    nbs = np.zeros((S, N))
    if noise_on:
        # sigma^2 = mean |y|^2 / snr (noise/models.py:13-18), as k_rx evaluates it in double
        p = (py if power_sum is None else float(power_sum)) / (S * (N + cp))
        sigma = float(np.sqrt((p / 10 ** (snr_db / 10)) / 2.0))
        if want_bound:
            nz, nb = lane_noise(gen, S, N, sigma, with_bound=True, radius_fn=radius_fn, product_rel=prel)
            nbs += nb
        else:
            nz = lane_noise(gen, S, N, sigma, radius_fn=radius_fn)
        rxs = rxs + nz
    if prefix == "ZP" and cp > 0:
        if noise_on:
            t = np.tile(np.arange(tps), S)
            for i in range(E):
                k = t + i * tps
                w, ph = gen.noise_draw()  # noise sample E + i
                n, nb = noise_from_words(w, ph, sigma, with_bound=True, radius_fn=radius_fn, product_rel=prel)
                use = k < cp
                srow = np.repeat(np.arange(S), tps)[use]
                tail[srow, k[use]] += n[use]
                np.add.at(nbs, (srow, k[use]), nb[use])
        rxs[:, :cp] += tail
    nerr = nbs.sum(axis=1)  # per symbol: sum over its received samples of the deviation bound
    nerr2 = (nbs ** 2).sum(axis=1)  # ... and the sum of its squares (the 2-norm of the deviations)
    H = np.fft.fft(np.asarray(h_raw, np.complex128), N)
    Y = np.fft.fft(rxs, axis=1, norm="ortho")
    Z = O.equalize(Y, H, eq, snr_db)
    if modulator == "SC":
        Z = np.fft.ifft(Z, axis=1, norm="ortho")
    bracket = stat_bracket = None
    if precision is not None:
        delta = z_error_bound(precision, Y, H, eq, snr_db, nerr, modulator, N, np.sqrt(nerr2))
        dstat = None
        if stat_sigma is not None:
            # (a callable gets the stored samples -- (S, N + cp) with zero padding, else (S, N) -- and
            # returns the measured deviation of the GPU's from them)
            sig = stat_sigma(y if prefix == "ZP" else yk) if callable(stat_sigma) else float(stat_sigma)
            dstat = z_stat_bound(precision, Y, H, eq, snr_db, sig, np.sqrt(np.mean(np.abs(yk) ** 2)),
                                 modulator, N, stat_k)
        if orders is not None:
            bracket = adaptive_bracket(Z, idx, orders, bk, delta, scheme)
            if dstat is not None:
                stat_bracket = adaptive_bracket(Z, idx, orders, bk, dstat, scheme)
        else:
            bracket = decision_bracket(Z, idx, lut, b, delta, scheme)
            if dstat is not None:
                stat_bracket = decision_bracket(Z, idx, lut, b, dstat, scheme)
    if orders is not None:
        ridx = np.zeros((S, N), np.int64)
        for o, lt in luts.items():
            cols = np.flatnonzero(orders == o)
            ridx[:, cols] = O.nn_demap(Z[:, cols].ravel(), lt).reshape(S, len(cols))
        diff = (ridx ^ idx).astype(np.int64)
        be, se = adaptive_counts(diff, bk, S)
        return PhiloxLink(be, se, py, px, mx, idx, y if prefix == "ZP" else yk, bracket, stat_bracket)
    ridx = O.nn_demap(Z.ravel(), lut).reshape(S, N)
    diff = (ridx ^ idx).astype(np.uint64)
    be = int(sum(int(np.count_nonzero((diff >> np.uint64(j)) & np.uint64(1))) for j in range(b)))
    se = int(np.count_nonzero(ridx != idx))
    return PhiloxLink(be, se, py, px, mx, idx, y if prefix == "ZP" else yk, bracket, stat_bracket)


def adaptive_counts(diff: np.ndarray, bk: np.ndarray, S: int):
    """Bit / symbol errors of CAPACITY_BASED decisions (diff = rx ^ tx index per (s, k)): the
    stream position of bit j (MSB first) of subcarrier k in symbol s is s*tot + off_k + j, and a
    trailing partial byte of the run is not compared (constellation/adaptive.py:259-263)."""
    tot = int(bk.sum())
    valid = (S * tot // 8) * 8
    off = np.concatenate([[0], np.cumsum(bk)[:-1]])
    be = 0
    for j in range(int(bk.max(initial=0))):
        has = bk > j
        bit = (diff >> np.maximum(bk - 1 - j, 0)[None, :]) & 1
        pos = np.arange(S)[:, None] * tot + (off + j)[None, :]
        be += int(np.count_nonzero(bit.astype(bool) & has[None, :] & (pos < valid)))
    se = int(np.count_nonzero(diff[:, bk > 0]))
    return be, se


# --------------------------------------------------------------------------- decision brackets
# A GPU run and this restatement see the same bits and the same noise words, but not bit-identical
# received points: the GPU evaluates the noise radius with float32 hardware log2 / sqrt (bounded per
# word by noise_from_words) and runs its FFTs in its own arithmetic.  z_error_bound turns these into
# a bound on |Z_gpu - Z| per element; decision_bracket then counts the errors of every decision
# consistent with that bound.  A correct kernel's integer counts lie inside [lo, hi]; the bracket
# is empty of slack (lo = hi) unless a received point lies within the bound of a decision boundary.

def z_error_bound(precision: str, Y: np.ndarray, H: np.ndarray, eq: str, snr_db: float,
                  noise_err: np.ndarray, modulator: str, N: int, noise_err2=None) -> np.ndarray:
    """(S, N) bound on the deviation of the GPU's equalised points from this restatement's.

    * noise: each received sample deviates by at most its noise_from_words bound; through the
      ortho FFT a subcarrier deviates by at most the sum over the symbol's samples / sqrt(N);
    * arithmetic: the FFT / FIR rounding of the kernel, bounded through the 2-norm, c log2(N) u
      sqrt(N) rms(Y) per symbol (u = 2^-24 complex64 with c = 6 for the TX and RX transforms and
      the FIR, u = 2^-53 complex128);
    * equaliser: the deviation times the subcarrier's gain |dZ/dY| (ZF 1/|H|, MMSE
      |H| / (|H|^2 + nv)), plus a relative term for the MMSE noise variance computed from the
      GPU's own received power;
    * single carrier: the IFFT after the equaliser preserves the 2-norm, so a sample deviates by at
      most the 2-norm of the equalised deviation: max gain x (2-norm of the noise deviations,
      noise_err2, + the arithmetic term) + the relative terms x ||Z||, plus the IFFT's own rounding
      (c log2(N) u ||Z||)."""
    S = Y.shape[0]
    logn = max(1.0, np.log2(N))
    u = 2.0 ** -24 if precision == "f32" else 2.0 ** -53
    rms = np.sqrt(np.mean(np.abs(Y) ** 2, axis=1))
    dy = noise_err / np.sqrt(N) + 6.0 * logn * u * np.sqrt(N) * rms  # (S,)
    if eq == "NONE":
        g = np.ones((S, N))
        rel = 0.0
    elif eq == "ZF":
        h = np.where(H == 0, 1e-10, H)
        g = np.broadcast_to(1.0 / np.abs(h), (S, N))
        rel = 4 * u
    else:
        gm = np.mean(np.abs(H) ** 2)
        nv = (np.mean(np.abs(Y) ** 2, axis=1) / 10 ** (snr_db / 10)) / gm
        g = np.abs(H)[None, :] / (np.abs(H)[None, :] ** 2 + nv[:, None])
        # nv from the GPU's received power: relative deviation <= 2 dy / rms + rounding
        rel = 8 * u + 2 * np.max(dy / np.maximum(rms, 1e-300))
    Zabs = np.abs(Y) * g
    d = g * dy[:, None] + rel * Zabs + 1e-300
    if modulator == "SC":
        n2 = noise_err if noise_err2 is None else noise_err2
        e2 = n2 + 6.0 * logn * u * np.sqrt(N) * rms  # 2-norm of the symbol's deviation (FFT: ortho)
        z2 = np.sqrt(np.sum(Zabs ** 2, axis=1))
        d = g.max(axis=1) * e2 + (rel + 6.0 * logn * u) * z2 + 1e-300
        d = np.broadcast_to(d[:, None], (S, N))
    return np.asarray(d)


def z_stat_bound(precision: str, Y: np.ndarray, H: np.ndarray, eq: str, snr_db: float, sigma_tx: float,
                 rms_y: float, modulator: str, N: int, k: float = STAT_K) -> np.ndarray:
    """(S, N) per-point deviation scale of the GPU's equalised points from this restatement's: k
    times the standard deviation of a model calibrated by the GPU's own transmitter.

    sigma_tx is the measured per-sample standard deviation of the GPU's channel samples from the
    restatement's (its IFFT, FIR and stores).  The receiver adds the noise product's rounding (u
    rms(y)) and its FFT, taken to deviate no more than the transmitter (which carries an IFFT and
    the FIR), so a received sample deviates by sd_t = sqrt(2 sigma_tx^2 + (u rms_y)^2) per sample;
    the ortho FFT preserves it per subcarrier.  The equaliser multiplies it by the subcarrier's gain
    g (ZF 1/|H|, MMSE |H| / (|H|^2 + nv)) and adds a few roundings of |Z| (8 u; MMSE: its noise
    variance from the GPU's own received power, relative 2 sd_t / rms).  Single carrier: the IFFT
    after the equaliser spreads the subcarriers' deviations over every sample, sqrt(mean g^2) sd_t,
    plus its own rounding (sd_t relative to the equalised signal)."""
    S = Y.shape[0]
    u = 2.0 ** -24 if precision == "f32" else 2.0 ** -53
    sd_t = np.sqrt(2.0 * sigma_tx ** 2 + (u * rms_y) ** 2)
    rms = np.sqrt(np.mean(np.abs(Y) ** 2, axis=1))
    if eq == "NONE":
        g = np.ones((S, N))
        rel = 0.0
    elif eq == "ZF":
        h = np.where(H == 0, 1e-10, H)
        g = np.broadcast_to(1.0 / np.abs(h), (S, N))
        rel = 8 * u
    else:
        gm = np.mean(np.abs(H) ** 2)
        nv = (np.mean(np.abs(Y) ** 2, axis=1) / 10 ** (snr_db / 10)) / gm
        g = np.abs(H)[None, :] / (np.abs(H)[None, :] ** 2 + nv[:, None])
        rel = 8 * u + 2 * sd_t / np.maximum(np.max(rms), 1e-300)
    Zabs = np.abs(Y) * g
    d = g * sd_t + rel * Zabs
    if modulator == "SC":
        zr = np.sqrt(np.mean(Zabs ** 2, axis=1))
        d = np.sqrt(np.mean(g ** 2, axis=1)) * sd_t + (rel + sd_t / np.maximum(np.max(rms), 1e-300)) * zr
        d = np.broadcast_to(d[:, None], (S, N))
    return k * np.asarray(d) + 1e-300


def _qam_levels(lut: np.ndarray):
    """Sorted axis levels, their step and the (kq, ki) -> index table of a square-QAM LUT."""
    lev = np.unique(np.round(lut.real, 12))
    side = len(lev)
    table = np.zeros((side, side), np.int64)
    ki = np.searchsorted(lev, np.round(lut.real, 12))
    kq = np.searchsorted(lev, np.round(lut.imag, 12))
    table[kq, ki] = np.arange(len(lut))
    return lev, lev[1] - lev[0], table


def _axis_candidates(u: np.ndarray, lev0: float, step: float, side: int, d: np.ndarray):
    """Decided level of each coordinate and the alternative level across the nearest interior
    threshold when the coordinate lies within d of it (else the decided level again)."""
    y = (u - lev0) / step
    k = np.clip(np.rint(y), 0, side - 1).astype(np.int64)
    if side < 2:
        return k, k
    th = np.clip(np.floor(y), 0, side - 2) + 0.5
    near = np.abs(y - th) * step <= d
    alt = np.where(k <= th, th + 0.5, th - 0.5).astype(np.int64)
    return k, np.where(near, alt, k)


def _popcount(v: np.ndarray) -> np.ndarray:
    return np.bitwise_count(np.asarray(v, np.uint64)).astype(np.int64)


def decision_candidates(Z: np.ndarray, lut: np.ndarray, delta: np.ndarray, scheme: str = "QAM") -> list:
    """Four candidate LUT indices per point (flattened): every decision of a point within delta
    of Z.  QAM (the reference's square LUTs are separable): per axis the decided
    level and, near an interior threshold, the level across it.  PSK (LUT[gray(i)] =
    exp(2 pi j i / M), constellation/models.py:356-380): the decided sector and, when the point
    lies within delta of a sector boundary ray, the sector across it (listed twice)."""
    Z = np.asarray(Z).ravel()
    d = np.broadcast_to(delta, np.asarray(delta).shape).ravel()
    if scheme == "PSK":
        M = len(lut)
        w = 2 * np.pi / M
        th = np.mod(np.angle(Z), 2 * np.pi)
        k = np.mod(np.rint(th / w), M).astype(np.int64)
        off = th - np.rint(th / w) * w                 # angle from the decided point, |off| <= w/2
        dist = np.abs(Z) * np.sin(np.abs(np.abs(off) - w / 2))  # distance to the nearer boundary ray
        near = (dist <= d) & (M > 1)
        alt = np.mod(k + np.where(off >= 0, 1, -1), M)
        g0, g1 = k ^ (k >> 1), np.where(near, alt ^ (alt >> 1), k ^ (k >> 1))
        return [g0, g1, g0, g1]
    lev, step, table = _qam_levels(lut)
    side = len(lev)
    ki, ki2 = _axis_candidates(Z.real, lev[0], step, side, d)
    kq, kq2 = _axis_candidates(Z.imag, lev[0], step, side, d)
    return [table[kq, ki], table[kq, ki2], table[kq2, ki], table[kq2, ki2]]


def decision_bracket(Z: np.ndarray, idx: np.ndarray, lut: np.ndarray, b: int, delta: np.ndarray,
                     scheme: str = "QAM") -> tuple:
    """(bit_lo, bit_hi, sym_lo, sym_hi) over every decision of points within delta of Z
    (decision_candidates)."""
    idx = np.asarray(idx).ravel().astype(np.int64)
    cands = decision_candidates(Z, lut, delta, scheme)
    be = np.stack([_popcount(c ^ idx) for c in cands])
    ne = np.stack([c != idx for c in cands])
    return (int(be.min(0).sum()), int(be.max(0).sum()), int(ne.all(0).sum()), int(ne.any(0).sum()))


def adaptive_bracket(Z: np.ndarray, idx: np.ndarray, orders: np.ndarray, bk: np.ndarray,
                     delta: np.ndarray, scheme: str = "QAM") -> tuple:
    """decision_bracket for CAPACITY_BASED loading: per order, the candidates of its subcarriers
    over that order's LUT (QAM or PSK); bit errors counted as adaptive_counts does (trailing
    partial byte excluded)."""
    S, N = Z.shape
    d = np.broadcast_to(delta, (S, N))
    cand = [np.array(idx, np.int64) for _ in range(4)]
    make = O.psk_lut if scheme == "PSK" else O.qam_lut
    for o in np.unique(orders):
        if o <= 0:
            continue
        cols = np.flatnonzero(orders == o)
        cs = decision_candidates(Z[:, cols], make(int(o)), d[:, cols], scheme)
        for c, v in zip(cand, cs):
            c[:, cols] = v.reshape(S, len(cols))
    be0, _ = adaptive_counts((cand[0] ^ idx).astype(np.int64), bk, S)
    # the other candidates change an element's bit count by at most the spread of its popcounts
    diffs = np.stack([_popcount(c ^ idx) for c in cand])
    used = (bk > 0)[None, :]
    slack = int(np.where(used, diffs.max(0) - diffs.min(0), 0).sum())
    ne = np.stack([(c != idx) & used for c in cand])
    return (be0 - slack, be0 + slack, int(ne.all(0).sum()), int(ne.any(0).sum()))
