"""CPU oracle for the OFDM modem hot path -- TEST INFRASTRUCTURE ONLY.

This module is a vectorised NumPy restatement of the reference's per-symbol
modem path (JomarJunior/ofdm-based-systems, ``src/ofdm_based_systems``).  It is
the CHECKER: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product (``ofdm_based_systems`` in
``ofdm-based-systems_amd/``) never imports it and has no CPU fallback.

Parity pinning: every function below is checked against golden vectors that
were produced by running the reference itself in the build container
(``tests/golden/make_golden.py``; fixtures ``tests/golden/*.npz|json``), see
``tests/test_oracle_golden.py``.  References are ``file:line`` under
``/root/reference/src/ofdm_based_systems``.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import numpy as np

# --------------------------------------------------------------------------- constellations


def gray(i: int) -> int:
    """constellation/models.py:75-77 -- ``i ^ (i >> 1)``."""
    return i ^ (i >> 1)


def qam_lut(order: int) -> np.ndarray:
    """Square-QAM LUT, constellation/models.py:180-218 with GrayWordCoder :70-109.

    ``constellation[i] = grid[gray(i)]`` over the row-major grid (top row = most
    positive Q, left to right = increasing I), then odd rows of the *index*
    space reversed (zig-zag, :94-109), then scaled to unit mean power (:211-213).
    """
    side = int(np.sqrt(order))
    if side * side != order:
        raise ValueError("Order must be a perfect square (e.g., 4, 16, 64).")
    lv = np.arange(-side + 1, side, 2)
    grid = [complex(i, q) for q in lv[::-1] for i in lv]
    c = np.zeros(order, dtype=np.complex128)
    for i in range(order):
        c[i] = grid[gray(i)]
    out = np.zeros_like(c)
    for r in range(side):
        row = c[r * side:(r + 1) * side]
        out[r * side:(r + 1) * side] = row[::-1] if r % 2 == 1 else row
    out /= np.sqrt(np.mean(np.abs(out) ** 2))
    return out


def psk_lut(order: int) -> np.ndarray:
    """M-PSK LUT, constellation/models.py:356-380: ``constellation[gray(i)] = exp(2*pi*j*i/M)``."""
    pts = np.exp(1j * 2 * np.pi * np.arange(order) / order)
    c = np.zeros(order, dtype=np.complex128)
    for i in range(order):
        c[gray(i)] = pts[i]
    return c


# --------------------------------------------------------------------------- bits


def bytes_to_bits(data: bytes | np.ndarray) -> np.ndarray:
    """MSB-first unpacking, simulation/models.py:59-69 and constellation/models.py:227-233."""
    return np.unpackbits(np.frombuffer(bytes(data), dtype=np.uint8))


def bits_to_indices(bits: np.ndarray, b: int) -> np.ndarray:
    """Zero-pad to a multiple of b (constellation/models.py:235-237), MSB-first index (:240-243)."""
    bits = np.asarray(bits, dtype=np.int64)
    if len(bits) % b:
        bits = np.concatenate([bits, np.zeros(b - len(bits) % b, dtype=np.int64)])
    return bits.reshape(-1, b) @ (1 << np.arange(b - 1, -1, -1))


def indices_to_bytes(idx: np.ndarray, b: int) -> bytes:
    """decode's packing, constellation/models.py:269-295 (tail byte zero-padded)."""
    bits = ((np.asarray(idx)[:, None] >> np.arange(b - 1, -1, -1)) & 1).astype(np.uint8).ravel()
    return np.packbits(bits).tobytes()


def generate_bits(num_bits: int, rng: np.random.Generator) -> bytes:
    """RandomBitsGenerator.generate_bits, bits_generation/models.py:27-55 (tail byte masked)."""
    nbytes = math.ceil(num_bits / 8)
    raw = bytearray(rng.bytes(nbytes))
    keep = num_bits % 8
    if keep:
        raw[-1] &= (0xFF << (8 - keep)) & 0xFF
    return bytes(raw)


# --------------------------------------------------------------------------- demap


def nn_demap(z: np.ndarray, lut: np.ndarray, chunk: int = 1 << 16) -> np.ndarray:
    """NNClassifier.classify + constellation_map lookup, constellation/models.py:19-27, :259-267.

    argmin over |z - C_m| (first index on ties); the LUT points are distinct so
    the tuple-key dict maps the classified point back to its own index.
    """
    z = np.asarray(z, dtype=np.complex128).ravel()
    out = np.empty(len(z), dtype=np.int64)
    for s in range(0, len(z), chunk):
        zz = z[s:s + chunk]
        out[s:s + chunk] = np.argmin(np.abs(zz[:, None] - lut[None, :]), axis=1)
    return out


# --------------------------------------------------------------------------- modem


def add_cp(x: np.ndarray, cp: int) -> np.ndarray:
    """CyclicPrefixScheme.add_prefix per row, prefix/models.py:34-44 (cp=0 -> unchanged)."""
    if cp == 0:
        return x
    return np.concatenate([x[:, -cp:], x], axis=1)


def modulate(X: np.ndarray, cp: int) -> np.ndarray:
    """OFDMModulator.modulate, modulation/models.py:27-39: ifft(axis=1, ortho) + prefix."""
    return add_cp(np.fft.ifft(X, axis=1, norm="ortho"), cp)


def normalize_h(h: np.ndarray) -> np.ndarray:
    """ChannelModel.normalize_impulse_response, channel/models.py:37-44."""
    p = np.sum(np.abs(h) ** 2)
    if p == 0:
        raise ValueError("Impulse response cannot be all zeros.")
    return h / np.sqrt(p)


def channel_conv(s: np.ndarray, h_raw: np.ndarray) -> np.ndarray:
    """ChannelModel.transmit convolution part, channel/models.py:52-55 (full, truncated)."""
    return np.convolve(s, normalize_h(h_raw), mode="full")[: s.shape[0]].astype(np.complex128)


def awgn(y: np.ndarray, snr_db: float, nr: np.ndarray, ni: np.ndarray) -> np.ndarray:
    """AWGNoiseModel.add_noise, noise/models.py:13-22 with the normals supplied."""
    p = np.mean(np.abs(y) ** 2)
    npow = p / 10 ** (snr_db / 10)
    return y + np.sqrt(npow / 2) * (nr + 1j * ni)


def equalize(Y: np.ndarray, H: np.ndarray, eq: str, snr_db: float) -> np.ndarray:
    """Per-row equalisers, equalization/models.py:22-68 (MMSE nv per OFDM symbol, :39-49)."""
    if eq == "NONE":
        return Y
    if eq == "ZF":
        h = np.where(H == 0, 1e-10, H)
        return Y / h[None, :]
    if eq == "MMSE":
        g = np.mean(np.abs(H) ** 2)
        sp = np.mean(np.abs(Y) ** 2, axis=1, keepdims=True)
        nv = (sp / 10 ** (snr_db / 10)) / g if g != 0 else np.full_like(sp, np.inf)
        return Y * (np.conj(H)[None, :] / (np.abs(H)[None, :] ** 2 + nv))
    raise ValueError(eq)


def demodulate(Yt: np.ndarray, cp: int, H: np.ndarray, eq: str, snr_db: float) -> np.ndarray:
    """OFDMModulator.demodulate, modulation/models.py:41-55: strip prefix, fft(ortho), equalise."""
    Y = np.fft.fft(Yt[:, cp:], axis=1, norm="ortho")
    return equalize(Y, H, eq, snr_db)


def papr_db(x: np.ndarray) -> float:
    """simulation/models.py:519-522 over the modulated array incl. the CP."""
    p = np.abs(x) ** 2
    avg = np.mean(p)
    return float(10 * np.log10(np.max(p) / avg)) if avg > 0 else float("inf")


# --------------------------------------------------------------------------- full path


@dataclass
class LinkResult:
    bit_errors: int
    symbol_errors: int
    total_bits: int
    papr_db: float
    num_symbols: int
    rx_bytes: bytes
    Z: Optional[np.ndarray] = None


def run_fixed(
    tx_bytes: bytes,
    total_bits: int,
    N: int,
    M: int,
    h_raw: np.ndarray,
    cp: int,
    eq: str,
    snr_db: float,
    noise: Optional[tuple] = None,
    keep_Z: bool = False,
) -> LinkResult:
    """Simulation.run FIXED/QAM/OFDM data path, simulation/models.py:454-609.

    ``noise`` = (normal_re, normal_im) of length S*(N+cp) or None for NoNoiseModel.
    """
    b = int(np.log2(M))
    lut = qam_lut(M)
    tx_bits = bytes_to_bits(tx_bytes)
    idx = bits_to_indices(tx_bits, b)
    if len(idx) % N:
        raise ValueError("Length of data must be divisible by number of streams.")
    X = lut[idx].reshape(-1, N)
    x = modulate(X, cp)
    pp = papr_db(x)
    s = x.ravel()
    y = channel_conv(s, h_raw)
    if noise is not None:
        y = awgn(y, snr_db, noise[0], noise[1])
    H = np.fft.fft(h_raw, N)
    Z = demodulate(y.reshape(-1, N + cp), cp, H, eq, snr_db)
    ridx = nn_demap(Z.ravel(), lut)
    rx = indices_to_bytes(ridx, b)
    rx_bits = bytes_to_bits(rx)
    n = min(len(tx_bits), len(rx_bits))
    be = int(np.count_nonzero(tx_bits[:n] != rx_bits[:n]))
    ridx2 = bits_to_indices(rx_bits, b)
    se = int(np.count_nonzero(lut[idx] != lut[ridx2[: len(idx)]])) if len(ridx2) >= len(idx) else -1
    return LinkResult(be, se, total_bits, pp, len(idx), rx, Z if keep_Z else None)


def reference_streams(seed: int, total_bits: int, n_samples: int, noise: bool = True):
    """The reference's seeded random streams.

    Bits: ``Generator(PCG64(seed)).bytes`` (bits_generation/models.py:24, :37).
    Noise: legacy global ``np.random.seed(seed)`` then ``normal(size)`` twice,
    real array first (noise/models.py:19-21).
    """
    tx = generate_bits(total_bits, np.random.Generator(np.random.PCG64(seed)))
    if not noise:
        return tx, None
    rs = np.random.RandomState(seed)
    nr = rs.normal(size=n_samples)
    ni = rs.normal(size=n_samples)
    return tx, (nr, ni)


def prefix_length(h_raw: np.ndarray, ratio: float, prefix: str) -> int:
    """simulation/models.py:251-253."""
    if prefix == "NONE":
        return 0
    return int(ratio * (len(h_raw) - 1))


def run_reference_fixed(seed: int, num_symbols: Optional[int], num_bits: Optional[int], N: int,
                        M: int, h_raw: np.ndarray, ratio: float, prefix: str, eq: str,
                        snr_db: float, noise: bool = True) -> LinkResult:
    """Seeded FIXED-mode run with the reference's streams (simulation/models.py:405-410, :454)."""
    b = int(np.log2(M))
    total_bits = num_bits if num_symbols is None else num_symbols * b
    cp = prefix_length(h_raw, ratio, prefix)
    nbytes = math.ceil(total_bits / 8)
    nsym = math.ceil(nbytes * 8 / b)
    S = nsym // N
    tx, nz = reference_streams(seed, total_bits, S * (N + cp), noise)
    return run_fixed(tx, total_bits, N, M, h_raw, cp, eq, snr_db, nz)


# --------------------------------------------------------------------------- power allocation / bit loading


def uniform_allocation(total_power: float, n: int) -> np.ndarray:
    """UniformPowerAllocation.allocate, power_allocation/models.py:61-69."""
    return np.full(n, total_power / n, dtype=np.float64)


def waterfilling_allocation(total_power: float, gains: np.ndarray, noise_power: float,
                            tol: float = 1e-8) -> np.ndarray:
    """WaterfillingPowerAllocation.allocate, power_allocation/models.py:140-225 (floor /K at :161)."""
    g = np.asarray(gains, dtype=np.float64)
    floor = noise_power / (g * len(g))
    lo, hi = 0.0, total_power + np.max(floor)
    mu = (lo + hi) / 2
    for _ in range(100):
        mu = (lo + hi) / 2
        ps = np.sum(np.maximum(0, mu - floor))
        if np.abs(ps - total_power) < tol:
            break
        if ps < total_power:
            lo = mu
        else:
            hi = mu
    p = np.maximum(0, mu - floor)
    s = np.sum(p)
    if s > 0:
        p = p * (total_power / s)
    return p


def qam_bit_loading_order(ser: float, snr: float) -> int:
    """QAMConstellationMapper.calculate_bit_loading_order, constellation/models.py:297-321."""
    from scipy.stats import norm

    q = norm.isf(ser / 4)
    gamma = (1 / 3) * q ** 2
    b = int(np.round(np.log2(1 + snr / gamma)))
    if b % 2:
        b -= 1
    return 0 if b <= 0 else 2 ** b


def psk_bit_loading_order(ser: float, snr: float) -> int:
    """PSKConstellationMapper.calculate_bit_loading_order, constellation/models.py:460-474:
    gamma* = Q^-1(SER/2)^2 / (2 pi^2), gamma = sqrt(snr gamma*) / (1 - sqrt(gamma* / (snr + 1e-10))),
    b = floor(log2(1 + snr / (gamma + 1e-10)) + 1e-10), 0 if b <= 0."""
    from scipy.stats import norm

    q = norm.isf(ser / 2)
    g_star = (q ** 2) / (2 * (np.pi ** 2))
    gamma = (np.sqrt(snr * g_star)) / (1 - np.sqrt(g_star / (snr + 1e-10)))
    b = int(np.floor(np.log2(1 + snr / (gamma + 1e-10)) + 1e-10))
    return 0 if b <= 0 else 2 ** b


# --------------------------------------------------------------------------- adaptive (CAPACITY_BASED)


def adaptive_orders(N: int, h_raw: np.ndarray, snr_db: float, ser: float, waterfilling: bool,
                    scheme: str = "QAM"):
    """simulation/models.py:278-352: orders from the base mapper's gap formula after power
    allocation (P_tot = N); scheme "QAM" | "PSK" selects the base mapper class (:330-332)."""
    H = np.fft.fft(h_raw, N)
    g = np.abs(H) ** 2
    n0 = 10 ** (-snr_db / 10)
    p = waterfilling_allocation(N, g, n0) if waterfilling else uniform_allocation(N, N)
    rule = psk_bit_loading_order if scheme == "PSK" else qam_bit_loading_order
    orders = np.array([rule(ser, pa * hg / n0) for pa, hg in zip(p, g)], dtype=np.int64)
    wl = None
    if waterfilling:
        wl = float(np.mean((p + n0 / g)[p > 1e-10]))
    return orders, p, wl


def run_adaptive(tx_bytes: bytes, orders: np.ndarray, N: int, h_raw: np.ndarray, cp: int, eq: str,
                 snr_db: float, noise=None, scheme: str = "QAM") -> LinkResult:
    """CAPACITY_BASED data path: AdaptiveConstellationMapper.encode/decode (constellation/adaptive.py:130-265)
    over the base mapper's LUT per order (QAM or PSK)."""
    bps = np.array([int(np.log2(o)) if o > 0 else 0 for o in orders], dtype=np.int64)
    tot = int(bps.sum())
    tx_bits = bytes_to_bits(tx_bytes)
    if len(tx_bits) % tot:
        raise ValueError(f"Bits length ({len(tx_bits)}) must be multiple of bits_per_symbol ({tot})")
    S = len(tx_bits) // tot
    make = psk_lut if scheme == "PSK" else qam_lut
    luts = {int(o): make(int(o)) for o in np.unique(orders) if o > 0}
    offs = np.concatenate([[0], np.cumsum(bps)[:-1]])
    bits2 = tx_bits.reshape(S, tot).astype(np.int64)
    idx = np.zeros((S, N), dtype=np.int64)
    X = np.zeros((S, N), dtype=np.complex128)
    for k in range(N):
        if bps[k] == 0:
            continue
        w = bits2[:, offs[k]:offs[k] + bps[k]] @ (1 << np.arange(bps[k] - 1, -1, -1))
        idx[:, k] = w
        X[:, k] = luts[int(orders[k])][w]
    x = modulate(X, cp)
    pp = papr_db(x)
    y = channel_conv(x.ravel(), h_raw)
    if noise is not None:
        y = awgn(y, snr_db, noise[0], noise[1])
    H = np.fft.fft(h_raw, N)
    Z = demodulate(y.reshape(-1, N + cp), cp, H, eq, snr_db)
    ridx = np.zeros((S, N), dtype=np.int64)
    rbits = np.zeros((S, tot), dtype=np.uint8)
    for k in range(N):
        if bps[k] == 0:
            continue
        r = nn_demap(Z[:, k], luts[int(orders[k])])
        ridx[:, k] = r
        rbits[:, offs[k]:offs[k] + bps[k]] = (r[:, None] >> np.arange(bps[k] - 1, -1, -1)) & 1
    allb = rbits.ravel()
    nfull = (len(allb) // 8) * 8
    rx = np.packbits(allb[:nfull]).tobytes()
    rx_bits = bytes_to_bits(rx)
    n = min(len(tx_bits), len(rx_bits))
    be = int(np.count_nonzero(tx_bits[:n] != rx_bits[:n]))
    # symbol errors: symbols != encode(received_bits) (simulation/models.py:604-605); inactive
    # subcarriers carry 0+0j on both sides.
    if len(rx_bits) % tot == 0 and len(rx_bits) // tot == S:
        se = int(np.count_nonzero((ridx != idx) & (bps[None, :] > 0)))
    else:
        se = -1
    return LinkResult(be, se, S * tot, pp, S * N, rx)
