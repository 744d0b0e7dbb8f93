"""The throughput-mode stream definition restated in the oracle (oracle/philox_streams.py).

CPU-only: Philox4x32-10 against the Random123 known-answer vectors, and the statistical
and structural properties of the lane streams that the GPU parity tests
(test_gpu_philox_parity.py) then hold the fused kernels to.
"""

import numpy as np
import pytest

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


def test_sfc32_counter_starts_at_one():
    g = P.Sfc32([1], [2], [3])
    assert int(g.next()[0]) == 1 + 2 + 1
    assert int(g.a[0]) == 2 ^ (2 >> 9) and int(g.b[0]) == 3 + (3 << 3)


def test_lane_streams_depend_only_on_seed_and_symbol():
    a = P.lane_generators(7, np.arange(10, 20), 1024)
    b = P.lane_generators(7, np.arange(15, 20), 1024)
    wa, wb = a.next(), b.next()
    assert np.array_equal(wa[5 * 64:], wb)
    c = P.lane_generators(8, np.arange(10, 20), 1024)
    assert not np.array_equal(c.next(), wa)


@pytest.mark.parametrize("N,b", [(1024, 6), (64, 2), (16, 4), (4096, 8)])
def test_payload_bits_uniform(N, b):
    S = max(1, 200_000 // N)
    idx = P.tx_indices(P.lane_generators(3, np.arange(S), N), S, N, b)
    assert idx.shape == (S, N) and idx.min() >= 0 and idx.max() < 2 ** b
    counts = np.bincount(idx.ravel(), minlength=2 ** b)
    exp = idx.size / 2 ** b
    assert np.all(np.abs(counts - exp) < 6 * np.sqrt(exp))


def test_noise_is_complex_gaussian():
    S, N, sigma = 400, 1024, 0.3
    g = P.lane_generators(5, np.arange(S), N)
    P.tx_indices(g, S, N, 6)
    n = P.lane_noise(g, S, N, sigma).ravel()
    for comp in (n.real, n.imag):
        assert abs(comp.mean()) < 5 * sigma / np.sqrt(n.size)
        assert abs(comp.var() / sigma ** 2 - 1) < 0.01
        k = np.mean((comp / sigma) ** 4)
        assert abs(k - 3) < 0.05
    # tails: P(|n_re| > 3 sigma) = 2.7e-3
    tail = np.mean(np.abs(n.real) > 3 * sigma)
    assert abs(tail / 2.6998e-3 - 1) < 0.05
    assert abs(np.corrcoef(n.real, n.imag)[0, 1]) < 0.01


def test_oracle_link_noise_free_is_error_free():
    r = P.run_philox(2, 32, 1024, 64, np.array([0.8, 0.3j, 0.1]), 2, "MMSE", 30.0, noise_on=False)
    assert r.bit_errors == 0 and r.symbol_errors == 0
