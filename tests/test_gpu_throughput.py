"""Throughput mode (Philox bits + noise generated inside the kernels).

Bit-exact properties at full size (noise-free links decode perfectly, results do not
depend on how the symbols are batched) and the statistical bar of the north star:
the BER curve within +-0.05 dB of the reference's at BER ~ 1e-4, measured against
the reference-stream GPU path (bit-exact with the reference, test_gpu_parity.py).
"""

import math

import numpy as np
import pytest
import torch
from conftest import channel

import ofdm_oracle as O
from ofdm_based_systems import _backend as B
from ofdm_based_systems.engine import LinkEngine

pytestmark = pytest.mark.gpu


def engine(N, M, ch, eq, precision=B.OFDM_F32, ratio=1.0):
    h = channel(ch)
    cp = int(ratio * (len(h) - 1))
    return LinkEngine(N, cp, h, eq, [O.qam_lut(M)], None, precision), cp


@pytest.mark.parametrize("N,M,ch,eq", [
    (1024, 64, "flat_fading", B.EQ_NONE),
    (1024, 64, "severe_multipath", B.EQ_MMSE),
    (2048, 16, "Lin-Phoong_P1", B.EQ_ZF),
    (4096, 256, "Lin-Phoong_P1", B.EQ_MMSE),
    (64, 4, "rayleigh_fading", B.EQ_ZF),
])
def test_noise_free_links_are_error_free(gpu, N, M, ch, eq):
    eng, _ = engine(N, M, ch, eq)
    res = eng.run(4096 if N <= 1024 else 512, 30.0, seed=11, noise_on=False)
    assert res.bit_errors == 0 and res.symbol_errors == 0
    assert 0.5 < res.power_sum / res.samples < 2.0


def test_philox_results_independent_of_batching(gpu):
    eng, _ = engine(1024, 64, "severe_multipath", B.EQ_MMSE)
    a = eng.run(3000, 22.0, seed=5)
    b = eng.run(3000, 22.0, seed=5, batch=1000)
    c = eng.run(3000, 22.0, seed=5, batch=777)
    assert (a.bit_errors, a.symbol_errors) == (b.bit_errors, b.symbol_errors) == (c.bit_errors, c.symbol_errors)
    assert a.bit_errors > 0
    d = eng.run(3000, 22.0, seed=6)
    assert d.bit_errors != a.bit_errors  # the seed matters


def test_one_plan_on_concurrent_streams(gpu):
    """Runs of one plan enqueued on three streams at once (as an SNR sweep or a pipelined
    bench does) give the same counts and statistics as the same runs one after another:
    the power reduction keeps a workspace per stream."""
    eng, _ = engine(1024, 64, "severe_multipath", B.EQ_MMSE)
    seeds = list(range(40, 49))
    serial = [eng.run(20000, 26.0, seed=s) for s in seeds]
    streams = [torch.cuda.Stream() for _ in range(3)]
    pend = []
    for i, s in enumerate(seeds):
        with torch.cuda.stream(streams[i % 3]):
            pend.append(eng.run_async(20000, 26.0, seed=s))
    for a, p in zip(serial, pend):
        b = p.result()
        assert (a.bit_errors, a.symbol_errors) == (b.bit_errors, b.symbol_errors)
        assert (a.power_sum, a.x_power_sum, a.x_peak) == (b.power_sum, b.x_power_sum, b.x_peak)


def test_philox_bits_are_uniform(gpu):
    """Map statistics: mean |x|^2 = 1 and PAPR in the usual range for random 64-QAM OFDM."""
    eng, _ = engine(1024, 64, "flat_fading", B.EQ_NONE)
    res = eng.run(20000, 24.0, seed=1)
    assert abs(res.x_power_sum / res.samples - 1.0) < 2e-3
    assert 9.0 < res.papr_db < 14.0


def reference_mode_ber(eng, N, cp, M, snr, S, seed):
    b = int(np.log2(M))
    tx, nz = O.reference_streams(seed, S * N * b, S * (N + cp))
    r = eng.run(S, snr, bits=np.frombuffer(tx, np.uint8), normals=nz)
    return r.bit_errors / (S * N * b)


@pytest.mark.parametrize("prec", [B.OFDM_F64, B.OFDM_F32], ids=["c128", "c64"])
@pytest.mark.parametrize("N,M,ch,eq,snr_lo,snr_hi", [
    (1024, 64, "flat_fading", B.EQ_NONE, 24.0, 25.0),          # config (b): BER 1e-4 near 24.4 dB
    (1024, 64, "severe_multipath", B.EQ_MMSE, 27.5, 28.5),    # config (c): BER 1e-4 near 27.7 dB
])
def test_ber_curve_within_005_db_of_reference(gpu, N, M, ch, eq, snr_lo, snr_hi, prec):
    """The throughput kernels the bench times (complex128 headline, complex64 companion) against
    the reference-stream path at the BER 1e-4 crossing (noise/models.py:13-22 with the reference's
    own normals; simulation/models.py:596-606 counts)."""
    S_ref, S_phx = 12000, 60000
    mid = 0.5 * (snr_lo + snr_hi)
    eng64, cp = engine(N, M, ch, eq, precision=B.OFDM_F64)
    ref_mid = reference_mode_ber(eng64, N, cp, M, mid, S_ref, seed=1)
    ref_hi = reference_mode_ber(eng64, N, cp, M, snr_hi, S_ref, seed=2)
    slope = (math.log10(ref_hi) - math.log10(ref_mid)) / (snr_hi - mid)  # decades / dB (< 0)
    eng_t, _ = engine(N, M, ch, eq, precision=prec)
    bits = S_phx * N * int(np.log2(M))
    phx = eng_t.run(S_phx, mid, seed=1234).bit_errors / bits
    # horizontal distance between the curves at the reference's BER, via the local slope
    delta_db = (math.log10(phx) - math.log10(ref_mid)) / slope
    assert 3e-5 < ref_mid < 1e-3
    assert abs(delta_db) <= 0.05, (ref_mid, ref_hi, phx, delta_db)
