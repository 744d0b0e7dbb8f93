"""Size-independent properties of the throughput path at the benchmark's full sizes
(BASELINE configs (b) and (e): 1e6 OFDM symbols of N = 1024, 2.5e5 of N = 4096 -- 16.4 GB of
channel samples per launch in complex128, the bench's headline precision, 8.2 GB in complex64),
where the oracle cannot follow:

* a noise-free link decodes every bit (map -> IFFT -> channel -> FFT -> equaliser -> slicer
  are exact inverses up to float rounding far below the decision distance);
* error counts are additive: one RX launch over [0, S) counts exactly what two RX launches over
  [0, S/2) and [S/2, S) count with the same TX statistics (sigma from the whole stream);
* results do not depend on batching: the batched schedule (power pass, then TX+RX per batch)
  gives the counts of the single-launch schedule.
"""

import numpy as np
import pytest
import torch
from conftest import channel

import ofdm_oracle as O
from ofdm_based_systems import _backend as B
from ofdm_based_systems.engine import LinkEngine, new_stats

pytestmark = pytest.mark.gpu

FULL = [  # N, M, channel, equaliser, symbols, SNR dB
    (1024, 64, "flat_fading", B.EQ_NONE, 1_000_000, 24.0),
    (4096, 256, "Lin-Phoong_P1", B.EQ_MMSE, 250_000, 34.0),
]


PRECS = pytest.mark.parametrize("prec", [B.OFDM_F64, B.OFDM_F32], ids=["c128", "c64"])


def _engine(N, M, ch, eq, prec):
    h = channel(ch)
    return LinkEngine(N, len(h) - 1, h, eq, [O.qam_lut(M)], None, prec)


@PRECS
@pytest.mark.parametrize("N,M,ch,eq,S,snr", FULL, ids=["b", "e"])
def test_full_size_noise_free_is_error_free(gpu, N, M, ch, eq, S, snr, prec):
    eng = _engine(N, M, ch, eq, prec)
    r = eng.run(S, snr, seed=3, noise_on=False)
    assert r.bit_errors == 0 and r.symbol_errors == 0
    assert 0.9 < r.power_sum / r.samples < 1.1  # unit-power constellation, unit-power channel
    assert 8.0 < r.papr_db < 14.0


@PRECS
@pytest.mark.parametrize("N,M,ch,eq,S,snr", FULL, ids=["b", "e"])
def test_full_size_counts_are_additive(gpu, N, M, ch, eq, S, snr, prec):
    eng = _engine(N, M, ch, eq, prec)
    st = eng.stream()
    y = torch.empty((S, eng.ystride), dtype=eng.cdtype, device="cuda")
    stats = new_stats("cuda")
    eng.tx(st, None, 7, 0, S, y, stats)
    samples = S * (N + eng.cp)
    whole = torch.zeros(2, dtype=torch.int64, device="cuda")
    eng.rx(st, y, None, None, 7, stats, samples, snr, 1, None, 0, S, eng.valid_bits(S), whole)
    parts = torch.zeros(2, dtype=torch.int64, device="cuda")
    h = S // 2
    eng.rx(st, y[:h], None, None, 7, stats, samples, snr, 1, None, 0, h, eng.valid_bits(S), parts)
    eng.rx(st, y[h:], None, None, 7, stats, samples, snr, 1, None, h, S - h, eng.valid_bits(S), parts)
    torch.cuda.synchronize()
    w, p = whole.cpu().numpy(), parts.cpu().numpy()
    assert w[0] > 1000 and np.array_equal(w, p), (w, p)
    # and the same run through the engine's own schedule
    del y
    r = eng.run(S, snr, seed=7)
    assert (r.bit_errors, r.symbol_errors) == (int(w[0]), int(w[1]))


@PRECS
def test_full_size_batching_invariance(gpu, prec):
    N, M, ch, eq, S, snr = FULL[0]
    eng = _engine(N, M, ch, eq, prec)
    a = eng.run(S, snr, seed=21)
    b = eng.run(S, snr, seed=21, batch=250_000)
    assert a.bit_errors > 1000
    assert (a.bit_errors, a.symbol_errors) == (b.bit_errors, b.symbol_errors)
    # the fixed-point power sum is exact: the same bits whatever the batching
    assert a.power_sum == b.power_sum
    c = eng.run(S, snr, seed=21, batch=333_333)
    assert (c.bit_errors, c.symbol_errors, c.power_sum) == (a.bit_errors, a.symbol_errors, a.power_sum)
