"""Edge cases of the fused path through the C ABI: empty runs, fewer symbols than a
workgroup holds (8 symbols per 512-thread block at N = 1024, 16 per multipath TX group),
ragged counts and offsets, and one-symbol runs, each against the oracle on the same streams.

The reference's own edge cases are the ValueErrors of SURVEY 8(b) (tests/test_api_contract.py);
these are the launch-shape edges of the kernels (partial blocks, partial symbol groups, the
predecessor tail of the first symbol of a shard).
"""

import numpy as np
import pytest
import torch
from conftest import channel

import philox_streams as P
import ofdm_oracle as O
from ofdm_based_systems import _backend as B
from ofdm_based_systems.engine import LinkEngine, new_stats

pytestmark = pytest.mark.gpu

EQ = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}

# N, M, channel, equaliser, SNR (BER ~1e-2 so that even one symbol counts errors)
SHAPES = [
    (1024, 64, "flat_fading", "NONE", 16.0),        # flat TX, 512-thread blocks
    (1024, 64, "severe_multipath", "MMSE", 18.0),   # window-FIR TX (16-symbol groups)
    (256, 16, "Lin-Phoong_P1", "ZF", 12.0),
    (32, 16, "flat_fading", "NONE", 10.0),          # generic kernel (N < 64)
]


def make(N, M, ch, eq):
    h = channel(ch)
    cp = len(h) - 1
    return LinkEngine(N, cp, h, EQ[eq], [O.qam_lut(M)], None, B.OFDM_F32), h, cp


@pytest.mark.parametrize("N,M,ch,eq,snr", SHAPES, ids=[f"N{s[0]}-{s[2]}" for s in SHAPES])
def test_empty_run(gpu, N, M, ch, eq, snr):
    eng, _, _ = make(N, M, ch, eq)
    r = eng.run(0, snr, seed=1)
    assert (r.bit_errors, r.symbol_errors, r.samples, r.power_sum) == (0, 0, 0, 0.0)


@pytest.mark.parametrize("S", [1, 3, 7, 9, 13, 17, 33])
@pytest.mark.parametrize("N,M,ch,eq,snr", SHAPES, ids=[f"N{s[0]}-{s[2]}" for s in SHAPES])
def test_ragged_counts_match_oracle(gpu, N, M, ch, eq, snr, S):
    eng, h, cp = make(N, M, ch, eq)
    seed = 31
    y = torch.empty((S, eng.ystride), dtype=eng.cdtype, device="cuda")
    stats = new_stats("cuda")
    eng.tx(eng.stream(), None, seed, 0, S, y, stats)
    torch.cuda.synchronize()
    ref_y = P.run_philox(seed, S, N, M, h, cp, eq, snr, noise_on=False)
    rms = np.sqrt(np.mean(np.abs(ref_y.y) ** 2))
    assert np.max(np.abs(y.cpu().numpy() - ref_y.y)) <= 1e-4 * rms
    res = eng.run(S, snr, seed=seed)
    ref = P.run_philox(seed, S, N, M, h, cp, eq, snr)
    for got, want in ((res.bit_errors, ref.bit_errors), (res.symbol_errors, ref.symbol_errors)):
        assert abs(got - want) <= 3 + 1e-3 * want, (S, got, want)
    assert res.power_sum == pytest.approx(ref.power_sum, rel=1e-5)


@pytest.mark.parametrize("N,M,ch,eq,snr", SHAPES[:3], ids=[f"N{s[0]}-{s[2]}" for s in SHAPES[:3]])
def test_ragged_offsets_tile_the_run(gpu, N, M, ch, eq, snr):
    """TX over [0, S) in pieces starting at ragged symbol offsets (a shard boundary inside a
    workgroup's symbols and inside a multipath group, whose first symbol regenerates its
    predecessor's tail) writes exactly the samples of one launch over [0, S)."""
    eng, _, _ = make(N, M, ch, eq)
    S, seed = 101, 4
    whole = torch.empty((S, eng.ystride), dtype=eng.cdtype, device="cuda")
    eng.tx(eng.stream(), None, seed, 0, S, whole, new_stats("cuda"))
    parts = torch.empty_like(whole)
    st = new_stats("cuda")
    cuts = [0, 1, 6, 23, 40, 57, 100, S]
    for a, b in zip(cuts[:-1], cuts[1:]):
        eng.tx(eng.stream(), None, seed, a, b - a, parts[a:b], st)
    torch.cuda.synchronize()
    assert torch.equal(whole, parts)


# the same launch-shape edges on the variant kernels: SC-OFDM + zero padding with 16-PSK sector
# decisions (throughput FB = 4), 8-PSK (FB = 3), a prefix shorter than the channel, and adaptive
# bit loading (FB = 1) -- through the case setup of the parity suite
VARIANTS = [
    (256, 16, "Lin-Phoong_P1", "MMSE", 14.0, {"scheme": "PSK", "modulator": "SC", "prefix": "ZP"}),
    (1024, 8, "severe_multipath", "MMSE", 14.0, {"scheme": "PSK"}),
    (256, 16, "severe_multipath", "MMSE", 12.0, {"cp": 2}),
    (2048, 0, "Lin-Phoong_P1", "MMSE", 12.0, {"adaptive": True}),
]


@pytest.mark.parametrize("S", [1, 5, 11])
@pytest.mark.parametrize("N,M,ch,eq,snr,var", VARIANTS, ids=[f"N{v[0]}-{'-'.join(map(str, v[5]))}" for v in VARIANTS])
def test_ragged_variant_counts_match_oracle(gpu, N, M, ch, eq, snr, var, S):
    from test_gpu_philox_parity import setup

    eng, h, cp, kw = setup(N, M, ch, eq, B.OFDM_F32, var, snr)
    res = eng.run(S, snr, seed=17)
    ref = P.run_philox(17, S, N, M, h, cp, eq, snr, **kw)
    for got, want in ((res.bit_errors, ref.bit_errors), (res.symbol_errors, ref.symbol_errors)):
        assert abs(got - want) <= 3 + 1e-3 * want, (S, got, want)
    assert res.power_sum == pytest.approx(ref.power_sum, rel=1e-5)
