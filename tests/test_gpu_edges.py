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
SID = [f"N{s[0]}-{s[2]}" for s in SHAPES]
PRECS = pytest.mark.parametrize("prec", [B.OFDM_F64, B.OFDM_F32], ids=["c128", "c64"])


def make(N, M, ch, eq, prec):
    h = channel(ch)
    cp = len(h) - 1
    return LinkEngine(N, cp, h, EQ[eq], [O.qam_lut(M)], None, prec), h, cp


def assert_in_bracket(res, seed, S, N, M, h, cp, eq, snr, prec, **kw):
    """The run's counts inside the oracle's decision bracket (the receivers' own noise radii and
    sigma: complex128 pinned to within 2 counts)."""
    from test_gpu_philox_parity import gpu_radius

    ref = P.run_philox(seed, S, N, M, h, cp, eq, snr, precision="f64" if prec == B.OFDM_F64 else "f32",
                       radius_fn=gpu_radius, power_sum=res.power_sum, **kw)
    lo, hi, slo, shi = ref.bracket
    assert lo <= res.bit_errors <= hi and slo <= res.symbol_errors <= shi, (S, res.bit_errors, ref.bracket)
    if prec == B.OFDM_F64:
        assert hi - lo <= 2 and shi - slo <= 2, ref.bracket
    assert res.power_sum == pytest.approx(ref.power_sum, rel=1e-5 if prec == B.OFDM_F32 else 1e-12)


@PRECS
@pytest.mark.parametrize("N,M,ch,eq,snr", SHAPES, ids=SID)
def test_empty_run(gpu, N, M, ch, eq, snr, prec):
    eng, _, _ = make(N, M, ch, eq, prec)
    r = eng.run(0, snr, seed=1)
    assert (r.bit_errors, r.symbol_errors, r.samples, r.power_sum) == (0, 0, 0, 0.0)


@PRECS
@pytest.mark.parametrize("S", [1, 3, 7, 9, 13, 17, 33])
@pytest.mark.parametrize("N,M,ch,eq,snr", SHAPES, ids=SID)
def test_ragged_counts_match_oracle(gpu, N, M, ch, eq, snr, S, prec):
    eng, h, cp = make(N, M, ch, eq, prec)
    seed = 31
    y = torch.empty((S, eng.ystride), dtype=eng.cdtype, device="cuda")
    stats = new_stats("cuda")
    eng.tx(eng.stream(), None, seed, 0, S, y, stats)
    torch.cuda.synchronize()
    ref_y = P.run_philox(seed, S, N, M, h, cp, eq, snr, noise_on=False)
    rms = np.sqrt(np.mean(np.abs(ref_y.y) ** 2))
    assert np.max(np.abs(y.cpu().numpy() - ref_y.y)) <= (1e-4 if prec == B.OFDM_F32 else 1e-12) * rms
    res = eng.run(S, snr, seed=seed)
    assert_in_bracket(res, seed, S, N, M, h, cp, eq, snr, prec)


@PRECS
@pytest.mark.parametrize("N,M,ch,eq,snr", SHAPES[:3], ids=SID[:3])
def test_ragged_offsets_tile_the_run(gpu, N, M, ch, eq, snr, prec):
    """TX over [0, S) in pieces starting at ragged symbol offsets (a shard boundary inside a
    workgroup's symbols and inside a multipath group, whose first symbol regenerates its
    predecessor's tail) writes exactly the samples of one launch over [0, S)."""
    eng, _, _ = make(N, M, ch, eq, prec)
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
    (1024, 64, "severe_multipath", "MMSE", 16.0, {"modulator": "SC"}),
    (4096, 64, "Lin-Phoong_P1", "MMSE", 18.0, {"prefix": "ZP"}),
]


@PRECS
@pytest.mark.parametrize("S", [1, 5, 11])
@pytest.mark.parametrize("N,M,ch,eq,snr,var", VARIANTS, ids=[f"N{v[0]}-{'-'.join(map(str, v[5]))}" for v in VARIANTS])
def test_ragged_variant_counts_match_oracle(gpu, N, M, ch, eq, snr, var, S, prec):
    from test_gpu_philox_parity import setup

    eng, h, cp, kw = setup(N, M, ch, eq, prec, var, snr)
    res = eng.run(S, snr, seed=17)
    assert_in_bracket(res, 17, S, N, M, h, cp, eq, snr, prec, **kw)


# The largest shapes the plan accepts: N = 4096, a 32-tap channel with a prefix of twice its order
# (prefix_length_ratio 2, configuration/models.py:128-133), SC-OFDM with zero padding and MMSE, and
# the cyclic-prefix OFDM twin: every throughput kernel either fits the 160 KB of LDS or the launcher
# runs the generic kernel (kLdsPerCu in ofdm_kernels_inst.hpp) -- no launch may fail.
@PRECS
@pytest.mark.parametrize("var", [{"modulator": "SC", "prefix": "ZP"}, {}], ids=["sc-zp", "ofdm-cp"])
def test_lds_limit_shapes_run(gpu, prec, var):
    rng = np.random.default_rng(8)
    h = (rng.normal(size=32) + 1j * rng.normal(size=32)) * np.exp(-np.arange(32) / 6.0)
    N, M, S, snr, cp = 4096, 16, 9, 22.0, 62
    eng = LinkEngine(N, cp, h, B.EQ_MMSE, [O.qam_lut(M)], None, prec,
                     prefix=B.PREFIX_ZERO if var.get("prefix") == "ZP" else B.PREFIX_CYCLIC,
                     modulator=B.MOD_SC if var.get("modulator") == "SC" else B.MOD_OFDM)
    res = eng.run(S, snr, seed=5)
    assert_in_bracket(res, 5, S, N, M, h, cp, "MMSE", snr, prec, **var)
