"""Throughput mode against the oracle on identical inputs.

The fused kernels generate their bits and noise from the throughput-mode stream
definition; oracle/philox_streams.py restates that definition and runs the link through
the oracle's (reference-pinned) arithmetic.  Checked here, per configuration:

* TX: the kept channel samples y of the complex64 kernel vs the oracle's modulate +
  channel on the same bits (relative 1e-4 of the rms sample: float32 IFFT/FIR rounding),
  and the power / PAPR statistics (relative 1e-5);
* RX: bit and symbol error counts vs the oracle's on the same bits and noise, inside the
  oracle's decision bracket (philox_streams.decision_bracket): the GPU evaluates the noise
  radius with the float32 hardware log2 / sqrt and its FFTs in its own arithmetic, so a
  decision may differ from the oracle's only for a received point within the oracle's bound
  on that deviation (z_error_bound) of a decision boundary; the bracket counts the errors of
  every such alternative decision.  The oracle takes the receivers' noise radii from the GPU
  (ofdm_noise_radius: the float32 hardware log2 / sqrt, the one non-IEEE step of the stream
  definition) and sigma from the GPU run's exact power: complex128 brackets are then a single
  value (width asserted <= 2, printed), i.e. bit-exact counts; complex64 brackets carry the
  float32 transform rounding (width asserted per case, printed).

Sizes cover both workgroup shapes of the throughput kernels (512 threads at N <= 1024
without equaliser, 256 otherwise), the multipath FIR, all three equalisers, QPSK to
256-QAM, and the generic kernel in throughput mode (N < 64 and complex128).
"""

import numpy as np
import pytest
import torch
from conftest import channel

import philox_streams as P
import ofdm_oracle as O
from ofdm_based_systems import _backend as B
from ofdm_based_systems.constellation.adaptive import AdaptiveConstellationMapper
from ofdm_based_systems.constellation.models import PSKConstellationMapper, QAMConstellationMapper
from ofdm_based_systems.engine import LinkEngine, new_stats

pytestmark = pytest.mark.gpu

EQ = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}

# N, M, channel, equaliser, OFDM symbols, SNR dB (BER ~1e-3 .. 1e-2), precision, variant
CASES = [
    (1024, 64, "flat_fading", "NONE", 512, 20.0, B.OFDM_F32, {}),
    (1024, 64, "severe_multipath", "MMSE", 512, 24.0, B.OFDM_F32, {}),
    (256, 16, "Lin-Phoong_P1", "ZF", 1024, 22.0, B.OFDM_F32, {}),
    (64, 4, "rayleigh_fading", "ZF", 4096, 14.0, B.OFDM_F32, {}),
    (4096, 256, "Lin-Phoong_P1", "MMSE", 96, 31.0, B.OFDM_F32, {}),
    (2048, 16, "flat_fading", "NONE", 256, 14.0, B.OFDM_F32, {}),
    (32, 16, "flat_fading", "NONE", 8192, 14.0, B.OFDM_F32, {}),
    (1024, 64, "severe_multipath", "MMSE", 256, 24.0, B.OFDM_F64, {}),
    # complex128 throughput kernels (the headline precision): flat TX + no equaliser (config b),
    # register-window FIR (4 / 8 taps), the run-time-tap FIR (cp > lanes per symbol), N = 64 ..
    # 4096 (two-level twiddles and two-wave symbols from 2048, preloaded equaliser at 4096)
    (1024, 64, "flat_fading", "NONE", 512, 20.0, B.OFDM_F64, {}),
    (256, 16, "Lin-Phoong_P1", "ZF", 1024, 22.0, B.OFDM_F64, {}),
    (64, 4, "rayleigh_fading", "ZF", 4096, 14.0, B.OFDM_F64, {}),
    (64, 16, "severe_multipath", "MMSE", 2048, 18.0, B.OFDM_F64, {}),
    (2048, 16, "flat_fading", "NONE", 256, 14.0, B.OFDM_F64, {}),
    (4096, 256, "Lin-Phoong_P1", "MMSE", 96, 31.0, B.OFDM_F64, {}),
    # N = 4096 with one symbol per workgroup: ZF through the late coefficient loads, and no equaliser
    (4096, 16, "Lin-Phoong_P1", "ZF", 64, 16.0, B.OFDM_F64, {}),
    (4096, 64, "flat_fading", "NONE", 64, 20.0, B.OFDM_F64, {}),
    (256, 16, "severe_multipath", "MMSE", 512, 16.0, B.OFDM_F64, {"cp": 2}),
    (512, 4, "default_multipath", "ZF", 512, 12.0, B.OFDM_F64, {"cp": 0}),
    # SURVEY 8(f) variants on the complex128 throughput kernels (the bench precision): SC-OFDM
    # (FFT -> EQ -> IFFT), zero padding (run-time-tap FIR, overlap-add RX), 4/8/16/32-PSK sector
    # decisions (FB = 2 / 3 / 4 / 5), N = 4096 with one symbol per workgroup
    (1024, 64, "severe_multipath", "MMSE", 256, 20.0, B.OFDM_F64, {"modulator": "SC"}),
    (1024, 16, "severe_multipath", "MMSE", 256, 21.0, B.OFDM_F64, {"prefix": "ZP"}),
    (1024, 16, "severe_multipath", "MMSE", 128, 16.0, B.OFDM_F64, {"scheme": "PSK"}),
    (1024, 8, "Lin-Phoong_P2", "MMSE", 128, 22.0, B.OFDM_F64, {"scheme": "PSK", "modulator": "SC", "prefix": "ZP"}),
    (256, 32, "severe_multipath", "MMSE", 256, 24.0, B.OFDM_F64, {"scheme": "PSK", "prefix": "ZP"}),
    (128, 4, "severe_multipath", "ZF", 1024, 10.0, B.OFDM_F64, {"scheme": "PSK", "prefix": "ZP"}),
    (4096, 64, "Lin-Phoong_P1", "MMSE", 64, 22.0, B.OFDM_F64, {"modulator": "SC"}),
    (2048, 16, "Lin-Phoong_P1", "MMSE", 128, 19.0, B.OFDM_F64, {"prefix": "ZP", "modulator": "SC"}),
    (256, 16, "flat_fading", "NONE", 1024, 12.0, B.OFDM_F64, {"modulator": "SC"}),
    # SURVEY 8(f) variants on the generic kernel
    (64, 4, "Lin-Phoong_P2", "ZF", 2048, 20.0, B.OFDM_F32, {"modulator": "SC"}),
    (1024, 16, "severe_multipath", "MMSE", 256, 21.0, B.OFDM_F32, {"prefix": "ZP"}),
    (256, 8, "Lin-Phoong_P1", "MMSE", 512, 17.0, B.OFDM_F32, {"scheme": "PSK"}),
    (128, 4, "Lin-Phoong_P2", "MMSE", 1024, 10.0, B.OFDM_F64, {"modulator": "SC", "prefix": "ZP", "scheme": "PSK"}),
    (2048, 16, "Lin-Phoong_P1", "MMSE", 128, 19.0, B.OFDM_F32, {"prefix": "ZP", "modulator": "SC"}),
    # SC-OFDM on the throughput kernels (FFT -> EQ -> IFFT with the per-pass tables)
    (1024, 64, "severe_multipath", "MMSE", 256, 20.0, B.OFDM_F32, {"modulator": "SC"}),
    (256, 16, "flat_fading", "NONE", 1024, 12.0, B.OFDM_F32, {"modulator": "SC"}),
    # complex64 M-PSK: sector decisions (octant fold + tangent thresholds) vs the oracle's search
    (64, 2, "two_ray", "ZF", 2048, 4.0, B.OFDM_F32, {"scheme": "PSK"}),
    (128, 4, "severe_multipath", "MMSE", 1024, 8.0, B.OFDM_F32, {"scheme": "PSK"}),
    (1024, 16, "severe_multipath", "MMSE", 128, 16.0, B.OFDM_F32, {"scheme": "PSK"}),
    (512, 32, "Lin-Phoong_P1", "ZF", 128, 22.0, B.OFDM_F32, {"scheme": "PSK"}),
    # 4- and 16-PSK take the throughput kernels (FB = 2 / 4) with sector decisions: with
    # SC-OFDM's unscaled IFFT, with the zero-padding overlap-add and its tail noise, and both
    (256, 16, "Lin-Phoong_P1", "MMSE", 256, 20.0, B.OFDM_F32, {"scheme": "PSK", "modulator": "SC", "prefix": "ZP"}),
    (128, 4, "severe_multipath", "ZF", 1024, 10.0, B.OFDM_F32, {"scheme": "PSK", "prefix": "ZP"}),
    (256, 16, "two_ray", "MMSE", 256, 18.0, B.OFDM_F32, {"scheme": "PSK", "modulator": "SC"}),
    (512, 4, "Lin-Phoong_P1", "MMSE", 256, 9.0, B.OFDM_F32, {"scheme": "PSK", "modulator": "SC"}),
    # 8- and 32-PSK (odd bits) on their own throughput kernels (FB = 3 / 5), with SC-OFDM and
    # zero padding; (256, 8, ...) and (512, 32, ...) above cover plain OFDM
    (1024, 8, "Lin-Phoong_P2", "MMSE", 128, 22.0, B.OFDM_F32, {"scheme": "PSK", "modulator": "SC", "prefix": "ZP"}),
    (256, 32, "severe_multipath", "MMSE", 256, 24.0, B.OFDM_F32, {"scheme": "PSK", "prefix": "ZP"}),
    (64, 8, "rayleigh_fading", "ZF", 2048, 20.0, B.OFDM_F32, {"scheme": "PSK", "prefix": "ZP"}),  # 4 lanes/symbol
    (128, 32, "two_ray", "MMSE", 1024, 26.0, B.OFDM_F32, {"scheme": "PSK", "modulator": "SC"}),
    # prefix shorter than the channel (prefix_length_ratio < 1): inter-symbol interference
    # through the FIR's tail of the previous symbol; no prefix at all on a 4-tap channel
    (256, 16, "severe_multipath", "MMSE", 512, 16.0, B.OFDM_F32, {"cp": 2}),
    (1024, 64, "Lin-Phoong_P2", "MMSE", 256, 30.0, B.OFDM_F32, {"cp": 1}),
    (512, 4, "default_multipath", "ZF", 512, 12.0, B.OFDM_F32, {"cp": 0}),
    # CAPACITY_BASED bit loading (config d): per-subcarrier orders from water-filling at the SNR;
    # an odd symbol count leaves a trailing partial byte that is not compared
    (2048, 0, "Lin-Phoong_P1", "MMSE", 255, 20.0, B.OFDM_F32, {"adaptive": True}),
    (1024, 0, "severe_multipath", "ZF", 257, 22.0, B.OFDM_F32, {"adaptive": True}),
    (256, 0, "two_ray", "ZF", 1023, 30.0, B.OFDM_F32, {"adaptive": True}),   # up to 256-QAM
    (256, 0, "two_ray", "MMSE", 1024, 16.0, B.OFDM_F32, {"adaptive": True}),  # unused subcarriers
    (4096, 0, "Lin-Phoong_P1", "MMSE", 160, 26.0, B.OFDM_F32, {"adaptive": True}),
    (64, 0, "default_multipath", "MMSE", 4097, 18.0, B.OFDM_F32, {"adaptive": True}),
    # ... and on the complex128 adaptive throughput kernel (FB = 1, double per-order tables)
    (2048, 0, "Lin-Phoong_P1", "MMSE", 255, 20.0, B.OFDM_F64, {"adaptive": True}),
    (2048, 0, "two_ray", "ZF", 129, 24.0, B.OFDM_F64, {"adaptive": True}),  # one symbol per workgroup, ZF
    (256, 0, "two_ray", "ZF", 1023, 30.0, B.OFDM_F64, {"adaptive": True}),
    (1024, 0, "severe_multipath", "ZF", 257, 24.0, B.OFDM_F64, {"adaptive": True}),
    # CAPACITY_BASED with the PSK base mapper (orders 2..32 and unused subcarriers at an aggressive
    # SER target): the generic kernel, nearest point within each subcarrier's own LUT
    (64, 0, "Lin-Phoong_P2", "MMSE", 1024, 20.0, B.OFDM_F32, {"adaptive": True, "scheme": "PSK", "ser": 0.1}),
    (128, 0, "two_ray", "ZF", 511, 26.0, B.OFDM_F64, {"adaptive": True, "scheme": "PSK", "ser": 0.05}),
]


def _id(c):
    v = "".join(f"-{k}={w}" for k, w in c[7].items())
    return f"N{c[0]}-M{c[1]}-{c[2]}-{c[3]}-{'f32' if c[6] == B.OFDM_F32 else 'f64'}{v}"


IDS = [_id(c) for c in CASES]


def setup(N, M, ch, eq, prec, var=None, snr=None):
    """Engine of a case; returns (engine, CIR, cp, keyword arguments for P.run_philox)."""
    var = dict(var or {})
    h = channel(ch)
    cp = var.pop("cp", len(h) - 1)
    sc = None
    ser = var.pop("ser", 1e-3)
    if var.pop("adaptive", False):
        psk = var.get("scheme") == "PSK"
        orders, _, _ = O.adaptive_orders(N, h, snr, ser, True, "PSK" if psk else "QAM")
        base = PSKConstellationMapper if psk else QAMConstellationMapper
        luts, sc = AdaptiveConstellationMapper(orders, base, N).lut_tables()
        var["orders"] = orders
    else:
        luts = [O.psk_lut(M) if var.get("scheme") == "PSK" else O.qam_lut(M)]
    eng = LinkEngine(N, cp, h, EQ[eq], luts, sc, prec,
                     prefix=B.PREFIX_ZERO if var.get("prefix") == "ZP" else B.PREFIX_CYCLIC,
                     modulator=B.MOD_SC if var.get("modulator") == "SC" else B.MOD_OFDM)
    return eng, h, cp, var


@pytest.mark.parametrize("N,M,ch,eq,S,snr,prec,var", CASES, ids=IDS)
def test_tx_samples_match_oracle(gpu, N, M, ch, eq, S, snr, prec, var):
    eng, h, cp, var = setup(N, M, ch, eq, prec, var, snr)
    seed = 1234
    y = torch.empty((S, eng.ystride), dtype=eng.cdtype, device="cuda")
    stats = new_stats("cuda")
    eng.tx(eng.stream(), None, seed, 0, S, y, stats)
    torch.cuda.synchronize()
    ref = P.run_philox(seed, S, N, M, h, cp, eq, snr, noise_on=False, **var)
    got = y.cpu().numpy()
    rms = np.sqrt(np.mean(np.abs(ref.y) ** 2))
    tol = 1e-4 if prec == B.OFDM_F32 else 1e-12
    assert got.shape == ref.y.shape
    assert np.max(np.abs(got - ref.y)) <= tol * rms
    st = stats.cpu().numpy()
    rt = 1e-5 if prec == B.OFDM_F32 else 1e-12
    assert st[0] == pytest.approx(ref.power_sum, rel=rt)
    assert st[1] == pytest.approx(ref.x_power_sum, rel=rt)
    assert st[2] == pytest.approx(ref.x_peak, rel=rt)


def gpu_radius(words: np.ndarray) -> np.ndarray:
    """The receivers' noise radius of each lane word on this GPU (ofdm_noise_radius: the same
    float32 hardware log2 / sqrt the fused kernels evaluate)."""
    w = torch.from_numpy(np.ascontiguousarray(words, np.uint32).view(np.int32)).to("cuda")
    r = torch.empty(w.numel(), dtype=torch.float32, device="cuda")
    B.check(B.lib().ofdm_noise_radius(B.stream_ptr(), B.ptr(w), w.numel(), B.ptr(r)))
    return r.cpu().numpy()


def bracket_width_bound(prec, var, count):
    """Widest rigorous decision bracket the test accepts (bit errors).  complex128: the oracle holds
    the receivers' noise bit for bit (their radii, their sigma), so only FFT / FIR / equaliser
    rounding at 2^-53 remains -- the counts are pinned to within 2 (in practice exactly, width 0).
    complex64: the float32 transforms' rounding, bounded through the 2-norm (philox_streams.
    z_error_bound), leaves up to ~8 % of the count at N = 4096 / 256-QAM and a few tens of counts on
    the ~200-error adaptive cases (asserted <= max(64, 10 %)); single-carrier complex64 spreads the
    worst subcarrier's equaliser gain over every sample and is not bounded here.  complex64 is
    also held to the per-point statistical bracket (stat_width_bound)."""
    if prec == B.OFDM_F64:
        return max(2, count // 1000)
    return None if var.get("modulator") == "SC" else max(64, count // 10)


def stat_width_bound(count):
    """Widest per-point statistical bracket (philox_streams.z_stat_bound, 16 standard deviations of
    a model calibrated by the GPU transmitter's own measured deviation) the complex64 cases accept:
    5 % of the count, and at least 4 counts."""
    return max(4, count // 20)


def tx_deviation(eng, seed, S):
    """The complex64 transmitter's per-sample deviation from the oracle's stored samples, as a
    function for run_philox(stat_sigma=...): the same seed's channel samples from the GPU."""
    y = torch.empty((S, eng.ystride), dtype=eng.cdtype, device="cuda")
    eng.tx(eng.stream(), None, seed, 0, S, y, new_stats("cuda"))
    torch.cuda.synchronize()
    got = y.cpu().numpy().astype(np.complex128)
    return lambda yref: float(np.sqrt(np.mean(np.abs(got - yref) ** 2)))


@pytest.mark.parametrize("N,M,ch,eq,S,snr,prec,var", CASES, ids=IDS)
def test_error_counts_match_oracle(gpu, N, M, ch, eq, S, snr, prec, var):
    case_id = _id((N, M, ch, eq, S, snr, prec, var))
    eng, h, cp, var = setup(N, M, ch, eq, prec, var, snr)
    seed = 77
    res = eng.run(S, snr, seed=seed)
    f32 = prec == B.OFDM_F32
    ref = P.run_philox(seed, S, N, M, h, cp, eq, snr, precision="f32" if f32 else "f64",
                       radius_fn=gpu_radius, power_sum=res.power_sum,
                       stat_sigma=tx_deviation(eng, seed, S) if f32 else None, **var)
    assert ref.bit_errors > 100, "SNR too high for a meaningful count"
    be_lo, be_hi, se_lo, se_hi = ref.bracket
    print(f"bracket {case_id}: bits {res.bit_errors} in [{be_lo}, {be_hi}] "
          f"(width {be_hi - be_lo}), symbols {res.symbol_errors} in [{se_lo}, {se_hi}] (width {se_hi - se_lo})")
    if f32:
        # complex64: also inside the per-point statistical bracket, which is asserted narrow
        sb_lo, sb_hi, ss_lo, ss_hi = ref.stat_bracket
        print(f"stat bracket {case_id}: bits {res.bit_errors} in [{sb_lo}, {sb_hi}] (width {sb_hi - sb_lo}), "
              f"symbols {res.symbol_errors} in [{ss_lo}, {ss_hi}] (width {ss_hi - ss_lo})")
        assert sb_lo <= res.bit_errors <= sb_hi and ss_lo <= res.symbol_errors <= ss_hi, (res, ref.stat_bracket)
        wst = stat_width_bound(ref.bit_errors)
        assert sb_hi - sb_lo <= wst and ss_hi - ss_lo <= wst, (ref.stat_bracket, wst)
    assert be_lo <= ref.bit_errors <= be_hi and se_lo <= ref.symbol_errors <= se_hi
    assert be_lo <= res.bit_errors <= be_hi, (res.bit_errors, ref.bracket)
    assert se_lo <= res.symbol_errors <= se_hi, (res.symbol_errors, ref.bracket)
    wmax = bracket_width_bound(prec, var, ref.bit_errors)
    if wmax is not None:
        assert be_hi - be_lo <= wmax and se_hi - se_lo <= wmax, (ref.bracket, wmax)
    assert res.power_sum == pytest.approx(ref.power_sum, rel=1e-5 if prec == B.OFDM_F32 else 1e-12)


def test_gpu_noise_radius_within_its_bound(gpu):
    """The receivers' float32 hardware radius stays inside the float64 restatement's bound
    (noise_from_words) on 2^22 words spread over the whole 32-bit range, and is exact at 0."""
    rng = np.random.default_rng(5)
    w = np.concatenate([rng.integers(0, 2 ** 32, size=1 << 22, dtype=np.uint64).astype(np.uint32),
                        np.arange(0, 4096, dtype=np.uint32),
                        np.array([0x1F8, 0xFFFFFE07, 0xFFFFFF7F, 0xFFFFFF80, 0xFFFFFFFF], np.uint32)])
    ph = rng.integers(0, P.NOISE_PHASES, size=w.size)
    n64, b64 = P.noise_from_words(w, ph, 1.0, with_bound=True)
    n32 = P.noise_from_words(w, ph, 1.0, radius_fn=gpu_radius)
    assert np.all(np.abs(n32 - n64) <= b64)
    r = gpu_radius(w)
    # stream version 3: the whole word -- 6.660 sigma at words 0 / 1, 6.493 sigma at words 2 / 3
    assert np.all(np.isfinite(r)) and r.min() >= 0.0 and r.max() < 6.661 / P.SQRT_2LN2
    assert r[(1 << 22) + 0] == r[(1 << 22) + 1] and abs(r[(1 << 22) + 2] * P.SQRT_2LN2 - 6.4934) < 1e-3


def test_sharded_halves_add_up_to_the_whole(gpu):
    """Symbols [0, S) in two launches at different offsets = one launch (stream is per symbol)."""
    eng, h, cp, _ = setup(1024, 64, "severe_multipath", "MMSE", B.OFDM_F32)
    S = 600
    whole = eng.run(S, 24.0, seed=9)
    y = torch.empty((S, 1024), dtype=eng.cdtype, device="cuda")
    st = new_stats("cuda")
    eng.tx(eng.stream(), None, 9, 0, 250, y[:250], st)
    eng.tx(eng.stream(), None, 9, 250, S - 250, y[250:], st)
    y2 = torch.empty_like(y)
    eng.tx(eng.stream(), None, 9, 0, S, y2, new_stats("cuda"))
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    assert whole.bit_errors > 0
