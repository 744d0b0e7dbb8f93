"""Run-to-run bit identity of the complex128 throughput kernels at the bench's full sizes.

Round 4 found a silent store hazard in the window-FIR TX (a buffer store with an SGPR offset whose
data VGPRs the next VALU instruction overwrote before the store had read them: ~20 % of config-e
rows differed in the low bits of their real parts between identical launches).
These tests launch the bench configs' transmitters twice over the whole step and require the
channel samples and the statistics record to be identical bit for bit, and require two launches
over the halves of the range (split at an offset that is no multiple of the symbol-group size) to
tile the one launch exactly -- the stream is defined per (seed, global symbol).  The receivers'
counts of two identical runs must agree as well.  tests/test_isa_guard.py keeps buffer stores out
of the device code statically.
"""

import pytest
import torch

import bench
from ofdm_based_systems.engine import new_stats

pytestmark = pytest.mark.gpu

# config, OFDM symbols per launch (the bench step), split offset for the two half launches
SHAPES = [
    ("c", 1_000_000, 499_999),   # N = 1024, 8-tap window FIR (LT = 8)
    ("d", 500_000, 250_013),     # N = 2048, adaptive loading, 4-tap window FIR
    ("e", 250_000, 124_997),     # N = 4096, 256-QAM, 4-tap window FIR at 3 waves per SIMD
    ("b", 1_000_000, 333_331),   # N = 1024, flat TX
]


@pytest.mark.parametrize("cfg,S,split", SHAPES, ids=[s[0] for s in SHAPES])
def test_full_size_tx_is_bit_identical_across_launches(gpu, cfg, S, split):
    eng = bench.make_engine(bench.CONFIGS[cfg], "f64")
    seed = 4242
    y1 = torch.empty((S, eng.ystride), dtype=eng.cdtype, device="cuda")
    s1 = new_stats("cuda")
    eng.tx(eng.stream(), None, seed, 0, S, y1, s1)
    y2 = torch.empty_like(y1)
    s2 = new_stats("cuda")
    eng.tx(eng.stream(), None, seed, 0, S, y2, s2)
    torch.cuda.synchronize()
    same = torch.equal(y1, y2)
    if not same:  # say how many rows differ before failing
        rows = int((y1 != y2).any(dim=1).sum())
        pytest.fail(f"config {cfg}: {rows} of {S} rows differ between two identical launches")
    assert torch.equal(s1, s2), (s1.cpu().tolist(), s2.cpu().tolist())
    # the halves [0, split) and [split, S) in two launches tile the one launch
    s3 = new_stats("cuda")
    eng.tx(eng.stream(), None, seed, 0, split, y2[:split], s3)
    eng.tx(eng.stream(), None, seed, split, S - split, y2[split:], s3)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2), f"config {cfg}: half launches differ from the whole"
    # exact fixed-point power: the two launches' limbs add to the one launch's
    assert s3[0].item() == s1[0].item()
    del y1, y2
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cfg", ["c", "e"])
def test_full_size_runs_repeat_their_counts(gpu, cfg):
    N, M, ch, ratio, eq, snr, _ = bench.CONFIGS[cfg]
    eng = bench.make_engine(bench.CONFIGS[cfg], "f64")
    S = 1_000_000 // max(1, N // 1024)
    a = eng.run(S, snr, seed=99)
    b = eng.run(S, snr, seed=99)
    assert a.bit_errors > 0
    assert (a.bit_errors, a.symbol_errors, a.power_sum) == (b.bit_errors, b.symbol_errors, b.power_sum)
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cfg,S,split", SHAPES, ids=[s[0] for s in SHAPES])
def test_full_size_rx_halves_add_up_to_the_whole(gpu, cfg, S, split):
    """The receiver over [0, S) and over [0, split) + [split, S) of one transmitted stream count the
    same errors: every symbol is decided exactly once whatever the launch's grid (the N = 1024
    receivers stride a grid of two resident rounds, the others up to kMaxGrid workgroups)."""
    N, M, ch, ratio, eq, snr, _ = bench.CONFIGS[cfg]
    eng = bench.make_engine(bench.CONFIGS[cfg], "f64")
    seed = 777
    y = torch.empty((S, eng.ystride), dtype=eng.cdtype, device="cuda")
    stats = new_stats("cuda")
    st = eng.stream()
    eng.tx(st, None, seed, 0, S, y, stats)
    samples = S * (N + eng.cp)
    n_valid = eng.valid_bits(S)
    whole = torch.zeros(2, dtype=torch.int64, device="cuda")
    eng.rx(st, y, None, None, seed, stats, samples, snr, True, None, 0, S, n_valid, whole)
    parts = torch.zeros(2, dtype=torch.int64, device="cuda")
    eng.rx(st, y[:split], None, None, seed, stats, samples, snr, True, None, 0, split, n_valid, parts)
    eng.rx(st, y[split:], None, None, seed, stats, samples, snr, True, None, split, S - split, n_valid, parts)
    torch.cuda.synchronize()
    w, p = whole.cpu().tolist(), parts.cpu().tolist()
    assert w[0] > 0
    assert w == p, f"config {cfg}: whole {w} != halves {p}"
    del y
    torch.cuda.empty_cache()
