"""Throughput of the fused path per modem variant (SURVEY 8(a) configs and the 8(f) rows).

Times ofdm_tx / ofdm_rx with HIP events on the launch stream, throughput mode (bits and noise
generated in the kernels), complex128 (the reference's arithmetic, default) or complex64, one GPU:

    python tools/bench_variants.py [--precision f64|f32] [--symbols 1000000] [--steps 5] > gpurun_out/variants.json

Prints one JSON object per variant and a summary table on stderr.  Which kernel runs:
square QAM or the reference's 4/16-PSK, OFDM or SC-OFDM, cyclic prefix or zero padding ->
the throughput specialisation on the bits per subcarrier; adaptive loading -> the adaptive
throughput kernel; 8-PSK (odd bits) -> the generic kernel.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-based-systems_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ofdm_based_systems import _backend as B  # noqa: E402
from ofdm_based_systems.constellation.adaptive import AdaptiveConstellationMapper  # noqa: E402
from ofdm_based_systems.constellation.models import PSKConstellationMapper, QAMConstellationMapper  # noqa: E402
from ofdm_based_systems.power_allocation.models import WaterfillingPowerAllocation  # noqa: E402
from ofdm_based_systems.engine import LinkEngine  # noqa: E402

EQ = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}

# name, N, M, scheme, channel, eq, snr, modulator, prefix
VARIANTS = [
    ("b: OFDM CP 64-QAM flat", 1024, 64, "QAM", "flat_fading", "NONE", 24.0, "OFDM", "CP"),
    ("c: OFDM CP 64-QAM severe MMSE", 1024, 64, "QAM", "severe_multipath", "MMSE", 27.75, "OFDM", "CP"),
    ("d: adaptive QAM N=2048 P1 MMSE WF", 2048, 0, "ADAPTIVE", "Lin-Phoong_P1", "MMSE", 20.0, "OFDM", "CP"),
    ("e: OFDM CP 256-QAM N=4096 P1 MMSE", 4096, 256, "QAM", "Lin-Phoong_P1", "MMSE", 30.0, "OFDM", "CP"),
    ("f1: SC-OFDM CP 64-QAM severe MMSE", 1024, 64, "QAM", "severe_multipath", "MMSE", 27.75, "SC", "CP"),
    ("f2: OFDM ZP 64-QAM severe MMSE", 1024, 64, "QAM", "severe_multipath", "MMSE", 27.75, "OFDM", "ZP"),
    ("f3: OFDM CP 16-PSK severe MMSE", 1024, 16, "PSK", "severe_multipath", "MMSE", 27.75, "OFDM", "CP"),
    # MMSE at 25 dB (BER ~2e-3): with ZF, SC-OFDM spreads P2's spectral-null noise enhancement
    # over every symbol and the BER (0.43) says nothing about correctness
    ("f1+f2+f3: SC-OFDM ZP 8-PSK P2 MMSE", 1024, 8, "PSK", "Lin-Phoong_P2", "MMSE", 25.0, "SC", "ZP"),
]


def adaptive_tables(N, h, snr_db, ser=1e-3):
    """Config (d): CAPACITY_BASED bit loading over the water-filling allocation with P_tot = N
    (simulation/models.py:289-395, as Simulation.run computes it): per-subcarrier QAM orders
    from calculate_bit_loading_order, their LUTs and the subcarrier -> LUT table."""
    gains = np.abs(np.fft.fft(h, N)) ** 2
    noise_power = 10 ** (-snr_db / 10)
    alloc = WaterfillingPowerAllocation(N, gains, noise_power).allocate()
    orders = np.array([QAMConstellationMapper.calculate_bit_loading_order(ser=ser, snr=p * g / noise_power)
                       for p, g in zip(alloc, gains)], dtype=np.int64)
    mapper = AdaptiveConstellationMapper(orders, QAMConstellationMapper, N)
    luts, sc = mapper.lut_tables()
    return luts, sc, int(np.sum(mapper.get_bits_per_subcarrier()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--symbols", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated variant name prefixes (e.g. b,d)")
    ap.add_argument("--precision", default="f64", choices=("f64", "f32"))
    args = ap.parse_args()
    only = [o for o in args.only.split(",") if o]
    torch.cuda.set_device(0)
    rows = []
    for name, N, M, scheme, ch, eq, snr, mod, pre in VARIANTS:
        if only and not any(name.split(":")[0] == o for o in only):
            continue
        h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
        cp = len(h) - 1
        sc = None
        if scheme == "ADAPTIVE":
            luts, sc, bps = adaptive_tables(N, h, snr)
            M = 2.0 ** (bps / N)  # mean bits per subcarrier, for the BER denominator
        else:
            luts = [(QAMConstellationMapper(M) if scheme == "QAM" else PSKConstellationMapper(M)).constellation]
        eng = LinkEngine(N, cp, h, EQ[eq], luts, sc, B.OFDM_F64 if args.precision == "f64" else B.OFDM_F32,
                         prefix=B.PREFIX_ZERO if pre == "ZP" else B.PREFIX_CYCLIC,
                         modulator=B.MOD_SC if mod == "SC" else B.MOD_OFDM)
        S = args.symbols if N <= 1024 else args.symbols // (N // 1024)
        eng.run(S, snr, seed=99)  # warm-up (plan, allocator)
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < 0.3:  # clock ramp (bench.py --ramp-seconds)
            eng.run(S, snr, seed=98)
        torch.cuda.synchronize()
        ev = []
        t0 = time.perf_counter()
        pend = [eng.run_async(S, snr, seed=k, events=ev) for k in range(args.steps)]
        bits = sum(p.result().bit_errors for p in pend)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        ms = {}
        for kname, n, e0, e1 in ev:
            ms.setdefault(kname, []).append(e0.elapsed_time(e1))
        row = {"variant": name, "precision": args.precision, "n_fft": N, "order": M, "scheme": scheme, "modulator": mod, "prefix": pre,
               "channel": ch, "equalizer": eq, "snr_db": snr, "symbols_per_step": S,
               "ofdm_symbols_per_s": S / dt,
               "ms_per_1e6_symbols": {k: float(np.mean(v)) * 1e6 / S for k, v in ms.items()},
               "ber": bits / (args.steps * S * N * np.log2(M))}
        rows.append(row)
        print(json.dumps(row), flush=True)
    for r in rows:
        k = r["ms_per_1e6_symbols"]
        print(f"{r['variant']:38s} {r['ofdm_symbols_per_s']:10.3e} sym/s   tx {k['ofdm_tx']:6.2f}  rx {k['ofdm_rx']:6.2f}"
              f" ms/1e6   BER {r['ber']:.2e}", file=sys.stderr)


if __name__ == "__main__":
    main()
