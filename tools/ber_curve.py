"""BER curve of a SURVEY config on the GPU, throughput streams vs the reference streams.

For every SNR point of the sweep (config (c): 0..30 dB in 1 dB steps plus 0.25 dB steps over
26..29 dB) this runs

* the throughput path (Philox / MWC64X bits and Box-Muller noise generated in the complex64
  kernels, or complex128 with ``--precision f64``), ``--symbols`` OFDM symbols per point, and
* the reference-stream path (the reference's PCG64 bytes and legacy normals through the
  complex128 kernels -- bit-exact with the reference NumPy code, tests/test_gpu_parity.py),
  ``--ref-symbols`` OFDM symbols per point (host stream generation bounds it),

then reports both curves, the SNR at which each crosses BER = 1e-4 (log-linear
interpolation) and the Delta dB between them (the north-star bar is +-0.05 dB).

    python tools/ber_curve.py --config c > gpurun_out/ber_curve_c.json
    torchrun --nproc-per-node N tools/ber_curve.py ...   # SNR points sharded over N GPUs

Multi-GPU: SNR points are independent, rank r takes points r, r+N, ...; rank 0 gathers.
"""

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-based-systems_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ofdm_based_systems import _backend as B  # noqa: E402
from ofdm_based_systems.constellation.models import QAMConstellationMapper  # noqa: E402
from ofdm_based_systems.engine import LinkEngine  # noqa: E402

CONFIGS = {
    # N, M, channel, eq, SNR grid
    "b": (1024, 64, "flat_fading", "NONE", [float(x) for x in range(0, 31)] + [23.5, 24.25, 24.5, 24.75, 25.25]),
    "c": (1024, 64, "severe_multipath", "MMSE",
          [float(x) for x in range(0, 31)] + [26 + 0.25 * i for i in range(13) if i % 4]),
    # config (e): 256-QAM, N = 4096, Lin-Phoong P1, MMSE; the 1e-4 crossing is near 38.5 dB
    "e": (4096, 256, "Lin-Phoong_P1", "MMSE",
          [float(x) for x in range(20, 43, 2)] + [37.5, 38.0, 38.5, 39.0, 39.5]),
    # config (d): CAPACITY_BASED loading re-derived at every SNR (orders from water-filling at
    # that SNR, desired SER 1e-3), so BER does not fall monotonically with SNR: per-point
    # comparison (no crossing)
    "d": (2048, 0, "Lin-Phoong_P1", "MMSE", [10.0, 15.0, 20.0, 25.0, 30.0]),
}
EQ = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}


def crossing(snrs, bers, target=1e-4):
    """SNR where the curve crosses `target` (log10 BER linear in dB between grid points)."""
    pts = sorted((s, b) for s, b in zip(snrs, bers) if b > 0)
    for (s0, b0), (s1, b1) in zip(pts[:-1], pts[1:]):
        if b0 >= target > b1:
            l0, l1, lt = math.log10(b0), math.log10(b1), math.log10(target)
            return s0 + (s1 - s0) * (l0 - lt) / (l0 - l1)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c", choices=sorted(CONFIGS))
    ap.add_argument("--symbols", type=int, default=2_000_000, help="throughput-mode OFDM symbols per SNR point")
    ap.add_argument("--ref-symbols", type=int, default=12_000, help="reference-stream OFDM symbols per SNR point")
    ap.add_argument("--precision", default="f32", choices=("f32", "f64"),
                    help="arithmetic of the throughput-mode kernels (complex64 / complex128)")
    ap.add_argument("--grid", default="", help="comma-separated SNR points (dB) instead of the config's grid")
    ap.add_argument("--ref-min-snr", type=float, default=20.0,
                    help="below this SNR the reference-stream path runs --ref-symbols/8 (errors are plentiful)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    PREC = B.OFDM_F32 if args.precision == "f32" else B.OFDM_F64
    N, M, ch, eq, grid = CONFIGS[args.config]
    if args.grid:
        grid = [float(x) for x in args.grid.split(",")]
    grid = sorted(set(grid))
    h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
    cp = len(h) - 1
    scale = max(1, N // 1024)  # equal samples per point at any N
    n_phx, n_ref = args.symbols // scale, max(1, args.ref_symbols // scale)
    lut = None if M == 0 else [QAMConstellationMapper(M).constellation]

    def engines(snr):
        if M == 0:  # adaptive: the plan's orders depend on the SNR (bench.make_engine)
            sys.path.insert(0, ROOT)
            from bench import make_engine

            cfg = (N, M, ch, 1.0, eq, snr, "")
            return make_engine(cfg, args.precision), make_engine(cfg, "f64")
        return (LinkEngine(N, cp, h, EQ[eq], lut, None, PREC),
                LinkEngine(N, cp, h, EQ[eq], lut, None, B.OFDM_F64))

    e32 = e64 = None
    rows = []
    t0 = time.perf_counter()
    for i, snr in enumerate(grid):
        if i % world != rank:
            continue
        if e32 is None or M == 0:
            e32, e64 = engines(snr)
        r = e32.run(n_phx, snr, seed=1000 + i)
        S = n_ref if snr >= args.ref_min_snr else max(1, n_ref // 8)
        bits = np.random.Generator(np.random.PCG64(i)).bytes(math.ceil(S * e64.bps / 8))
        rs = np.random.RandomState(i)
        nr = rs.normal(size=S * (N + cp))
        ni = rs.normal(size=S * (N + cp))
        q = e64.run(S, snr, bits=np.frombuffer(bits, np.uint8), normals=(nr, ni))
        rows.append({"snr_db": snr, "bits_per_ofdm_symbol": e32.bps,
                     "throughput": {"symbols": n_phx, "bit_errors": r.bit_errors,
                                    "ber": r.bit_errors / e32.valid_bits(n_phx)},
                     "reference_streams": {"symbols": S, "bit_errors": q.bit_errors,
                                           "ber": q.bit_errors / e64.valid_bits(S)}})
        print(f"rank {rank}: {snr:6.2f} dB  BER {rows[-1]['throughput']['ber']:.3e} "
              f"(ref streams {rows[-1]['reference_streams']['ber']:.3e})", file=sys.stderr, flush=True)
    if world > 1:
        import torch.distributed as dist

        allrows = [None] * world
        dist.all_gather_object(allrows, rows)
        rows = [x for part in allrows for x in part]
    if rank == 0:
        rows.sort(key=lambda x: x["snr_db"])
        snrs = [x["snr_db"] for x in rows]
        c_phx = crossing(snrs, [x["throughput"]["ber"] for x in rows]) if M else None
        c_ref = crossing(snrs, [x["reference_streams"]["ber"] for x in rows]) if M else None
        for x in rows:  # per point: log10 of the BER ratio and its 1-sigma (Poisson counts)
            et, er = x["throughput"]["bit_errors"], x["reference_streams"]["bit_errors"]
            if et > 0 and er > 0:
                x["log10_ber_ratio"] = math.log10(x["throughput"]["ber"] / x["reference_streams"]["ber"])
                x["log10_ber_ratio_sigma"] = 0.4343 * math.sqrt(1.0 / et + 1.0 / er)
        out = {"config": args.config, "throughput_precision": args.precision, "n_fft": N, "qam_order": M, "channel": ch, "cp": cp, "equalizer": eq,
               "n_gpus": world, "wall_s": time.perf_counter() - t0,
               "ber_1e-4_crossing_db": {"throughput": c_phx, "reference_streams": c_ref},
               "delta_db_at_1e-4": None if c_phx is None or c_ref is None else c_phx - c_ref,
               "bar_db": 0.05, "points": rows}
        print(json.dumps(out), flush=True)
        print(f"BER=1e-4 crossing: throughput {c_phx} dB, reference streams {c_ref} dB, "
              f"Delta {out['delta_db_at_1e-4']}", file=sys.stderr)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
