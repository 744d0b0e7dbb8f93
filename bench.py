"""Headline benchmark: OFDM symbols/s through the fused GPU modem path.

Metric (BASELINE.json): OFDM symbols/sec at N_FFT=1024, 64-QAM.  Workload =
BASELINE config (b): N_FFT=1024, 64-QAM, flat channel (flat_fading.npy, cp=0),
no equaliser, AWGN at 24 dB (BER ~1e-4), complex64 arithmetic, Philox bits and
noise generated on the device.  One step = one complete Simulation-run of the hot
path over `--symbols` OFDM symbols per GPU (TX kernel, power all-reduce, RX
kernel, counter all-reduce, results on the host).  Default 10 steps x 1e6
symbols = the "1e7 symbols at one SNR" of config (b).  After the timed region rank 0
also reports the BER Delta dB of the run against the reference-stream path (the second
half of the BASELINE metric).

Multi-GPU (torchrun): each rank simulates its contiguous share of the global
symbol range of every step (weak scaling); exchanges: one all-reduce of the
AWGN power statistics and one of the error counters per step (RCCL).
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ofdm-based-systems_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

CONFIGS = {
    # name: (N, M, channel, ratio, eq, snr_db, description)
    "b": (1024, 64, "flat_fading", 1.0, "NONE", 24.0,
          "config (b): N_FFT=1024, 64-QAM, flat channel (flat_fading.npy, cp=0), no equaliser, AWGN 24 dB"),
    "c": (1024, 64, "severe_multipath", 1.0, "MMSE", 27.75,
          "config (c): N_FFT=1024, 64-QAM, severe_multipath.npy (8 taps, cp=7), MMSE, AWGN 27.75 dB"),
    # M = 0: CAPACITY_BASED adaptive bit loading (per-subcarrier square-QAM orders from the
    # water-filling allocation at the SNR, simulation/models.py:289-395)
    "d": (2048, 0, "Lin-Phoong_P1", 1.0, "MMSE", 20.0,
          "config (d): N_FFT=2048, adaptive bit loading (water-filling, desired SER 1e-3), Lin-Phoong_P1.npy "
          "(4 taps, cp=3), MMSE, AWGN 20 dB"),
    "e": (4096, 256, "Lin-Phoong_P1", 1.0, "MMSE", 30.0,
          "config (e): N_FFT=4096, 256-QAM, Lin-Phoong_P1.npy (4 taps, cp=3), MMSE, AWGN 30 dB"),
}


def make_engine(cfg, precision):
    """LinkEngine of a bench config; the constellation tables as Simulation builds them
    (QAMConstellationMapper, or the adaptive mapper over the water-filling orders)."""
    from ofdm_based_systems import _backend as B
    from ofdm_based_systems.constellation.adaptive import AdaptiveConstellationMapper
    from ofdm_based_systems.constellation.models import QAMConstellationMapper
    from ofdm_based_systems.engine import LinkEngine
    from ofdm_based_systems.power_allocation.models import WaterfillingPowerAllocation

    N, M, ch, ratio, eq_name, snr, _ = cfg
    h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
    cp = int(ratio * (len(h) - 1))
    eq = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}[eq_name]
    sc = None
    if M == 0:
        gains = np.abs(np.fft.fft(h, N)) ** 2
        noise_power = 10 ** (-snr / 10)
        alloc = WaterfillingPowerAllocation(N, gains, noise_power).allocate()
        orders = np.array([QAMConstellationMapper.calculate_bit_loading_order(ser=1e-3, snr=p * g / noise_power)
                           for p, g in zip(alloc, gains)], dtype=np.int64)
        luts, sc = AdaptiveConstellationMapper(orders, QAMConstellationMapper, N).lut_tables()
    else:
        luts = [QAMConstellationMapper(M).constellation]
    return LinkEngine(N, cp, h, eq, luts, sc, precision), h, cp
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def kernel_bytes_per_symbol(N: int, bps: int, cp: int) -> int:
    """Algorithmic bytes one OFDM symbol moves in ONE of the two kernels:
    B_alg = 2*ceil(bps/8) + 2*(N+cp)*8 per symbol (bps = N*b, or sum b_k with adaptive loading)
    is split evenly: each kernel touches the tx bits once (map / comparator) and the complex64
    channel stream once (write / read)."""
    return math.ceil(bps / 8) + (N + cp) * 8


def _cpu_worker(args):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ofdm_oracle as O

    seed, S, N, M, ch, cp, eq, snr = args
    h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
    if M == 0:  # CAPACITY_BASED: orders from water-filling, the adaptive data path
        orders, _, _ = O.adaptive_orders(N, h, snr, 1e-3, True)
        bps = int(sum(int(np.log2(o)) for o in orders if o > 0))
        tx, nz = O.reference_streams(seed, S * bps, S * (N + cp))
        t0 = time.perf_counter()
        O.run_adaptive(tx, orders, N, h, cp, eq, snr, nz)
        return S, time.perf_counter() - t0
    b = int(np.log2(M))
    tx, nz = O.reference_streams(seed, S * N * b, S * (N + cp))
    t0 = time.perf_counter()
    O.run_fixed(tx, S * N * b, N, M, h, cp, eq, snr, nz)
    return S, time.perf_counter() - t0


def cpu_baseline(cfg, per_worker: int):
    """The NumPy oracle (a port of the reference path) on the host cores, bounded sample."""
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    N, M, ch, ratio, eq, snr, _ = cfg
    h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
    cp = int(ratio * (len(h) - 1))
    workers = max(1, min(16, os.cpu_count() or 1))
    jobs = [(100 + i, per_worker, N, M, ch, cp, eq, snr) for i in range(workers)]
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        out = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t0
    syms = sum(o[0] for o in out)
    cpu_s = sum(o[1] for o in out)
    return {
        "value": syms / wall, "unit": "OFDM symbols/s", "cores": workers, "kind": "port",
        "sample": f"{workers} processes x {per_worker} OFDM symbols of the same config through the NumPy "
                  f"oracle (reference PCG64 bits + legacy-normal noise; stream generation untimed), "
                  f"{cpu_s:.1f} s of CPU work, {wall:.1f} s wall incl. process start",
        "per_core_symbols_per_s": syms / cpu_s,
    }


def ber_vs_reference(engine64, N, cp, snr, ber_phx, bits_phx, symbols=16000, seed=1):
    """BER Delta dB of the timed throughput run against the reference-stream path at the same SNR.

    The reference-stream path is the drop-in's default mode: the reference's own PCG64 bytes and
    legacy normal draws (real array first, noise/models.py:19-21) through the complex128 kernels,
    bit-exact with the reference NumPy code (tests/test_gpu_parity.py).  Delta dB is the
    horizontal distance between the two BER curves at the throughput run's BER, through the
    reference curve's local slope from a second point 0.5 dB higher; positive = the throughput
    run needs more SNR.  Outside the timed region."""
    def ref_ber(snr_db, sd):
        bits = np.random.Generator(np.random.PCG64(sd)).bytes(math.ceil(symbols * engine64.bps / 8))
        rs = np.random.RandomState(sd)  # = np.random.seed(sd) + np.random.normal (the reference's draws)
        nr = rs.normal(size=symbols * (N + cp))
        ni = rs.normal(size=symbols * (N + cp))
        r = engine64.run(symbols, snr_db, bits=np.frombuffer(bits, np.uint8), normals=(nr, ni))
        return r.bit_errors, engine64.valid_bits(symbols)

    e0, n0 = ref_ber(snr, seed)
    e1, n1 = ref_ber(snr + 0.5, seed + 1)
    if min(e0, e1, ber_phx * bits_phx) <= 0:
        return {"snr_db": snr, "ber": ber_phx, "ber_reference_streams": e0 / n0, "delta_db": None}
    slope = (math.log10(e1 / n1) - math.log10(e0 / n0)) / 0.5  # decades per dB (< 0)
    delta = (math.log10(ber_phx) - math.log10(e0 / n0)) / slope
    sd_db = 0.4343 * math.sqrt(1.0 / e0 + 1.0 / (ber_phx * bits_phx)) / abs(slope)
    return {"snr_db": snr, "ber": ber_phx, "ber_reference_streams": e0 / n0,
            "reference_symbols": symbols, "slope_decades_per_db": slope,
            "delta_db": delta, "delta_db_stderr": sd_db, "bar_db": 0.05}


def pmc_traffic(config_name: str, symbols_per_launch: int):
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3 --pmc summary
    (profiles/pmc_summary.json, produced by tools/pmc_summary.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pm = json.load(f)
    rec = pm.get(config_name)
    if not rec:
        return None
    return {k: v * symbols_per_launch / rec["symbols_per_launch"] for k, v in rec["bytes_per_launch"].items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--symbols", type=int, default=0,
                    help="OFDM symbols per GPU per step (default 1e6 x 1024/N: 8.2 GB of channel samples)")
    ap.add_argument("--config", default="b", choices=sorted(CONFIGS))
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="OFDM symbols per CPU worker (default 1500 x 1024/N)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ber-check", action="store_true", help="skip the BER Delta-dB check vs the reference streams")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--ramp-seconds", type=float, default=0.25,
                    help="untimed warmup beyond --warmup until this much GPU time has passed (clock ramp)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # OFDM_BENCH_DEVICE pins every rank to one device: a multi-rank rehearsal on a 1-GPU box
    # (with --backend gloo; RCCL refuses two ranks on one GPU)
    dev = int(os.environ.get("OFDM_BENCH_DEVICE", local))
    torch.cuda.set_device(dev)
    group = None
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.backend)
        group = dist.group.WORLD

    from ofdm_based_systems import _backend as B

    cfg = CONFIGS[args.config]
    N, M, ch, ratio, eq_name, snr, desc = cfg
    prec = B.OFDM_F32 if args.precision == "f32" else B.OFDM_F64
    engine, h, cp = make_engine(cfg, prec)
    bps = engine.bps  # bits per OFDM symbol
    per_gpu = args.symbols if args.symbols else 1_000_000 // max(1, N // 1024)
    total = per_gpu * world

    def barrier():
        if world > 1:
            import torch.distributed as dist

            dist.barrier()

    for i in range(args.warmup):
        engine.run(total, snr, seed=10_000 + i, group=group)
    torch.cuda.synchronize()
    # Clock ramp: a fresh box idles at ~100-350 MHz and its clock needs ~40 ms of load to reach
    # the steady state the power cap sets (tools/ramp_probe.py, profiles/r02_ramp_b.json), longer
    # than a few warmup steps.  Keep warming up (untimed, outside the K timed steps) until
    # --ramp-seconds of GPU work have run; the extra steps are reported.
    ramp_steps, t_ramp = 0, time.perf_counter()
    while args.ramp_seconds > 0:
        done = torch.tensor([time.perf_counter() - t_ramp >= args.ramp_seconds], dtype=torch.int32, device="cuda")
        if world > 1:
            import torch.distributed as dist

            dist.all_reduce(done, op=dist.ReduceOp.MIN)  # every rank runs the same number of steps
        if int(done.item()):
            break
        engine.run(total, snr, seed=20_000 + ramp_steps, group=group)
        ramp_steps += 1
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    events = []
    bit_errors = 0
    t0 = time.perf_counter()
    # every step is the whole hot path (bits -> ... -> error counts) of one run; the host
    # enqueues all steps (step k+1's TX ahead of step k's RX, so the ranks' statistics
    # exchange overlaps a transmitter) and reads every run's counts back inside the timed region
    pending = engine.run_pipelined(total, snr, range(args.steps), group=group, events=events)
    for p in pending:
        bit_errors += p.result().bit_errors
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel average launch duration from HIP events on the launch stream
    durs = {}
    for name, n, e0, e1 in events:
        durs.setdefault(name, []).append((e0.elapsed_time(e1) * 1e-3, n))
    avg = {k: sum(d for d, _ in v) / len(v) for k, v in durs.items()}
    dom = max(avg, key=avg.get)
    sym_per_launch = durs[dom][0][1]
    alg = kernel_bytes_per_symbol(N, bps, cp) * sym_per_launch
    achieved = alg / avg[dom] / 1e9
    traffic = pmc_traffic(args.config, sym_per_launch)
    value = total * args.steps / elapsed
    out = {
        "metric": "OFDM symbols/sec (1/2/4/8 GPU) at N_FFT=1024 64-QAM; BER ΔdB vs ref",
        "value": value,
        "unit": "OFDM symbols/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "clock_ramp": {"extra_untimed_steps": ramp_steps, "seconds": args.ramp_seconds},
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "c64 (f32)" if prec == B.OFDM_F32 else "c128 (f64)",
        "data": "synthetic: Philox4x32-10 / MWC64X bits and Box-Muller AWGN (64-point phase table) generated "
                "on the GPU per (seed, symbol)",
        "config": {
            "workload": f"{desc}; {per_gpu} OFDM symbols per GPU per step",
            "n_fft": N, "qam_order": M if M else "adaptive", "bits_per_ofdm_symbol": bps, "cp": cp,
            "channel": ch, "equalizer": eq_name, "snr_db": snr,
            "symbols_per_step": total, "parallelism": f"symbol-sharded x{world}",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": None if traffic is None else traffic.get(dom),
            "alg_bytes_per_symbol": kernel_bytes_per_symbol(N, bps, cp),
            "symbols_per_launch": sym_per_launch,
            "avg_launch_ms": {k: v * 1e3 for k, v in avg.items()},
        },
        "path_hbm_fraction": value * 2 * kernel_bytes_per_symbol(N, bps, cp) / (HBM_PEAK_GBS * 1e9 * world),
        "ber": bit_errors / (engine.valid_bits(total) * args.steps),
    }
    if rank == 0 and not args.no_ber_check:
        eng64, _, _ = make_engine(cfg, B.OFDM_F64)
        out["ber_vs_reference"] = ber_vs_reference(eng64, N, cp, snr, out["ber"],
                                                   engine.valid_bits(total) * args.steps,
                                                   symbols=max(2000, 16000 * 1024 // N))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_sample or max(100, 1500 * 1024 // N))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
