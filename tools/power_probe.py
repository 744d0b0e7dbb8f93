"""Steady-state clock, package power and kernel times of the bench path and of its ablations
(diagnostic: ablated runs are NOT numerically valid; OFDM_ABLATE_TX / _RX bit flags, see
ofdm_launch.hpp).  Each variant runs back-to-back steps for --seconds while rocm-smi is
sampled; the first 0.5 s (clock ramp) is not sampled.

    python tools/power_probe.py [--config b] [--precision f64] [--seconds 3] [--only full,rx_only,...]

The switches exist only in the ablation build of the library:
    make -C ofdm-based-systems_amd VARIANT=ablate EXTRA=-DOFDM_ABLATION=1
which this script selects (OFDM_LIB_VARIANT=ablate); the product library ignores them.
"""

import argparse
import json
import os
import re
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-based-systems_amd"))
sys.path.insert(0, ROOT)

os.environ.setdefault("OFDM_LIB_VARIANT", "ablate")  # before the library loads

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from ofdm_based_systems import _backend as B  # noqa: E402
from ofdm_based_systems.constellation.models import QAMConstellationMapper  # noqa: E402
from ofdm_based_systems.engine import LinkEngine  # noqa: E402

# name: (TX flags, RX flags); TX 1 no bits, 2 no FFT, 4 no store; RX 1 no noise, 2 no FFT,
# 4 no bits, 8 no demap, 16 no load
VARIANTS = {
    "full": (0, 0),
    "tx_only": (0, 31),
    "rx_only": (7, 0),
    "hbm_only": (1 | 2, 1 | 2 | 4 | 8),       # map + store / load only
    "compute_only": (4, 16),                  # no y store, no y load
    "rx_no_noise": (0, 1),
    "rx_no_fft": (0, 2),
}


def smi_sample():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks", "--showpower"], capture_output=True, text=True,
                             timeout=20).stdout
    except Exception:
        return None
    m = re.search(r"sclk clock level: \S+ \((\d+)Mhz\)", out)
    p = re.search(r"Package Power \(W\): ([\d.]+)", out)
    return (int(m.group(1)) if m else None, float(p.group(1)) if p else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="b")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--symbols", type=int, default=1_000_000)
    ap.add_argument("--only", default="")
    ap.add_argument("--precision", default="f32", choices=("f32", "f64"))
    args = ap.parse_args()
    N, M, ch, ratio, eq_name, snr, _ = CONFIGS[args.config]
    h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
    cp = int(ratio * (len(h) - 1))
    eq = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}[eq_name]
    eng = LinkEngine(N, cp, h, eq, [QAMConstellationMapper(M).constellation], None,
                     B.OFDM_F64 if args.precision == "f64" else B.OFDM_F32)
    eng.run(1000, snr, seed=1)
    names = [n for n in VARIANTS if not args.only or n in args.only.split(",")]
    res = {}
    for name in names:
        tf, rf = VARIANTS[name]
        os.environ["OFDM_ABLATE_TX"] = str(tf)
        os.environ["OFDM_ABLATE_RX"] = str(rf)
        samples, stop = [], threading.Event()

        def sampler():
            time.sleep(0.5)
            while not stop.is_set():
                s = smi_sample()
                if s:
                    samples.append(s)
                time.sleep(0.2)

        th = threading.Thread(target=sampler)
        th.start()
        t0 = time.perf_counter()
        events, k = [], 0
        while time.perf_counter() - t0 < args.seconds:
            pend = [eng.run_async(args.symbols, snr, seed=k + j, events=events) for j in range(20)]
            for p in pend:
                p.result()
            k += 20
            if len(events) > 400:
                events = events[-200:]
        stop.set()
        th.join()
        torch.cuda.synchronize()
        per = {}
        for nm, n, e0, e1 in events[-100:]:
            per.setdefault(nm, []).append(e0.elapsed_time(e1))
        sclk = [s[0] for s in samples if s[0]]
        pw = [s[1] for s in samples if s[1]]
        res[name] = {"tx_rx_flags": [tf, rf], "kernel_ms": {k2: round(float(np.median(v)), 4) for k2, v in per.items()},
                     "sclk_mhz": round(float(np.mean(sclk)), 1) if sclk else None,
                     "power_w": round(float(np.mean(pw)), 1) if pw else None, "smi_samples": len(samples)}
        print(name, json.dumps(res[name]), flush=True)
    os.environ.pop("OFDM_ABLATE_TX")
    os.environ.pop("OFDM_ABLATE_RX")
    print(json.dumps({"config": args.config, "precision": args.precision, "symbols": args.symbols, "variants": res}))


if __name__ == "__main__":
    main()
