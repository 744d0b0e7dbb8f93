"""Clock ramp of the bench from a cold (idle-clocked) GPU: per-step kernel times over the
first steps of a run, HIP events on the launch stream.

    python tools/ramp_probe.py [--config b] [--steps 600]

Prints one JSON line: ms per step (TX + RX) at selected step indices and the running time.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-based-systems_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402
from ofdm_based_systems import _backend as B  # noqa: E402
from ofdm_based_systems.constellation.models import QAMConstellationMapper  # noqa: E402
from ofdm_based_systems.engine import LinkEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="b")
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--symbols", type=int, default=1_000_000)
    ap.add_argument("--idle", type=float, default=2.0, help="seconds idle before the run")
    args = ap.parse_args()
    N, M, ch, ratio, eq_name, snr, _ = CONFIGS[args.config]
    h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
    cp = int(ratio * (len(h) - 1))
    eq = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}[eq_name]
    eng = LinkEngine(N, cp, h, eq, [QAMConstellationMapper(M).constellation], None, B.OFDM_F32)
    eng.run(1000, snr, seed=1)  # plan, workspaces, code objects
    torch.cuda.synchronize()
    time.sleep(args.idle)
    events = []
    t0 = time.perf_counter()
    pending = [eng.run_async(args.symbols, snr, seed=k, events=events) for k in range(args.steps)]
    for p in pending:
        p.result()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    per = {}
    for name, n, e0, e1 in events:
        per.setdefault(name, []).append(e0.elapsed_time(e1))
    steps = np.array(per["ofdm_tx"]) + np.array(per["ofdm_rx"])
    cum = np.cumsum(steps)
    marks = [0, 1, 2, 5, 10, 20, 30, 50, 100, 200, 400, args.steps - 1]
    out = {"config": args.config, "steps": args.steps, "wall_s": wall,
           "step_ms": {str(i): round(float(steps[i]), 4) for i in marks if i < len(steps)},
           "tx_ms": {str(i): round(float(per["ofdm_tx"][i]), 4) for i in marks if i < len(steps)},
           "rx_ms": {str(i): round(float(per["ofdm_rx"][i]), 4) for i in marks if i < len(steps)},
           "cum_kernel_ms": {str(i): round(float(cum[i]), 2) for i in marks if i < len(steps)},
           "mean_first_20": float(steps[:20].mean()), "mean_last_100": float(steps[-100:].mean())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
