"""Ablation timing of the fused kernels (diagnostic; results are NOT numerically valid).

Each variant sets OFDM_ABLATE_TX / OFDM_ABLATE_RX (bit flags, see ofdm_launch.hpp) and
times ofdm_tx / ofdm_rx with HIP events on the launch stream.

    python tools/ablate.py [--config b|c|e] [--symbols 1000000]

The switches exist only in the ablation build of the library:
    make -C ofdm-based-systems_amd VARIANT=ablate EXTRA=-DOFDM_ABLATION=1
which this script selects (OFDM_LIB_VARIANT=ablate); the product library ignores them.
"""

import argparse
import json
import os
import sys

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

RX = {"full": 0, "no_noise": 1, "no_fft": 2, "no_bits": 4, "no_demap": 8, "no_load": 16,
      "only_fft": 1 | 4 | 8 | 16, "only_noise": 2 | 4 | 8 | 16, "only_bits": 1 | 2 | 8 | 16,
      "only_demap": 1 | 2 | 16, "only_load": 1 | 2 | 4 | 8, "nothing": 31}
TX = {"full": 0, "no_bits": 1, "no_fft": 2, "no_store": 4, "only_fft": 1 | 4, "nothing": 7}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="b")
    ap.add_argument("--symbols", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--precision", default="f32")
    args = ap.parse_args()
    N, M, ch, ratio, eq_name, snr, _ = CONFIGS[args.config]
    h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
    cp = int(ratio * (len(h) - 1))
    eq = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}[eq_name]
    prec = B.OFDM_F32 if args.precision == "f32" else B.OFDM_F64
    eng = LinkEngine(N, cp, h, eq, [QAMConstellationMapper(M).constellation], None, prec)
    eng.run(args.symbols, snr, seed=1)
    res = {}
    for tname, tf in TX.items():
        for rname, rf in RX.items():
            if tname != "full" and rname != "full":
                continue
            os.environ["OFDM_ABLATE_TX"] = str(tf)
            os.environ["OFDM_ABLATE_RX"] = str(rf)
            ev = []
            for r in range(args.reps):
                eng.run(args.symbols, snr, seed=r, events=ev)
            torch.cuda.synchronize()
            t = {}
            for name, n, e0, e1 in ev:
                t.setdefault(name, []).append(e0.elapsed_time(e1))
            res[f"tx:{tname} rx:{rname}"] = {k: float(np.median(v)) for k, v in t.items()}
            print(f"tx:{tname:9s} rx:{rname:11s} " +
                  "  ".join(f"{k}={np.median(v):7.3f} ms" for k, v in t.items()), flush=True)
    os.environ.pop("OFDM_ABLATE_TX")
    os.environ.pop("OFDM_ABLATE_RX")
    print(json.dumps({"config": args.config, "symbols": args.symbols, "ms": res}))


if __name__ == "__main__":
    main()
