"""Does running independent bench steps on several HIP streams overlap the write-bound TX
of step k+1 with the issue-bound RX of step k?  Config (b), wall time per 1e6 symbols.

    python tools/overlap_probe.py > gpurun_out/overlap.json
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-based-systems_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    torch.cuda.set_device(0)
    from ofdm_based_systems import _backend as B
    from ofdm_based_systems.constellation.models import QAMConstellationMapper
    from ofdm_based_systems.engine import LinkEngine

    h = np.array([1.0 + 0j])
    eng = LinkEngine(1024, 0, h, B.EQ_NONE, [QAMConstellationMapper(64).constellation], None, B.OFDM_F32)
    out = {}
    for n_streams in (1, 2, 3):
        for per in (1_000_000, 500_000):
            streams = [torch.cuda.Stream() for _ in range(n_streams)]
            steps = max(6, 12 * 1_000_000 // per)

            def go(k0):
                pend = []
                for k in range(steps):
                    with torch.cuda.stream(streams[k % n_streams]):
                        pend.append(eng.run_async(per, 24.0, seed=k0 + k))
                errs = 0
                for p in pend:
                    errs += p.result().bit_errors
                torch.cuda.synchronize()
                return errs

            go(1000)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            errs = go(0)
            dt = time.perf_counter() - t0
            key = f"streams{n_streams}_per{per}"
            out[key] = {"symbols_per_s": steps * per / dt, "ms_per_1e6": dt / (steps * per) * 1e9,
                        "ber": errs / (steps * per * 1024 * 6)}
            print(key, out[key], file=sys.stderr, flush=True)
            del streams
            torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
