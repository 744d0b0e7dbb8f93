"""Summarise tools/counters.sh output: per fused kernel, counters per OFDM symbol (one wave
per symbol at N = 1024) and the wave-cycle split (quad-cycles, MI355X_MICROARCH.md SQ row).

    python tools/ctr_report.py gpurun_out/ctr_<tag> [symbols_per_launch] [f32|f64]

Only the fused throughput kernels of the profiled precision are counted (pmc_summary.kernel_key).
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary  # noqa: E402


def main():
    d = sys.argv[1]
    syms = float(sys.argv[2]) if len(sys.argv) > 2 else 1e6
    pmc_summary.PREC = sys.argv[3] if len(sys.argv) > 3 else "f32"
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/g*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            k = {"ofdm_rx": "rx", "ofdm_tx": "tx"}.get(pmc_summary.kernel_key(n))
            if k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in sorted(agg.items()):
        m = {n: sum(v) / len(v) for n, v in c.items()}
        print(f"== {k}")
        for n in sorted(m):
            print(f"  {n:24s} {m[n]:14.4g}   per symbol {m[n] / syms:10.2f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if n in m:
                    print(f"  {n:24s} {100 * m[n] / wc:6.1f} % of wave cycles")


if __name__ == "__main__":
    main()
