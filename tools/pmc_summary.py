"""Condense a tools/profile.sh run into committed summaries under profiles/.

    python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> <config> <symbols_per_launch> [f32|f64]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary),
profiles/<tag>_summary.json and merges the per-launch HBM traffic of the two fused
kernels into profiles/pmc_summary.json (read by bench.py for roofline.traffic).

Traffic correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64-B units of
TCC_EA0_RDREQ and reports half the bytes of a wide coalesced read; it is doubled.
Calibration on these kernels: k_rx at 1e6 symbols reads exactly 8.19 GB of channel
samples and FETCH_SIZE reports 4.0e6 KB, i.e. 0.5x.  WRITE_SIZE is taken as is (k_tx
writes 8.19 GB and WRITE_SIZE reports 8.0e6 KB, 1.0x).
"""

import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


PREC = "f32"


def kernel_key(name: str):
    """The bench's fused throughput kernels in the profiled precision (k_tx<R, LOGN, FB, LT>,
    k_rx<R, LOGN, EQ, FB> with FB > 0); the generic kernel's reference-stream launches of the
    BER check (FB = 0) are not the timed workload."""
    if ("<float" if PREC == "f32" else "<double") not in name or "<" not in name:
        return None
    args = [a.strip() for a in name[name.index("<") + 1:name.index(">")].split(",")]
    if "k_rx" in name and len(args) >= 4 and int(args[3]) > 0:  # k_rx<R, LOGN, EQ, FB, MV>
        return "ofdm_rx"
    if "k_tx" in name and len(args) >= 4 and int(args[2]) > 0:  # k_tx<R, LOGN, FB, LT, ZPW>
        return "ofdm_tx"
    return None


def counters(path, counter):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            k = kernel_key(r["Kernel_Name"])
            if k and r["Counter_Name"] == counter:
                out.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def main():
    global PREC
    src, tag, config, syms = sys.argv[1], sys.argv[2], sys.argv[3], int(float(sys.argv[4]))
    PREC = sys.argv[5] if len(sys.argv) > 5 else "f32"
    key = config if PREC == "f32" else f"{config}_{PREC}"  # bench.py pmc_traffic key
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats_csv = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    durations = {}
    with open(stats_csv) as f:
        for r in csv.DictReader(f):
            k = kernel_key(r["Name"])
            if k:
                durations[k] = {"name": r["Name"], "calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                "percent": float(r["Percentage"])}
    fetch = counters(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    per_launch = {}
    for k in set(fetch) | set(write):
        rd = 2 * fetch.get(k, 0.0) * 1024
        wr = write.get(k, 0.0) * 1024
        per_launch[k] = {"read_bytes": rd, "write_bytes": wr, "total_bytes": rd + wr,
                         "raw_FETCH_SIZE_KB": fetch.get(k), "raw_WRITE_SIZE_KB": write.get(k)}
    summary = {"tag": tag, "config": config, "precision": PREC, "symbols_per_launch": syms, "kernels": durations,
               "hbm_per_launch": per_launch,
               "correction": "read_bytes = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write_bytes = WRITE_SIZE x 1024"}
    pm_path = os.path.join(prof, "pmc_summary.json")
    pm = json.load(open(pm_path)) if os.path.exists(pm_path) else {}
    sys.path.insert(0, os.path.join(ROOT, "ofdm-based-systems_amd"))
    from ofdm_based_systems._backend import build_id

    pm[key] = {"tag": tag, "symbols_per_launch": syms, "build_id": build_id(),
               "bytes_per_launch": {k: v["total_bytes"] for k, v in per_launch.items()}}
    summary["build_id"] = pm[key]["build_id"]
    with open(pm_path, "w") as f:
        json.dump(pm, f, indent=1)
    with open(os.path.join(prof, f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
