"""Condense a tools/profile.sh run into committed summaries under profiles/.

    python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> <config> <symbols_per_launch> [f32|f64]
    python tools/pmc_summary.py --counters gpurun_out/ctr_<tag> <tag> <config> <symbols_per_launch> [f32|f64]

The second form condenses a tools/counters.sh run (SQ issue counters, each pass with the kernel's
GRBM_GUI_ACTIVE) into the fraction of the SIMDs' time each fused kernel issues VALU and LDS
instructions, merged into profiles/pmc_summary.json under the same key and build id (read by
bench.py for roofline.issue).

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


SIMDS = 256 * 4  # MI355X: 256 CUs x 4 SIMDs
XCDS = 8         # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS)


def issue_fractions(m: dict) -> dict:
    """Issue fractions of one kernel from its mean counters (quad-cycles, MI355X_MICROARCH.md SQ row):
    the SIMDs' time is GRBM_GUI_ACTIVE / 8 cycles (one XCD's share) / 4 x 1024 SIMDs in quad-cycles;
    SQ_ACTIVE_INST_VALU / _LDS / _ANY summed over the kernel's waves over it are the fractions of every
    SIMD's time spent issuing VALU / LDS / any instruction, SQ_WAVE_CYCLES over it the mean resident
    waves per SIMD.  (Per wave: ACTIVE / WAVE_CYCLES x waves per SIMD, the same number.)"""
    g = m["GRBM_GUI_ACTIVE"]
    quads = SIMDS * g / XCDS / 4.0
    out = {"simd_quad_cycles": quads, "grbm_gui_active": g}
    for name, key in (("valu", "SQ_ACTIVE_INST_VALU"), ("lds", "SQ_ACTIVE_INST_LDS"), ("any", "SQ_ACTIVE_INST_ANY")):
        if key in m:
            out[name] = m[key] / quads
    if "SQ_WAVE_CYCLES" in m:
        out["waves_per_simd"] = m["SQ_WAVE_CYCLES"] / quads
        for name, key in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst_any", "SQ_WAIT_INST_ANY"),
                          ("active_any", "SQ_ACTIVE_INST_ANY")):
            if key in m:
                out[name + "_of_wave_cycles"] = m[key] / m["SQ_WAVE_CYCLES"]
    return out


def counters_main(argv):
    """--counters: per fused kernel, mean counters per launch (GRBM_GUI_ACTIVE per pass, so every
    fraction uses the duration of the pass its SQ counter came from) -> pmc_summary.json[key]['issue']."""
    import collections
    import glob

    global PREC
    src, tag, config, syms = argv[0], argv[1], argv[2], int(float(argv[3]))
    PREC = argv[4] if len(argv) > 4 else "f32"
    key = config if PREC == "f32" else f"{config}_{PREC}"
    per_kernel = {}
    for g in sorted(glob.glob(os.path.join(src, "g*", "*counter_collection.csv"))):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(g)):
            k = kernel_key(r["Kernel_Name"])
            if k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, c in agg.items():
            m = {n: statistics.mean(v) for n, v in c.items()}
            if "GRBM_GUI_ACTIVE" not in m:
                continue
            fr = issue_fractions(m)
            d = per_kernel.setdefault(k, {"per_symbol": {}})
            for n, v in m.items():
                if n.startswith("SQ_INSTS") or n in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"):
                    d["per_symbol"][n] = v / syms
            for n, v in fr.items():
                if n not in ("simd_quad_cycles", "grbm_gui_active"):
                    d[n] = v
            d.setdefault("grbm_gui_active_per_pass", []).append(m["GRBM_GUI_ACTIVE"])
    prof = os.path.join(ROOT, "profiles")
    pm_path = os.path.join(prof, "pmc_summary.json")
    pm = json.load(open(pm_path)) if os.path.exists(pm_path) else {}
    sys.path.insert(0, os.path.join(ROOT, "ofdm-based-systems_amd"))
    from ofdm_based_systems._backend import build_id

    bid = build_id()
    rec = pm.setdefault(key, {})
    rec["issue"] = {"tag": tag, "build_id": bid, "symbols_per_launch": syms, "kernels": per_kernel,
                    "method": "SQ_ACTIVE_INST_{VALU,LDS,ANY} / (GRBM_GUI_ACTIVE / 8 / 4 x 1024 SIMDs), quad-cycles, "
                              "per rocprofv3 --pmc pass (tools/counters.sh)"}
    with open(pm_path, "w") as f:
        json.dump(pm, f, indent=1)
    with open(os.path.join(prof, f"{tag}_issue.json"), "w") as f:
        json.dump(rec["issue"], f, indent=1)
    print(json.dumps(rec["issue"], indent=1))


def main():
    global PREC
    if sys.argv[1] == "--counters":
        return counters_main(sys.argv[2:])
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

    old = pm.get(key, {})
    pm[key] = {"tag": tag, "symbols_per_launch": syms, "build_id": build_id(),
               "bytes_per_launch": {k: v["total_bytes"] for k, v in per_launch.items()}}
    if "issue" in old:  # the counters of this key (their own build id) are kept
        pm[key]["issue"] = old["issue"]
    summary["build_id"] = pm[key]["build_id"]
    with open(pm_path, "w") as f:
        json.dump(pm, f, indent=1)
    with open(os.path.join(prof, f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
