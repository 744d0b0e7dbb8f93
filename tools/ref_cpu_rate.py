"""The literal reference's CPU rate per bench config, from the timings the golden generators took.

tests/golden/make_golden*.py ran the reference's own Simulation.run (pure Python + NumPy, one
process) in the build container for every seeded run and kept its wall time (`_ref_seconds`,
Simulation.run alone).  The GPU box has no copy of the reference, so bench.py cannot time it
there; this writes the container's measurement, per bench config, to
profiles/literal_reference_cpu.json, which bench.py puts beside its own CPU baseline (the NumPy
oracle port, timed on the box) as cpu_baseline.literal_reference.

    python tools/ref_cpu_rate.py
"""

import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# bench config -> golden run tags of the same shape (N, constellation, channel, equaliser)
SHAPES = {
    "b": ["cfg_b_n1024_m64_flat_none_24", "n1024_m64_flat_none_18"],
    "c": ["cfg_c_n1024_m64_severe_mmse", "r06_cfg_c_n1024_m64_severe_mmse_2775"],
    "d": ["r06_cfg_d_n2048_adaptive"],
    "e": ["cfg_e_n4096_m256_p1_wf"],
}


def main():
    with open(os.path.join(ROOT, "tests", "golden", "runs.json")) as f:
        runs = json.load(f)
    out = {}
    for cfg, tags in SHAPES.items():
        syms = secs = 0.0
        used = []
        for c in runs:
            if c["tag"] not in tags:
                continue
            p = c["params"]
            n = p["num_symbols"] if p.get("adaptive_modulation_mode") == "CAPACITY_BASED" else \
                p["num_symbols"] // p["num_subcarriers"]
            syms += n
            secs += c["result"]["_ref_seconds"]
            used.append(f"{c['tag']} seed {c['seed']} {p['snr_db']} dB: {n} OFDM symbols in "
                        f"{c['result']['_ref_seconds']:.2f} s")
        out[cfg] = {"per_core_symbols_per_s": syms / secs, "cores": 1, "kind": "reference",
                    "runs": used,
                    "measured": "the reference's Simulation.run (/root/reference/src, pure Python + NumPy, one "
                                "process) in the build container by tests/golden/make_golden*.py; wall time of "
                                "run() alone; not re-timed on the GPU box, which holds no copy of the reference"}
    path = os.path.join(ROOT, "profiles", "literal_reference_cpu.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: round(v["per_core_symbols_per_s"], 1) for k, v in out.items()}))


if __name__ == "__main__":
    main()
