"""Add the round-6 reference runs to runs.json: config (d) at its own size with enough errors to
pin the N = 2048 CAPACITY_BASED decode, and config (c) at its bench SNR (the BER 1e-4 crossing).

Run ONLY in the build container, where the reference is importable (see make_golden.py):

    PYTHONPATH=/root/reference/src PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg \\
        python tests/golden/make_golden_r06.py

Seeded exactly like make_golden.run_sim; cases tagged "r06_*" are replaced on every run, the rest
of runs.json is kept.  The adaptive symbol counts are multiples of 8 (whole-byte bit streams).
"""

from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden as G  # noqa: E402  (imports the reference)


def main() -> None:
    path = os.path.join(G.OUT, "runs.json")
    with open(path) as f:
        cases = [c for c in json.load(f) if not c["tag"].startswith("r06_")]
    new = []

    def add(tag, seed, ch, **kw):
        h = G.channel(ch)
        res = G.run_sim(seed, channel_impulse_response=h, **kw)
        params = {k: (v.value if hasattr(v, "value") else v) for k, v in kw.items()}
        new.append(dict(tag=tag, seed=seed, channel=ch, params=params, result=res))
        print(f"  {tag} seed={seed} snr={kw['snr_db']} be={res['bit_errors']} se={res['symbol_errors']} "
              f"bits={res['total_bits']} t={res['_ref_seconds']:.1f}s", file=sys.stderr, flush=True)

    base = dict(constellation_scheme=G.ConstellationType.QAM, modulator_type=G.ModulationType.OFDM,
                noise_scheme=G.NoiseType.AWGN, power_allocation_type=G.PowerAllocationType.UNIFORM,
                adaptive_modulation_mode=G.AdaptiveModulationMode.FIXED)
    ad = dict(base, power_allocation_type=G.PowerAllocationType.WATERFILLING,
              adaptive_modulation_mode=G.AdaptiveModulationMode.CAPACITY_BASED)
    MM = G.EqualizationMethod.MMSE
    # config (d) as BASELINE names it: N = 2048, Lin-Phoong P1, MMSE, water-filling + CAPACITY_BASED
    # loading at SER 1e-3, at the sweep's SNRs (config/simulation_settings_adaptive.json: 15/20/25 dB)
    for seed, snr, nsym in ((11, 20.0, 320), (12, 15.0, 240), (13, 25.0, 240)):
        add("r06_cfg_d_n2048_adaptive", seed, "Lin-Phoong_P1", num_symbols=nsym, num_subcarriers=2048,
            constellation_order=16, prefix_scheme=G.PrefixType.CYCLIC, prefix_length_ratio=1.0,
            equalizator_type=MM, snr_db=snr, desired_symbol_error_rate=1e-3, **ad)
    # config (c) at the bench SNR 27.75 dB (its BER 1e-4 crossing): 400 OFDM symbols, ~2.5e6 bits
    add("r06_cfg_c_n1024_m64_severe_mmse_2775", 21, "severe_multipath", num_symbols=1024 * 400,
        num_subcarriers=1024, constellation_order=64, prefix_scheme=G.PrefixType.CYCLIC,
        prefix_length_ratio=1.0, equalizator_type=MM, snr_db=27.75, **base)
    with open(path, "w") as f:
        json.dump(cases + new, f, indent=1, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o))


if __name__ == "__main__":
    main()
