"""Add CAPACITY_BASED runs with the PSK base mapper to runs.json.

Run ONLY in the build container, where the reference is importable (see make_golden.py):

    PYTHONPATH=/root/reference/src PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg \\
        python tests/golden/make_golden_adaptive_psk.py

The reference builds its AdaptiveConstellationMapper from whichever base mapper class the
settings name (simulation/models.py:330-373), PSK included, with orders from
PSKConstellationMapper.calculate_bit_loading_order (constellation/models.py:460-474).  Seeded
exactly like make_golden.run_sim; cases tagged "adaptive_psk_*" are replaced on every run, the
rest of runs.json is kept.  Symbol counts are multiples of 8, so every run's bit stream is whole
bytes.
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
        cases = [c for c in json.load(f) if not c["tag"].startswith("adaptive_psk_")]
    new = []

    def add(tag, seed, ch, **kw):
        h = G.channel(ch)
        res = G.run_sim(seed, channel_impulse_response=h, **kw)
        params = {k: (v.value if hasattr(v, "value") else v) for k, v in kw.items()}
        new.append(dict(tag=tag, seed=seed, channel=ch, params=params, result=res))
        print(f"  {tag} seed={seed} snr={kw['snr_db']} orders={sorted(set(res['constellation_order_per_subcarrier']))} "
              f"be={res['bit_errors']} se={res['symbol_errors']} t={res['_ref_seconds']:.1f}s", file=sys.stderr)

    ad = dict(constellation_scheme=G.ConstellationType.PSK, modulator_type=G.ModulationType.OFDM,
              noise_scheme=G.NoiseType.AWGN, power_allocation_type=G.PowerAllocationType.WATERFILLING,
              adaptive_modulation_mode=G.AdaptiveModulationMode.CAPACITY_BASED, prefix_scheme=G.PrefixType.CYCLIC,
              prefix_length_ratio=1.0, constellation_order=16, desired_symbol_error_rate=1e-3)
    MM, ZF = G.EqualizationMethod.MMSE, G.EqualizationMethod.ZF
    for snr in (15.0, 20.0, 25.0):
        add("adaptive_psk_n64_p1_mmse", 1, "Lin-Phoong_P1", num_symbols=200, num_subcarriers=64,
            equalizator_type=MM, snr_db=snr, **ad)
    add("adaptive_psk_n256_severe_zf_uniform", 2, "severe_multipath", num_symbols=40, num_subcarriers=256,
        equalizator_type=ZF, snr_db=24.0, **dict(ad, power_allocation_type=G.PowerAllocationType.UNIFORM))
    add("adaptive_psk_n128_tworay_mmse", 3, "two_ray", num_symbols=48, num_subcarriers=128,
        equalizator_type=MM, snr_db=32.0, **ad)
    # an aggressive loading target (SER 1e-1): hundreds of errors to compare
    add("adaptive_psk_n64_p2_mmse_ser1e-1", 4, "Lin-Phoong_P2", num_symbols=160, num_subcarriers=64,
        equalizator_type=MM, snr_db=20.0, **dict(ad, desired_symbol_error_rate=1e-1))
    with open(path, "w") as f:
        json.dump(cases + new, f, indent=1, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o))


if __name__ == "__main__":
    main()
