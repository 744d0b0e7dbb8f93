"""Fused GPU hot path vs the reference: seeded Simulation.run results must equal the
reference's (tests/golden/runs.json) -- integer counts bit-exact, PAPR to 1e-9."""

import math

import numpy as np
import pytest
from conftest import channel, load_runs, load_stages, stage_arrays
from numpy.random import PCG64, Generator

import ofdm_oracle as O
import ofdm_based_systems.bits_generation.models as bg
from ofdm_based_systems import _backend as B
from ofdm_based_systems.configuration.enums import (
    AdaptiveModulationMode,
    ConstellationType,
    EqualizationMethod,
    ModulationType,
    NoiseType,
    PowerAllocationType,
    PrefixType,
)
from ofdm_based_systems.engine import LinkEngine
from ofdm_based_systems.simulation.models import Simulation

pytestmark = pytest.mark.gpu

ENUMS = {
    "constellation_scheme": ConstellationType, "modulator_type": ModulationType, "prefix_scheme": PrefixType,
    "equalizator_type": EqualizationMethod, "noise_scheme": NoiseType,
    "power_allocation_type": PowerAllocationType, "adaptive_modulation_mode": AdaptiveModulationMode,
}


def seeded_run(case, **extra):
    """The reference's seeding recipe applied to this package."""
    seed = case["seed"]
    bg.RandomBitsGenerator.__init__.__defaults__ = (Generator(PCG64(seed)),)
    bg.AdaptiveBitsGenerator.__init__.__defaults__ = (Generator(PCG64(seed)),)
    np.random.seed(seed)
    kw = {}
    for k, v in case["params"].items():
        if k in ENUMS:
            v = ENUMS[k]("SC-OFDM" if v == "SC_OFDM" else v)
        kw[k] = v
    ch = case["channel"]
    h = None if ch is None else channel(ch)
    return Simulation(verbose=False, channel_impulse_response=h, make_plot=False, **kw, **extra).run()


def _id(c):
    return f"{c['tag']}-s{c['seed']}-{c['params']['snr_db']}"


@pytest.mark.parametrize("case", load_runs(), ids=_id)
def test_simulation_run_matches_reference(gpu, case):
    r = case["result"]
    got = seeded_run(case)
    assert got["bit_errors"] == r["bit_errors"]
    assert got["symbol_errors"] == r["symbol_errors"]
    assert got["total_bits"] == r["total_bits"]
    assert math.isclose(got["papr_db"], r["papr_db"], rel_tol=1e-9)
    assert got["constellation_order_per_subcarrier"] == r["constellation_order_per_subcarrier"]
    np.testing.assert_allclose(got["allocated_power"], r["allocated_power"], rtol=1e-12, atol=1e-300)
    if r["water_level"] is None:
        assert got["water_level"] is None
    else:
        assert math.isclose(got["water_level"], r["water_level"], rel_tol=1e-9)
    for key in ("title", "subtitle", "prefix_acronym", "power_allocation_acronym", "num_subcarriers",
                "constellation_scheme", "modulator_type", "equalizator_type"):
        assert got[key] == r[key], key
    assert set(r) - {"_ref_seconds", "_received_symbols_len"} <= set(got)


@pytest.mark.parametrize("case", [c for c in load_runs() if c["tag"] in
                                  ("n1024_m64_p1_mmse_20", "cfg_c_n1024_m64_severe_mmse", "n64_m16_p1_mmse_15")],
                         ids=_id)
def test_f32_hot_path_tracks_reference(gpu, case):
    """complex64 arithmetic with the reference's streams: counts within 0.2 % (decision flips
    only at near-ties)."""
    r = case["result"]
    got = seeded_run(case, precision="f32")
    assert abs(got["bit_errors"] - r["bit_errors"]) <= max(2, 2e-3 * r["bit_errors"])
    assert abs(got["symbol_errors"] - r["symbol_errors"]) <= max(2, 2e-3 * r["symbol_errors"])
    assert math.isclose(got["papr_db"], r["papr_db"], rel_tol=1e-5)


@pytest.mark.parametrize("st", load_stages(), ids=lambda s: s["name"])
def test_fused_engine_stage_parity(gpu, st):
    """ofdm_tx/ofdm_rx on the stage fixtures: counts, received symbols, PAPR."""
    a = stage_arrays(st["name"])
    N, M, cp = st["N"], st["M"], st["cp"]
    eq = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}[st["eq"]]
    eng = LinkEngine(N, cp, a["h_raw"], eq, [O.qam_lut(M)])
    S = st["S"]
    res = eng.run(S, st["snr_db"], bits=a["tx_bytes"], normals=(a["noise_re"], a["noise_im"]), keep_symbols=S)
    assert res.bit_errors == st["bit_errors"]
    assert res.symbol_errors == st["symbol_errors"]
    assert math.isclose(res.papr_db, st["papr_db"], rel_tol=1e-12)
    np.testing.assert_allclose(res.received, a["Z"].ravel(), rtol=1e-9, atol=1e-9)
    assert math.isclose(res.power_sum, float(np.sum(np.abs(a["y_clean"]) ** 2)), rel_tol=1e-12)


@pytest.mark.parametrize("batch", [1, 3, 7])
def test_batched_power_pass_is_identical(gpu, batch):
    """Forcing the two-pass (power pass + per-batch TX/RX) schedule changes nothing."""
    case = next(c for c in load_runs() if c["tag"] == "n1024_m64_p1_mmse_20" and c["seed"] == 1)
    r = case["result"]
    got = seeded_run(case, batch_symbols=batch)
    assert (got["bit_errors"], got["symbol_errors"]) == (r["bit_errors"], r["symbol_errors"])
    assert math.isclose(got["papr_db"], r["papr_db"], rel_tol=1e-9)


def test_settings_json_entry_point(gpu, tmp_path, monkeypatch):
    """SimulationSettings.from_json -> create_from_simulation_settings -> run, from a cwd
    holding config/ (simulation/models.py:175-177)."""
    import os

    from conftest import ROOT
    from ofdm_based_systems.configuration.models import SimulationSettings

    monkeypatch.chdir(ROOT)
    st = SimulationSettings.from_json(os.path.join("config", "simulation_settings_test.json"))
    sims = Simulation.create_from_simulation_settings(st)
    exp = {c["params"]["snr_db"]: c["result"] for c in load_runs()
           if c["tag"] == "settings_test_json" and c["seed"] == 0}
    for sim in sims:
        bg.RandomBitsGenerator.__init__.__defaults__ = (Generator(PCG64(0)),)
        np.random.seed(0)
        sim.verbose = False
        out = sim.run()
        assert out["bit_errors"] == exp[sim.snr_db]["bit_errors"]
        assert out["constellation_plot"] is not None
