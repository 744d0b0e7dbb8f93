"""The benched throughput kernels on the reference's own streams.

The bench times the complex128 throughput kernels (k_tx / k_rx specialised on 64-QAM at N = 1024
for configs b and c, adaptive square-QAM loading at N = 2048 for config d, 256-QAM at N = 4096 for
config e), which generate their bits and noise on the device; the reference's seeded runs (tests/golden/runs.json) pin them only through the oracle's
restatement of those streams.  Here the reference's PCG64 bytes and legacy normals go through the
REF instantiations of the same kernels -- the same template body with the bit source (ref_lane:
the caller's bytes in the lane-block layout; adaptive: ref_lane_adaptive, each subcarrier's b_k bits
at its offset in the symbol's subcarrier-major bit stream) and the noise source (the caller's
normals) swapped,
selected by the launcher for caller bits on these shapes (ofdm_kernels_inst.hpp ref_shape) -- and
the integer bit / symbol error counts must equal the reference's Simulation.run counts exactly
(simulation/models.py:289-395 and :596-606; noise/models.py:13-22; constellation/adaptive.py:130-265).

(A received-symbol tap -- Simulation's keep_symbols -- sends the receiver to the generic kernel,
so these runs ask for none; the transmitter takes the REF kernel either way.)
"""

import math

import numpy as np
import pytest
from conftest import channel, load_runs

import ofdm_oracle as O
from ofdm_based_systems import _backend as B
from ofdm_based_systems.constellation.adaptive import AdaptiveConstellationMapper
from ofdm_based_systems.constellation.models import QAMConstellationMapper
from ofdm_based_systems.engine import LinkEngine

pytestmark = pytest.mark.gpu

EQ = {"NONE": B.EQ_NONE, "ZF": B.EQ_ZF, "MMSE": B.EQ_MMSE}


def _ref_shape_cases():
    out = []
    for c in load_runs():
        p = c["params"]
        if (p.get("adaptive_modulation_mode", "FIXED") == "FIXED" and p["modulator_type"] == "OFDM"
                and p["prefix_scheme"] == "CYCLIC" and p["constellation_scheme"] == "QAM"
                and p.get("num_symbols") and p["noise_scheme"] == "AWGN"
                and (p["num_subcarriers"], p["constellation_order"]) in ((1024, 64), (4096, 256))):
            out.append(c)
    return out


CASES = _ref_shape_cases()


def test_cases_cover_the_bench_shapes():
    tags = {c["tag"] for c in CASES}
    # config (b) and (c) at fixture scale, config (c) at its bench SNR, config (e)'s 256-QAM
    assert {"cfg_b_n1024_m64_flat_none_24", "cfg_c_n1024_m64_severe_mmse", "r06_cfg_c_n1024_m64_severe_mmse_2775",
            "cfg_e_n4096_m256_p1_wf", "n1024_m64_flat_none_18", "n1024_m64_p1_mmse_20"} <= tags, tags


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['tag']}-s{c['seed']}-{c['params']['snr_db']}")
def test_reference_streams_through_the_benched_kernels(gpu, case):
    p, r = case["params"], case["result"]
    h = channel(case["channel"])
    N, M = p["num_subcarriers"], p["constellation_order"]
    b = int(math.log2(M))
    S = p["num_symbols"] // N
    cp = O.prefix_length(h, p["prefix_length_ratio"], "CP")
    tx, nz = O.reference_streams(case["seed"], S * N * b, S * (N + cp))
    eng = LinkEngine(N, cp, h, EQ[p["equalizator_type"]], [O.qam_lut(M)], None, B.OFDM_F64)
    res = eng.run(S, p["snr_db"], bits=np.frombuffer(tx, np.uint8), normals=nz)
    print(f"{case['tag']} seed {case['seed']} {p['snr_db']} dB: bits {res.bit_errors} (reference {r['bit_errors']}), "
          f"symbols {res.symbol_errors} (reference {r['symbol_errors']})")
    assert r["bit_errors"] > 0 or p["snr_db"] >= 30.0
    assert (res.bit_errors, res.symbol_errors) == (r["bit_errors"], r["symbol_errors"])
    assert math.isclose(res.papr_db, r["papr_db"], rel_tol=1e-9)
    # the same run in two batches (power pass, then TX + RX per batch): the same counts
    res2 = eng.run(S, p["snr_db"], bits=np.frombuffer(tx, np.uint8), normals=nz, batch=max(1, S // 2 + 1))
    assert (res2.bit_errors, res2.symbol_errors) == (r["bit_errors"], r["symbol_errors"])


def _adaptive_cases():
    # CAPACITY_BASED square-QAM loading at config (d)'s N = 2048, OFDM with a cyclic prefix
    return [c for c in load_runs()
            if c["params"].get("adaptive_modulation_mode") == "CAPACITY_BASED" and c["params"]["num_subcarriers"] == 2048
            and c["params"]["constellation_scheme"] == "QAM" and c["params"]["modulator_type"] == "OFDM"
            and c["params"]["prefix_scheme"] == "CYCLIC" and c["params"]["noise_scheme"] == "AWGN"]


ADAPTIVE = _adaptive_cases()


def test_adaptive_cases_cover_config_d():
    assert {(c["tag"], c["params"]["snr_db"]) for c in ADAPTIVE} >= {
        ("r06_cfg_d_n2048_adaptive", 15.0), ("r06_cfg_d_n2048_adaptive", 20.0), ("r06_cfg_d_n2048_adaptive", 25.0)}


@pytest.mark.parametrize("case", ADAPTIVE, ids=lambda c: f"{c['tag']}-s{c['seed']}-{c['params']['snr_db']}")
def test_reference_streams_through_the_benched_adaptive_kernels(gpu, case):
    """Config (d): the reference's per-subcarrier orders (water-filling at the run's SNR), its PCG64
    bytes laid out subcarrier-major per OFDM symbol and its legacy normals through the adaptive
    kernels' REF instantiations (k_tx / k_rx FB = 1 at N = 2048): the reference's counts exactly."""
    p, r = case["params"], case["result"]
    h = channel(case["channel"])
    N = p["num_subcarriers"]
    orders, _, _ = O.adaptive_orders(N, h, p["snr_db"], p.get("desired_symbol_error_rate", 1e-3),
                                     p["power_allocation_type"] == "WATERFILLING", "QAM")
    assert orders.tolist() == r["constellation_order_per_subcarrier"]
    assert max(orders) <= 256  # the adaptive kernels' orders (the plan's upat)
    bps = sum(int(np.log2(o)) for o in orders if o > 0)
    S = p["num_symbols"]
    cp = O.prefix_length(h, p["prefix_length_ratio"], "CP")
    tx, nz = O.reference_streams(case["seed"], bps * S, S * (N + cp))
    luts, sc = AdaptiveConstellationMapper(orders, QAMConstellationMapper, N).lut_tables()
    eng = LinkEngine(N, cp, h, EQ[p["equalizator_type"]], luts, sc, B.OFDM_F64)
    assert eng.adaptive and eng.bps == bps
    res = eng.run(S, p["snr_db"], bits=np.frombuffer(tx, np.uint8), normals=nz)
    print(f"{case['tag']} seed {case['seed']} {p['snr_db']} dB: bits {res.bit_errors} (reference {r['bit_errors']}), "
          f"symbols {res.symbol_errors} (reference {r['symbol_errors']})")
    assert r["bit_errors"] > 0
    assert (res.bit_errors, res.symbol_errors) == (r["bit_errors"], r["symbol_errors"])
    assert math.isclose(res.papr_db, r["papr_db"], rel_tol=1e-9)
    res2 = eng.run(S, p["snr_db"], bits=np.frombuffer(tx, np.uint8), normals=nz, batch=max(1, S // 2 + 1))
    assert (res2.bit_errors, res2.symbol_errors) == (r["bit_errors"], r["symbol_errors"])
