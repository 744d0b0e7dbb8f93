"""The benched throughput kernels on the reference's own streams.

The bench times the complex128 throughput kernels (k_tx / k_rx specialised on 64-QAM at N = 1024
for configs b and c, 256-QAM at N = 4096 for config e), which generate their bits and noise on the
device; the reference's seeded runs (tests/golden/runs.json) pin them only through the oracle's
restatement of those streams.  Here the reference's PCG64 bytes and legacy normals go through the
REF instantiations of the same kernels -- the same template body with the bit source (ref_lane:
the caller's bytes in the lane-block layout) and the noise source (the caller's normals) swapped,
selected by the launcher for caller bits on these shapes (ofdm_kernels_inst.hpp ref_shape) -- and
the integer bit / symbol error counts must equal the reference's Simulation.run counts exactly
(simulation/models.py:289-395 and :596-606; noise/models.py:13-22).

(A received-symbol tap -- Simulation's keep_symbols -- sends the receiver to the generic kernel,
so these runs ask for none; the transmitter takes the REF kernel either way.)
"""

import math

import numpy as np
import pytest
from conftest import channel, load_runs

import ofdm_oracle as O
from ofdm_based_systems import _backend as B
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
