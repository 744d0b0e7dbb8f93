"""Pin the CPU oracle (oracle/ofdm_oracle.py) to the reference's own outputs.

Every fixture under tests/golden was produced by running the reference itself
(tests/golden/make_golden.py).  The oracle must reproduce integer counts and
LUTs exactly and floating-point stages to 1e-12.
"""

import math

import numpy as np
import pytest
from conftest import channel, load_runs, load_stages, stage_arrays, GOLDEN

import ofdm_oracle as O


def test_luts_match_reference():
    luts = np.load(f"{GOLDEN}/luts.npz")
    for m in (4, 16, 64, 256):
        assert np.array_equal(O.qam_lut(m), luts[f"qam{m}"])
    for m in (2, 4, 8, 16):
        assert np.array_equal(O.psk_lut(m), luts[f"psk{m}"])


def test_qam_lut_is_separable_and_not_gray_above_16():
    # I from the low b/2 bits, Q = -I pattern from the high bits
    for m in (4, 16, 64, 256):
        lut = O.qam_lut(m)
        side = int(np.sqrt(m))
        h = int(np.log2(m)) // 2
        i_lev = np.array([lut[i].real for i in range(side)])
        for i in range(m):
            assert lut[i].real == i_lev[i & (side - 1)]
            assert lut[i].imag == -i_lev[i >> h]


@pytest.mark.parametrize("st", load_stages(), ids=lambda s: s["name"])
def test_stages_match_reference(st):
    a = stage_arrays(st["name"])
    N, M, cp = st["N"], st["M"], st["cp"]
    b = int(np.log2(M))
    lut = O.qam_lut(M)
    tx = a["tx_bytes"].tobytes()
    idx = O.bits_to_indices(O.bytes_to_bits(tx), b)
    X = lut[idx].reshape(-1, N)
    assert np.array_equal(X, a["X"])
    x = O.modulate(X, cp)
    np.testing.assert_allclose(x, a["x"], rtol=0, atol=1e-12)
    y_clean = O.channel_conv(x.ravel(), a["h_raw"])
    np.testing.assert_allclose(y_clean, a["y_clean"], rtol=0, atol=1e-12)
    y = O.awgn(y_clean, st["snr_db"], a["noise_re"], a["noise_im"])
    np.testing.assert_allclose(y, a["y"], rtol=0, atol=1e-12)
    Z = O.demodulate(a["y"].reshape(-1, N + cp), cp, a["H"], st["eq"], st["snr_db"])
    np.testing.assert_allclose(Z, a["Z"], rtol=1e-9, atol=1e-9)
    rx = O.indices_to_bytes(O.nn_demap(a["Z"].ravel(), lut), b)
    assert rx == a["rx_bytes"].tobytes()
    assert np.isclose(O.papr_db(a["x"]), st["papr_db"], rtol=1e-12)


def _fixed_cases():
    return [c for c in load_runs()
            if c["params"].get("adaptive_modulation_mode", "FIXED") == "FIXED"
            and c["params"]["modulator_type"] == "OFDM"
            and c["params"]["prefix_scheme"] != "ZERO"
            and c["params"]["constellation_scheme"] == "QAM"]


@pytest.mark.parametrize("case", _fixed_cases(), ids=lambda c: f"{c['tag']}-s{c['seed']}-{c['params']['snr_db']}")
def test_fixed_runs_match_reference(case):
    p, r = case["params"], case["result"]
    res = O.run_reference_fixed(
        case["seed"], p.get("num_symbols"), p.get("num_bits"), p["num_subcarriers"], p["constellation_order"],
        channel(case["channel"]), p["prefix_length_ratio"], "NONE" if p["prefix_scheme"] == "NONE" else "CP",
        p["equalizator_type"], p["snr_db"], noise=p["noise_scheme"] == "AWGN")
    assert res.bit_errors == r["bit_errors"]
    assert res.symbol_errors == r["symbol_errors"]
    assert res.total_bits == r["total_bits"]
    assert math.isclose(res.papr_db, r["papr_db"], rel_tol=1e-9)


def _adaptive_cases():
    return [c for c in load_runs() if c["params"].get("adaptive_modulation_mode") == "CAPACITY_BASED"]


@pytest.mark.parametrize("case", _adaptive_cases(), ids=lambda c: f"{c['tag']}-{c['params']['snr_db']}")
def test_adaptive_runs_match_reference(case):
    p, r = case["params"], case["result"]
    h = channel(case["channel"])
    N = p["num_subcarriers"]
    scheme = p.get("constellation_scheme", "QAM")
    orders, power, wl = O.adaptive_orders(N, h, p["snr_db"], p.get("desired_symbol_error_rate", 1e-3),
                                          p["power_allocation_type"] == "WATERFILLING", scheme)
    assert orders.tolist() == r["constellation_order_per_subcarrier"]
    np.testing.assert_array_equal(power, np.array(r["allocated_power"]))
    if wl is not None:
        assert math.isclose(wl, r["water_level"], rel_tol=1e-12)
    bps = sum(int(np.log2(o)) for o in orders if o > 0)
    S = p["num_symbols"]
    cp = O.prefix_length(h, p["prefix_length_ratio"], "CP")
    tx, nz = O.reference_streams(case["seed"], bps * S, S * (N + cp))
    res = O.run_adaptive(tx, orders, N, h, cp, p["equalizator_type"], p["snr_db"], nz, scheme)
    assert (res.bit_errors, res.symbol_errors, res.total_bits) == (
        r["bit_errors"], r["symbol_errors"], r["total_bits"])
    assert math.isclose(res.papr_db, r["papr_db"], rel_tol=1e-9)


def test_power_allocation_matches_reference():
    pa = np.load(f"{GOLDEN}/power_allocation.npz")
    for key in pa.files:
        if not key.startswith("wf_"):
            continue
        ch, n, snr, tot = key[3:].rsplit("_", 3)
        n, snr, tot = int(n[1:]), float(snr[3:]), float(tot[1:])
        g = np.abs(np.fft.fft(channel(ch), n)) ** 2
        np.testing.assert_array_equal(O.waterfilling_allocation(tot, g, 10 ** (-snr / 10)), pa[key])
    np.testing.assert_array_equal(O.uniform_allocation(1.0, 64), pa["uniform_64_1"])


def test_bit_loading_matches_reference():
    import json

    with open(f"{GOLDEN}/bitloading.json") as f:
        bl = json.load(f)
    for ser, vals in bl["orders"].items():
        got = [O.qam_bit_loading_order(float(ser), s) for s in bl["snrs"]]
        assert got == vals["qam"]
        assert [O.psk_bit_loading_order(float(ser), s) for s in bl["snrs"]] == vals["psk"]
