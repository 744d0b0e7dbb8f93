"""Generate the golden vectors that pin the oracle and the HIP path.

Run ONLY in the build container, where the reference is importable:

    PYTHONPATH=/root/reference/src PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg \
        python tests/golden/make_golden.py

It imports the reference (read-only, never shipped), drives it with seeded
random streams and writes numbers only:

* ``luts.npz``            - QAM / PSK constellation LUTs (constellation/models.py:180-218, :356-380)
* ``stage_<case>.npz``    - every intermediate of the operator chain for tiny
                            cases (tests/integration/test_end_to_end.py:42-94 order)
* ``runs.json``           - seeded ``Simulation.run()`` results (simulation/models.py:214-818)
* ``power_allocation.npz``- water-filling / uniform allocations (power_allocation/models.py:61-225)
* ``bitloading.json``     - ``calculate_bit_loading_order`` on an SNR grid (constellation/models.py:297-321)

Determinism recipe: the default ``Generator(PCG64())``
instances bound at def-time (bits_generation/models.py:24, :74) are replaced by
``Generator(PCG64(seed))`` and the legacy global RNG used by AWGN
(noise/models.py:19-21) is seeded with ``np.random.seed(seed)``.  Consumers
regenerate the same streams from the seed, so the fixtures store seeds, not
megabytes of noise.
"""

from __future__ import annotations

import contextlib
import hashlib
import io
import json
import os
import sys
import time

import numpy as np
from numpy.random import PCG64, Generator

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
CH = os.path.join(REF, "config", "channel_models")

import ofdm_based_systems.bits_generation.models as bg  # noqa: E402
from ofdm_based_systems.channel.models import ChannelModel  # noqa: E402
from ofdm_based_systems.configuration.enums import (  # noqa: E402
    AdaptiveModulationMode,
    ConstellationType,
    EqualizationMethod,
    ModulationType,
    NoiseType,
    PowerAllocationType,
    PrefixType,
)
from ofdm_based_systems.configuration.models import SimulationSettings  # noqa: E402
from ofdm_based_systems.constellation.models import (  # noqa: E402
    PSKConstellationMapper,
    QAMConstellationMapper,
)
from ofdm_based_systems.equalization.models import (  # noqa: E402
    MMSEEqualizator,
    NoEqualizator,
    ZeroForcingEqualizator,
)
from ofdm_based_systems.modulation.models import OFDMModulator  # noqa: E402
from ofdm_based_systems.noise.models import AWGNoiseModel, NoNoiseModel  # noqa: E402
from ofdm_based_systems.power_allocation.models import (  # noqa: E402
    UniformPowerAllocation,
    WaterfillingPowerAllocation,
)
from ofdm_based_systems.prefix.models import (  # noqa: E402
    CyclicPrefixScheme,
    NoPrefixScheme,
)
from ofdm_based_systems.serial_parallel.models import SerialToParallelConverter  # noqa: E402
from ofdm_based_systems.simulation.models import Simulation  # noqa: E402

DEFAULT_4TAP = np.array(
    [
        (7.767824138452235072e-01 + 4.560896742466611919e-01j),
        (-6.669848996328063551e-02 + 2.839935704583463338e-01j),
        (1.398968327715586490e-01 - 1.591963958343969865e-01j),
        (2.229949514514480494e-02 + 2.409945439452868821e-01j),
    ],
    dtype=np.complex128,
)


def channel(name: str) -> np.ndarray:
    if name == "FLAT_DEFAULT":
        return DEFAULT_4TAP.copy()
    return np.load(os.path.join(CH, name + ".npy"))


def seed_all(seed: int) -> None:
    bg.RandomBitsGenerator.__init__.__defaults__ = (Generator(PCG64(seed)),)
    bg.AdaptiveBitsGenerator.__init__.__defaults__ = (Generator(PCG64(seed)),)
    np.random.seed(seed)


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()[:16]


# --------------------------------------------------------------------------- LUTs
def make_luts() -> None:
    out = {}
    for m in (4, 16, 64, 256):
        out[f"qam{m}"] = QAMConstellationMapper(m).constellation
    for m in (2, 4, 8, 16):
        out[f"psk{m}"] = PSKConstellationMapper(m).constellation
    np.savez_compressed(os.path.join(OUT, "luts.npz"), **out)


# --------------------------------------------------------------------------- stages
STAGES = [
    # name, N, M, channel, prefix ("CP"/"NONE"), ratio, eq, snr, S, seed
    ("n64_m16_severe_cp_mmse", 64, 16, "severe_multipath", "CP", 1.0, "MMSE", 15.0, 8, 3),
    ("n64_m4_flat_none", 64, 4, "flat_fading", "CP", 1.0, "NONE", 5.0, 8, 4),
    ("n1024_m64_p1_cp_zf", 1024, 64, "Lin-Phoong_P1", "CP", 1.0, "ZF", 25.0, 4, 5),
    ("n256_m256_default_cp034_mmse", 256, 256, "FLAT_DEFAULT", "CP", 0.34, "MMSE", 30.0, 4, 6),
    ("n128_m16_tworay_noprefix_mmse", 128, 16, "two_ray", "NONE", 1.0, "MMSE", 20.0, 4, 7),
    ("n4096_m64_p2_cp_mmse", 4096, 64, "Lin-Phoong_P2", "CP", 1.0, "MMSE", 28.0, 2, 8),
    ("n2048_m16_rayleigh_cp_zf", 2048, 16, "rayleigh_fading", "CP", 1.0, "ZF", 18.0, 2, 9),
    ("n16_m4_default_cp_mmse", 16, 4, "default_multipath", "CP", 1.0, "MMSE", 10.0, 8, 10),
    ("n8_m16_severe_cp_zf", 8, 16, "severe_multipath", "CP", 1.0, "ZF", 30.0, 16, 11),
    ("n512_m64_severe_cp050_mmse", 512, 64, "severe_multipath", "CP", 0.5, "MMSE", 22.0, 4, 12),
]

EQ = {"MMSE": MMSEEqualizator, "ZF": ZeroForcingEqualizator, "NONE": NoEqualizator}


def make_stage(name, n, m, ch, prefix, ratio, eq, snr, s, seed) -> dict:
    """Operator chain exactly as Simulation.run wires it (simulation/models.py:248-606)."""
    h_raw = channel(ch)
    b = int(np.log2(m))
    mapper = QAMConstellationMapper(m)
    cm = ChannelModel(h_raw, snr, AWGNoiseModel())
    cp = int(ratio * cm.order)
    if prefix == "NONE":
        cp = 0
    pscheme = CyclicPrefixScheme(cp) if prefix == "CP" else NoPrefixScheme(cp)
    H = np.fft.fft(h_raw, n)
    eqz = EQ[eq](channel_frequency_response=H, snr_db=snr)
    mod = OFDMModulator(num_subcarriers=n, prefix_scheme=pscheme, equalizator=eqz)
    sp = SerialToParallelConverter()

    nbits = s * n * b
    gen = bg.RandomBitsGenerator(Generator(PCG64(seed)))
    bits = gen.generate_bits(nbits)
    tx_bytes = bits.getvalue()
    X = sp.to_parallel(mapper.encode(io.BytesIO(tx_bytes)), n)
    x = mod.modulate(X)
    ser = sp.to_serial(x)
    y_clean = ChannelModel(h_raw, snr, NoNoiseModel()).transmit(ser)
    np.random.seed(seed)
    y = cm.transmit(ser)
    np.random.seed(seed)
    nr = np.random.normal(size=ser.shape)
    ni = np.random.normal(size=ser.shape)
    Yp = sp.to_parallel(y, n + cp)
    Z = mod.demodulate(Yp)
    z = sp.to_serial(Z)
    rx = mapper.decode(z).getvalue()
    txb = np.unpackbits(np.frombuffer(tx_bytes, np.uint8))
    rxb = np.unpackbits(np.frombuffer(rx, np.uint8))
    bit_errors = int(np.sum(txb[: len(rxb)] != rxb[: len(txb)]))
    sym_err = int(np.sum(mapper.encode(io.BytesIO(rx)) != mapper.encode(io.BytesIO(tx_bytes))))
    p = np.abs(x) ** 2
    papr = float(10 * np.log10(np.max(p) / np.mean(p)))
    np.savez_compressed(
        os.path.join(OUT, f"stage_{name}.npz"),
        h_raw=h_raw, H=H, tx_bytes=np.frombuffer(tx_bytes, np.uint8), X=X, x=x, y_clean=y_clean,
        noise_re=nr, noise_im=ni, y=y, Z=Z, rx_bytes=np.frombuffer(rx, np.uint8),
    )
    return dict(
        name=name, N=n, M=m, channel=ch, prefix=prefix, ratio=ratio, cp=cp, eq=eq, snr_db=snr,
        S=s, seed=seed, bit_errors=bit_errors, symbol_errors=sym_err, papr_db=papr,
        tx_sha=sha(tx_bytes), rx_sha=sha(rx),
    )


# --------------------------------------------------------------------------- runs
def run_sim(seed: int, **kw) -> dict:
    seed_all(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        t0 = time.perf_counter()
        r = Simulation(verbose=False, **kw).run()
        dt = time.perf_counter() - t0
    keep = {}
    for k, v in r.items():
        if k in ("received_symbols", "constellation_plot"):
            continue
        if isinstance(v, (np.integer,)):
            v = int(v)
        elif isinstance(v, (np.floating,)):
            v = float(v)
        keep[k] = v
    keep["_ref_seconds"] = dt
    keep["_received_symbols_len"] = int(len(r["received_symbols"]))
    return keep


def runs() -> list:
    cases = []

    def add(tag, seed, ch, **kw):
        kw = dict(kw)
        h = None if ch is None else channel(ch)
        res = run_sim(seed, channel_impulse_response=h, **kw)
        params = {k: (v.value if hasattr(v, "value") else v) for k, v in kw.items()}
        cases.append(dict(tag=tag, seed=seed, channel=ch, params=params, result=res))
        print(f"  {tag} seed={seed} ber={res['bit_error_rate']:.3e} "
              f"be={res['bit_errors']} t={res['_ref_seconds']:.1f}s", file=sys.stderr)

    Q, O = ConstellationType.QAM, ModulationType.OFDM
    CP, NP, ZP = PrefixType.CYCLIC, PrefixType.NONE, PrefixType.ZERO
    MM, ZF, NE = EqualizationMethod.MMSE, EqualizationMethod.ZF, EqualizationMethod.NONE
    WF, UN = PowerAllocationType.WATERFILLING, PowerAllocationType.UNIFORM

    # config (a): simulation_settings_test.json as written (via the settings loader)
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        st = SimulationSettings.from_json("config/simulation_settings_test.json")
        for seed in (0, 1):
            for sim in Simulation.create_from_simulation_settings(st):
                seed_all(seed)
                with contextlib.redirect_stdout(io.StringIO()):
                    sim.verbose = False
                    r = sim.run()
                cases.append(dict(
                    tag="settings_test_json", seed=seed, channel="severe_multipath",
                    params=dict(num_symbols=st.num_symbols, num_subcarriers=st.num_bands,
                                constellation_order=st.constellation_order, constellation_scheme="QAM",
                                modulator_type="OFDM", prefix_scheme="CYCLIC", prefix_length_ratio=1.0,
                                equalizator_type="ZF", snr_db=sim.snr_db, noise_scheme="AWGN",
                                power_allocation_type="WATERFILLING", adaptive_modulation_mode="FIXED"),
                    result={k: (int(v) if isinstance(v, np.integer) else float(v) if isinstance(v, np.floating) else v)
                            for k, v in r.items() if k not in ("received_symbols", "constellation_plot")},
                ))
                print(f"  settings_test seed={seed} snr={sim.snr_db} be={r['bit_errors']}", file=sys.stderr)
    finally:
        os.chdir(cwd)

    base = dict(constellation_scheme=Q, modulator_type=O, noise_scheme=NoiseType.AWGN,
                power_allocation_type=UN, adaptive_modulation_mode=AdaptiveModulationMode.FIXED)
    # literal-intent variant of config (a)
    for snr in (0.0, 5.0, 10.0):
        add("n64_qpsk_flat_none", 1, "flat_fading", num_symbols=10240, num_subcarriers=64,
            constellation_order=4, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=NE,
            snr_db=snr, **base)
    for seed in (1, 7):
        add("n64_m16_p1_mmse_15", seed, "Lin-Phoong_P1", num_symbols=32768, num_subcarriers=64,
            constellation_order=16, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=MM,
            snr_db=15.0, **base)
        add("n1024_m64_p1_mmse_20", seed, "Lin-Phoong_P1", num_symbols=102400, num_subcarriers=1024,
            constellation_order=64, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=MM,
            snr_db=20.0, **base)
        add("n1024_m64_flat_none_18", seed, "flat_fading", num_symbols=102400, num_subcarriers=1024,
            constellation_order=64, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=NE,
            snr_db=18.0, **base)
        add("n256_m256_p1_mmse_28", seed, "Lin-Phoong_P1", num_symbols=25600, num_subcarriers=256,
            constellation_order=256, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=MM,
            snr_db=28.0, **base)
        add("n64_qpsk_p1_mmse_8", seed, "Lin-Phoong_P1", num_symbols=12800, num_subcarriers=64,
            constellation_order=4, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=MM,
            snr_db=8.0, **base)
    # config (b) and (c) at fixture scale (200 OFDM symbols)
    add("cfg_b_n1024_m64_flat_none_24", 1, "flat_fading", num_symbols=1024 * 200,
        num_subcarriers=1024, constellation_order=64, prefix_scheme=CP, prefix_length_ratio=1.0,
        equalizator_type=NE, snr_db=24.0, **base)
    for snr in (10.0, 26.0):
        add("cfg_c_n1024_m64_severe_mmse", 1, "severe_multipath", num_symbols=1024 * 200,
            num_subcarriers=1024, constellation_order=64, prefix_scheme=CP, prefix_length_ratio=1.0,
            equalizator_type=MM, snr_db=snr, **base)
    # ISI cases: prefix shorter than the channel, and no prefix at all
    add("n256_m16_severe_cp043_mmse", 2, "severe_multipath", num_symbols=256 * 40,
        num_subcarriers=256, constellation_order=16, prefix_scheme=CP, prefix_length_ratio=0.43,
        equalizator_type=MM, snr_db=25.0, **base)
    add("n64_m4_default4tap_noprefix_zf", 3, None, num_symbols=64 * 50, num_subcarriers=64,
        constellation_order=4, prefix_scheme=NP, prefix_length_ratio=1.0, equalizator_type=ZF,
        snr_db=20.0, **base)
    # no-noise run: every count must be zero
    add("n128_m64_severe_nonoise_zf", 4, "severe_multipath", num_symbols=128 * 20,
        num_subcarriers=128, constellation_order=64, prefix_scheme=CP, prefix_length_ratio=1.0,
        equalizator_type=ZF, snr_db=10.0, **{**base, "noise_scheme": NoiseType.NONE})
    # num_bits path (FIXED mode): total_bits = num_bits
    add("n64_m16_numbits_p2_mmse", 5, "Lin-Phoong_P2", num_bits=64 * 4 * 30, num_subcarriers=64,
        constellation_order=16, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=MM,
        snr_db=12.0, **base)
    # config (e): waterfilling FIXED at N=4096 (water-filling computed, not applied)
    for m in (16, 64, 256):
        add(f"cfg_e_n4096_m{m}_p1_wf", 1, "Lin-Phoong_P1", num_symbols=4096 * 4,
            num_subcarriers=4096, constellation_order=m, prefix_scheme=CP, prefix_length_ratio=1.0,
            equalizator_type=MM, snr_db=30.0,
            **{**base, "power_allocation_type": WF})
    # config (d): adaptive bit loading (CAPACITY_BASED), N=64 as written and N=2048
    ad = dict(base, power_allocation_type=WF,
              adaptive_modulation_mode=AdaptiveModulationMode.CAPACITY_BASED)
    for snr in (15.0, 20.0, 25.0):
        add("cfg_d_n64_adaptive", 1, "Lin-Phoong_P1", num_symbols=200, num_subcarriers=64,
            constellation_order=16, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=MM,
            snr_db=snr, min_constellation_order=4, max_constellation_order=256,
            desired_symbol_error_rate=1e-3, **ad)
    add("cfg_d_n2048_adaptive", 1, "Lin-Phoong_P1", num_symbols=4, num_subcarriers=2048,
        constellation_order=16, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=MM,
        snr_db=20.0, desired_symbol_error_rate=1e-3, **ad)
    add("cfg_d_n64_adaptive_uniform", 2, "severe_multipath", num_symbols=100, num_subcarriers=64,
        constellation_order=16, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=MM,
        snr_db=22.0, **dict(ad, power_allocation_type=UN))
    # published BER table rows (docs/OFDM-Based Systems.tex:200-264): 64-QAM, N=64,
    # Lin-Phoong P2, 30 dB, 6e6 bits, MMSE with CP ratios 0.34 and 1.00
    for ratio in (0.34, 1.0):
        add(f"published_cp{ratio:.2f}_mmse", 1, "Lin-Phoong_P2", num_bits=6_000_000,
            num_subcarriers=64, constellation_order=64, prefix_scheme=CP, prefix_length_ratio=ratio,
            equalizator_type=MM, snr_db=30.0, **base)
    # next-row variants, pinned now for later rounds (ZP prefix, SC-OFDM, PSK)
    add("next_zp_n64_m16_p2_mmse", 1, "Lin-Phoong_P2", num_symbols=64 * 100, num_subcarriers=64,
        constellation_order=16, prefix_scheme=ZP, prefix_length_ratio=1.0, equalizator_type=MM,
        snr_db=20.0, **base)
    add("next_scofdm_n64_qpsk_p1_zf", 1, "Lin-Phoong_P1", num_symbols=64 * 100, num_subcarriers=64,
        constellation_order=4, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=ZF,
        snr_db=10.0, **dict(base, modulator_type=ModulationType.SC_OFDM))
    add("next_psk8_n64_p1_mmse", 1, "Lin-Phoong_P1", num_symbols=64 * 100, num_subcarriers=64,
        constellation_order=8, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=MM,
        snr_db=18.0, **dict(base, constellation_scheme=ConstellationType.PSK))
    # SURVEY 8(f) rows on the fused path: published ZP rows (docs tex:257-260), SC-OFDM, PSK
    for ratio in (0.34, 1.0):
        add(f"published_zp{ratio:.2f}_mmse", 1, "Lin-Phoong_P2", num_bits=6_000_000,
            num_subcarriers=64, constellation_order=64, prefix_scheme=ZP, prefix_length_ratio=ratio,
            equalizator_type=MM, snr_db=30.0, **base)
    add("next_zp_n256_m64_severe_zf", 2, "severe_multipath", num_symbols=256 * 40, num_subcarriers=256,
        constellation_order=64, prefix_scheme=ZP, prefix_length_ratio=1.0, equalizator_type=ZF,
        snr_db=28.0, **base)
    add("next_zp_n128_m16_severe_cp050_mmse", 3, "severe_multipath", num_symbols=128 * 40,
        num_subcarriers=128, constellation_order=16, prefix_scheme=ZP, prefix_length_ratio=0.5,
        equalizator_type=MM, snr_db=24.0, **base)
    add("next_scofdm_n256_m16_severe_mmse", 2, "severe_multipath", num_symbols=256 * 40,
        num_subcarriers=256, constellation_order=16, prefix_scheme=CP, prefix_length_ratio=1.0,
        equalizator_type=MM, snr_db=22.0, **dict(base, modulator_type=ModulationType.SC_OFDM))
    add("next_scofdm_zp_n64_qpsk_p2_zf", 3, "Lin-Phoong_P2", num_symbols=64 * 60, num_subcarriers=64,
        constellation_order=4, prefix_scheme=ZP, prefix_length_ratio=1.0, equalizator_type=ZF,
        snr_db=15.0, **dict(base, modulator_type=ModulationType.SC_OFDM))
    add("next_scofdm_n128_m64_flat_none", 4, "flat_fading", num_symbols=128 * 40, num_subcarriers=128,
        constellation_order=64, prefix_scheme=CP, prefix_length_ratio=1.0, equalizator_type=NE,
        snr_db=20.0, **dict(base, modulator_type=ModulationType.SC_OFDM))
    for m, ch, eq, snr, ratio in ((2, "severe_multipath", ZF, 8.0, 1.0), (4, "flat_fading", NE, 6.0, 1.0),
                                  (16, "Lin-Phoong_P1", MM, 22.0, 1.0), (8, "severe_multipath", MM, 20.0, 0.5)):
        add(f"next_psk{m}_n128_{ch}_r{ratio:.1f}", 2, ch, num_symbols=128 * 40, num_subcarriers=128,
            constellation_order=m, prefix_scheme=CP, prefix_length_ratio=ratio, equalizator_type=eq,
            snr_db=snr, **dict(base, constellation_scheme=ConstellationType.PSK))
    add("next_psk8_zp_scofdm_n64_p1_mmse", 5, "Lin-Phoong_P1", num_symbols=64 * 60, num_subcarriers=64,
        constellation_order=8, prefix_scheme=ZP, prefix_length_ratio=1.0, equalizator_type=MM,
        snr_db=16.0, **dict(base, constellation_scheme=ConstellationType.PSK,
                            modulator_type=ModulationType.SC_OFDM))
    return cases


# --------------------------------------------------------------------------- power allocation
def power_allocation() -> None:
    out = {}
    for ch in ("Lin-Phoong_P1", "Lin-Phoong_P2", "severe_multipath", "two_ray", "rayleigh_fading"):
        h = channel(ch)
        for n in (64, 1024, 4096):
            g = np.abs(np.fft.fft(h, n)) ** 2
            for snr in (0.0, 10.0, 20.0, 30.0):
                n0 = 10 ** (-snr / 10)
                for tot in (1.0, float(n)):
                    key = f"{ch}_n{n}_snr{int(snr)}_p{int(tot)}"
                    out["wf_" + key] = WaterfillingPowerAllocation(tot, g, n0).allocate()
    out["uniform_64_1"] = UniformPowerAllocation(1.0, 64).allocate()
    out["uniform_2048_2048"] = UniformPowerAllocation(2048.0, 2048).allocate()
    np.savez_compressed(os.path.join(OUT, "power_allocation.npz"), **out)


def bitloading() -> None:
    snrs = [0.0, 0.5, 1.0, 2.0, 5.0, 10.0, 20.0, 31.6, 100.0, 316.0, 1000.0, 3162.0, 1e4, 1e5, 1e6]
    res = {}
    with contextlib.redirect_stdout(io.StringIO()):
        for ser in (1e-2, 1e-3, 1e-4, 1e-6):
            res[str(ser)] = {
                "qam": [QAMConstellationMapper.calculate_bit_loading_order(ser, s) for s in snrs],
                "psk": [PSKConstellationMapper.calculate_bit_loading_order(ser, s) for s in snrs],
            }
    with open(os.path.join(OUT, "bitloading.json"), "w") as f:
        json.dump({"snrs": snrs, "orders": res}, f, indent=1)


def main() -> None:
    t0 = time.time()
    make_luts()
    power_allocation()
    bitloading()
    stages = [make_stage(*c) for c in STAGES]
    with open(os.path.join(OUT, "stages.json"), "w") as f:
        json.dump(stages, f, indent=1)
    print(f"stages done {time.time() - t0:.1f}s", file=sys.stderr)
    cases = runs()
    with open(os.path.join(OUT, "runs.json"), "w") as f:
        json.dump(cases, f, indent=1, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o))
    print(f"all done {time.time() - t0:.1f}s", file=sys.stderr)


if __name__ == "__main__":
    main()
