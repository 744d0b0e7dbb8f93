"""The drop-in's host-side contract on CPU (no GPU): what the reference's own unit tests pin
 -- exception types and messages raised before any kernel call,
the Gray word coder tables, constellation tables, serial/parallel ordering, guard-interval
slicing, power allocation, bit loading, seeded bit streams and the settings surface -- checked
on the product package ``ofdm_based_systems`` (the oracle only supplies reference-pinned
numbers: tests/golden was produced by the reference itself).

Reference tests mirrored (behaviour, not code): tests/ofdm_based_systems/{constellation,
serial_parallel,prefix,channel,equalization,modulation,bits_generation,simulation}/
test_models.py and tests/integration/test_power_allocation.py.
"""

import io
import json
import os

import numpy as np
import pytest
from conftest import GOLDEN, ROOT, channel

from ofdm_based_systems.bits_generation.models import AdaptiveBitsGenerator, IGenerator, RandomBitsGenerator
from ofdm_based_systems.channel.models import ChannelModel
from ofdm_based_systems.configuration.enums import (AdaptiveModulationMode, ChannelType, ConstellationType,
                                                    EqualizationMethod, ModulationType, NoiseType,
                                                    PowerAllocationType, PrefixType)
from ofdm_based_systems.configuration.models import SimulationSettings
from ofdm_based_systems.constellation.models import (GrayWordCoder, NoWordCoder, PSKConstellationMapper,
                                                     QAMConstellationMapper)
from ofdm_based_systems.equalization.models import MMSEEqualizator, NoEqualizator, ZeroForcingEqualizator
from ofdm_based_systems.modulation.models import OFDMModulator
from ofdm_based_systems.power_allocation.models import (UniformPowerAllocation, WaterfillingPowerAllocation,
                                                        calculate_capacity)
from ofdm_based_systems.prefix.models import CyclicPrefixScheme, NoPrefixScheme, ZeroPaddingPrefixScheme
from ofdm_based_systems.serial_parallel.models import SerialToParallelConverter
from ofdm_based_systems.simulation.models import Simulation, read_bits_from_stream

# ----------------------------------------------------------------- word coders (constellation/models.py:30-109)


def test_gray_coder_tables():
    c = GrayWordCoder(bits_per_word=3)
    assert [c.encode(i) for i in range(8)] == [0, 1, 3, 2, 6, 7, 5, 4]
    assert [c.decode(i) for i in range(8)] == [0, 1, 3, 2, 7, 6, 4, 5]
    c5 = GrayWordCoder(bits_per_word=5)
    assert all(c5.decode(c5.encode(i)) == i for i in range(32))
    with pytest.raises(ValueError):
        c.decode(8)


def test_no_word_coder_range():
    c = NoWordCoder(bits_per_word=2)
    assert [c.encode(i) for i in range(4)] == [0, 1, 2, 3]
    with pytest.raises(ValueError):
        c.encode(4)
    with pytest.raises(ValueError):
        c.decode(4)


# ----------------------------------------------------------------- constellations


@pytest.mark.parametrize("order", [3, 5, 10, 15, 17])
def test_qam_rejects_non_square_orders(order):
    with pytest.raises(ValueError, match="Order must be a perfect square"):
        QAMConstellationMapper(order)


def test_constellation_tables_match_reference():
    luts = np.load(os.path.join(GOLDEN, "luts.npz"))
    for m in (4, 16, 64, 256):
        mp = QAMConstellationMapper(m)
        assert mp.bits_per_symbol == int(np.log2(m))
        assert mp.constellation_name == f"{m}-QAM"
        assert np.array_equal(mp.constellation, luts[f"qam{m}"])
        assert len(mp.constellation_map) == m
        assert np.isclose(np.mean(np.abs(mp.constellation) ** 2), 1.0)
    for m in (2, 4, 8, 16):
        assert np.array_equal(PSKConstellationMapper(m).constellation, luts[f"psk{m}"])


def test_bit_loading_orders_match_reference():
    with open(os.path.join(GOLDEN, "bitloading.json")) as f:
        bl = json.load(f)
    for ser, vals in bl["orders"].items():
        got = [QAMConstellationMapper.calculate_bit_loading_order(ser=float(ser), snr=s) for s in bl["snrs"]]
        assert got == vals["qam"]
        got = [PSKConstellationMapper.calculate_bit_loading_order(ser=float(ser), snr=s) for s in bl["snrs"]]
        assert got == vals["psk"]


# ----------------------------------------------------------------- serial / parallel (serial_parallel/models.py:6-21)


def test_serial_parallel_ordering_and_errors():
    s = np.arange(12) + 0j
    p = SerialToParallelConverter.to_parallel(s, 4)
    assert p.shape == (3, 4) and np.array_equal(p[1], [4, 5, 6, 7])  # row-major
    assert np.array_equal(SerialToParallelConverter.to_serial(p), s)
    with pytest.raises(ValueError, match="Length of data must be divisible by number of streams."):
        SerialToParallelConverter.to_parallel(s, 5)
    with pytest.raises(ValueError, match="Number of streams must be a positive integer"):
        SerialToParallelConverter.to_parallel(s, 0)
    with pytest.raises(ValueError, match="Input data must be a 1D array"):
        SerialToParallelConverter.to_parallel(p, 4)
    with pytest.raises(ValueError, match="Input data must be a 2D array"):
        SerialToParallelConverter.to_serial(s)


# ----------------------------------------------------------------- guard intervals (prefix/models.py:7-113)


def test_cyclic_prefix_slicing():
    x = np.arange(8) + 1j
    cp = CyclicPrefixScheme(3)
    assert cp.acronym == "CP" and cp.prefix_length == 3
    y = cp.add_prefix(x)
    assert np.array_equal(y, np.concatenate((x[-3:], x)))
    assert np.array_equal(cp.remove_prefix(y), x)
    with pytest.raises(ValueError, match="Input symbols must be a 1D array"):
        cp.add_prefix(x.reshape(2, 4))
    with pytest.raises(ValueError, match="Prefix length must be a non-negative integer"):
        CyclicPrefixScheme(-1)


def test_zero_padding_overlap_add():
    x = np.arange(1, 9) + 0j
    zp = ZeroPaddingPrefixScheme(2)
    assert zp.acronym == "ZP"
    y = zp.add_prefix(x)
    assert np.array_equal(y, np.concatenate((x, [0, 0])))
    r = y.copy()
    r[-2:] = [10, 20]  # a channel tail in the guard folds back onto the first samples
    back = zp.remove_prefix(r)
    assert np.array_equal(back, x + np.array([10, 20, 0, 0, 0, 0, 0, 0]))
    with pytest.raises(ValueError, match="Input symbols must be a 1D array"):
        zp.remove_prefix(r.reshape(2, 5))


def test_no_prefix_is_identity():
    x = np.arange(4) + 0j
    npf = NoPrefixScheme()
    assert npf.prefix_length == 0 and npf.acronym == ""  # prefix/models.py:104-106
    assert np.array_equal(npf.add_prefix(x), x) and np.array_equal(npf.remove_prefix(x), x)


# ----------------------------------------------------------------- channel / equalisers / modulator validation


def test_channel_model_normalises_and_validates():
    h = channel("Lin-Phoong_P1") * 3.0
    ch = ChannelModel(h, 20.0)
    assert ch.order == len(h) - 1
    assert np.isclose(np.sum(np.abs(ch.impulse_response) ** 2), 1.0)
    with pytest.raises(ValueError, match="Impulse response cannot be all zeros."):
        ChannelModel(np.zeros(3, complex), 20.0)
    with pytest.raises(ValueError, match=r"Signal must be serial \(1D array\)"):
        ch.transmit(np.zeros((2, 2), complex))


def test_equalisers_validate_before_the_gpu():
    H = np.ones(8, complex)
    with pytest.raises(ValueError, match="must have the same shape"):
        ZeroForcingEqualizator(H).equalize(np.ones(4, complex))
    with pytest.raises(ValueError, match="must have the same shape"):
        MMSEEqualizator(H, snr_db=10.0).equalize(np.ones(4, complex))
    with pytest.raises(ValueError, match="SNR in dB must be provided"):
        MMSEEqualizator(H).equalize(np.ones(8, complex))
    assert np.array_equal(NoEqualizator(H).equalize(np.arange(8) + 0j), np.arange(8) + 0j)


def test_modulator_checks_the_symbol_count():
    mod = OFDMModulator(16, CyclicPrefixScheme(1), NoEqualizator(np.ones(16, complex)))
    with pytest.raises(ValueError, match="Number of symbols must be 16"):
        mod.modulate(np.zeros((2, 8), complex))


# ----------------------------------------------------------------- power allocation (power_allocation/models.py)


def test_power_allocation_matches_reference():
    pa = np.load(os.path.join(GOLDEN, "power_allocation.npz"))
    for key in pa.files:
        if not key.startswith("wf_"):
            continue
        ch, n, snr, tot = key[3:].rsplit("_", 3)
        n, snr, tot = int(n[1:]), float(snr[3:]), float(tot[1:])
        g = np.abs(np.fft.fft(channel(ch), n)) ** 2
        got = WaterfillingPowerAllocation(tot, g, 10 ** (-snr / 10)).allocate()
        np.testing.assert_array_equal(got, pa[key])
    np.testing.assert_array_equal(UniformPowerAllocation(1.0, 64).allocate(), pa["uniform_64_1"])
    np.testing.assert_array_equal(UniformPowerAllocation(2048, 2048).allocate(), pa["uniform_2048_2048"])


def test_power_allocation_rejects_invalid_inputs():
    for kw in ({"total_power": -1.0, "num_subcarriers": 64}, {"total_power": 1.0, "num_subcarriers": 0}):
        with pytest.raises(ValueError):
            UniformPowerAllocation(**kw)
    g = np.array([1.0, 0.8, 0.6])
    for kw in ({"total_power": -1.0, "channel_gains": g, "noise_power": 0.1},
               {"total_power": 1.0, "channel_gains": g, "noise_power": -0.1},
               {"total_power": 1.0, "channel_gains": np.array([]), "noise_power": 0.1}):
        with pytest.raises(ValueError):
            WaterfillingPowerAllocation(**kw)


def test_waterfilling_beats_uniform_capacity():
    g = np.abs(np.fft.fft(channel("Lin-Phoong_P2"), 64)) ** 2
    n0 = 10 ** (-10 / 10)
    wf = WaterfillingPowerAllocation(64.0, g, n0).allocate()
    un = UniformPowerAllocation(64.0, 64).allocate()
    assert np.isclose(wf.sum(), 64.0) and np.all(wf >= 0)
    assert calculate_capacity(wf, g, n0) >= calculate_capacity(un, g, n0)


# ----------------------------------------------------------------- bit streams (bits_generation/models.py:12-128)


def test_generator_interface_is_abstract():
    with pytest.raises(TypeError):
        IGenerator()


def test_seeded_bits_are_reproducible_and_tail_masked():
    a = RandomBitsGenerator(np.random.Generator(np.random.PCG64(7))).generate_bits(37).read()
    b = RandomBitsGenerator(np.random.Generator(np.random.PCG64(7))).generate_bits(37).read()
    assert a == b and len(a) == 5
    assert a[-1] & 0x07 == 0  # 37 bits: the last byte keeps its 5 leading bits
    assert a == np.random.Generator(np.random.PCG64(7)).bytes(5)[:4] + bytes([a[-1]])
    bits = read_bits_from_stream(io.BytesIO(a))
    assert len(bits) == 40 and bits[:8] == [int(c) for c in f"{a[0]:08b}"]  # MSB first


def test_adaptive_bits_cover_whole_symbols():
    gen = AdaptiveBitsGenerator(np.array([2, 4, 0, 6]), 3, np.random.Generator(np.random.PCG64(1)))
    data = gen.generate_bits(12 * 3).read()
    assert len(data) * 8 >= 36


# ----------------------------------------------------------------- settings and the Simulation front door


@pytest.mark.parametrize("name", sorted(f for f in os.listdir(os.path.join(ROOT, "config"))
                                        if f.startswith("simulation_settings") and f.endswith(".json")))
def test_every_shipped_settings_file_loads(name):
    s = SimulationSettings.from_json(os.path.join(ROOT, "config", name))
    assert s.num_bands > 0 and len(s.signal_noise_ratios) > 0
    assert (s.num_bits is None) != (s.num_symbols is None)
    assert isinstance(s.constellation_type, ConstellationType)
    assert isinstance(s.modulation_type, ModulationType)
    assert isinstance(s.prefix_type, PrefixType)
    assert isinstance(s.equalization_method, EqualizationMethod)
    assert isinstance(s.channel_type, ChannelType)
    assert isinstance(s.noise_type, NoiseType)
    assert isinstance(s.power_allocation_type, PowerAllocationType)
    assert isinstance(s.adaptive_modulation_mode, AdaptiveModulationMode)
    assert s.rng_mode == "reference" and s.precision == "f64"  # build-only knobs default to parity


def test_simulation_requires_exactly_one_size():
    with pytest.raises(ValueError, match="Either num_bits or num_symbols must be provided."):
        Simulation()
    with pytest.raises(ValueError, match="Only one of"):
        Simulation(num_bits=64, num_symbols=64)
