"""Simulation orchestrator (simulation/models.py:59-818 of the reference).

Same constructor, strategy maps, ``create_from_simulation_settings`` and result
keys.  ``run()`` keeps the reference's setup (channel, prefix length, power
allocation, bit loading -- host precompute on <= 4096 values) and replaces the
data path with the fused GPU engine (:mod:`ofdm_based_systems.engine`):

* every built-in modulator / prefix / constellation (OFDM or SC-OFDM, cyclic, zero or no
  prefix, QAM or PSK, FIXED or CAPACITY_BASED): the two fused kernels (ofdm_tx / ofdm_rx);
* a user-supplied strategy class: the GPU operators composed as in the reference
  (encode -> modulate -> transmit -> demodulate -> decode), calling its own methods.

``rng_mode='reference'`` (default) draws the bits (PCG64 ``Generator.bytes``) and
the AWGN normals (legacy ``np.random.normal``, real part first) exactly as the
reference does, so seeded runs give the reference's integer error counts.
``rng_mode='philox'`` generates both inside the kernels (Monte-Carlo scale).
"""

from __future__ import annotations

import math
import os
import time
from io import BytesIO
from typing import Any, BinaryIO, Dict, List, Optional, Type

import numpy as np
import torch
from numpy.typing import NDArray

from ofdm_based_systems import _backend as B
from ofdm_based_systems.bits_generation.models import AdaptiveBitsGenerator, IGenerator, RandomBitsGenerator
from ofdm_based_systems.channel.models import ChannelModel
from ofdm_based_systems.configuration.enums import (
    AdaptiveModulationMode,
    ConstellationType,
    EqualizationMethod,
    ModulationType,
    NoiseType,
    PowerAllocationType,
    PrefixType,
)
from ofdm_based_systems.configuration.models import SimulationSettings
from ofdm_based_systems.constellation.adaptive import AdaptiveConstellationMapper
from ofdm_based_systems.constellation.models import (
    IConstellationMapper,
    PSKConstellationMapper,
    QAMConstellationMapper,
)
from ofdm_based_systems.engine import LinkEngine
from ofdm_based_systems.equalization.models import MMSEEqualizator, NoEqualizator, ZeroForcingEqualizator
from ofdm_based_systems.modulation.models import IModulator, OFDMModulator, SingleCarrierOFDMModulator
from ofdm_based_systems.noise.models import AWGNoiseModel, NoNoiseModel
from ofdm_based_systems.power_allocation.models import UniformPowerAllocation, WaterfillingPowerAllocation
from ofdm_based_systems.prefix.models import CyclicPrefixScheme, NoPrefixScheme, ZeroPaddingPrefixScheme
from ofdm_based_systems.serial_parallel.models import SerialToParallelConverter

# channel used when no CIR is configured (channel_type FLAT), simulation/models.py:237-245
DEFAULT_CHANNEL = np.array(
    [
        0.7767824138452235072 + 0.4560896742466611919j,
        -0.06669848996328063551 + 0.2839935704583463338j,
        0.1398968327715586490 - 0.1591963958343969865j,
        0.02229949514514480494 + 0.2409945439452868821j,
    ],
    dtype=np.complex128,
)

_EQ_KIND = {EqualizationMethod.NONE: B.EQ_NONE, EqualizationMethod.ZF: B.EQ_ZF,
            EqualizationMethod.MMSE: B.EQ_MMSE}


def read_bits_from_stream(stream: BinaryIO) -> List[int]:
    """All bits of a byte stream, MSB first; rewinds the stream (simulation/models.py:59-69)."""
    data = stream.read()
    stream.seek(0)
    return np.unpackbits(np.frombuffer(data, dtype=np.uint8)).astype(int).tolist()


def _stream_bytes(stream: BinaryIO) -> np.ndarray:
    data = np.frombuffer(stream.read(), dtype=np.uint8).copy()
    stream.seek(0)
    return data


class Simulation:
    CONSTELLATION_SCHEME_MAPPERS = {
        ConstellationType.QAM: QAMConstellationMapper,
        ConstellationType.PSK: PSKConstellationMapper,
    }
    MODULATOR_SCHEME_MAPPERS = {
        ModulationType.OFDM: OFDMModulator,
        ModulationType.SC_OFDM: SingleCarrierOFDMModulator,
    }
    PREFIX_SCHEME_MAPPERS = {
        PrefixType.NONE: NoPrefixScheme,
        PrefixType.CYCLIC: CyclicPrefixScheme,
        PrefixType.ZERO: ZeroPaddingPrefixScheme,
    }
    EQUALIZATOR_SCHEME_MAPPERS = {
        EqualizationMethod.NONE: NoEqualizator,
        EqualizationMethod.ZF: ZeroForcingEqualizator,
        EqualizationMethod.MMSE: MMSEEqualizator,
    }
    NOISE_SCHEME_MAPPERS = {NoiseType.AWGN: AWGNoiseModel, NoiseType.NONE: NoNoiseModel}
    POWER_ALLOCATION_MAPPERS = {
        PowerAllocationType.UNIFORM: UniformPowerAllocation,
        PowerAllocationType.WATERFILLING: WaterfillingPowerAllocation,
    }

    def __init__(
        self,
        num_bits: Optional[int] = None,
        num_symbols: Optional[int] = None,
        num_subcarriers: int = 64,
        constellation_order: int = 16,
        constellation_scheme: ConstellationType = ConstellationType.QAM,
        modulator_type: ModulationType = ModulationType.OFDM,
        prefix_scheme: PrefixType = PrefixType.CYCLIC,
        prefix_length_ratio: float = 1.0,
        equalizator_type: EqualizationMethod = EqualizationMethod.MMSE,
        snr_db: float = 20.0,
        noise_scheme: NoiseType = NoiseType.AWGN,
        power_allocation_type: PowerAllocationType = PowerAllocationType.UNIFORM,
        adaptive_modulation_mode: AdaptiveModulationMode = AdaptiveModulationMode.FIXED,
        min_constellation_order: int = 4,
        max_constellation_order: int = 256,
        desired_symbol_error_rate: float = 1e-3,
        channel_impulse_response: Optional[NDArray[np.complex128]] = None,
        verbose: bool = True,
        *,
        rng_mode: str = "reference",
        seed: Optional[int] = None,
        precision: str = "f64",
        batch_symbols: Optional[int] = None,
        received_symbols_keep: int = 64,
        make_plot: bool = True,
        process_group=None,
    ):
        if num_bits is None and num_symbols is None:
            raise ValueError("Either num_bits or num_symbols must be provided.")
        if num_bits is not None and num_symbols is not None:
            raise ValueError("Only one of num_bits or num_symbols should be provided.")
        if rng_mode not in ("reference", "philox"):
            raise ValueError("rng_mode must be 'reference' or 'philox'")
        self.num_bits = num_bits
        self.num_symbols = num_symbols
        self.num_subcarriers = num_subcarriers
        self.constellation_order = constellation_order
        self.constellation_scheme = constellation_scheme
        self.modulator_type = modulator_type
        self.prefix_scheme = prefix_scheme
        self.prefix_length_ratio = prefix_length_ratio
        self.equalizator_type = equalizator_type
        self.snr_db = snr_db
        self.noise_scheme = noise_scheme
        self.power_allocation_type = power_allocation_type
        self.adaptive_modulation_mode = adaptive_modulation_mode
        self.min_constellation_order = min_constellation_order
        self.max_constellation_order = max_constellation_order
        self.desired_symbol_error_rate = desired_symbol_error_rate
        self.channel_impulse_response = channel_impulse_response
        self.verbose = verbose
        self.rng_mode = rng_mode
        self.seed = seed
        self.precision = precision
        self.batch_symbols = batch_symbols
        self.received_symbols_keep = received_symbols_keep
        self.make_plot = make_plot
        self.process_group = process_group

    def _log(self, message: str) -> None:
        if self.verbose:
            print(message)

    @classmethod
    def create_from_simulation_settings(cls, simulation_settings: SimulationSettings) -> List["Simulation"]:
        """One Simulation per SNR; CUSTOM channels load their .npy relative to the cwd (:167-188)."""
        s = simulation_settings
        cir = None
        if s.channel_type.value == "CUSTOM":
            path = s.channel_model_path
            if not path:
                raise ValueError("channel_model_path must be specified when channel_type is CUSTOM")
            if not path.startswith("/"):
                path = os.path.abspath(path)
            if not os.path.exists(path):
                raise FileNotFoundError(f"Channel model file not found: {path}")
            try:
                cir = np.load(path)  # allow_pickle=False (default)
            except Exception as e:  # noqa: BLE001
                raise ValueError(f"Failed to load channel model from {path}: {e}")
        extra = {"rng_mode": s.rng_mode, "seed": s.seed, "precision": s.precision,
                 "batch_symbols": s.batch_symbols}
        return [
            cls(num_bits=s.num_bits, num_symbols=s.num_symbols, num_subcarriers=s.num_bands,
                constellation_order=s.constellation_order, constellation_scheme=s.constellation_type,
                modulator_type=s.modulation_type, prefix_scheme=s.prefix_type,
                prefix_length_ratio=s.prefix_length_ratio, equalizator_type=s.equalization_method,
                snr_db=snr, noise_scheme=s.noise_type, power_allocation_type=s.power_allocation_type,
                adaptive_modulation_mode=s.adaptive_modulation_mode,
                min_constellation_order=s.min_constellation_order,
                max_constellation_order=s.max_constellation_order,
                desired_symbol_error_rate=s.desired_symbol_error_rate, channel_impulse_response=cir, **extra)
            for snr in s.signal_noise_ratios
        ]

    # ------------------------------------------------------------------ helpers
    def _channel_gains(self, h_raw: np.ndarray) -> np.ndarray:
        """|fft(h_raw, N)|^2 of the un-normalised CIR (simulation/models.py:278-279), on the GPU."""
        plan = B.Plan(n_fft=self.num_subcarriers, h_raw=h_raw)
        H = torch.empty(self.num_subcarriers, dtype=torch.complex128, device=B.device())
        g = torch.empty(self.num_subcarriers, dtype=torch.float64, device=B.device())
        B.check(B.lib().ofdm_plan_response(plan.handle, B.stream_ptr(), B.ptr(H), B.ptr(g)))
        return g.cpu().numpy()

    def _plot(self, received: np.ndarray, mapper: IConstellationMapper, ber: float, papr_db: float,
              title: str, orders: np.ndarray):
        if not self.make_plot:
            return None
        import matplotlib

        matplotlib.use("Agg", force=False)
        import matplotlib.pyplot as plt
        from PIL import Image

        fig = plt.figure(figsize=(8, 8))
        ax = fig.add_subplot(1, 1, 1)
        ax.scatter(received.real, received.imag, color="blue", marker=".", alpha=0.1, label="Received Symbols")
        pts = mapper.constellation
        ax.scatter(pts.real, pts.imag, color="red", marker="o", label="Ideal Constellation Points")
        ax.set_title(title)
        ax.set_xlabel("In-Phase")
        ax.set_ylabel("Quadrature")
        ax.axhline(0, color="black", lw=0.5)
        ax.axvline(0, color="black", lw=0.5)
        ax.legend(loc="upper right")
        ax.grid(True)
        ax.set_xlim(-1.5, 1.5)
        ax.set_ylim(-1.5, 1.5)
        fig.text(0.15, 0.75, f"BER: {ber:.6f}\nSNR: {self.snr_db} dB\nPAPR: {papr_db:.2f} dB", fontsize=10,
                 bbox=dict(facecolor="white", alpha=0.5))
        buf = BytesIO()
        fig.savefig(buf, format="png")
        plt.close(fig)
        buf.seek(0)
        return Image.open(buf)

    # ------------------------------------------------------------------ run
    def run(self) -> Dict[str, Any]:
        results: Dict[str, Any] = {}
        sp = SerialToParallelConverter()
        noise_model = self.NOISE_SCHEME_MAPPERS.get(self.noise_scheme, AWGNoiseModel)()
        h_raw = np.asarray(DEFAULT_CHANNEL if self.channel_impulse_response is None
                           else self.channel_impulse_response, dtype=np.complex128)
        channel = ChannelModel(impulse_response=h_raw, snr_db=self.snr_db, noise_model=noise_model)
        cp = 0 if self.prefix_scheme == PrefixType.NONE else int(self.prefix_length_ratio * channel.order)
        prefix_scheme = self.PREFIX_SCHEME_MAPPERS.get(self.prefix_scheme, NoPrefixScheme)(prefix_length=cp)
        N = self.num_subcarriers
        gains = self._channel_gains(h_raw)
        noise_power = 10 ** (-self.snr_db / 10)
        water_level: Optional[float] = None
        base_mapper: Type[IConstellationMapper] = self.CONSTELLATION_SCHEME_MAPPERS.get(
            self.constellation_scheme, QAMConstellationMapper)

        if self.adaptive_modulation_mode == AdaptiveModulationMode.CAPACITY_BASED:
            # bit loading from the allocation with P_tot = N (simulation/models.py:289-395)
            if self.power_allocation_type == PowerAllocationType.WATERFILLING:
                allocation = WaterfillingPowerAllocation(N, gains, noise_power).allocate()
                level = allocation + noise_power / gains
                water_level = float(np.mean(level[allocation > 1e-10]))
            else:
                allocation = UniformPowerAllocation(N, N).allocate()
            orders = np.array([base_mapper.calculate_bit_loading_order(
                ser=self.desired_symbol_error_rate, snr=p * g / noise_power) for p, g in zip(allocation, gains)],
                dtype=np.int64)
            mapper: IConstellationMapper = AdaptiveConstellationMapper(orders, base_mapper, N)
            bps = int(np.sum(mapper.get_bits_per_subcarrier()))
            if self.num_symbols is not None:
                n_ofdm = self.num_symbols
            else:
                if bps == 0:
                    raise ValueError("All subcarriers have zero order - cannot transmit data")
                n_ofdm = self.num_bits // bps
            bits_gen: IGenerator = AdaptiveBitsGenerator(mapper.get_bits_per_subcarrier(), n_ofdm)
            total_bits = bits_gen.get_total_bits()
        else:
            orders = np.full(N, self.constellation_order, dtype=np.int64)
            mapper = base_mapper(order=self.constellation_order)
            bits_gen = RandomBitsGenerator()
            total_bits = self.num_bits
            if self.num_symbols is not None:
                total_bits = self.num_symbols * int(np.log2(self.constellation_order))
            allocation = None

        results.update({
            "num_bits": self.num_bits,
            "num_symbols": self.num_symbols,
            "num_subcarriers": N,
            "constellation_order": self.constellation_order,
            "constellation_scheme": self.constellation_scheme.name,
            "modulator_type": self.modulator_type.name,
            "prefix_scheme": self.prefix_scheme.name,
            "prefix_acronym": prefix_scheme.acronym,
            "equalizator_type": self.equalizator_type.name,
            "snr_db": self.snr_db,
            "noise_scheme": self.noise_scheme.name,
            "power_allocation_type": self.power_allocation_type.name,
            "power_allocation_acronym": (
                "WF" if self.power_allocation_type == PowerAllocationType.WATERFILLING else "UNIFORM"),
            "adaptive_modulation_mode": self.adaptive_modulation_mode.name,
            "constellation_order_per_subcarrier": orders.tolist(),
            "water_level": water_level,
            "title": f"{prefix_scheme.acronym}-{self.modulator_type.name}-{self.equalizator_type.name}",
            "subtitle": (f"{self.constellation_order}{self.constellation_scheme.name}-"
                         f"SNR{self.snr_db}dB-{self.power_allocation_type.name}"),
        })
        if total_bits is None:
            raise ValueError("Total bits could not be determined.")

        adaptive = self.adaptive_modulation_mode == AdaptiveModulationMode.CAPACITY_BASED
        if adaptive:
            n_ofdm_syms = n_ofdm
            valid_bits = (total_bits // 8) * 8
            # AdaptiveConstellationMapper.encode needs whole OFDM symbols, both for the tx stream
            # and for the re-encode of the received (whole-byte) stream (simulation/models.py:604)
            for nbits in (8 * math.ceil(total_bits / 8), valid_bits):
                if nbits % bps:
                    raise ValueError(f"Bits length ({nbits}) must be multiple of bits_per_symbol ({bps})")
        else:
            b = int(np.log2(self.constellation_order))
            n_const = math.ceil(8 * math.ceil(total_bits / 8) / b)
            if n_const % N:
                raise ValueError("Length of data must be divisible by number of streams.")
            n_ofdm_syms = n_const // N
            valid_bits = 8 * math.ceil(total_bits / 8)

        # FIXED-mode allocation: computed, reported, never applied (simulation/models.py:483-509)
        if not adaptive:
            if self.power_allocation_type == PowerAllocationType.WATERFILLING:
                allocation = WaterfillingPowerAllocation(1.0, gains, noise_power).allocate()
                level = allocation + noise_power / gains
                water_level = float(np.mean(level[allocation > 1e-10]))
            else:
                allocation = UniformPowerAllocation(1.0, N).allocate()
        results["allocated_power"] = allocation.tolist()

        # ---------------- data path
        reference = self.rng_mode == "reference"
        tx_bytes = _stream_bytes(bits_gen.generate_bits(total_bits)) if reference else None
        # every built-in strategy runs on the fused kernels (SC-OFDM, zero padding and PSK on
        # the generic kernel); a user-supplied strategy class falls back to the composed
        # GPU operators, which call its own methods
        mod_cls = self.MODULATOR_SCHEME_MAPPERS.get(self.modulator_type, OFDMModulator)
        pre_cls = self.PREFIX_SCHEME_MAPPERS.get(self.prefix_scheme, NoPrefixScheme)
        fused = (mod_cls in (OFDMModulator, SingleCarrierOFDMModulator)
                 and pre_cls in (CyclicPrefixScheme, ZeroPaddingPrefixScheme, NoPrefixScheme)
                 and type(mapper) in (QAMConstellationMapper, PSKConstellationMapper, AdaptiveConstellationMapper)
                 and not (adaptive and self.modulator_type == ModulationType.SC_OFDM)
                 and len(h_raw) - 1 <= N and cp <= N)
        if not fused and not reference:
            raise ValueError("rng_mode='philox' needs the built-in modulators, prefixes and constellations")
        t0 = time.perf_counter()
        if fused:
            luts, sc = (mapper.lut_tables() if adaptive else ([mapper.constellation], None))
            prec = B.OFDM_F32 if self.precision == "f32" else B.OFDM_F64
            engine = LinkEngine(N, cp, h_raw, _EQ_KIND[self.equalizator_type], luts, sc, prec,
                                prefix=B.PREFIX_ZERO if pre_cls is ZeroPaddingPrefixScheme else B.PREFIX_CYCLIC,
                                modulator=B.MOD_SC if mod_cls is SingleCarrierOFDMModulator else B.MOD_OFDM)
            noise_on = isinstance(noise_model, AWGNoiseModel)
            normals = None
            if reference and noise_on:
                n_samp = n_ofdm_syms * (N + cp)
                normals = (np.random.normal(size=n_samp), np.random.normal(size=n_samp))
            seed = self.seed if self.seed is not None else 0
            st = engine.run(n_ofdm_syms, self.snr_db, bits=tx_bytes, normals=normals, seed=seed,
                            noise_on=noise_on, keep_symbols=self.received_symbols_keep,
                            group=self.process_group, batch=self.batch_symbols, n_valid_bits=valid_bits)
            torch.cuda.synchronize()
            bit_errors, symbol_errors, papr_db = st.bit_errors, st.symbol_errors, st.papr_db
            received = st.received if st.received is not None else np.zeros(0, np.complex128)
            n_syms_total = n_ofdm_syms * N
        else:
            bit_errors, symbol_errors, papr_db, received, n_syms_total = self._composed_path(
                tx_bytes, mapper, prefix_scheme, channel, sp, valid_bits)
        elapsed = time.perf_counter() - t0

        ber = bit_errors / total_bits if total_bits > 0 else 0.0
        ser = symbol_errors / n_syms_total if n_syms_total > 0 else 0.0
        results.update({
            "papr_db": papr_db,
            "bit_errors": bit_errors,
            "symbol_errors": symbol_errors,
            "total_bits": total_bits,
            "bit_error_rate": ber,
            "symbol_error_rate": ser,
            "received_symbols": received,
        })
        results["constellation_plot"] = self._plot(received, mapper, ber, papr_db, results["title"], orders)
        results["transmission_time_ms"] = elapsed * 1000
        results["bitrate_mbps"] = total_bits / 1e6  # the reference reports Mbit, not a rate (:807)
        self._log(f"BER {ber:.6e}  SER {ser:.6e}  PAPR {papr_db:.2f} dB  ({elapsed * 1e3:.1f} ms)")
        return results

    # ------------------------------------------------------------------ composed GPU operators
    def _composed_path(self, tx_bytes, mapper, prefix_scheme, channel, sp, valid_bits):
        """SC-OFDM / zero padding / PSK: the reference's operator chain on GPU operators."""
        N = self.num_subcarriers
        eq = self.EQUALIZATOR_SCHEME_MAPPERS.get(self.equalizator_type, NoEqualizator)(
            channel_frequency_response=self._raw_response(channel), snr_db=self.snr_db)
        modulator: IModulator = self.MODULATOR_SCHEME_MAPPERS.get(self.modulator_type, OFDMModulator)(
            num_subcarriers=N, prefix_scheme=prefix_scheme, equalizator=eq)
        symbols = mapper.encode(BytesIO(tx_bytes.tobytes()))
        x = modulator.modulate(sp.to_parallel(symbols, N))
        p = np.abs(x) ** 2
        papr_db = float(10 * np.log10(np.max(p) / np.mean(p))) if np.mean(p) > 0 else float("inf")
        y = channel.transmit(sp.to_serial(x))
        Z = modulator.demodulate(sp.to_parallel(y, N + prefix_scheme.prefix_length))
        z = sp.to_serial(Z)
        rx = np.frombuffer(mapper.decode(z).read(), dtype=np.uint8)
        be, se = _compare_on_device(tx_bytes, rx, symbols, mapper, valid_bits)
        keep = z[: self.received_symbols_keep * N]
        return be, se, papr_db, keep, len(symbols)

    def _raw_response(self, channel: ChannelModel) -> np.ndarray:
        """fft(h_raw, N) of the configured (un-normalised) CIR, as the reference's equaliser gets it."""
        plan = B.Plan(n_fft=self.num_subcarriers, h_raw=channel._h_raw)
        H = torch.empty(self.num_subcarriers, dtype=torch.complex128, device=B.device())
        B.check(B.lib().ofdm_plan_response(plan.handle, B.stream_ptr(), B.ptr(H), None))
        return H.cpu().numpy()


def _compare_on_device(tx: np.ndarray, rx: np.ndarray, symbols: np.ndarray, mapper, valid_bits: int):
    """bit_errors = popcount(tx ^ rx) over the compared bits; symbol_errors = symbols != encode(rx)
    (simulation/models.py:596-606)."""
    n = min(len(tx), len(rx))
    a = torch.from_numpy(tx[:n].copy()).to(B.device())
    b = torch.from_numpy(rx[:n].copy()).to(B.device())
    xor = torch.bitwise_xor(a, b)
    tail = min(valid_bits, 8 * n)
    bits = torch.bitwise_and(xor.unsqueeze(1) >> torch.arange(7, -1, -1, device=a.device), 1).reshape(-1)
    be = int(bits[:tail].sum().item())
    recoded = mapper.encode(BytesIO(rx.tobytes()))
    m = min(len(recoded), len(symbols))
    se = int(np.count_nonzero(symbols[:m] != recoded[:m]))
    return be, se
