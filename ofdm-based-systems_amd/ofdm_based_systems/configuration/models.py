"""Settings models loaded from ``config/*.json`` (configuration/models.py:19-151 of the reference).

Same field names, defaults and validation messages as the reference, so the
reference's JSON files load unchanged (unknown keys such as
``capacity_scaling_factor`` are ignored, as pydantic does there).  Build-only
fields (``rng_mode``, ``seed``, ``precision``, ``batch_symbols``) are optional
with defaults that reproduce the reference's behaviour.
"""

from __future__ import annotations

import json
import os
from typing import Literal, Optional

from pydantic import BaseModel, Field, field_validator

from ofdm_based_systems.configuration.enums import (
    AdaptiveModulationMode,
    ChannelType,
    ConstellationType,
    EqualizationMethod,
    ModulationType,
    NoiseType,
    PowerAllocationType,
    PrefixType,
)


class BaseSettings(BaseModel):
    @classmethod
    def from_json(cls, file_path: str):
        """Build the model from a JSON file (FileNotFoundError if absent)."""
        if not os.path.exists(file_path):
            raise FileNotFoundError(f"Configuration file not found: {file_path}")
        with open(file_path, "r", encoding="utf-8") as fh:
            return cls(**json.load(fh))


class Settings(BaseSettings):
    """Project metadata (config/settings.json)."""

    project_name: str = Field(..., description="The name of the project")
    version: str = Field(..., description="The version of the project")
    debug: bool = Field(False, description="Enable or disable debug mode")

    def __str__(self) -> str:
        return "\n".join([self.project_name, self.version, f"Debug Mode: {self.debug}"])


class SimulationSettings(BaseSettings):
    """Parameters of one SNR sweep (one Simulation per entry of signal_noise_ratios)."""

    num_bands: int = Field(..., description="Number of frequency bands")
    signal_noise_ratios: list[float] = Field(..., description="SNR values in dB")
    channel_model_path: str = Field(..., description="Path to the channel model file")
    channel_type: ChannelType = Field(ChannelType.FLAT)
    noise_type: NoiseType = Field(NoiseType.AWGN)
    num_bits: Optional[int] = Field(None)
    num_symbols: Optional[int] = Field(None)
    constellation_order: int = Field(16)
    constellation_type: ConstellationType = Field(ConstellationType.PSK)
    prefix_type: PrefixType = Field(PrefixType.CYCLIC)
    prefix_length_ratio: float = Field(0.25)
    equalization_method: EqualizationMethod = Field(EqualizationMethod.MMSE)
    modulation_type: ModulationType = Field(ModulationType.OFDM)
    power_allocation_type: PowerAllocationType = Field(PowerAllocationType.UNIFORM)
    adaptive_modulation_mode: AdaptiveModulationMode = Field(AdaptiveModulationMode.FIXED)
    min_constellation_order: int = Field(4)
    max_constellation_order: int = Field(256)
    desired_symbol_error_rate: float = Field(1e-3)
    # ---- build-only knobs (absent from the reference's JSON files)
    rng_mode: Literal["reference", "philox"] = Field(
        "reference", description="'reference': PCG64 bits + legacy-normal noise drawn on the host "
        "exactly as the reference does; 'philox': counter-based bits/noise generated on the GPU")
    seed: Optional[int] = Field(None, description="seed for rng_mode='philox'")
    precision: Literal["f64", "f32"] = Field("f64", description="arithmetic precision of the GPU path")
    batch_symbols: Optional[int] = Field(None, description="OFDM symbols per device batch")

    def __str__(self) -> str:
        lines = [
            f"Number of Bands: {self.num_bands}",
            f"Signal-to-Noise Ratios: {self.signal_noise_ratios}",
            f"Channel Type: {self.channel_type}",
            f"Channel Model Path: '{self.channel_model_path}'",
            f"Noise Type: {self.noise_type}",
        ]
        if self.num_bits is not None:
            lines.append(f"Number of Bits: {self.num_bits}")
        if self.num_symbols is not None:
            lines.append(f"Number of Symbols: {self.num_symbols}")
        lines += [
            f"Constellation Type: '{self.constellation_type}'",
            f"Constellation Order: {self.constellation_order}",
            f"Prefix Type: {self.prefix_type}",
            f"Prefix Length Ratio: {self.prefix_length_ratio}",
            f"Equalization Method: {self.equalization_method}",
            f"Modulation Type: {self.modulation_type}",
            f"Power Allocation Type: {self.power_allocation_type}",
        ]
        return "\n".join(lines)

    @field_validator("num_symbols")
    @classmethod
    def check_bits_or_symbols(cls, v, info):
        has_bits = info.data.get("num_bits") is not None
        if not has_bits and v is None:
            raise ValueError("Either num_bits or num_symbols must be specified.")
        if has_bits and v is not None:
            raise ValueError("Only one of num_bits or num_symbols should be specified.")
        return v

    @field_validator("prefix_length_ratio")
    @classmethod
    def validate_prefix_length_ratio(cls, v):
        # the reference accepts [0, 2] although its message says [0, 1]
        if v < 0.0 or v > 2.0:
            raise ValueError("prefix_length_ratio must be between 0 and 1 (inclusive).")
        return v

    @field_validator("min_constellation_order", "max_constellation_order")
    @classmethod
    def validate_constellation_order(cls, v):
        if not 2 <= v <= 4096:
            raise ValueError("Constellation order must be between 2 and 4096.")
        if v & (v - 1):
            raise ValueError(f"Constellation order must be a power of 2, got {v}.")
        return v

    @field_validator("desired_symbol_error_rate")
    @classmethod
    def validate_desired_symbol_error_rate(cls, v):
        if v <= 0:
            raise ValueError("desired_symbol_error_rate must be positive.")
        if v >= 0.5:
            raise ValueError("desired_symbol_error_rate must be less than 0.5.")
        return v
