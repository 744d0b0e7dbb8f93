"""Configuration enums (configuration/enums.py:4-67 of the reference).

String-valued so ``SimulationSettings.from_json`` accepts the JSON spellings and
``str(member)`` prints the value.
"""

from enum import Enum


class _ValueStr(str, Enum):
    def __str__(self) -> str:  # "QAM", not "ConstellationType.QAM"
        return self.value


ConstellationType = _ValueStr("ConstellationType", [("QAM", "QAM"), ("PSK", "PSK")])
PrefixType = _ValueStr("PrefixType", [("CYCLIC", "CYCLIC"), ("ZERO", "ZERO"), ("NONE", "NONE")])
EqualizationMethod = _ValueStr("EqualizationMethod", [("ZF", "ZF"), ("MMSE", "MMSE"), ("NONE", "NONE")])
ModulationType = _ValueStr("ModulationType", [("OFDM", "OFDM"), ("SC_OFDM", "SC-OFDM")])
ChannelType = _ValueStr("ChannelType", [("FLAT", "FLAT"), ("CUSTOM", "CUSTOM")])
NoiseType = _ValueStr("NoiseType", [("AWGN", "AWGN"), ("NONE", "NONE")])
PowerAllocationType = _ValueStr("PowerAllocationType", [("UNIFORM", "UNIFORM"), ("WATERFILLING", "WATERFILLING")])
AdaptiveModulationMode = _ValueStr(
    "AdaptiveModulationMode", [("FIXED", "FIXED"), ("CAPACITY_BASED", "CAPACITY_BASED")])

__all__ = [
    "ConstellationType", "PrefixType", "EqualizationMethod", "ModulationType", "ChannelType",
    "NoiseType", "PowerAllocationType", "AdaptiveModulationMode",
]
