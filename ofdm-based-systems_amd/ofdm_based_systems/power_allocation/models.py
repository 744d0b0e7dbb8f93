"""Power allocation (power_allocation/models.py:13-334 of the reference).

Host-side precompute over K <= 4096 subcarriers (microseconds).  In FIXED mode
the reference computes the allocation but never applies it to the data
(simulation/models.py:508); in CAPACITY_BASED mode it feeds the bit-loading
orders, which the GPU path then uses.
"""

from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np
from numpy.typing import NDArray


class IPowerAllocation(ABC):
    @abstractmethod
    def allocate(self) -> NDArray[np.float64]:
        """Power per subcarrier."""


class UniformPowerAllocation(IPowerAllocation):
    def __init__(self, total_power: float, num_subcarriers: int):
        if total_power < 0:
            raise ValueError(f"Total power must be non-negative, got {total_power}")
        if num_subcarriers <= 0:
            raise ValueError(f"Number of subcarriers must be positive, got {num_subcarriers}")
        self.total_power = total_power
        self.num_subcarriers = num_subcarriers

    def allocate(self) -> NDArray[np.float64]:
        return np.full(self.num_subcarriers, self.total_power / self.num_subcarriers, dtype=np.float64)


class WaterfillingPowerAllocation(IPowerAllocation):
    """P[k] = max(0, mu - floor[k]), mu found by bisection so that sum P = P_total.

    The floor is N0 / (|H[k]|^2 K) -- the reference divides by K
    (power_allocation/models.py:161) -- and the result is renormalised to P_total.
    """

    def __init__(self, total_power: float, channel_gains: NDArray[np.float64], noise_power: float,
                 tolerance: float = 1e-8):
        if total_power < 0:
            raise ValueError(f"Total power must be non-negative, got {total_power}")
        if noise_power < 0:
            raise ValueError(f"Noise power must be non-negative, got {noise_power}")
        gains = np.asarray(channel_gains, dtype=np.float64)
        if gains.size == 0:
            raise ValueError("Channel gains array cannot be empty")
        if np.any(gains <= 0):
            raise ValueError("All channel gains must be positive, "
                             f"got min={np.min(gains)}, max={np.max(gains)}")
        self.total_power = total_power
        self.channel_gains = gains
        self.noise_power = noise_power
        self.tolerance = tolerance
        self.num_subcarriers = gains.size

    def _find_water_level(self, floor: NDArray[np.float64]) -> float:
        lo, hi = 0.0, self.total_power + np.max(floor)
        mu = 0.5 * (lo + hi)
        for _ in range(100):
            mu = 0.5 * (lo + hi)
            filled = np.sum(np.maximum(0, mu - floor))
            if np.abs(filled - self.total_power) < self.tolerance:
                break
            lo, hi = (mu, hi) if filled < self.total_power else (lo, mu)
        return mu

    def allocate(self) -> NDArray[np.float64]:
        floor = self.noise_power / (self.channel_gains * self.num_subcarriers)
        power = np.maximum(0, self._find_water_level(floor) - floor)
        total = np.sum(power)
        return power * (self.total_power / total) if total > 0 else power


def calculate_capacity_per_subcarrier(power_allocation, channel_gains, noise_power) -> NDArray[np.float64]:
    """log2(1 + P |H|^2 / N0 + 1e-12) per subcarrier."""
    return np.log2(1 + np.asarray(power_allocation) * np.asarray(channel_gains) / noise_power + 1e-12)


def calculate_capacity(power_allocation, channel_gains, noise_power) -> float:
    return np.sum(calculate_capacity_per_subcarrier(power_allocation, channel_gains, noise_power))


def compare_allocations(uniform, waterfilling, channel_gains, noise_power) -> dict:
    cu = calculate_capacity(uniform, channel_gains, noise_power)
    cw = calculate_capacity(waterfilling, channel_gains, noise_power)
    return {
        "uniform_capacity": cu,
        "waterfilling_capacity": cw,
        "capacity_gain": cw - cu,
        "capacity_gain_percent": 100 * (cw - cu) / cu if cu > 0 else 0,
    }
