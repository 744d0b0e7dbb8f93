"""Bit sources (bits_generation/models.py:12-163 of the reference).

``RandomBitsGenerator`` and ``AdaptiveBitsGenerator`` draw their bytes from a
NumPy ``Generator`` exactly like the reference (PCG64 by default, tail byte
masked MSB-first), so a seeded run feeds the GPU path the very bits the
reference would use.  For large Monte-Carlo runs ``Simulation`` can instead
generate bits on the GPU (``rng_mode='philox'``); these classes are the
reference-compatible source.
"""

from __future__ import annotations

import math
from abc import ABC, abstractmethod
from io import BytesIO
from typing import BinaryIO, Tuple

import numpy as np
from numpy.random import PCG64, Generator
from numpy.typing import NDArray


def _masked_bytes(generator: Generator, num_bits: int) -> bytes:
    """ceil(num_bits/8) random bytes; the bits past num_bits in the last byte are zeroed."""
    data = bytearray(generator.bytes(math.ceil(num_bits / 8)))
    spare = (-num_bits) % 8
    if spare and data:
        data[-1] &= (0xFF << spare) & 0xFF
    return bytes(data)


class IGenerator(ABC):
    @abstractmethod
    def generate_bits(self, num_bits: int) -> BinaryIO:
        """Return a stream holding ``num_bits`` bits, packed MSB-first."""


class RandomBitsGenerator(IGenerator):
    """Uniform random bits from a NumPy ``Generator``.

    Like the reference, the default generator instance is created once, when the
    function is defined (bits_generation/models.py:24), so successive default-
    constructed generators continue one PCG64 stream.
    """

    def __init__(self, generator: Generator = Generator(PCG64())):
        self.generator = generator

    def generate_bits(self, num_bits: int) -> BinaryIO:
        stream = BytesIO(_masked_bytes(self.generator, num_bits))
        stream.seek(0)
        return stream


class AdaptiveBitsGenerator(IGenerator):
    """Exactly ``sum(bits_per_subcarrier) * num_ofdm_symbols`` bits for adaptive loading."""

    def __init__(
        self,
        bits_per_subcarrier: NDArray[np.int64],
        num_ofdm_symbols: int,
        generator: Generator = Generator(PCG64()),
    ):
        if len(bits_per_subcarrier) == 0:
            raise ValueError("bits_per_subcarrier cannot be empty")
        if num_ofdm_symbols <= 0:
            raise ValueError(f"num_ofdm_symbols must be positive, got {num_ofdm_symbols}")
        self.bits_per_subcarrier = np.array(bits_per_subcarrier, dtype=np.int64)
        self.num_ofdm_symbols = num_ofdm_symbols
        self.generator = generator

    def get_total_bits(self) -> int:
        return int(self.bits_per_subcarrier.sum() * self.num_ofdm_symbols)

    def generate_bits(self, num_bits: int = 0) -> BinaryIO:
        """``num_bits`` is ignored: the size follows from the bit allocation."""
        stream = BytesIO(_masked_bytes(self.generator, self.get_total_bits()))
        stream.seek(0)
        return stream

    @staticmethod
    def calculate_requirements(
        constellation_orders: NDArray[np.int64], num_ofdm_symbols: int
    ) -> Tuple[int, NDArray[np.int64]]:
        """(total bits, log2 order per subcarrier; 0 for order 0)."""
        orders = np.asarray(constellation_orders)
        bits = np.array([int(np.log2(o)) if o > 0 else 0 for o in orders], dtype=np.int64)
        return int(bits.sum() * num_ofdm_symbols), bits
