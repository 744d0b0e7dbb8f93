"""Guard-interval schemes (prefix/models.py:7-113 of the reference).

These objects describe the guard interval (``prefix_length``, ``acronym``) that
``OFDMModulator`` applies inside its HIP kernels.  Their 1-D ``add_prefix`` /
``remove_prefix`` helpers are kept for API compatibility; they are single-row
layout operations (slicing / concatenation, plus the zero-padding overlap-add)
on host arrays and are not used by the GPU modem path.
"""

from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np
from numpy.typing import NDArray


class IPrefixScheme(ABC):
    prefix_length: int

    def __init__(self, prefix_length: int = 0):
        if prefix_length < 0:
            raise ValueError("Prefix length must be a non-negative integer.")
        self.prefix_length = prefix_length

    @property
    @abstractmethod
    def acronym(self) -> str: ...

    @abstractmethod
    def add_prefix(self, symbols: NDArray[np.complex128]) -> NDArray[np.complex128]: ...

    @abstractmethod
    def remove_prefix(self, symbols: NDArray[np.complex128]) -> NDArray[np.complex128]: ...


def _require_1d(symbols) -> None:
    if symbols.ndim != 1:
        raise ValueError("Input symbols must be a 1D array.")


class CyclicPrefixScheme(IPrefixScheme):
    """Copy of the last ``prefix_length`` samples in front of each symbol."""

    @property
    def acronym(self) -> str:
        return "CP"

    def add_prefix(self, symbols):
        _require_1d(symbols)
        if len(symbols) < self.prefix_length:
            raise ValueError("Input symbols length must be greater than prefix length.")
        cp = self.prefix_length
        return symbols if cp == 0 else np.concatenate((symbols[len(symbols) - cp:], symbols))

    def remove_prefix(self, symbols):
        _require_1d(symbols)
        if len(symbols) <= self.prefix_length:
            raise ValueError("Input symbols length must be greater than prefix length.")
        return symbols[self.prefix_length:]


class ZeroPaddingPrefixScheme(IPrefixScheme):
    """``prefix_length`` zeros appended; removal folds the tail onto the head (overlap-add)."""

    @property
    def acronym(self) -> str:
        return "ZP"

    def add_prefix(self, symbols):
        _require_1d(symbols)
        return np.concatenate((symbols, np.zeros(self.prefix_length, dtype=symbols.dtype)))

    def remove_prefix(self, symbols):
        _require_1d(symbols)
        if len(symbols) <= self.prefix_length:
            raise ValueError("Input symbols length must be greater than prefix length.")
        n = len(symbols) - self.prefix_length
        if n < self.prefix_length:
            raise ValueError("negative dimensions are not allowed")
        out = np.array(symbols[:n], copy=True)
        out[: self.prefix_length] += symbols[n:]
        return out


class NoPrefixScheme(IPrefixScheme):
    @property
    def acronym(self) -> str:
        return ""

    def add_prefix(self, symbols):
        return symbols

    def remove_prefix(self, symbols):
        return symbols
