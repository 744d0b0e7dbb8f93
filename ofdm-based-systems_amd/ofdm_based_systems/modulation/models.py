"""OFDM / SC-OFDM modulators (modulation/models.py:9-91 of the reference).

``OFDMModulator.modulate`` = one GPU launch (IFFT(ortho) + guard interval for all
rows); ``demodulate`` = one launch (guard removal, FFT(ortho), per-row ZF/MMSE).
Custom prefix schemes or equalisers (user subclasses) are honoured by calling
their own ``add_prefix`` / ``remove_prefix`` / ``equalize`` around the GPU FFT.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional, Tuple

import numpy as np
import torch
from numpy.typing import NDArray

from ofdm_based_systems import _backend as B
from ofdm_based_systems.equalization.models import (
    IEqualizator,
    MMSEEqualizator,
    NoEqualizator,
    ZeroForcingEqualizator,
)
from ofdm_based_systems.prefix.models import (
    CyclicPrefixScheme,
    IPrefixScheme,
    NoPrefixScheme,
    ZeroPaddingPrefixScheme,
)


class IModulator(ABC):
    @abstractmethod
    def modulate(self, symbols: NDArray[np.complex128]) -> NDArray[np.complex128]: ...

    @abstractmethod
    def demodulate(self, symbols: NDArray[np.complex128]) -> NDArray[np.complex128]: ...


def guard_of(prefix_scheme: IPrefixScheme) -> Optional[Tuple[int, int]]:
    """(length, kind) of a built-in guard interval; None for a user-defined scheme."""
    if type(prefix_scheme) is CyclicPrefixScheme:
        return prefix_scheme.prefix_length, B.PREFIX_CYCLIC
    if type(prefix_scheme) is ZeroPaddingPrefixScheme:
        return prefix_scheme.prefix_length, B.PREFIX_ZERO
    if type(prefix_scheme) is NoPrefixScheme:
        return 0, B.PREFIX_CYCLIC
    return None


_BUILTIN_EQ = (ZeroForcingEqualizator, MMSEEqualizator, NoEqualizator)


class _DeviceRows:
    """Plan cache + row-block helpers shared by the two modulators."""

    def _plan(self, n: int, cp: int, kind: int) -> B.Plan:
        cache = self.__dict__.setdefault("_plan_cache", {})
        key = (n, cp, kind)
        if key not in cache:
            cache[key] = B.Plan(n_fft=n, cp=cp, prefix=kind)
        return cache[key]

    def _eq_plan(self, n: int, cp: int, kind: int) -> B.Plan:
        eq = self.equalizator
        if type(eq) in _BUILTIN_EQ and type(eq) is not NoEqualizator:
            if np.shape(eq.channel_frequency_response) != (n,):
                raise ValueError("Received symbols and channel frequency response must have the same shape.")
            if isinstance(eq, MMSEEqualizator) and eq.snr_db is None:
                raise ValueError("SNR in dB must be provided to calculate noise variance.")
            return eq.device_plan(cp, kind)
        return self._plan(n, cp, kind)

    @staticmethod
    def _fft_rows(plan: B.Plan, rows: np.ndarray, inverse: bool) -> np.ndarray:
        d = B.to_device(np.ascontiguousarray(rows, dtype=np.complex128))
        B.check(B.lib().ofdm_fft(plan.handle, B.stream_ptr(), B.ptr(d), d.shape[0], int(inverse)))
        return d.cpu().numpy()

    def _demodulate_fft_eq(self, symbols: np.ndarray, n: int) -> np.ndarray:
        """Guard removal + FFT(ortho) + equalisation of every row."""
        y = np.asarray(symbols, dtype=np.complex128)
        g = guard_of(self.prefix_scheme)
        eq = self.equalizator
        builtin_eq = type(eq) in _BUILTIN_EQ
        if g is not None and builtin_eq and y.ndim == 2 and y.shape[1] == n + g[0]:
            plan = self._eq_plan(n, g[0], g[1])
            yd = B.to_device(np.ascontiguousarray(y))
            zd = torch.empty((y.shape[0], n), dtype=torch.complex128, device=yd.device)
            snr = float(eq.snr_db) if eq.snr_db is not None else 0.0
            B.check(B.lib().ofdm_demodulate(plan.handle, B.stream_ptr(), B.ptr(yd), y.shape[0], snr, B.ptr(zd)))
            return zd.cpu().numpy()
        # generic composition: the scheme's own remove_prefix, GPU FFT, the equaliser's own rows
        t = np.array([self.prefix_scheme.remove_prefix(row) for row in y])
        if t.ndim != 2 or t.shape[1] != n:
            raise ValueError(f"Number of symbols must be {n}")
        Y = self._fft_rows(self._plan(n, 0, B.PREFIX_CYCLIC), t, inverse=False)
        if builtin_eq:
            return Y if type(eq) is NoEqualizator else eq.equalize_rows(Y)
        return np.array([eq.equalize(row) for row in Y])


class OFDMModulator(IModulator, _DeviceRows):
    def __init__(self, num_subcarriers: int, prefix_scheme: IPrefixScheme, equalizator: IEqualizator):
        self.num_subcarriers = num_subcarriers
        self.prefix_scheme = prefix_scheme
        self.equalizator = equalizator

    def modulate(self, symbols: NDArray[np.complex128]) -> NDArray[np.complex128]:
        """ifft(rows, norm="ortho") with the guard interval added to every row."""
        n = self.num_subcarriers
        if symbols.shape[1] != n:
            raise ValueError(f"Number of symbols must be {n}")
        X = np.ascontiguousarray(symbols, dtype=np.complex128)
        g = guard_of(self.prefix_scheme)
        if g is None:
            x = self._fft_rows(self._plan(n, 0, B.PREFIX_CYCLIC), X, inverse=True)
            return np.array([self.prefix_scheme.add_prefix(row) for row in x])
        plan = self._plan(n, g[0], g[1])
        Xd = B.to_device(X)
        xd = torch.empty((X.shape[0], n + g[0]), dtype=torch.complex128, device=Xd.device)
        B.check(B.lib().ofdm_modulate(plan.handle, B.stream_ptr(), B.ptr(Xd), X.shape[0], B.ptr(xd)))
        return xd.cpu().numpy()

    def demodulate(self, symbols: NDArray[np.complex128]) -> NDArray[np.complex128]:
        return self._demodulate_fft_eq(symbols, self.num_subcarriers)


class SingleCarrierOFDMModulator(IModulator, _DeviceRows):
    """SC-FDE: guard interval only on transmit; FFT, equalise, IFFT on receive (:58-91)."""

    def __init__(self, prefix_scheme: IPrefixScheme, equalizator: IEqualizator, num_subcarriers: int):
        self.prefix_scheme = prefix_scheme
        self.equalizator = equalizator
        self.num_subcarriers = num_subcarriers

    def modulate(self, symbols: NDArray[np.complex128]) -> NDArray[np.complex128]:
        return np.array([self.prefix_scheme.add_prefix(row) for row in symbols])

    def demodulate(self, symbols: NDArray[np.complex128]) -> NDArray[np.complex128]:
        n = self.num_subcarriers
        Z = self._demodulate_fft_eq(symbols, n)
        return self._fft_rows(self._plan(n, 0, B.PREFIX_CYCLIC), Z, inverse=True)
