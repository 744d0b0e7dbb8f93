"""One-tap frequency-domain equalisers (equalization/models.py:8-68 of the reference).

``equalize`` runs on the GPU (``ofdm_equalize``) on one row of N subcarriers
(the reference's per-OFDM-symbol call) or on a (rows, N) block.  The MMSE noise
variance is estimated per row from the received power, as in the reference.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Optional

import numpy as np
import torch
from numpy.typing import NDArray

from ofdm_based_systems import _backend as B


class IEqualizator(ABC):
    KIND = B.EQ_NONE

    def __init__(self, channel_frequency_response: NDArray[np.complex128], snr_db: Optional[float] = None):
        self.channel_frequency_response = channel_frequency_response
        self.snr_db = snr_db

    @abstractmethod
    def equalize(self, received_symbols: NDArray[np.complex128]) -> NDArray[np.complex128]: ...

    def _check_shape(self, y) -> None:
        if np.shape(y) != np.shape(self.channel_frequency_response):
            raise ValueError("Received symbols and channel frequency response must have the same shape.")

    def equalize_rows(self, rows: NDArray[np.complex128]) -> NDArray[np.complex128]:
        """``equalize`` applied to every row of a (S, N) block in one GPU launch."""
        y = np.asarray(rows, dtype=np.complex128)
        if y.ndim != 2 or y.shape[1] != np.shape(self.channel_frequency_response)[0]:
            raise ValueError("Received symbols and channel frequency response must have the same shape.")
        if self.KIND == B.EQ_MMSE and self.snr_db is None:
            raise ValueError("SNR in dB must be provided to calculate noise variance.")
        return self._run(y)

    def device_plan(self, cp: int = 0, prefix: int = B.PREFIX_CYCLIC) -> B.Plan:
        """Plan carrying this equaliser's H (and a guard interval, for OFDMModulator)."""
        key = (cp, prefix)
        plans = self.__dict__.setdefault("_plans", {})
        if key not in plans:
            H = np.asarray(self.channel_frequency_response, dtype=np.complex128)
            plans[key] = B.Plan(n_fft=len(H), cp=cp, prefix=prefix, equalizer=self.KIND, H=H)
        return plans[key]

    def _run(self, received_symbols) -> NDArray[np.complex128]:
        y = np.asarray(received_symbols, dtype=np.complex128)
        rows = 1 if y.ndim == 1 else y.shape[0]
        yd = B.to_device(np.ascontiguousarray(y))
        zd = torch.empty_like(yd)
        snr = 0.0 if self.snr_db is None else float(self.snr_db)
        B.check(B.lib().ofdm_equalize(self.device_plan().handle, B.stream_ptr(), B.ptr(yd), rows, snr, B.ptr(zd)))
        return zd.cpu().numpy()


class ZeroForcingEqualizator(IEqualizator):
    """Y / H, with H == 0 replaced by 1e-10 (equalization/models.py:22-35)."""

    KIND = B.EQ_ZF

    def equalize(self, received_symbols):
        y = np.asarray(received_symbols)
        self._check_shape(y)
        return self._run(y)


class MMSEEqualizator(IEqualizator):
    """Y conj(H) / (|H|^2 + nv), nv = mean|Y|^2 / snr_lin / mean|H|^2 per row (:38-63)."""

    KIND = B.EQ_MMSE

    def calculate_noise_variance(self, received_signal: NDArray[np.complex128]) -> float:
        """Host helper kept for API parity; the GPU path computes nv inside the kernels."""
        if self.snr_db is None:
            raise ValueError("SNR in dB must be provided to calculate noise variance.")
        gain = np.mean(np.abs(self.channel_frequency_response) ** 2)
        if gain == 0:
            return float("inf")
        return float(np.mean(np.abs(received_signal) ** 2) / 10 ** (self.snr_db / 10) / gain)

    def equalize(self, received_symbols):
        if self.snr_db is None:
            raise ValueError("SNR in dB must be provided to calculate noise variance.")
        y = np.asarray(received_symbols)
        self._check_shape(y)
        return self._run(y)


class NoEqualizator(IEqualizator):
    def equalize(self, received_symbols):
        return received_symbols
