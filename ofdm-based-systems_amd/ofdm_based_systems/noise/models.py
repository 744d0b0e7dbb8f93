"""Noise models (noise/models.py:6-27 of the reference).

``AWGNoiseModel`` keeps the reference's random stream: two ``np.random.normal``
draws from NumPy's legacy global generator (real part first).  The power
measurement and the scaled addition run on the GPU (``ofdm_power`` /
``ofdm_awgn``).
"""

from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np
import torch
from numpy.typing import NDArray

from ofdm_based_systems import _backend as B


class INoiseModel(ABC):
    @abstractmethod
    def add_noise(self, signal: NDArray[np.complex128], snr_db: float) -> NDArray[np.complex128]: ...


def reference_normals(shape) -> tuple:
    """The reference's draws: ``normal(size)`` for the real parts, then for the imaginary parts."""
    return np.random.normal(size=shape), np.random.normal(size=shape)


_power_plan = None


def _scratch_plan() -> B.Plan:
    global _power_plan
    if _power_plan is None:
        _power_plan = B.Plan(n_fft=1)
    return _power_plan


class AWGNoiseModel(INoiseModel):
    """y + sqrt(P / snr_lin / 2) (n_re + j n_im), P = mean |y|^2 over the whole signal."""

    def add_noise_device(self, y: torch.Tensor, power_sum: torch.Tensor, snr_db: float) -> torch.Tensor:
        """In-place on a complex128 device vector whose sum |y|^2 is already in ``power_sum``."""
        nr, ni = reference_normals(tuple(y.shape))
        nr_d, ni_d = B.to_device(nr), B.to_device(ni)
        B.check(B.lib().ofdm_awgn(_scratch_plan().handle, B.stream_ptr(), B.ptr(y), y.numel(), B.ptr(nr_d),
                                  B.ptr(ni_d), B.ptr(power_sum), float(snr_db)))
        return y

    def add_noise(self, signal: NDArray[np.complex128], snr_db: float) -> NDArray[np.complex128]:
        sig = np.asarray(signal, dtype=np.complex128)
        y = B.to_device(np.ascontiguousarray(sig).ravel())
        ps = torch.zeros(1, dtype=torch.float64, device=y.device)
        B.check(B.lib().ofdm_power(_scratch_plan().handle, B.stream_ptr(), B.ptr(y), y.numel(), B.ptr(ps)))
        self.add_noise_device(y, ps, snr_db)
        return y.cpu().numpy().reshape(sig.shape)


class NoNoiseModel(INoiseModel):
    def add_noise(self, signal: NDArray[np.complex128], snr_db: float) -> NDArray[np.complex128]:
        return signal
