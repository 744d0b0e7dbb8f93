"""Multipath channel (channel/models.py:7-62 of the reference).

``transmit`` convolves the whole serial stream with the unit-power CIR on the
GPU (``ofdm_channel``, which also accumulates sum |y|^2 for the noise model) and
adds the noise there too when the noise model is one of this package's.
"""

from __future__ import annotations

import numpy as np
import torch
from numpy.typing import NDArray

from ofdm_based_systems import _backend as B
from ofdm_based_systems.noise.models import AWGNoiseModel, INoiseModel, NoNoiseModel


class ChannelModel:
    def __init__(self, impulse_response: NDArray[np.complex128], snr_db: float,
                 noise_model: INoiseModel = AWGNoiseModel()):
        self._h_raw = np.asarray(impulse_response, dtype=np.complex128)
        self.impulse_response: NDArray[np.complex128] = self.normalize_impulse_response(self._h_raw)
        self.snr_db: float = snr_db
        self.noise_model: INoiseModel = noise_model
        self.frequency_response_cache: dict[int, NDArray[np.complex128]] = {}
        self._plans: dict = {}

    @property
    def order(self) -> int:
        return len(self.impulse_response) - 1

    def normalize_impulse_response(self, impulse_response: NDArray[np.complex128]) -> NDArray[np.complex128]:
        """h / sqrt(sum |h|^2) (channel/models.py:37-44)."""
        h = np.asarray(impulse_response)
        energy = np.sum(np.abs(h) ** 2)
        if energy == 0:
            raise ValueError("Impulse response cannot be all zeros.")
        return h / np.sqrt(energy)

    def _response_plan(self, n_fft: int) -> B.Plan:
        key = ("resp", n_fft)
        if key not in self._plans:
            self._plans[key] = B.Plan(n_fft=n_fft, h_raw=self.impulse_response)
        return self._plans[key]

    def get_frequency_response(self, n_fft: int) -> NDArray[np.complex128]:
        """fft(h, n_fft) of the normalised CIR, computed on the GPU and cached."""
        if n_fft not in self.frequency_response_cache:
            plan = self._response_plan(n_fft)
            H = torch.empty(n_fft, dtype=torch.complex128, device=B.device())
            B.check(B.lib().ofdm_plan_response(plan.handle, B.stream_ptr(), B.ptr(H), None))
            self.frequency_response_cache[n_fft] = H.cpu().numpy()
        return self.frequency_response_cache[n_fft]

    def get_gains(self, n_fft: int) -> NDArray[np.float64]:
        """|H|^2 per subcarrier (np.abs(H)**2 semantics: hypot squared)."""
        plan = self._response_plan(n_fft)
        H = torch.empty(n_fft, dtype=torch.complex128, device=B.device())
        g = torch.empty(n_fft, dtype=torch.float64, device=B.device())
        B.check(B.lib().ofdm_plan_response(plan.handle, B.stream_ptr(), B.ptr(H), B.ptr(g)))
        return g.cpu().numpy()

    @property
    def conv_plan(self) -> B.Plan:
        if "conv" not in self._plans:
            self._plans["conv"] = B.Plan(n_fft=1, h_raw=self._h_raw)
        return self._plans["conv"]

    def convolve_device(self, s: torch.Tensor):
        """(y, sum |y|^2) on the device for a complex128 device vector s."""
        y = torch.empty_like(s)
        ps = torch.zeros(1, dtype=torch.float64, device=s.device)
        B.check(B.lib().ofdm_channel(self.conv_plan.handle, B.stream_ptr(), B.ptr(s), s.numel(), B.ptr(y),
                                     B.ptr(ps)))
        return y, ps

    def transmit(self, signal: NDArray[np.complex128]) -> NDArray[np.complex128]:
        """conv(signal, h)[:len] + noise (channel/models.py:46-62)."""
        if signal.ndim != 1:
            raise ValueError("Signal must be serial (1D array)")
        s = B.to_device(np.asarray(signal, dtype=np.complex128))
        y, ps = self.convolve_device(s)
        if isinstance(self.noise_model, AWGNoiseModel):
            self.noise_model.add_noise_device(y, ps, self.snr_db)
            return y.cpu().numpy()
        if isinstance(self.noise_model, NoNoiseModel):
            return y.cpu().numpy()
        return self.noise_model.add_noise(y.cpu().numpy(), self.snr_db)
