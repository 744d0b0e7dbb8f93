"""Per-subcarrier constellation orders (constellation/adaptive.py:16-329 of the reference).

One libofdm_hip plan carries every distinct LUT plus a per-subcarrier table
(LUT id, bits, bit offset inside the OFDM symbol), so encode / decode are single
GPU launches instead of the reference's per-(symbol, subcarrier) Python calls.
"""

from __future__ import annotations

from io import BytesIO
from typing import BinaryIO, Dict, List, Tuple, Type, Union

import numpy as np
import torch
from numpy.typing import NDArray

from ofdm_based_systems import _backend as B
from ofdm_based_systems.constellation.models import IConstellationMapper


class AdaptiveConstellationMapper(IConstellationMapper):
    """Subcarrier k uses ``constellation_orders[k]`` (0 = unused, carries 0+0j).

    Bits of one OFDM symbol are laid out subcarrier-major: subcarrier k takes the
    next ``log2(order_k)`` bits (constellation/adaptive.py:178-199).
    """

    def __init__(self, constellation_orders: NDArray[np.int64], base_mapper_class: Type[IConstellationMapper],
                 num_subcarriers: int):
        if len(constellation_orders) != num_subcarriers:
            raise ValueError(
                f"constellation_orders length ({len(constellation_orders)}) "
                f"must match num_subcarriers ({num_subcarriers})")
        self.constellation_orders = np.array(constellation_orders, dtype=np.int64)
        self.base_mapper_class = base_mapper_class
        self.num_subcarriers = num_subcarriers
        self.mappers: Dict[int, Tuple[List[int], IConstellationMapper]] = {}
        for order in np.unique(self.constellation_orders):
            if order > 0:
                idx = np.flatnonzero(self.constellation_orders == order).tolist()
                self.mappers[int(order)] = (idx, base_mapper_class(order=int(order)))
        self.bits_per_subcarrier = np.array(
            [int(np.log2(o)) if o > 0 else 0 for o in self.constellation_orders], dtype=np.int64)
        pts = [p for o in sorted(self.mappers) for p in self.mappers[o][1].constellation.tolist()]
        self.constellation = np.unique(np.array(pts, dtype=np.complex128))
        self.constellation_map = {(float(p.real), float(p.imag)): i for i, p in enumerate(self.constellation)}

    @property
    def order(self) -> int:
        return int(np.max(self.constellation_orders))

    @property
    def constellation_name(self) -> str:
        used = np.unique(self.constellation_orders[self.constellation_orders > 0])
        base = self.base_mapper_class.__name__.replace("ConstellationMapper", "")
        if len(used) == 0:
            return "No-Transmission"
        if len(used) == 1:
            return f"{int(used[0])}-{base}"
        return f"Adaptive-{int(used.min())}-to-{int(used.max())}-{base}"

    @property
    def bits_per_symbol(self) -> int:
        return int(np.max(self.bits_per_subcarrier))

    def get_bits_per_subcarrier(self) -> NDArray[np.int64]:
        return self.bits_per_subcarrier

    def get_constellation_orders(self) -> NDArray[np.int64]:
        return self.constellation_orders

    def lut_tables(self):
        """(LUT list, per-subcarrier LUT id with -1 = inactive) for a libofdm_hip plan."""
        orders = sorted(self.mappers)
        luts = [self.mappers[o][1].constellation for o in orders]
        pos = {o: i for i, o in enumerate(orders)}
        sc = np.array([pos.get(int(o), -1) if o > 0 else -1 for o in self.constellation_orders], np.int32)
        return luts, sc

    @property
    def device_plan(self) -> B.Plan:
        plan = getattr(self, "_plan", None)
        if plan is None:
            luts, sc = self.lut_tables()
            plan = B.Plan(n_fft=self.num_subcarriers, luts=luts, sc_lut=sc)
            self._plan = plan
        return plan

    def encode(self, bits: Union[BinaryIO, List[int]]) -> NDArray[np.complex128]:
        if isinstance(bits, list):
            arr = np.asarray(bits, dtype=np.uint8)
            nbits = len(arr)
            data = np.packbits(arr)
        else:
            data = np.frombuffer(bits.read(), dtype=np.uint8)
            nbits = 8 * len(data)
        per_sym = int(self.bits_per_subcarrier.sum())
        if per_sym == 0:
            raise ValueError("No active subcarriers (all orders are zero)")
        if nbits % per_sym:
            raise ValueError(f"Bits length ({nbits}) must be multiple of bits_per_symbol ({per_sym})")
        n_out = (nbits // per_sym) * self.num_subcarriers
        out = torch.empty(n_out, dtype=torch.complex128, device=B.device())
        src = B.to_device(data) if len(data) else None
        B.check(B.lib().ofdm_map(self.device_plan.handle, B.stream_ptr(), B.ptr(src), len(data), n_out,
                                 B.ptr(out)))
        return out.cpu().numpy()

    def decode(self, symbols) -> BinaryIO:
        z = (np.array([symbols], dtype=np.complex128) if np.isscalar(symbols)
             else np.asarray(symbols, dtype=np.complex128).ravel())
        if len(z) % self.num_subcarriers:
            raise ValueError(
                f"Symbols length ({len(z)}) must be multiple of num_subcarriers ({self.num_subcarriers})")
        nbytes = (len(z) // self.num_subcarriers) * int(self.bits_per_subcarrier.sum()) // 8
        out = torch.empty(max(nbytes, 0), dtype=torch.uint8, device=B.device())
        zd = B.to_device(z)
        B.check(B.lib().ofdm_demap(self.device_plan.handle, B.stream_ptr(), B.ptr(zd), len(z), B.ptr(out)))
        return BytesIO(out.cpu().numpy().tobytes())

    def calculate_bit_loading_order(self, ser: float, snr: float) -> int:
        raise NotImplementedError("This method is not implemented in AdaptiveConstellationMapper.")


def calculate_constellation_orders(capacity: NDArray[np.float64], min_order: int, max_order: int,
                                   scaling_factor: float, base_mapper_class: Type[IConstellationMapper]
                                   ) -> NDArray[np.int64]:
    """Capacity -> power-of-two orders (constellation/adaptive.py:271-329): scale, clip to
    [0, log2 max], even bits for QAM (floor for PSK), below log2 min -> 0."""
    from ofdm_based_systems.constellation.models import QAMConstellationMapper

    b = np.clip(np.asarray(capacity) * scaling_factor, 0, np.log2(max_order))
    b = b // 2 * 2 if base_mapper_class == QAMConstellationMapper else np.floor(b)
    b = np.where(b < np.log2(min_order), 0, b)
    return np.where(b > 0, 2 ** b, 0).astype(np.int64)
