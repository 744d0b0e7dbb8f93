"""Constellation mappers (constellation/models.py:11-474 of the reference).

The LUT itself is host setup (a few hundred constants, built exactly as the
reference builds it so it is bit-identical).  ``encode`` / ``decode`` /
``NNClassifier.classify`` run on the GPU through libofdm_hip
(``ofdm_map`` / ``ofdm_demap`` / ``ofdm_nn_classify``).
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from functools import cached_property
from io import BytesIO
from typing import BinaryIO, Dict, List, Tuple, Type, Union

import numpy as np
import torch
from numpy.typing import NDArray

from ofdm_based_systems import _backend as B


# --------------------------------------------------------------------------- classifiers
class ISymbolClassifier(ABC):
    @abstractmethod
    def classify(self, constellation: NDArray[np.complex128], symbols: NDArray[np.complex128]
                 ) -> NDArray[np.complex128]: ...


def nearest_indices(constellation: NDArray[np.complex128], symbols) -> np.ndarray:
    """argmin_m |z - C_m| (first index on ties) on the GPU (constellation/models.py:23-26)."""
    lut = np.ascontiguousarray(np.asarray(constellation, dtype=np.complex128))
    z = np.ascontiguousarray(np.asarray(symbols, dtype=np.complex128).ravel())
    handle = B.lib()
    lut_d = B.to_device(lut.view(np.float64))
    z_d = B.to_device(z)
    idx_d = torch.empty(len(z), dtype=torch.int64, device=B.device())
    B.check(handle.ofdm_nn_classify(B.stream_ptr(), B.ptr(lut_d), len(lut), B.ptr(z_d), len(z),
                                    B.ptr(idx_d)))
    return idx_d.cpu().numpy()


class NNClassifier(ISymbolClassifier):
    """Nearest-neighbour decision over the whole LUT (brute force, GPU)."""

    def classify(self, constellation, symbols):
        return np.asarray(constellation)[nearest_indices(constellation, symbols)]


# --------------------------------------------------------------------------- word coders
class IWordCoder(ABC):
    def __init__(self, bits_per_word: int):
        self.bits_per_word = bits_per_word

    @property
    def size(self) -> int:
        return 1 << self.bits_per_word

    def _check(self, w: int, what: str) -> None:
        if not 0 <= w < self.size:
            raise ValueError(f"{what} must be in range [0, {self.size})")

    @abstractmethod
    def encode(self, word: int) -> int: ...

    @abstractmethod
    def decode(self, coded_word: int) -> int: ...

    @abstractmethod
    def reorder_constellation(self, constellation: NDArray[np.complex128], constellation_name: str
                              ) -> NDArray[np.complex128]: ...


class NoWordCoder(IWordCoder):
    def encode(self, word: int) -> int:
        self._check(word, "Word")
        return word

    def decode(self, coded_word: int) -> int:
        self._check(coded_word, "Coded word")
        return coded_word

    def reorder_constellation(self, constellation, constellation_name):
        return constellation


class GrayWordCoder(IWordCoder):
    """Binary-reflected Gray code; QAM LUTs additionally get the zig-zag row order
    of constellation/models.py:94-109 (odd rows of the index space reversed)."""

    @cached_property
    def gray_table(self) -> Dict[int, int]:
        return {w: w ^ (w >> 1) for w in range(self.size)}

    @cached_property
    def inverse_gray_table(self) -> Dict[int, int]:
        return {g: w for w, g in self.gray_table.items()}

    def encode(self, word: int) -> int:
        self._check(word, "Word")
        return self.gray_table[word]

    def decode(self, coded_word: int) -> int:
        self._check(coded_word, "Gray word")
        return self.inverse_gray_table[coded_word]

    def reorder_constellation(self, constellation, constellation_name):
        if constellation_name != QAMConstellationMapper.__name__:
            return constellation
        side = int(np.sqrt(len(constellation)))
        grid = np.array(constellation).reshape(side, side)
        grid[1::2] = grid[1::2, ::-1]
        return grid.reshape(-1)


# --------------------------------------------------------------------------- bits helpers
def _stream_bytes(bits: Union[BinaryIO, List[int]], b: int) -> Tuple[np.ndarray, int]:
    """(packed bytes, number of symbols) for encode's two input kinds.

    Stream input is zero-padded to whole symbols (constellation/models.py:235-237);
    a bit list is used as is and must hold whole symbols (the reshape at :240).
    """
    if isinstance(bits, list):
        arr = np.asarray(bits, dtype=np.uint8)
        if len(arr) % b:
            raise ValueError(f"cannot reshape array of size {len(arr)} into shape ({b})")
        return np.packbits(arr), len(arr) // b
    data = np.frombuffer(bits.read(), dtype=np.uint8)
    return data, -(-8 * len(data) // b)


class IConstellationMapper(ABC):
    constellation: NDArray[np.complex128]
    constellation_map: Dict[Tuple[float, float], int]

    def __init__(self, order: int, word_coder: Type[IWordCoder] = GrayWordCoder,
                 classifier: Type[ISymbolClassifier] = NNClassifier):
        self.order = order
        self.word_coder = word_coder(bits_per_word=self.bits_per_symbol)
        self.classifier = classifier()

    @property
    @abstractmethod
    def constellation_name(self) -> str: ...

    @property
    @abstractmethod
    def bits_per_symbol(self) -> int: ...

    @abstractmethod
    def encode(self, bits: BinaryIO) -> NDArray[np.complex128]: ...

    @abstractmethod
    def decode(self, symbols: NDArray[np.complex128] | np.complex128) -> BinaryIO: ...

    @classmethod
    @abstractmethod
    def calculate_bit_loading_order(cls, ser: float, snr: float) -> int: ...


class _LutMapper(IConstellationMapper):
    """encode/decode through a libofdm_hip plan holding this mapper's LUT."""

    @property
    def device_plan(self) -> B.Plan:
        plan = getattr(self, "_plan", None)
        if plan is None:
            plan = B.Plan(n_fft=1, luts=[self.constellation])
            self._plan = plan
        return plan

    def encode(self, bits: Union[BinaryIO, List[int]]) -> NDArray[np.complex128]:
        b = self.bits_per_symbol
        data, n = _stream_bytes(bits, b)
        plan = self.device_plan
        out = torch.empty(n, dtype=torch.complex128, device=B.device())
        src = B.to_device(data) if len(data) else None
        B.check(B.lib().ofdm_map(plan.handle, B.stream_ptr(), B.ptr(src), len(data), n, B.ptr(out)))
        return out.cpu().numpy()

    def decode(self, symbols) -> BinaryIO:
        z = (np.array([symbols], dtype=np.complex128) if np.isscalar(symbols)
             else np.asarray(symbols, dtype=np.complex128).ravel())
        b = self.bits_per_symbol
        if not isinstance(self.classifier, NNClassifier):
            # a user-supplied classifier: classify with it, index through the map (:259-267)
            pts = self.classifier.classify(self.constellation, z)
            idx = np.array([self.constellation_map[(float(p.real), float(p.imag))] for p in pts],
                           dtype=np.int64)
            bits = ((idx[:, None] >> np.arange(b - 1, -1, -1)) & 1).astype(np.uint8).ravel()
            return BytesIO(np.packbits(bits).tobytes())
        nbytes = -(-len(z) * b // 8)
        out = torch.empty(nbytes, dtype=torch.uint8, device=B.device())
        zd = B.to_device(z)
        B.check(B.lib().ofdm_demap(self.device_plan.handle, B.stream_ptr(), B.ptr(zd), len(z), B.ptr(out)))
        return BytesIO(out.cpu().numpy().tobytes())

    def _index_map(self) -> Dict[Tuple[float, float], int]:
        return {(float(p.real), float(p.imag)): i for i, p in enumerate(self.constellation)}


class QAMConstellationMapper(_LutMapper):
    """Square M-QAM, unit mean energy, Gray-coded with the reference's zig-zag order."""

    def __init__(self, order: int, word_coder: Type[IWordCoder] = GrayWordCoder,
                 classifier: Type[ISymbolClassifier] = NNClassifier):
        super().__init__(order, word_coder, classifier)
        self.validate_order()
        self.constellation, self.constellation_map = self.generate_constellation()

    @property
    def constellation_name(self) -> str:
        return f"{self.order}-QAM"

    @property
    def bits_per_symbol(self) -> int:
        return int(np.log2(self.order))

    def validate_order(self) -> None:
        if int(np.sqrt(self.order)) ** 2 != self.order:
            raise ValueError("Order must be a perfect square (e.g., 4, 16, 64).")

    def generate_constellation(self):
        """LUT[i] = grid[coder.encode(i)] over the row-major grid (top row = +Q,
        left = -I), reordered by the coder, scaled to unit mean |C|^2
        (constellation/models.py:180-218)."""
        side = int(np.sqrt(self.order))
        levels = np.arange(1 - side, side, 2)
        grid = (levels[None, :] + 1j * levels[::-1, None]).reshape(-1)
        lut = np.array([grid[self.word_coder.encode(i)] for i in range(self.order)], dtype=np.complex128)
        lut = self.word_coder.reorder_constellation(lut, QAMConstellationMapper.__name__)
        lut = lut / np.sqrt(np.mean(np.abs(lut) ** 2))
        self.constellation = lut
        return lut, self._index_map()

    @classmethod
    def calculate_bit_loading_order(cls, ser: float, snr: float) -> int:
        """Gap approximation (constellation/models.py:297-321): Gamma = Q^-1(SER/4)^2 / 3,
        b = round(log2(1 + snr / Gamma)), made even by subtracting 1, 0 if <= 0."""
        from scipy.stats import norm

        gap = norm.isf(ser / 4) ** 2 / 3
        b = int(np.round(np.log2(1 + snr / gap)))
        b -= b % 2
        return 0 if b <= 0 else 2 ** b


class PSKConstellationMapper(_LutMapper):
    """M-PSK on the unit circle, Gray-coded (constellation/models.py:324-474)."""

    def __init__(self, order: int, word_coder: Type[IWordCoder] = GrayWordCoder,
                 classifier: Type[ISymbolClassifier] = NNClassifier):
        super().__init__(order, word_coder, classifier)
        self.validate_order()
        self.constellation, self.constellation_map = self.generate_constellation()

    @property
    def constellation_name(self) -> str:
        return f"{self.order}-PSK"

    @property
    def bits_per_symbol(self) -> int:
        return int(np.log2(self.order))

    def validate_order(self) -> None:
        b = np.log2(self.order)
        if b != int(b) or self.order < 2:
            raise ValueError("PSK order must be a power of 2 (e.g., 2, 4, 8, 16).")

    def generate_constellation(self):
        """LUT[coder.encode(i)] = exp(2 pi j i / M) (constellation/models.py:361-369)."""
        pts = np.exp(1j * 2 * np.pi * np.arange(self.order) / self.order)
        lut = np.zeros(self.order, dtype=np.complex128)
        for i in range(self.order):
            lut[self.word_coder.encode(i)] = pts[i]
        lut = self.word_coder.reorder_constellation(lut, PSKConstellationMapper.__name__)
        self.constellation = lut
        return lut, self._index_map()

    @classmethod
    def calculate_bit_loading_order(cls, ser: float, snr: float) -> int:
        from scipy.stats import norm

        q = norm.isf(ser / 2)
        g_star = q ** 2 / (2 * np.pi ** 2)
        gap = np.sqrt(snr * g_star) / (1 - np.sqrt(g_star / (snr + 1e-10)))
        b = int(np.floor(np.log2(1 + snr / (gap + 1e-10)) + 1e-10))
        return 0 if b <= 0 else 2 ** b
