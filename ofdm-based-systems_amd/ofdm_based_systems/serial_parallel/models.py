"""Serial <-> parallel layout (serial_parallel/models.py:6-21 of the reference).

Pure layout (row-major views), no arithmetic.  Accepts NumPy arrays and torch
tensors alike, so the GPU path can reshape device buffers without copies.
"""

import numpy as np
from numpy.typing import NDArray


class SerialToParallelConverter:
    @staticmethod
    def to_parallel(data: NDArray[np.complex128], num_streams: int) -> NDArray[np.complex128]:
        """(L,) -> (L / num_streams, num_streams), row-major."""
        if data.ndim != 1:
            raise ValueError("Input data must be a 1D array.")
        if num_streams <= 0:
            raise ValueError("Number of streams must be a positive integer.")
        if data.shape[0] % num_streams:
            raise ValueError("Length of data must be divisible by number of streams.")
        return data.reshape(-1, num_streams)

    @staticmethod
    def to_serial(data: NDArray[np.complex128]) -> NDArray[np.complex128]:
        """(S, n) -> (S * n,), row-major (a copy, like ndarray.flatten)."""
        if data.ndim != 2:
            raise ValueError("Input data must be a 2D array.")
        return data.flatten() if isinstance(data, np.ndarray) else data.reshape(-1).clone()
