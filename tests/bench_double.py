"""Engine factory for running bench.py without a GPU (test double, CPU tests only).

``bench.py --engine-factory bench_double:make_engine`` builds this instead of the HIP
LinkEngine: the production LinkEngine schedule (sharding, statistics exchange, pipelining,
counter reduction) with its two kernels computed by the oracle on CPU tensors
(test_distributed_cpu.OracleEngine), so the bench's rank launch and reporting can be checked
on CPU with gloo.
"""

import os

import numpy as np

from test_distributed_cpu import OracleEngine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class LazyStreamEngine(OracleEngine):
    """OracleEngine whose per-seed 'in-kernel' streams are made on first use."""

    def __init__(self, *a, symbols_hint=64, **kw):
        super().__init__(*a, **kw)
        self.hint = symbols_hint

    def _need(self, seed, n):
        if seed not in self.streams or len(self.streams[seed][0]) * 8 < n * self.bps:
            self.seed_streams(seed, max(n, self.hint))

    def tx(self, stream, bits_d, seed, sym0, n_sym, y, stats):
        if bits_d is None:
            self._need(seed, sym0 + n_sym)
        super().tx(stream, bits_d, seed, sym0, n_sym, y, stats)

    def rx(self, stream, y, nr, ni, seed, stats, total_samples, snr_db, noise_on, bits_d, sym0, n_sym, *rest, **kw):
        if bits_d is None:
            self._need(seed, sym0 + n_sym)
        super().rx(stream, y, nr, ni, seed, stats, total_samples, snr_db, noise_on, bits_d, sym0, n_sym, *rest, **kw)


def make_engine(cfg, precision):
    """The double of bench.make_engine.  CAPACITY_BASED configs (M = 0: config d) run a fixed 16-QAM
    stand-in -- the double checks the bench's rank launch, sweep groups and reporting, not the
    adaptive loading, which the GPU tests hold to the oracle and the reference."""
    N, M, ch, ratio, eq, snr, _ = cfg
    M = M or 16
    h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
    cp = int(ratio * (len(h) - 1))
    return LazyStreamEngine(N, M, h, cp, eq)
