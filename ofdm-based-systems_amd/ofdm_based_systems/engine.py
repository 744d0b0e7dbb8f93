"""Fused GPU link engine: the hot path of ``Simulation.run`` (simulation/models.py:454-606).

One :class:`LinkEngine` = one modem configuration (N, prefix, channel, LUTs,
equaliser) held in a libofdm_hip plan.  :meth:`LinkEngine.run` pushes S OFDM
symbols through

    ofdm_tx  : bits -> map -> IFFT(ortho) + CP -> FIR (across symbol boundaries)
               -> kept channel samples y (HBM) + sum|y|^2 / PAPR statistics
    [all-reduce of the statistics across ranks]
    ofdm_rx  : y + AWGN (sigma from the global mean power) -> FFT(ortho) -> ZF/MMSE
               -> slicer -> XOR/popcount against the tx bits -> u64 counters
    [all-reduce of the counters across ranks]

Bit / noise sources:
  * reference mode -- the caller passes the reference's packed PCG64 bytes and its
    legacy-RNG normals (the whole serial stream): integer counts are bit-exact with
    the reference;
  * philox mode    -- bits and noise are generated inside the kernels from a
    counter-based Philox4x32-10 keyed by (seed, global symbol), so nothing but y
    touches HBM and results do not depend on the number of GPUs.

Multi-GPU: symbols [r*S/R, (r+1)*S/R) go to rank r; the only exchanges are one
all-gather of the 40-byte ofdm_stats record per rank (the AWGN power is a whole-stream
mean, noise/models.py:14, kept as an exact fixed-point sum so that sigma does not depend
on the rank count) and one all-reduce of the two u64 counters.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from ofdm_based_systems import _backend as B

DEFAULT_Y_BUDGET = 64 << 30  # bytes of kept channel samples held at once per GPU


@dataclass
class LinkStats:
    bit_errors: int
    symbol_errors: int
    num_ofdm_symbols: int
    power_sum: float      # sum |y|^2 over the whole serial stream (all ranks)
    x_power_sum: float    # sum |x|^2 over the modulated stream incl. prefix
    x_peak: float         # max |x|^2
    samples: int          # S * (N + cp)
    papr_db: float
    received: Optional[np.ndarray] = None
    timings: dict = field(default_factory=dict)


def new_stats(dev) -> torch.Tensor:
    """A zeroed ofdm_stats record (include/ofdm_hip.h): power_sum, x_power_sum, x_peak as
    float64 and the two int64 fixed-point limbs of sum |y|^2, 5 x 8 bytes."""
    return torch.zeros(B.STATS_WORDS, dtype=torch.float64, device=dev)


def combine_stats(stats: torch.Tensor, parts) -> None:
    """Reduce every rank's ofdm_stats record into ``stats`` (the same on every rank): the
    fixed-point power limbs add as integers -- exact, so power_sum and sigma equal the
    single-GPU values bit for bit -- then power_sum is recomputed from them as the kernels do;
    sum |x|^2 adds in rank order, max |x|^2 is the maximum."""
    g = torch.stack(list(parts))                      # (world, 5) float64
    limbs = g.view(torch.int64)[:, 3:5].sum(0)        # exact
    l0 = limbs[0] & 0xFFFFFFFF
    l1 = limbs[1] + (limbs[0] >> 32)
    si = stats.view(torch.int64)
    si[3] = l0
    si[4] = l1
    stats[0] = l1.to(torch.float64) * B.FX_HI + l0.to(torch.float64) * B.FX_LO
    stats[1] = g[:, 1].sum()
    stats[2] = g[:, 2].max()


def shard(n: int, rank: int, world: int) -> tuple:
    """Contiguous [lo, hi) share of n items for one rank."""
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return lo, hi


class LinkEngine:
    def __init__(self, n_fft: int, cp: int, h_raw: np.ndarray, equalizer: int, luts: Sequence[np.ndarray],
                 sc_lut: Optional[np.ndarray] = None, precision: int = B.OFDM_F64,
                 prefix: int = B.PREFIX_CYCLIC, modulator: int = B.MOD_OFDM):
        """prefix: cyclic prefix (or none, cp = 0) or zero padding; modulator: OFDM or
        single-carrier OFDM; non-square constellations (PSK) are decided by
        brute-force nearest point."""
        self.plan = B.Plan(n_fft=n_fft, cp=cp, precision=precision, equalizer=equalizer, luts=list(luts),
                           sc_lut=sc_lut, h_raw=np.asarray(h_raw, np.complex128), prefix=prefix,
                           modulator=modulator)
        self.n_fft = n_fft
        self.cp = cp
        # stored channel samples per OFDM symbol: the post-prefix N, or all N + cp with
        # zero padding (the receiver overlap-adds the guard)
        self.ystride = n_fft + cp if prefix == B.PREFIX_ZERO else n_fft
        self.bps = self.plan.bits_per_ofdm_symbol
        self.adaptive = self.plan.adaptive
        self.cdtype = self.plan.cdtype
        self._lib = B.lib()

    # ------------------------------------------------------------------ helpers
    def device(self) -> torch.device:
        return B.device()

    def stream(self):
        return B.stream_ptr()

    def upload(self, a: np.ndarray) -> torch.Tensor:
        a = np.ascontiguousarray(a)
        if not a.flags.writeable:  # e.g. np.frombuffer(bytes): torch wants a writable array
            a = a.copy()
        return torch.from_numpy(a).to(self.device())

    def valid_bits(self, n_sym: int) -> int:
        """Bits the reference compares: all of them in FIXED mode, whole bytes in adaptive mode
        (AdaptiveConstellationMapper.decode drops a partial byte, constellation/adaptive.py:259-263)."""
        total = n_sym * self.bps
        return (total // 8) * 8 if self.adaptive else total

    @staticmethod
    def _timed(events, name, n_sym, fn):
        if events is None:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        events.append((name, n_sym, e0, e1))

    def tx(self, stream, bits_d, seed, sym0, n_sym, y, stats):
        B.check(self._lib.ofdm_tx(self.plan.handle, stream, B.ptr(bits_d), int(seed), int(sym0), int(n_sym),
                                  B.ptr(y), B.ptr(stats)))

    def rx(self, stream, y, nr, ni, seed, stats, total_samples, snr_db, noise_on, bits_d, sym0, n_sym,
           n_valid, counters, z_out=None, z_keep=0):
        B.check(self._lib.ofdm_rx(self.plan.handle, stream, B.ptr(y), B.ptr(nr), B.ptr(ni), int(seed),
                                  B.ptr(stats), int(total_samples), float(snr_db), int(noise_on), B.ptr(bits_d),
                                  int(sym0), int(n_sym), int(n_valid), B.ptr(counters), B.ptr(z_out),
                                  int(z_keep)))

    def reserve(self, n_sym: int, runs_in_flight: int = 2, group=None, lanes: int = 1) -> None:
        """Allocate, and hand back to torch's caching allocator, the channel-sample buffers of
        ``runs_in_flight`` concurrent runs of n_sym global symbols (run_pipelined keeps two
        alive), so that later runs reuse them instead of paying for a multi-GB hipMalloc; with
        lanes > 1, spread over run_pipelined's lane streams (the allocator pools buffers per
        stream): run k lives on lane k mod lanes, so a lane holds ceil(runs_in_flight / lanes) of
        them at once -- one each with two lanes."""
        if lanes > 1 and self.device().type == "cuda":
            per_lane = -(-runs_in_flight // lanes)
            for st in self.lane_streams(lanes):
                with torch.cuda.stream(st):
                    self.reserve(n_sym, per_lane, group)
            return
        world, rank = 1, 0
        if group is not None:
            import torch.distributed as dist

            world, rank = dist.get_world_size(group), dist.get_rank(group)
        lo, hi = shard(n_sym, rank, world)
        bufs = [torch.empty((max(hi - lo, 1), self.ystride), dtype=self.cdtype, device=self.device())
                for _ in range(runs_in_flight)]
        del bufs

    # ------------------------------------------------------------------ run
    def run(self, n_sym: int, snr_db: float, **kw) -> LinkStats:
        """Simulate global OFDM symbols [0, n_sym) and return the counts (see :meth:`run_async`)."""
        return self.run_async(n_sym, snr_db, **kw).result()

    def run_async(self, n_sym: int, snr_db: float, *, bits: Optional[np.ndarray] = None,
                  normals: Optional[tuple] = None, seed: int = 0, noise_on: bool = True, keep_symbols: int = 0,
                  group=None, y_budget: int = DEFAULT_Y_BUDGET, batch: Optional[int] = None,
                  n_valid_bits: Optional[int] = None, events: Optional[list] = None) -> "PendingLink":
        """Enqueue global OFDM symbols [0, n_sym) (this rank's shard when ``group`` is set) on
        the current stream without waiting for them; :meth:`PendingLink.result` reads the
        counts back.  Back-to-back calls therefore keep the GPU busy while the host prepares
        the next batch.

        bits    : packed tx bytes of the whole run (reference mode) or None (Philox)
        normals : (nr, ni) float64 arrays of length n_sym*(N+cp) (reference mode), or None
                  for Philox noise
        events  : if a list, (kernel, n_symbols, start, end) HIP events are appended around
                  every ofdm_tx / ofdm_rx launch (recorded on the launch stream)
        """
        dev = self.device()
        stream = self.stream()
        world, rank = 1, 0
        if group is not None:
            import torch.distributed as dist

            world, rank = dist.get_world_size(group), dist.get_rank(group)
        lo, hi = shard(n_sym, rank, world)
        mine = hi - lo
        N, cp = self.n_fft, self.cp
        samples = n_sym * (N + cp)
        n_valid = self.valid_bits(n_sym) if n_valid_bits is None else int(n_valid_bits)

        bits_d = None
        if bits is not None:
            need = math.ceil(n_sym * self.bps / 8)
            if len(bits) < need:
                raise ValueError(f"need {need} tx bytes for {n_sym} OFDM symbols, got {len(bits)}")
            bits_d = self.upload(np.asarray(bits, dtype=np.uint8)[: math.ceil(hi * self.bps / 8) + 1])
        nr_d = ni_d = None
        if normals is not None and noise_on:
            nr_d = self.upload(np.asarray(normals[0], np.float64))
            ni_d = self.upload(np.asarray(normals[1], np.float64))

        stats = new_stats(dev)
        counters = torch.zeros(2, dtype=torch.int64, device=dev)
        csize = 8 if self.cdtype == torch.complex64 else 16
        per_batch = batch or max(1, min(mine, y_budget // (self.ystride * csize)))
        keep = min(keep_symbols, mine)
        z_out = torch.empty((keep, N), dtype=self.cdtype, device=dev) if keep else None

        def reduce_stats():
            # one collective on the TX -> RX critical path: every rank gathers all ranks'
            # ofdm_stats records and reduces them (combine_stats), so all ranks hold the
            # statistics -- and sigma -- of a single-GPU run, bit for bit
            # (run with any process group, one rank included: a 1-rank RCCL group exercises the
            # same collectives, tests/test_gpu_multirank.py)
            if group is not None:
                import torch.distributed as dist

                parts = [torch.empty_like(stats) for _ in range(world)]
                dist.all_gather(parts, stats, group=group)
                combine_stats(stats, parts)

        if per_batch >= mine:
            # whole shard resident: one TX, one RX
            y = torch.empty((max(mine, 1), self.ystride), dtype=self.cdtype, device=dev)
            self._timed(events, "ofdm_tx", mine, lambda: self.tx(stream, bits_d, seed, lo, mine, y, stats))
            reduce_stats()
            self._timed(events, "ofdm_rx", mine, lambda: self.rx(
                stream, y, nr_d, ni_d, seed, stats, samples, snr_db, noise_on, bits_d, lo, mine, n_valid,
                counters, z_out, keep))
        else:
            # power pass first (the AWGN power is a whole-stream mean), then TX+RX per batch
            self.tx(stream, bits_d, seed, lo, mine, None, stats)
            reduce_stats()
            scratch = new_stats(dev)
            y = torch.empty((per_batch, self.ystride), dtype=self.cdtype, device=dev)
            for b0 in range(lo, hi, per_batch):
                nb = min(per_batch, hi - b0)
                self.tx(stream, bits_d, seed, b0, nb, y, scratch)
                zk = keep if b0 == lo else 0
                self.rx(stream, y, nr_d, ni_d, seed, stats, samples, snr_db, noise_on, bits_d, b0, nb,
                        n_valid, counters, z_out if zk else None, zk)
        work = None
        if group is not None:
            import torch.distributed as dist

            # off the critical path: the next run's TX does not wait for this reduction;
            # result() waits for it before reading the counters
            work = dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group, async_op=True)
        done = None
        if dev.type == "cuda":
            done = torch.cuda.Event()
            done.record()  # on the launch stream: result() may be called under another stream
        return PendingLink(n_sym, samples, stats, counters, z_out, done, work)


    def lane_streams(self, lanes: int) -> list:
        """The current stream and lanes - 1 more, kept per engine (their allocator pools persist:
        reserve() fills them before a timed region)."""
        if lanes <= 1 or self.device().type != "cuda":
            return [None]
        cur = torch.cuda.current_stream()
        extra = getattr(self, "_lanes", [])
        while len(extra) < lanes - 1:
            extra.append(torch.cuda.Stream())
        self._lanes = extra
        return [cur] + extra[:lanes - 1]

    def run_pipelined(self, n_sym: int, snr_db, seeds, *, group=None,
                      events: Optional[list] = None, y_budget: int = DEFAULT_Y_BUDGET, lanes: int = 1) -> list:
        """Independent throughput-mode runs (one per seed) of global OFDM symbols [0, n_sym),
        software-pipelined across runs: run k+1's TX is enqueued before run k's RX, so with
        several ranks the statistics exchange of run k (the one collective on a run's
        TX -> RX path) is in flight while the GPU transmits run k+1.  Every run is complete
        and its counts are those of :meth:`run_async` with the same seed; returns the
        PendingLink of each run.  Two runs' channel samples are live at once; when they do not
        fit ``y_budget`` the runs go through :meth:`run_async` one after another (batched).

        snr_db: one SNR for every run, or one per seed -- an SNR sweep (the reference's one
        Simulation per SNR point, simulation/models.py:190-211, run in order by main.py:234-239),
        its points pipelined the same way (the SNR enters only the receiver).

        lanes: HIP streams the runs alternate over (run k on lane k mod lanes, each run's TX,
        exchanges and RX in order on its lane): with 2, one run's receiver overlaps the next run's
        transmitter -- the launch tails and the one-workgroup statistics kernel between them of
        short runs (a sweep's points) fill with the other lane's work.  One y buffer per lane."""
        seeds = list(seeds)
        snrs = list(snr_db) if isinstance(snr_db, (list, tuple, np.ndarray)) else [snr_db] * len(seeds)
        if len(snrs) != len(seeds):
            raise ValueError("one SNR per seed")
        dev = self.device()
        stream = self.stream()
        world, rank = 1, 0
        if group is not None:
            import torch.distributed as dist

            world, rank = dist.get_world_size(group), dist.get_rank(group)
        lo, hi = shard(n_sym, rank, world)
        mine = hi - lo
        N, cp = self.n_fft, self.cp
        samples = n_sym * (N + cp)
        n_valid = self.valid_bits(n_sym)
        csize = 8 if self.cdtype == torch.complex64 else 16
        if 2 * max(mine, 1) * self.ystride * csize > y_budget:
            return [self.run_async(n_sym, q, seed=s, group=group, events=events, y_budget=y_budget)
                    for s, q in zip(seeds, snrs)]

        lane_list = self.lane_streams(lanes) if lanes > 1 and dev.type == "cuda" else None

        def on(k):
            """Context of run k's lane (the current stream when not alternating)."""
            import contextlib

            return torch.cuda.stream(lane_list[k % len(lane_list)]) if lane_list else contextlib.nullcontext()

        def tx(k):
            seed = seeds[k]
            with on(k):
                st = self.stream()
                stats = new_stats(dev)
                y = torch.empty((max(mine, 1), self.ystride), dtype=self.cdtype, device=dev)
                self._timed(events, "ofdm_tx", mine, lambda: self.tx(st, None, seed, lo, mine, y, stats))
                work = None
                if group is not None:
                    import torch.distributed as dist

                    parts = [torch.empty_like(stats) for _ in range(world)]
                    work = (dist.all_gather(parts, stats, group=group, async_op=True), parts)
            return seed, y, stats, work

        def rx(state, snr, k):
            with on(k):
                return rx_on(state, snr, self.stream())

        def rx_on(state, snr, stream):
            seed, y, stats, work = state
            if work is not None:  # reduce the gathered statistics (as run_async)
                work[0].wait()
                combine_stats(stats, work[1])
            counters = torch.zeros(2, dtype=torch.int64, device=dev)
            self._timed(events, "ofdm_rx", mine, lambda: self.rx(
                stream, y, None, None, seed, stats, samples, snr, True, None, lo, mine, n_valid, counters))
            red = None
            if group is not None:
                import torch.distributed as dist

                red = dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group, async_op=True)
            done = torch.cuda.Event() if dev.type == "cuda" else None
            if done is not None:
                done.record()
            return PendingLink(n_sym, samples, stats, counters, None, done, red)

        out = []
        cur = tx(0) if seeds else None
        for k in range(len(seeds)):
            nxt = tx(k + 1) if k + 1 < len(seeds) else None
            out.append(rx(cur, snrs[k], k))
            cur = nxt
        return out


class PendingLink:
    """Device-side results of one :meth:`LinkEngine.run_async` call."""

    def __init__(self, n_sym, samples, stats, counters, z_out, done=None, work=None):
        self.n_sym, self.samples = n_sym, samples
        self.stats, self.counters, self.z_out = stats, counters, z_out
        self.done = done
        self.work = work  # the asynchronous counter all-reduce (multi-rank), or None

    def result(self) -> LinkStats:
        if self.done is not None:
            self.done.synchronize()
        if self.work is not None:
            self.work.wait()  # the reduced counters (host-blocking for gloo, stream-ordered for RCCL)
            self.work = None
            if self.counters.is_cuda:
                torch.cuda.current_stream().synchronize()
        st = self.stats.cpu().numpy()
        cnt = self.counters.cpu().numpy()
        samples = self.samples
        avg = st[1] / samples if samples else 0.0
        papr = float(10 * np.log10(st[2] / avg)) if avg > 0 else float("inf")
        z = self.z_out
        return LinkStats(
            bit_errors=int(cnt[0]), symbol_errors=int(cnt[1]), num_ofdm_symbols=self.n_sym,
            power_sum=float(st[0]), x_power_sum=float(st[1]), x_peak=float(st[2]), samples=samples,
            papr_db=papr, received=None if z is None else z.cpu().numpy().reshape(-1),
        )
