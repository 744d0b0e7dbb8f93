"""Multi-rank path of LinkEngine.run on CPU (gloo, world_size 2).

The GPU kernels are replaced by a test double that computes ofdm_tx / ofdm_rx with
the oracle on CPU tensors; everything else -- the symbol sharding, the all-reduce of
the AWGN power statistics between TX and RX, the batched power-pass schedule and the
counter all-reduce -- is the production LinkEngine.run.  The sharded result must equal
the single-process oracle run bit for bit.
"""

import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from conftest import channel

import ofdm_oracle as O
from ofdm_based_systems.engine import LinkEngine, shard


def fx_add(stats: torch.Tensor, p: float) -> None:
    """Add one symbol's sum |y|^2 to an ofdm_stats record the way the kernels do (fx_accum:
    2^-40 fixed point in 32-bit limbs, normalised; power_sum recomputed from the limbs)."""
    a = p * 256.0
    hi = math.floor(a)
    lo = round((a - hi) * 2.0 ** 32)  # round half to even, as rint
    si = stats.view(torch.int64)
    l0, l1 = int(si[3]) + lo, int(si[4]) + hi
    l1, l0 = l1 + (l0 >> 32), l0 & 0xFFFFFFFF
    si[3], si[4] = l0, l1
    stats[0] = l1 * 2.0 ** -8 + l0 * 2.0 ** -40


class OracleEngine(LinkEngine):
    """LinkEngine whose two kernels are computed by the oracle on the CPU (test double)."""

    def __init__(self, N, M, h_raw, cp, eq):
        self.n_fft, self.cp, self.h, self.eq = N, cp, np.asarray(h_raw, np.complex128), eq
        self.ystride = N  # cyclic prefix: the kept samples
        self.b = int(np.log2(M))
        self.bps = N * self.b
        self.adaptive = False
        self.cdtype = torch.complex128
        self.lut = O.qam_lut(M)
        self.hn = O.normalize_h(self.h)
        self.H = np.fft.fft(self.h, N)

        self.streams = {}  # seed -> (bits, nr, ni) standing in for the in-kernel streams

    def device(self):
        return torch.device("cpu")

    def seed_streams(self, seed, S):
        """Throughput-mode stand-in: the double's 'in-kernel' bits and noise of a seed."""
        tx, nz = O.reference_streams(seed, S * self.bps, S * (self.n_fft + self.cp))
        self.streams[seed] = (torch.from_numpy(np.frombuffer(tx, np.uint8).copy()),
                              torch.from_numpy(nz[0]), torch.from_numpy(nz[1]))

    def stream(self):
        return None

    def _ext(self, bits, s):
        """Modulated OFDM symbol s with its prefix (zeros before the stream starts)."""
        N, cp = self.n_fft, self.cp
        if s < 0:
            return np.zeros(N + cp, np.complex128)
        nb = self.bps // 8
        raw = bits[s * nb:(s + 1) * nb].numpy().tobytes()
        X = self.lut[O.bits_to_indices(O.bytes_to_bits(raw), self.b)]
        return O.add_cp(np.fft.ifft(X[None, :], norm="ortho"), cp)[0]

    def tx(self, stream, bits_d, seed, sym0, n_sym, y, stats):
        if bits_d is None:
            bits_d = self.streams[seed][0]
        L = len(self.h)
        for s in range(sym0, sym0 + n_sym):
            ext = self._ext(bits_d, s)
            prev = self._ext(bits_d, s - 1)[len(ext) - (L - 1):] if L > 1 else np.zeros(0)
            full = np.convolve(np.concatenate([prev, ext]), self.hn)[L - 1:L - 1 + len(ext)]
            fx_add(stats, float(np.sum(np.abs(full) ** 2)))
            stats[1] += float(np.sum(np.abs(ext) ** 2))
            stats[2] = max(float(stats[2]), float(np.max(np.abs(ext) ** 2)))
            if y is not None:
                y[s - sym0] = torch.from_numpy(full[self.cp:])

    def rx(self, stream, y, nr, ni, seed, stats, total_samples, snr_db, noise_on, bits_d, sym0, n_sym,
           n_valid, counters, z_out=None, z_keep=0):
        N, cp = self.n_fft, self.cp
        if bits_d is None:
            bits_d, nr, ni = self.streams[seed]
        sigma = np.sqrt(float(stats[0]) / total_samples / 10 ** (snr_db / 10) / 2) if noise_on else 0.0
        nb = self.bps // 8
        for s in range(sym0, sym0 + n_sym):
            v = y[s - sym0].numpy().copy()
            if noise_on:
                g = s * (N + cp) + cp
                v = v + sigma * (nr[g:g + N].numpy() + 1j * ni[g:g + N].numpy())
            Z = O.equalize(np.fft.fft(v[None, :], norm="ortho"), self.H, self.eq, snr_db)[0]
            ridx = O.nn_demap(Z, self.lut)
            tidx = O.bits_to_indices(O.bytes_to_bits(bits_d[s * nb:(s + 1) * nb].numpy().tobytes()), self.b)
            d = ridx ^ tidx
            counters[0] += int(sum(bin(int(x)).count("1") for x in d))
            counters[1] += int(np.count_nonzero(d))


CASE = dict(N=64, M=16, ch="severe_multipath", eq="MMSE", snr=14.0, S=48, seed=5)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, batch, S, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = dict(CASE, S=S)
    h = channel(c["ch"])
    cp = len(h) - 1
    b = int(np.log2(c["M"]))
    tx, nz = O.reference_streams(c["seed"], c["S"] * c["N"] * b, c["S"] * (c["N"] + cp))
    eng = OracleEngine(c["N"], c["M"], h, cp, c["eq"])
    st = eng.run(c["S"], c["snr"], bits=np.frombuffer(tx, np.uint8), normals=nz, group=dist.group.WORLD,
                 batch=batch)
    out[rank] = (st.bit_errors, st.symbol_errors, st.papr_db, st.power_sum)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,batch,S", [(2, None, 48), (2, 5, 48), (3, None, 48),
                                           (4, None, 50), (4, 5, 50), (8, None, 53), (8, 3, 53)])
def test_sharded_engine_matches_single_process_oracle(world, batch, S):
    """world 4 / 8 with S not divisible by the rank count (shards of unequal length, 53 = 6 x 8 + 5)"""
    c = dict(CASE, S=S)
    h = channel(c["ch"])
    cp = len(h) - 1
    b = int(np.log2(c["M"]))
    tx, nz = O.reference_streams(c["seed"], c["S"] * c["N"] * b, c["S"] * (c["N"] + cp))
    ref = O.run_fixed(tx, c["S"] * c["N"] * b, c["N"], c["M"], h, cp, c["eq"], c["snr"], nz)
    assert ref.bit_errors > 0
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), batch, S, out), nprocs=world, join=True)
    for r in range(world):
        be, se, papr, _ = out[r]
        assert (be, se) == (ref.bit_errors, ref.symbol_errors), (r, be, se, ref)
        assert abs(papr - ref.papr_db) < 1e-9
    # every rank holds the power of the single-process run, bit for bit (exact fixed-point sum)
    single = OracleEngine(c["N"], c["M"], h, cp, c["eq"]).run(
        c["S"], c["snr"], bits=np.frombuffer(tx, np.uint8), normals=nz, batch=batch)
    assert {out[r][3] for r in range(world)} == {single.power_sum}


def _pipelined_worker(rank, world, port, S, lanes, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = dict(CASE, S=S)
    h = channel(c["ch"])
    eng = OracleEngine(c["N"], c["M"], h, len(h) - 1, c["eq"])
    seeds = [11, 12, 13]
    for sd in seeds:
        eng.seed_streams(sd, c["S"])
    piped = [p.result() for p in eng.run_pipelined(c["S"], c["snr"], seeds, group=dist.group.WORLD, lanes=lanes)]
    # a y budget below two shards' buffers: the runs go through batched run_async instead
    # (8 symbols per batch: a rank's shard spans several batches at world 2)
    small = [p.result() for p in eng.run_pipelined(c["S"], c["snr"], seeds, group=dist.group.WORLD,
                                                   y_budget=8 * c["N"] * 16, lanes=lanes)]
    serial = [eng.run(c["S"], c["snr"], seed=sd, group=dist.group.WORLD) for sd in seeds]
    out[rank] = ([(r.bit_errors, r.symbol_errors, r.power_sum) for r in piped],
                 [(r.bit_errors, r.symbol_errors, r.power_sum) for r in serial],
                 [(r.bit_errors, r.symbol_errors, r.power_sum) for r in small])
    dist.destroy_process_group()


@pytest.mark.parametrize("world,S,lanes", [(2, 48, 1), (4, 50, 2), (8, 53, 2)])
def test_pipelined_runs_match_serial_runs(world, S, lanes):
    """bench.py's schedule (run k+1's TX enqueued before run k's RX, asynchronous exchanges)
    gives every run the counts and statistics of LinkEngine.run with the same seed, on every
    rank, and those of the single-process oracle; so does its batched fallback when the two
    runs' channel-sample buffers exceed y_budget.  World 4 / 8 with uneven shards, and the
    two-lane schedule of --sweep (on CPU tensors the lanes share the one host stream)."""
    c = dict(CASE, S=S)
    h = channel(c["ch"])
    cp = len(h) - 1
    b = int(np.log2(c["M"]))
    out = mp.Manager().dict()
    mp.spawn(_pipelined_worker, args=(world, _free_port(), S, lanes, out), nprocs=world, join=True)
    for r in range(world):
        piped, serial, small = out[r]
        assert piped == serial, (r, piped, serial)
        assert small == serial, (r, small, serial)
    for k, sd in enumerate([11, 12, 13]):
        tx, nz = O.reference_streams(sd, c["S"] * c["N"] * b, c["S"] * (c["N"] + cp))
        ref = O.run_fixed(tx, c["S"] * c["N"] * b, c["N"], c["M"], h, cp, c["eq"], c["snr"], nz)
        assert out[0][0][k][:2] == (ref.bit_errors, ref.symbol_errors)


def test_shard_covers_range_exactly():
    for n in (0, 1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            parts = [shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert max(hi - lo for lo, hi in parts) - min(hi - lo for lo, hi in parts) <= 1
