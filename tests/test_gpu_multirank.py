"""The multi-rank path with the real kernels: two ranks share device 0 over gloo
(RCCL refuses two ranks on one GPU; on a node each rank binds its own GPU and the group is RCCL --
the same LinkEngine code).  The whole-stream AWGN power (noise/models.py:14) is the one exchange:
the ranks all-gather their ofdm_stats records and add the fixed-point limbs, so sigma -- and every
decision -- must be bit-identical to the single-process run.  Checked on the complex128 throughput
kernels of configs (b) and (c) at 2 x 1e5 OFDM symbols: one launch per rank, the batched schedule
(power pass + TX/RX per batch) and the pipelined schedule bench.py times; then bench.py --gpus 2
itself (its rank launch, barrier and max-over-ranks timing)."""

import json
import os
import socket
import subprocess
import sys

import pytest
from conftest import ROOT

import bench

pytestmark = pytest.mark.gpu

S = 200_000


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    env = dict(os.environ, OFDM_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    return env


def _launch(args, timeout, nproc=2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}"] + args
    return subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=timeout)


def _record(st):
    return [st.bit_errors, st.symbol_errors, st.power_sum.hex(), st.x_power_sum, st.x_peak]


def test_two_ranks_match_one_rank_bit_for_bit(gpu, tmp_path):
    out = tmp_path / "ranks.json"
    r = _launch([os.path.join(ROOT, "tests", "multirank_worker.py"), str(out), str(S)], timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    got = json.loads(out.read_text())
    assert got["world"] == 2
    for cfg in ("b", "c"):
        c = bench.CONFIGS[cfg]
        eng = bench.make_engine(c, "f64")
        one = _record(eng.run(S, c[5], seed=3))
        piped = [_record(eng.run(S, c[5], seed=sd)) for sd in (4, 5)]
        runs = got["runs"][cfg]
        assert one[0] > 1000, one  # a meaningful error count at the BER 1e-4 point
        # counts and the exact power limbs' value: identical; sum |x|^2 adds in rank order (rel 1e-12)
        for name, rec in (("whole", runs["whole"]), ("batched", runs["batched"])):
            assert rec[:3] == one[:3], (cfg, name, rec, one)
            assert abs(rec[3] - one[3]) <= 1e-12 * one[3] and rec[4] == one[4], (cfg, name, rec, one)
        for rec, ref in zip(runs["pipelined"], piped):
            assert rec[:3] == ref[:3], (cfg, "pipelined", rec, ref)


def test_bench_two_ranks_on_one_gpu(gpu):
    r = _launch([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--symbols", "100000",
                 "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-ber-check", "--no-variant",
                 "--ramp-seconds", "0"], timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["devices"] == [0, 0], d
    assert d["config"]["symbols_per_step"] == 200_000 and d["scaling"] == "weak" and d["value"] > 0
    assert d["dtype"].startswith("c128") and 1e-5 < d["ber"] < 1e-3


def test_bench_one_rank_rccl_runs_the_node_path(gpu):
    """bench.py under torch.distributed.run with one rank: the Runtime a node's N-GPU run builds --
    an RCCL process group bound with device_id, the gloo host group, the barriers and the
    max-over-ranks timing on RCCL, the device gather, the CPU baseline on rank 0 while the host
    group waits -- on the one GPU a box has.  The line reports its process group and the same BER as
    the plain one-process run over the same symbols."""
    common = ["--gpus", "1", "--symbols", "100000", "--steps", "2", "--warmup", "1", "--no-ber-check",
              "--no-variant", "--ramp-seconds", "0", "--cpu-sample", "100"]
    r = _launch([os.path.join(ROOT, "bench.py"), "--backend", "nccl"] + common, timeout=600, nproc=1)
    assert r.returncode == 0, r.stderr[-4000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert d["process_group"] == "nccl" and d["n_gpus"] == 1 and d["devices"] == [0], d
    assert d["value"] > 0 and d["cpu_baseline"]["value"] > 0
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + common, env=_env(), capture_output=True,
                        text=True, timeout=600)
    assert r1.returncode == 0, r1.stderr[-4000:]
    d1 = json.loads([x for x in r1.stdout.splitlines() if x.startswith("{")][0])
    assert d1["process_group"] is None
    assert d["ber"] == d1["ber"] and d["config"]["symbols_per_step"] == d1["config"]["symbols_per_step"]


@pytest.mark.parametrize("config", ["c", "d", "e"])
def test_bench_sweep_two_ranks_on_one_gpu(gpu, config):
    """bench.py --gpus 2 --sweep on device 0 (gloo; the rehearsal of the driver's multi-GPU sweep
    line): every point's BER equals the one-rank sweep's over the same global symbols (2 ranks x S
    against 1 rank x 2S), and the line carries n_gpus / devices of the two ranks."""
    per = {"c": 2000, "d": 1000, "e": 500}[config]
    common = ["--sweep", "--config", config, "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
              "--no-ber-check"]
    r = _launch([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--symbols", str(per)] + common,
                timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    d2 = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    env = _env()
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--symbols", str(2 * per)] + common,
                        env=env, capture_output=True, text=True, timeout=600)
    assert r1.returncode == 0, r1.stderr[-4000:]
    d1 = json.loads([x for x in r1.stdout.splitlines() if x.startswith("{")][0])
    assert d2["n_gpus"] == 2 and d2["devices"] == [0, 0] and d1["n_gpus"] == 1
    assert d2["config"]["symbols_per_step"] == d1["config"]["symbols_per_step"]
    assert d2["sweep"]["snr_db"] == d1["sweep"]["snr_db"]
    assert d2["sweep"]["ber"] == d1["sweep"]["ber"], (d2["sweep"]["ber"], d1["sweep"]["ber"])
    assert d2["roofline"] is not None and d2["value"] > 0


def test_rccl_group_of_one_rank_matches_no_group(gpu, tmp_path):
    """The RCCL branch of the multi-GPU path on the one GPU a box has: one rank in an "nccl" (RCCL)
    process group bound with device_id, as bench.py binds every rank of a node.  LinkEngine runs its
    collectives for any group (engine.py: the device all-gather of the ofdm_stats records, the exact
    limb reduction, the asynchronous counter all-reduce -- in run_async and in the pipelined
    schedule), so this executes RCCL on the device tensors the 8-GPU run exchanges; the counts and
    the power bits must equal the group-less run's."""
    out = tmp_path / "rccl.json"
    r = _launch([os.path.join(ROOT, "tests", "multirank_worker.py"), str(out), str(S), "nccl"], timeout=600, nproc=1)
    assert r.returncode == 0, r.stderr[-4000:]
    got = json.loads(out.read_text())
    assert got["world"] == 1 and got["backend"] == "nccl"
    for cfg in ("b", "c"):
        c = bench.CONFIGS[cfg]
        eng = bench.make_engine(c, "f64")
        one = _record(eng.run(S, c[5], seed=3))
        piped = [_record(eng.run(S, c[5], seed=sd)) for sd in (4, 5)]
        runs = got["runs"][cfg]
        assert runs["whole"] == one and runs["batched"] == one, (cfg, runs, one)
        assert runs["pipelined"] == piped, (cfg, runs["pipelined"], piped)
