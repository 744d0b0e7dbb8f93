"""bench.py's measurement definitions on CPU: the algorithmic bytes per OFDM symbol against
SURVEY.md 8(d)'s worked values, the configs against BASELINE.json, and the adaptive config's
bit loading (built exactly as Simulation builds it)."""

import json
import os

import numpy as np
import pytest
from conftest import ROOT

import bench


def test_algorithmic_bytes_match_the_survey():
    # B_alg = 2 ceil(bps / 8) + 2 (N + cp) 8 per symbol, split evenly over TX / RX;
    # worked values (b) 17 920 B, (c) 18 032 B, (e) 1024 b + 65 584 B at b = 8
    assert 2 * bench.kernel_bytes_per_symbol(1024, 1024 * 6, 0) == 17920
    assert 2 * bench.kernel_bytes_per_symbol(1024, 1024 * 6, 7) == 18032
    assert 2 * bench.kernel_bytes_per_symbol(4096, 4096 * 8, 3) == 1024 * 8 + 65584


def test_configs_follow_baseline():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert "N_FFT=1024 64-QAM" in base["metric"]
    N, M, ch, ratio, eq, snr, _ = bench.CONFIGS["b"]  # configs[1]: AWGN only, one SNR
    assert (N, M, ch, eq) == (1024, 64, "flat_fading", "NONE")
    N, M, ch, ratio, eq, snr, _ = bench.CONFIGS["c"]  # configs[2]: custom multipath + MMSE
    assert (N, M, ch, eq) == (1024, 64, "severe_multipath", "MMSE")
    N, M, ch, ratio, eq, snr, _ = bench.CONFIGS["d"]  # configs[3]: adaptive, N = 2048
    assert (N, M, eq) == (2048, 0, "MMSE")
    N, M, ch, ratio, eq, snr, _ = bench.CONFIGS["e"]  # configs[4]: N = 4096, up to 256-QAM
    assert (N, M, eq) == (4096, 256, "MMSE")
    for cfg in bench.CONFIGS.values():
        assert os.path.exists(os.path.join(ROOT, "config", "channel_models", cfg[2] + ".npy"))


def test_adaptive_config_orders_follow_the_reference_rule():
    import ofdm_oracle as O

    N, M, ch, ratio, eq, snr, _ = bench.CONFIGS["d"]
    h = np.load(os.path.join(ROOT, "config", "channel_models", ch + ".npy"))
    orders, _, _ = O.adaptive_orders(N, h, snr, 1e-3, True)
    bps = sum(int(np.log2(o)) for o in orders if o > 0)
    assert 0 < bps < 8 * N and all(o == 0 or (o & (o - 1)) == 0 for o in orders)


@pytest.mark.parametrize("gpus", [2, 4])
def test_bench_gpus_flag_launches_ranks(gpus):
    """`bench.py --gpus N` (no torch.distributed environment) launches N ranks itself and
    reports n_gpus N from the process group (gloo, CPU engine double instead of the kernels); the
    line carries the CPU baseline beside the N-rank measurement (north star: 1/2/4/8 GPUs alongside
    the reference CPU path timed on the node's own host cores, in the same run)."""
    import subprocess
    import sys

    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                                         os.path.join(ROOT, "ofdm-based-systems_amd"), env.get("PYTHONPATH", "")])
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--backend", "gloo",
                        "--engine-factory", "bench_double:make_engine", "--config", "b", "--symbols", "3",
                        "--steps", "2", "--warmup", "1", "--cpu-sample", "2", "--no-ber-check", "--no-variant",
                        "--ramp-seconds", "0"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout
    d = json.loads(line[0])
    assert d["n_gpus"] == gpus and d["devices"] == ["cpu"] * gpus
    assert d["config"]["symbols_per_step"] == 3 * gpus and d["scaling"] == "weak"
    assert d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port" and cb["unit"] == "OFDM symbols/s"


def test_bench_one_rank_under_torchrun_takes_the_process_group():
    """A torch.distributed.run launch builds the process group even for one rank (bench.Runtime), so
    one device rehearses the barriers, max-over-ranks timing and gather of a node's run; a plain
    one-process run has none.  CPU engine double, gloo."""
    import socket
    import subprocess
    import sys

    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                                         os.path.join(ROOT, "ofdm-based-systems_amd"), env.get("PYTHONPATH", "")])
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    args = [os.path.join(ROOT, "bench.py"), "--gpus", "1", "--backend", "gloo", "--engine-factory",
            "bench_double:make_engine", "--config", "b", "--symbols", "3", "--steps", "2", "--warmup", "1",
            "--cpu-sample", "2", "--no-ber-check", "--no-variant", "--ramp-seconds", "0"]
    lines = {}
    for name, cmd in (("torchrun", [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                                    "--master-addr=127.0.0.1", f"--master-port={port}"] + args),
                      ("plain", [sys.executable] + args)):
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, (name, r.stderr[-3000:])
        lines[name] = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert lines["torchrun"]["process_group"] == "gloo" and lines["plain"]["process_group"] is None
    for d in lines.values():
        assert d["n_gpus"] == 1 and d["devices"] == ["cpu"] and d["cpu_baseline"]["value"] > 0
    assert lines["torchrun"]["ber"] == lines["plain"]["ber"]


def test_sweep_grid_and_crossing():
    """--sweep: BASELINE configs[2]'s 0..30 dB in 1 dB steps plus SURVEY 8(d)'s 0.25 dB refinement
    over 26..29 dB; the crossing interpolates log10 BER linearly in dB."""
    g = bench.SWEEP_GRID
    assert len(g) == 40 and g[0] == 0.0 and g[-1] == 30.0 and 27.75 in g and 26.25 in g
    assert abs(bench.crossing([20.0, 21.0], [1e-3, 1e-5]) - 20.5) < 1e-12
    assert bench.crossing([20.0, 21.0], [1e-3, 1e-3]) is None


def test_bench_sweep_two_ranks():
    """`bench.py --sweep --gpus 2` (config (c) by default): one step = every point of the sweep, sharded over the ranks,
    pipelined through run_pipelined (one SNR per run); the line carries the per-point BER."""
    import subprocess
    import sys

    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                                         os.path.join(ROOT, "ofdm-based-systems_amd"), env.get("PYTHONPATH", "")])
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--engine-factory", "bench_double:make_engine", "--sweep", "--symbols", "1",
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-ber-check"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["config"]["symbols_per_step"] == 80
    # --sweep without --config measures the sweep BASELINE configs[2] names: config (c)
    assert d["config"]["workload"].startswith("config (c)"), d["config"]["workload"]
    sw = d["sweep"]
    assert sw["points"] == 40 and len(sw["ber"]) == 40 and sw["snr_db"] == bench.SWEEP_GRID
    assert sw["ber"][0] > sw["ber"][-1]  # 0 dB vs 30 dB


def test_bench_sweep_config_e_two_ranks():
    """`bench.py --sweep --config e --gpus 2`: BASELINE configs[4] as config/simulation_settings_waterfilling.json
    runs it -- SNR 10..30 dB by 5 at 16-, 64- and 256-QAM, one engine per order, every point in one step."""
    import subprocess
    import sys

    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                                         os.path.join(ROOT, "ofdm-based-systems_amd"), env.get("PYTHONPATH", "")])
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--engine-factory", "bench_double:make_engine", "--sweep", "--config", "e", "--symbols", "1",
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-ber-check"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert d["n_gpus"] == 2 and d["config"]["symbols_per_step"] == 2 * 15
    assert d["config"]["qam_order"] == [16, 64, 256] and d["config"]["bits_per_ofdm_symbol"] == [4 * 4096, 6 * 4096,
                                                                                                 8 * 4096]
    sw = d["sweep"]
    assert sw["points"] == 15 and sw["snr_db"] == bench.SWEEP_SNRS_E * 3
    assert [p["qam_order"] for p in sw["per_point"]] == [16] * 5 + [64] * 5 + [256] * 5
    assert d["ber_1e-4_crossing_db"] is None


def _bench(args, timeout=900):
    """Run bench.py with the CPU engine double (gloo ranks); returns the JSON line."""
    import subprocess
    import sys

    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                                         os.path.join(ROOT, "ofdm-based-systems_amd"), env.get("PYTHONPATH", "")])
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--backend", "gloo",
                        "--engine-factory", "bench_double:make_engine", "--no-ber-check", "--ramp-seconds", "0"] + args,
                       env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout
    return json.loads(line[0])


@pytest.mark.parametrize("config,sweep", [("b", False), ("c", True), ("d", True), ("e", True)])
def test_bench_eight_ranks_count_what_one_rank_counts(config, sweep):
    """The N = 8 line the driver's scaling run prints, rehearsed with 8 gloo ranks on the CPU engine
    double: n_gpus / devices / symbols per step follow the rank count, the CPU baseline is on the
    line, and with the same global symbols per point (8 ranks x 1 symbol against 1 rank x 8 -- the
    streams are per symbol, the power exchange exact) every point's BER equals the one-rank run's."""
    extra = ["--sweep"] if sweep else ["--no-variant"]
    common = ["--config", config, "--steps", "1", "--warmup", "0", "--cpu-sample", "1"] + extra
    d8 = _bench(["--gpus", "8", "--symbols", "1"] + common)
    d1 = _bench(["--gpus", "1", "--symbols", "8"] + common)
    npts = d8["sweep"]["points"] if sweep else 1
    assert d8["n_gpus"] == 8 and d8["devices"] == ["cpu"] * 8 and d1["n_gpus"] == 1
    assert d8["config"]["symbols_per_step"] == d1["config"]["symbols_per_step"] == 8 * npts
    assert d8["scaling"] == "weak" and d8["value"] > 0
    cb = d8["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
    if sweep:
        assert d8["sweep"]["snr_db"] == d1["sweep"]["snr_db"]
        assert d8["sweep"]["ber"] == d1["sweep"]["ber"]
        assert [p["bits"] for p in d8["sweep"]["per_point"]] == [p["bits"] for p in d1["sweep"]["per_point"]]
    else:
        assert d8["ber"] == d1["ber"]
