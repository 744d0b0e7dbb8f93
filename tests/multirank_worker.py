"""Rank program of tests/test_gpu_multirank.py (not a test module): every rank binds device 0
(OFDM_BENCH_DEVICE semantics -- RCCL refuses two ranks on one GPU, so two ranks use gloo; one rank
may use RCCL, argv[3] = "nccl"), runs the complex128 throughput kernels of BASELINE configs (b) and
(c) through LinkEngine's sharded schedules and rank 0 writes the per-run results as JSON."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ofdm-based-systems_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def record(st):
    return [st.bit_errors, st.symbol_errors, st.power_sum.hex(), st.x_power_sum, st.x_peak]


def main():
    out_path, S = sys.argv[1], int(sys.argv[2])
    backend = sys.argv[3] if len(sys.argv) > 3 else "gloo"
    dev = int(os.environ.get("OFDM_BENCH_DEVICE", "0"))
    torch.cuda.set_device(dev)
    if backend == "nccl":  # as bench.py's Runtime binds it
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group(backend)
    g = dist.group.WORLD
    res = {}
    for cfg in ("b", "c"):
        c = bench.CONFIGS[cfg]
        eng = bench.make_engine(c, "f64")
        snr = c[5]
        whole = eng.run(S, snr, seed=3, group=g)
        batched = eng.run(S, snr, seed=3, group=g, batch=S // (2 * dist.get_world_size()) + 7)
        piped = [p.result() for p in eng.run_pipelined(S, snr, [4, 5], group=g)]
        res[cfg] = {"whole": record(whole), "batched": record(batched), "pipelined": [record(p) for p in piped]}
    if dist.get_rank() == 0:
        with open(out_path, "w") as f:
            json.dump({"world": dist.get_world_size(), "backend": dist.get_backend(), "runs": res}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
