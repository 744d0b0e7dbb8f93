"""Practical HBM ceilings on this GPU, for reading the fused kernels' roofline fraction.

Times PyTorch's own streaming kernels on buffers the size of one bench launch (1e6 OFDM
symbols x 1024 complex64 = 8.2 GB): a pure write (fill_), a pure read (sum), and a copy.

    python tools/hbm_ceiling.py > gpurun_out/hbm_ceiling.json
"""

import json

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / reps


def main():
    n = 1_000_000 * 1024 * 2  # float32 words of 1e6 complex64 OFDM symbols
    a = torch.empty(n, dtype=torch.float32, device="cuda")
    b = torch.empty(n, dtype=torch.float32, device="cuda")
    a.fill_(1.0)
    nbytes = a.numel() * 4
    out = {"buffer_bytes": nbytes}
    t = timed(lambda: a.fill_(0.5))
    out["write_GBps"] = nbytes / t / 1e9
    t = timed(lambda: a.sum())
    out["read_GBps"] = nbytes / t / 1e9
    t = timed(lambda: b.copy_(a))
    out["copy_GBps"] = 2 * nbytes / t / 1e9
    out["device"] = torch.cuda.get_device_name(0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
