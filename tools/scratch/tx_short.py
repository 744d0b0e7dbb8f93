"""Per-symbol time of the config-c complex128 TX at 1e5 against 1e6 symbols per launch (events)."""
import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench
from ofdm_based_systems.engine import new_stats
eng = bench.make_engine(bench.CONFIGS["c"], "f64")
st = eng.stream()
for S, reps in ((1_000_000, 6), (100_000, 40), (50_000, 40), (200_000, 20)):
    y = torch.empty((S, eng.ystride), dtype=eng.cdtype, device="cuda")
    ts = []
    for r in range(reps):
        s = new_stats("cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); eng.tx(st, None, 7 + r, 0, S, y, s); e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    d = sorted(a.elapsed_time(b) for a, b in ts[2:])
    print(S, "median ms %.4f" % d[len(d) // 2], "per 1e5 %.4f" % (d[len(d) // 2] * 1e5 / S), flush=True)
    del y
