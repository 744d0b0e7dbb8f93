"""The --sweep groups of configs c, d and e on the GPU (bench.measure_sweep in-process, small sizes):
every point of every group is one complete run of its own engine, so its counts equal a plain
LinkEngine.run of that engine with the same seed (the sweep only schedules: pipelining over two
lanes, all groups enqueued before any count is read)."""

import argparse
import os

import pytest

import bench

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["c", "d", "e"])
def test_sweep_groups_count_what_single_runs_count(gpu, name):
    os.environ.pop("WORLD_SIZE", None)
    rt = bench.Runtime("nccl", cpu=False)
    cfg = bench.CONFIGS[name]
    groups = bench.sweep_groups(name, cfg)
    per_gpu = 64
    args = argparse.Namespace(lanes=2, warmup=0, steps=2)
    engines, rec = bench.measure_sweep(rt, args, groups, "f64", per_gpu, bench.make_engine)
    sw = rec["sweep"]
    assert sw["points"] == sum(len(q) for _, q in groups) == len(sw["per_point"])
    assert rec["value"] > 0 and rec["roofline"] is not None
    # point k of group gi in step st ran seed 1e6 gi + 1000 st + k: recount both steps with run()
    i = 0
    for gi, ((gcfg, snrs), eng) in enumerate(zip(groups, engines)):
        for k, q in enumerate(snrs):
            errs = sum(eng.run(per_gpu, q, seed=1_000_000 * gi + 1000 * st + k).bit_errors for st in range(2))
            pt = sw["per_point"][i]
            assert pt["snr_db"] == q and pt["bits"] == eng.valid_bits(per_gpu) * 2
            assert pt["ber"] == errs / pt["bits"], (name, gi, q)
            i += 1
    if name == "e":
        assert [p["qam_order"] for p in sw["per_point"]] == [16] * 5 + [64] * 5 + [256] * 5
        assert sw["bits_per_point"] == [e.valid_bits(per_gpu) * 2 for e in engines]
    elif name == "d":
        assert [p["qam_order"] for p in sw["per_point"]] == ["adaptive"] * 3
    else:  # config (c): BASELINE configs[2]'s 40-point 0..30 dB sweep on one 64-QAM engine
        assert [p["snr_db"] for p in sw["per_point"]] == bench.SWEEP_GRID and len(groups) == 1
        assert [p["qam_order"] for p in sw["per_point"]] == [64] * 40
        assert sw["bits_per_point"] == engines[0].valid_bits(per_gpu) * 2
