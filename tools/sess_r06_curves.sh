#!/bin/bash
# Stream-v3 BER curves of configs b-e against the reference-stream path (tools/ber_curve.py, complex128)
# and the d / e sweeps with as many timed steps as round 5 measured them (10, warmup 2).  Every GPU step
# has its own time limit; a fault, abort or timeout ends the script.
export PYTHONUNBUFFERED=1
TAG=${TAG:-r06c}
mkdir -p gpurun_out
for cfg in b c d e; do
    timeout -k 10 300 python tools/ber_curve.py --config $cfg --precision f64 > gpurun_out/${TAG}_ber_curve_${cfg}_f64.json \
        2> gpurun_out/${TAG}_ber_curve_${cfg}.err || { echo "curve $cfg rc=$?"; tail -3 gpurun_out/${TAG}_ber_curve_${cfg}.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_ber_curve_${cfg}_f64.json')); print('$cfg', d.get('ber_1e-4_crossing_db'), d.get('delta_db_at_1e-4'), round(d['wall_s'],1))"
done
for cfg in d e; do
    timeout -k 10 300 python bench.py --sweep --config $cfg --steps 10 --warmup 2 > gpurun_out/${TAG}_sweep_$cfg.json \
        2> gpurun_out/${TAG}_sweep_$cfg.err || { echo "sweep $cfg rc=$?"; tail -3 gpurun_out/${TAG}_sweep_$cfg.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_sweep_$cfg.json')); print('sweep $cfg', '%.4g'%d['value'], d['ms_per_step'])"
done
# the single point on one HIP stream lane (the bench default) against two and three (run k+1's TX
# beside run k's RX), configs b and c, interleaved twice
for rep in 1 2; do for cfg in b c; do for lanes in 1 2 3; do
    timeout -k 10 180 python bench.py --config $cfg --lanes $lanes --steps 40 --warmup 5 --no-cpu-baseline --no-ber-check \
        --no-variant > gpurun_out/${TAG}_lanes_${cfg}_${lanes}_$rep.json 2> gpurun_out/${TAG}_lanes.err || { echo "lanes rc=$?"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_lanes_${cfg}_${lanes}_$rep.json')); print('lanes', '$cfg', $lanes, $rep, '%.4g'%d['value'], round(d['ms_per_step'],3))"
done; done; done
exit 0
