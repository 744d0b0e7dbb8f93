#!/bin/bash
# One driver-shaped bench line of config b on whatever box this call drew (TAG names it): the spread
# of the headline across boxes (same build, same command as the driver's N = 1 run).
export PYTHONUNBUFFERED=1
TAG=${TAG:-r06box}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_b.json 2> gpurun_out/${TAG}_bench_b.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/${TAG}_bench_b.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_b.json')); r=d['roofline']; print('%.4g sym/s'%d['value'], '%.3f ms/step'%d['ms_per_step'], r['bound'], round(r['frac'],3), {k:round(v,3) for k,v in r['avg_launch_ms'].items()})"
