#!/bin/bash
# the config-c sweep on 2, 3 and 4 HIP stream lanes (product library)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in 1 2; do for l in 2 3 4; do
  timeout -k 10 200 python bench.py --sweep --steps 3 --warmup 1 --lanes $l --no-cpu-baseline --no-ber-check \
      > gpurun_out/lanes_$l.json 2> gpurun_out/lanes_$l.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/lanes_$l.json')); print($rep, 'lanes', $l, '%.4g'%d['value'], round(d['ms_per_step'],2))"
done; done > gpurun_out/r05q_lanes.txt
