#!/bin/bash
# the default bench line (warmup 10) of configs b and c, twice each
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in 1 2; do for c in b c; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-ber-check --no-variant > gpurun_out/warm_$c.json 2>/dev/null || exit $?
  python -c "import json; d=json.load(open('gpurun_out/warm_$c.json')); print($rep, '$c', d['warmup'], '%.4g'%d['value'], '%.4g'%d['value_after_ramp']['value'])"
done; done > gpurun_out/r05u_warm.txt
