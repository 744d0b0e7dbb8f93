#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
AB_REPS=3 AB_STEPS=100 AB_ARGS="--precision f64 --no-variant" bash tools/ab.sh "default e3" "e" > gpurun_out/r04q_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r04q_ab.txt
for v in default e3; do python -c "import json; d=json.load(open('gpurun_out/ab_${v}_e_1.json')); print('$v', d.get('ber'))"; done
exit $rc
