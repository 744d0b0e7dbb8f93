#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
AB_REPS=2 AB_STEPS=100 AB_ARGS="--precision f64 --no-variant" bash tools/ab.sh "default w3" "c d" > gpurun_out/r04t_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r04t_ab.txt
for v in default w3; do for c in c d; do python -c "import json; d=json.load(open('gpurun_out/ab_${v}_${c}_1.json')); print('$v','$c', d.get('ber'))"; done; done
exit $rc
