#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r04u_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04u_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=2 AB_STEPS=100 AB_ARGS="--precision f32 --no-variant" bash tools/ab.sh "default c64old" "b c d e" > gpurun_out/r04u_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r04u_ab.txt
for v in default c64old; do for c in b c d e; do python -c "import json; d=json.load(open('gpurun_out/ab_${v}_${c}_1.json')); print('$v','$c', d.get('ber'))"; done; done
exit $rc
