#!/bin/bash
# the MMSE scale folded into the slicers' level multiplier (fold, AB_ONLY build of the working tree)
# against the product library (default); then the complex128 MMSE parity cases on fold
set -o pipefail
export PYTHONUNBUFFERED=1
AB_REPS=2 AB_STEPS=60 bash tools/ab.sh "default fold" "c d e" > gpurun_out/r05v_ab.txt 2>&1 || exit $?
OFDM_LIB_VARIANT=fold timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py tests/test_gpu_determinism.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -s \
    -k "(N1024 and severe_multipath and MMSE and f64) or (N2048 and adaptive and f64) or (N4096 and MMSE and f64) or halves or repeat" \
    >> gpurun_out/r05v_ab.txt 2>&1
