#!/bin/bash
# config-d receiver with the next symbol's samples prefetched (pf1) against without (pf0)
set -o pipefail
export PYTHONUNBUFFERED=1
AB_REPS=2 AB_STEPS=60 bash tools/ab.sh "pf0 pf1" "d" > gpurun_out/r05m_ab.txt 2>&1 || exit $?
OFDM_LIB_VARIANT=pf1 timeout -k 10 300 python -u -m pytest tests/test_gpu_determinism.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "d" >> gpurun_out/r05m_ab.txt 2>&1
