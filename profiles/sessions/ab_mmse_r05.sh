#!/bin/bash
# config-d receiver: the MMSE's batched reciprocal (mb1) against one reciprocal per element (mb0),
# then the N = 2048 adaptive parity cases on mb1
set -o pipefail
export PYTHONUNBUFFERED=1
AB_REPS=2 AB_STEPS=60 bash tools/ab.sh "mb0 mb1" "d" > gpurun_out/r05o_ab.txt 2>&1 || exit $?
OFDM_LIB_VARIANT=mb1 timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py tests/test_gpu_determinism.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "N2048 and adaptive" -s >> gpurun_out/r05o_ab.txt 2>&1
