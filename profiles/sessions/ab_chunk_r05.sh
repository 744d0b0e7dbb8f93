#!/bin/bash
# multipath TX symbol-group length A/B: OFDM_TX_CHUNK 32 (default build), 64, 128 (each launch picks
# its chunk in [max/2, max], tx_chunk); configs c d e, then the config-c sweep
set -o pipefail
export PYTHONUNBUFFERED=1
AB_REPS=2 AB_STEPS=60 bash tools/ab.sh "default ch64 ch128" "c d e" > gpurun_out/r05n_ab.txt 2>&1 || exit $?
AB_REPS=1 AB_STEPS=3 AB_ARGS="--sweep" bash tools/ab.sh "default ch64 ch128" "c" >> gpurun_out/r05n_ab.txt 2>&1
