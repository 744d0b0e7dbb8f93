#!/bin/bash
# N = 1024 complex128 receiver grid A/B: OFDM_RX_GRID_ROUNDS 0 (up to kMaxGrid), 2, 3, 4 rounds of
# the resident workgroups; configs b c, then the config-c sweep
set -o pipefail
export PYTHONUNBUFFERED=1
AB_REPS=2 AB_STEPS=60 bash tools/ab.sh "r0 r2 r3 r4" "b c" > gpurun_out/r05k_ab.txt 2>&1 || exit $?
AB_REPS=2 AB_STEPS=3 AB_ARGS="--sweep" bash tools/ab.sh "r0 r2 r3 r4" "c" >> gpurun_out/r05k_ab.txt 2>&1
