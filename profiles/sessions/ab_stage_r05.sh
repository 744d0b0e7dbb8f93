#!/bin/bash
# staged workgroup prologue A/B: steady-state configs c d e, then the config-c sweep
set -o pipefail
export PYTHONUNBUFFERED=1
AB_REPS=2 AB_STEPS=60 bash tools/ab.sh "nostg stg stgg1" "c d e" > gpurun_out/r05i_ab.txt 2>&1 || exit $?
AB_REPS=2 AB_STEPS=3 AB_ARGS="--sweep" bash tools/ab.sh "nostg stg stgg1" "c" >> gpurun_out/r05i_ab.txt 2>&1
