#!/bin/bash
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/r06i_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06i_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
AB_REPS=3 AB_STEPS=60 timeout -k 10 900 bash tools/ab.sh "pk0 default" "b c" > gpurun_out/r06i_ab_peak_max.txt 2>&1
rc=$?; cat gpurun_out/r06i_ab_peak_max.txt; exit $rc
