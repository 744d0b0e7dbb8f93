#!/bin/bash
# Config (d) two-half N = 2048 transform (fft2048_d2): the parity and full-size tests that run the
# complex128 adaptive kernels at N = 2048, then a same-box A/B against the library before it
# (libofdm_hip_nod2.so).  Every GPU step has its own time limit; a failure ends the script.
export PYTHONUNBUFFERED=1
TAG=${TAG:-r06d}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    "tests/test_gpu_philox_parity.py::test_tx_samples_match_oracle[N2048-M0-Lin-Phoong_P1-MMSE-f64-adaptive=True]" \
    "tests/test_gpu_philox_parity.py::test_tx_samples_match_oracle[N2048-M0-two_ray-ZF-f64-adaptive=True]" \
    "tests/test_gpu_philox_parity.py::test_error_counts_match_oracle[N2048-M0-Lin-Phoong_P1-MMSE-f64-adaptive=True]" \
    "tests/test_gpu_philox_parity.py::test_error_counts_match_oracle[N2048-M0-two_ray-ZF-f64-adaptive=True]" \
    tests/test_gpu_determinism.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "bracket|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
AB_REPS=3 AB_STEPS=40 bash tools/ab.sh "nod2 default" "d" > gpurun_out/${TAG}_ab_d2.txt 2>&1 || { cat gpurun_out/${TAG}_ab_d2.txt; exit 1; }
cat gpurun_out/${TAG}_ab_d2.txt
exit 0
