#!/bin/bash
# One GPU-box session used while iterating: GPU tests (optionally filtered), then optional
# A/B of variant libraries and the per-variant throughput tool.  Every GPU step has its own
# time limit and a failure ends the script.
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_SECS:-600} python -m pytest ${PYTEST_FILES:-tests} -m gpu -q -p no:cacheprovider -x \
    --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$AB_VARIANTS" ]; then bash tools/ab.sh "$AB_VARIANTS" "$AB_CONFIGS" || exit $?; fi
if [ -n "$VARIANTS" ]; then
  timeout -k 10 300 python tools/bench_variants.py --only $VARIANTS > gpurun_out/variants.json 2> gpurun_out/variants.err
  rc=$?; grep -v amdgpu.ids gpurun_out/variants.err | tail -12; exit $rc
fi
