# round-3 session: exact stream-power limbs computed in float32 in the complex64 kernels (fx32)
# against the double path (base); parity first (complex64 counts + batching-invariant power)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OFDM_LIB_VARIANT=fx32 timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py tests/test_gpu_fullsize.py -k "(N1024-M64 or N4096-M256 or N2048-M0) or fullsize or batch" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03an_t.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03an_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=3 AB_STEPS=60 AB_ARGS="--precision f32 --no-variant --ramp-seconds 0" bash tools/ab.sh "base fx32" "b c" 2>&1 | grep -v amdgpu.ids
