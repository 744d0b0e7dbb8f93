# round-3 session: config e RX, one symbol per 256-thread workgroup at 3 waves/SIMD with the
# equaliser coefficients buffer-loaded after the FFT (solo3b), plus batched MMSE reciprocals
# (solo3bb), against the current kernels (base); parity of each variant first
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in solo3b solo3bb; do
  OFDM_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -k "(N4096-M256 or N1024-M64-severe_multipath-MMSE) and f64" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03y_t_$v.txt 2>&1; rc=$?; echo "pytest $v rc=$rc"; tail -2 gpurun_out/r03y_t_$v.txt; [ $rc -eq 0 ] || exit $rc
done
AB_REPS=3 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base solo3b solo3bb" "e" 2>&1 | grep -v amdgpu.ids
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base solo3bb" "c" 2>&1 | grep -v amdgpu.ids
