# round-3 session: complex128 RX at N <= 1024 with buffer loads of the channel samples (bl: one
# address VGPR, SGPR element offsets; bl4: the same at 4 waves/SIMD, 1024-thread workgroups)
# against global loads (base); parity first
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in bl bl4; do
  OFDM_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -k "(N4096-M256 or N1024-M64) and f64" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ab_t_$v.txt 2>&1; rc=$?; echo "pytest $v rc=$rc"; tail -2 gpurun_out/r03ab_t_$v.txt; [ $rc -eq 0 ] || exit $rc
done
AB_REPS=3 AB_STEPS=60 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base bl bl4" "b" 2>&1 | grep -v amdgpu.ids
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base bl" "c" 2>&1 | grep -v amdgpu.ids
