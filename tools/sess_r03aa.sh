# round-3 session: complex128 multipath TX mapping through the two axis tables of the square-QAM
# LUT (sep) against the complex LUT (base); parity first
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in sep; do
  OFDM_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -k "(N4096-M256 or N1024-M64-severe_multipath-MMSE) and f64" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03aa_t_$v.txt 2>&1; rc=$?; echo "pytest $v rc=$rc"; tail -2 gpurun_out/r03aa_t_$v.txt; [ $rc -eq 0 ] || exit $rc
done
AB_REPS=3 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base sep" "c e" 2>&1 | grep -v amdgpu.ids
