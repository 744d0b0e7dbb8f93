# round-3 session: multipath TX symbol groups of 32 / 64 consecutive symbols (ch32 / ch64: one
# regenerated predecessor tail per group) against 16 (base); parity first
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in ch32 ch64; do
OFDM_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -k "(N4096-M256 or N1024-M64-severe or N2048-M0) and f64" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ag_t_$v.txt 2>&1; rc=$?; echo "pytest $v rc=$rc"; tail -2 gpurun_out/r03ag_t_$v.txt; [ $rc -eq 0 ] || exit $rc
done
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base ch32 ch64" "c d e" 2>&1 | grep -v amdgpu.ids
