# round-3 session: complex128 window-FIR TX at 3 waves per SIMD (fir3: 168 VGPRs, 39-68 dwords
# spilled) against 2 (base: 221 / 249 VGPRs); parity first
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OFDM_LIB_VARIANT=fir3 timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -k "(N4096-M256 or N1024-M64-severe or N2048-M0) and f64" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03af_t.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03af_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base fir3" "c d e" 2>&1 | grep -v amdgpu.ids
