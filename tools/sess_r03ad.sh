# round-3 session: complex128 adaptive RX at N = 2048 (config d) with one symbol per 128-thread
# workgroup and the equaliser coefficients buffer-loaded after the FFT (dsolo) against four symbols
# per 512-thread workgroup with the LDS table (base); parity first
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OFDM_LIB_VARIANT=dsolo timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -k "N2048-M0 and f64" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ad_t.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03ad_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=3 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base dsolo" "d" 2>&1 | grep -v amdgpu.ids
