# round-3 session: complex128 flat TX (config b) in 768-thread workgroups at 3 waves/SIMD (tx3, no
# spills) against 1024 threads at 4 (base, 5 dwords spilled)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OFDM_LIB_VARIANT=tx3 timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -k "N1024-M64-flat and f64" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ap_t.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03ap_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=3 AB_STEPS=60 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base tx3" "b" 2>&1 | grep -v amdgpu.ids
