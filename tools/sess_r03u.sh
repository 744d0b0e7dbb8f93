# round-3 session: complex128 window-FIR TX with its outputs transposed through the row for
# whole-line stores (default) against direct lane-contiguous stores (direct); parity first
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03u_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/r03u_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "direct default" "c d e" 2>&1 | grep -v amdgpu.ids
