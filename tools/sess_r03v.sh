# round-3 session: complex64 window-FIR TX outputs transposed through the row (default, plain
# stores; ntc64, nontemporal stores) against direct lane-contiguous stores (direct32)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03v_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/r03v_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f32 --no-variant --ramp-seconds 0" bash tools/ab.sh "direct32 default ntc64" "c d e" 2>&1 | grep -v amdgpu.ids
