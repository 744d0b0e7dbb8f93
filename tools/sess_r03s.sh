# round-3 session: nontemporal complex128 TX stores (default) against plain stores (ntoff),
# configs b c d e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03s_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/r03s_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "ntoff default" "b c d e" 2>&1 | grep -v amdgpu.ids
