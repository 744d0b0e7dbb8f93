# round-3 session: new complex128 parity cases (N = 4096 ZF / no equaliser, N = 2048 adaptive ZF)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -k "f64 and (N4096 or N2048)" -x -v --timeout 120 --timeout-method thread > gpurun_out/r03ak_t.txt 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/r03ak_t.txt | tail -20; [ $rc -eq 0 ] || exit $rc
