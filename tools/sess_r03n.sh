# round-3 session: complex128 window FIR through a row of reals (default) against complex rows
# (cplx): parity, then A/B on configs c d e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03n_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/r03n_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "cplx default" "c d e" 2>&1 | grep -v amdgpu.ids
