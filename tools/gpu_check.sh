#!/bin/bash
# One GPU-box session: smoke, the GPU test suite, a short bench.  Every GPU step has its
# own time limit; anything other than pass/fail (a fault, abort, timeout) ends the script.
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -5 "gpurun_out/$name.log"
    case $rc in 0|1) return 0 ;; *) exit $rc ;; esac
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu ${PYTEST_SECS:-700} python -m pytest tests -m gpu -q -p no:cacheprovider -rf ${PYTEST_ARGS:-}
step bench ${BENCH_SECS:-240} python bench.py --steps 5 --warmup 1 ${BENCH_ARGS:-}
