#!/bin/bash
# One GPU-box session: smoke, the GPU test suite (verbose, with the tests' printed bracket
# widths), a bench line.  Every GPU step has its own time limit; anything other than
# pass/fail (a fault, abort, timeout) ends the script.  TAG names the output files.
export PYTHONUNBUFFERED=1
TAG=${TAG:-s}
mkdir -p gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -4 "gpurun_out/${TAG}_$name.log"
    case $rc in 0|1) return 0 ;; *) exit $rc ;; esac
}
[ -z "$NO_SMOKE" ] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ -z "$NO_TESTS" ] && step pytest_gpu ${PYTEST_SECS:-900} python -u -m pytest tests -m gpu -v -s -p no:cacheprovider \
    --timeout 300 --timeout-method thread -rf ${PYTEST_ARGS:-}
[ -z "$NO_BENCH" ] && step bench ${BENCH_SECS:-300} python bench.py ${BENCH_ARGS:-}
exit 0
