#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench.
# Usage (GPU box): bash tools/profile.sh <tag> [bench args, e.g. --config b --precision f64...]
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/prof_$tag
mkdir -p $out
args="--steps ${PROF_STEPS:-5} --warmup 1 --no-cpu-baseline --no-ber-check --no-variant --ramp-seconds 0 $*"
run() {  # name seconds rocprof-args...
    local name=$1 secs=$2; shift 2
    timeout -k 10 $secs rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- python3 bench.py $args \
        > $out/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc"; tail -2 $out/$name.log
    [ $rc -eq 0 ] || exit $rc
}
run trace 300 --kernel-trace --stats
run fetch 300 --pmc FETCH_SIZE
run write 300 --pmc WRITE_SIZE
find $out -name "*.csv" | head -20
