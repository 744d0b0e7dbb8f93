#!/bin/bash
# Final-build measurements (TAG names them): smoke and the GPU suite, the bench lines of configs
# b-e and the three sweeps, then per config a rocprofv3 kernel trace + PMC bytes (tools/profile.sh)
# and the SQ issue counters (tools/counters.sh).  Every GPU step has its own time limit; a fault,
# abort or timeout ends the script (rc 1 = test failures: recorded, the session goes on).
export PYTHONUNBUFFERED=1
TAG=${TAG:-r06z}
mkdir -p gpurun_out
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -3 "gpurun_out/${TAG}_$name.log" | cut -c1-400
    case $rc in 0|1) return 0 ;; *) exit $rc ;; esac
}
bstep() {  # name, seconds, bench args...: the JSON line to <name>.json, the log to <name>.err
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" python bench.py "$@" > "gpurun_out/${TAG}_$name.json" 2> "gpurun_out/${TAG}_$name.err"
    local rc=$?
    echo "$name rc=$rc"
    [ $rc -eq 0 ] || { tail -3 "gpurun_out/${TAG}_$name.err"; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_$name.json')); r=d['roofline']; print('%.4g sym/s'%d['value'], '%.3f ms/step'%d['ms_per_step'], r['bound'], round(r['frac'],3), {k:round(v,3) for k,v in r['avg_launch_ms'].items()})"
}
if [ -z "$NO_TESTS" ]; then
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    step pytest_gpu 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf
fi
if [ -z "$NO_PROF" ]; then
    # traces, PMC bytes and SQ counters first, condensed into profiles/pmc_summary.json on the box (the
    # same files come back under gpurun_out/ and are condensed again on the CPU side), so the bench
    # lines below carry roofline.traffic and roofline.issue of this build
    for cfg in ${PROF_CONFIGS:-b c d e}; do
        syms=1000000; [ $cfg = d ] && syms=500000; [ $cfg = e ] && syms=250000
        PROF_STEPS=10 bash tools/profile.sh ${TAG}_${cfg}_f64 --config $cfg --precision f64 || exit $?
        bash tools/counters.sh ${TAG}_${cfg}_f64 --config $cfg --precision f64 || exit $?
        python tools/pmc_summary.py gpurun_out/prof_${TAG}_${cfg}_f64 ${TAG}_${cfg}_f64 $cfg $syms f64 > /dev/null || exit $?
        python tools/pmc_summary.py --counters gpurun_out/ctr_${TAG}_${cfg}_f64 ${TAG}_${cfg}_f64 $cfg $syms f64 > /dev/null || exit $?
    done
fi
if [ -z "$NO_BENCH" ]; then
    for cfg in ${BENCH_CONFIGS:-b c d e}; do
        bstep bench_$cfg 300 --config $cfg --steps 20 --warmup 5
    done
    for cfg in ${SWEEP_CONFIGS:-c d e}; do
        bstep sweep_$cfg 300 --sweep --config $cfg --steps 3 --warmup 1
    done
fi
if [ -z "$NO_TAIL" ]; then
    step ber_tail 600 python tools/ber_tail.py --snrs 24 26 27 28 28.5 29 --min-errors 20000 --max-symbols 2000000000
fi
if [ -z "$NO_REFPROF" ]; then
    # which kernels the reference-stream parity test runs: the REF instantiations (..., true>)
    export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/refprof_${TAG} -o ref --output-format csv -- \
        python3 -m pytest tests/test_gpu_ref_streams.py -m gpu -q -p no:cacheprovider > gpurun_out/${TAG}_refprof.log 2>&1
    rc=$?; echo "refprof rc=$rc"; tail -2 gpurun_out/${TAG}_refprof.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
