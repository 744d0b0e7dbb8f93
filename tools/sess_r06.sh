#!/bin/bash
# Round-6 GPU session (TAG names the outputs): smoke, the GPU test suite, the driver-shaped bench
# line, the deep-tail BER of config b (stream v3, and the round-5 stream-v2 library beside it), a
# same-box A/B of the v2 and v3 libraries on configs b and c, then a rocprofv3 kernel trace and the
# SQ counters of config b.  Every GPU step has its own time limit; a fault, abort or timeout ends
# the script (rc 1 = test failures: recorded, the session goes on).
export PYTHONUNBUFFERED=1
TAG=${TAG:-r06b}
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
[ -z "$NO_BENCH" ] && step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
if [ -z "$NO_TAIL" ]; then
    step tail_v3 600 python tools/ber_tail.py --snrs ${TAIL_SNRS:-24 26 27 28 28.5 29}
    OFDM_LIB_VARIANT=v2 OFDM_LIB_VARIANT_ABI=4 step tail_v2 600 python tools/ber_tail.py --snrs ${TAIL_SNRS:-24 26 27 28 28.5 29}
fi
if [ -z "$NO_AB" ]; then
    export OFDM_LIB_VARIANT_ABI=4
    AB_REPS=2 AB_STEPS=60 bash tools/ab.sh "v2 default" "${AB_CONFIGS:-b c}" > gpurun_out/${TAG}_ab_v2_v3.txt 2>&1 || exit $?
    unset OFDM_LIB_VARIANT_ABI
    cat gpurun_out/${TAG}_ab_v2_v3.txt
fi
if [ -z "$NO_PROF" ]; then
    for cfg in ${PROF_CONFIGS:-b}; do
        PROF_STEPS=10 bash tools/profile.sh ${TAG}_${cfg}_f64 --config $cfg --precision f64 || exit $?
        bash tools/counters.sh ${TAG}_${cfg}_f64 --config $cfg --precision f64 || exit $?
    done
fi
exit 0
