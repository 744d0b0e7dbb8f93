#!/bin/bash
# round-5 final build: GPU suite, smoke, bench lines b-e, the config-c SNR sweep, rocprofv3 kernel
# traces + PMC bytes of b-e, pipe counters of the config-c TX and config-d RX.  Every GPU step has
# its own time limit; a failure ends the script.  T names the outputs.
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r05f}
step() {  # name seconds output command... (the command's stdout goes to the output file)
    local name=$1 secs=$2 out=$3; shift 3
    timeout -k 10 "$secs" "$@" > "$out"
    local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
if [ -z "$NO_TESTS" ]; then
  step tests 600 gpurun_out/${T}_gpu_tests.txt python -u -m pytest tests -m gpu -v -s -p no:cacheprovider \
      --timeout 300 --timeout-method thread 2>&1
  tail -1 gpurun_out/${T}_gpu_tests.txt
  step smoke 300 gpurun_out/${T}_smoke.txt python -c "import __graft_entry__ as g; g.smoke()" 2>&1
  tail -1 gpurun_out/${T}_smoke.txt
fi
for c in ${BENCH_CONFIGS:-b c d e}; do
  step bench_$c 300 gpurun_out/${T}_bench_$c.json python bench.py --config $c 2> gpurun_out/${T}_bench_$c.err
  python -c "import json; d=json.load(open('gpurun_out/${T}_bench_$c.json')); print('$c', '%.4g'%d['value'], round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['roofline']['avg_launch_ms'].items()}, 'cpu', '%.3g'%d['cpu_baseline']['value'])"
done
if [ -z "$NO_SWEEP" ]; then
  step sweep 400 gpurun_out/${T}_sweep_c.json python bench.py --sweep 2> gpurun_out/${T}_sweep_c.err
  python -c "import json; d=json.load(open('gpurun_out/${T}_sweep_c.json')); print('sweep', '%.4g'%d['value'], d['roofline'] and round(d['roofline']['frac'],3), d.get('delta_db_at_1e-4'))"
fi
if [ -z "$NO_PROF" ]; then
  for c in ${PROF_CONFIGS:-b c d e}; do
    PROF_STEPS=30 step prof_$c 600 gpurun_out/${T}_prof_$c.txt bash tools/profile.sh ${T}_${c}_f64 --config $c \
        --precision f64 --warmup 2 --ramp-seconds 0.25 2>&1
  done
fi
if [ -n "$CTR_CONFIGS" ]; then
  for c in $CTR_CONFIGS; do
    COUNTER_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64" \
      step ctr_$c 600 gpurun_out/${T}_ctr_$c.txt bash tools/counters.sh ${T}_$c --config $c --precision f64 2>&1
  done
fi
exit 0
