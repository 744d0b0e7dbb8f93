#!/bin/bash
# round-4 final build: GPU suite, smoke, bench lines b-e, the config-c SNR sweep, steady-state
# rocprofv3 traces + PMC bytes, stall counters of the config-c TX
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r04p}
timeout -k 10 300 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${T}_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${T}_smoke.txt; [ $rc -eq 0 ] || exit $rc
for c in b c d e; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/${T}_bench_$c.json 2> gpurun_out/${T}_bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench_$c.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_bench_$c.json')); print('$c', '%.4g'%d['value'], round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['roofline']['avg_launch_ms'].items()})"
done
timeout -k 10 400 python bench.py --sweep > gpurun_out/${T}_sweep_c.json 2> gpurun_out/${T}_sweep_c.err
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_sweep_c.err; exit $rc; }
for c in b c d e; do
  PROF_STEPS=30 bash tools/profile.sh ${T}_${c}_f64 --config $c --precision f64 --warmup 2 --ramp-seconds 0.25 > gpurun_out/${T}_prof_$c.txt 2>&1
  rc=$?; echo "prof $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_prof_$c.txt; exit $rc; }
done
COUNTER_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
  bash tools/counters.sh ${T}_c --config c --precision f64 > gpurun_out/${T}_ctr.txt 2>&1
rc=$?; echo "ctr rc=$rc"
exit $rc
