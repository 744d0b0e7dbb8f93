#!/bin/bash
# Same-box A/B of the round-4 final library (libofdm_hip_r04.so, built from commit a1b5083 = build
# b3fa4997) against the current in-tree library on config b: the driver's own command shape
# (steps 20, warmup 5, cpu baseline and BER check included) twice each, the steady-state A/B
# (tools/ab.sh, 60 timed steps) three times each, interleaved, then a rocprofv3 kernel trace of each.
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
out=gpurun_out/${TAG:-r06a}_ab_r04_vs_cur_b.txt
: > $out
for rep in 1 2; do for v in r04 default; do
  if [ "$v" = "default" ]; then unset OFDM_LIB_VARIANT; else export OFDM_LIB_VARIANT=$v; fi
  timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_${v}_$rep.json 2> gpurun_out/drv_${v}_$rep.err \
      || { echo "driver-shape $v rc=$?"; tail -3 gpurun_out/drv_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/drv_${v}_$rep.json')); print('driver-shape', '$rep', '$v', '%.4g sym/s'%d['value'], '%.4f ms/step'%d['ms_per_step'], {k:round(x,3) for k,x in d['roofline']['avg_launch_ms'].items()})" >> $out
done; done
unset OFDM_LIB_VARIANT
AB_REPS=3 AB_STEPS=60 bash tools/ab.sh "r04 default" "b" >> $out 2>&1 || exit $?
export OFDM_LIB_VARIANT=r04
PROF_STEPS=20 bash tools/profile.sh ${TAG:-r06a}_r04_b_f64 --config b --precision f64 || exit $?
unset OFDM_LIB_VARIANT
PROF_STEPS=20 bash tools/profile.sh ${TAG:-r06a}_cur_b_f64 --config b --precision f64 || exit $?
cat $out
