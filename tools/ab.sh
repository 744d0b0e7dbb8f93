#!/bin/bash
# A/B the variant libraries (_lib/libofdm_hip_<v>.so) on bench configs, steady state (the bench's
# clock-ramp warmup, 100 timed steps), variants interleaved over AB_REPS rounds to average out
# box drift.  Usage: bash tools/ab.sh "v1 v2 ..." "b c"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in $(seq 1 ${AB_REPS:-2}); do
for cfg in $2; do for v in $1; do
  if [ "$v" = "default" ]; then unset OFDM_LIB_VARIANT; else export OFDM_LIB_VARIANT=$v; fi
  out=gpurun_out/ab_${v}_${cfg}_${rep}
  timeout -k 10 120 python bench.py --config $cfg --steps ${AB_STEPS:-100} --warmup 2 --no-cpu-baseline --no-ber-check $AB_ARGS \
      > $out.json 2> $out.err
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v cfg $cfg rc=$rc"; tail -3 $out.err; exit $rc; }
  python -c "import json,sys; d=json.load(open('$out.json')); print('$rep', '$v', '$cfg', '%.4g sym/s'%d['value'], '%.4f ms/step'%d['ms_per_step'], {k:round(x,3) for k,x in d['roofline']['avg_launch_ms'].items()})"
done; done; done
