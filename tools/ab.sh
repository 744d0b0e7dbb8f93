#!/bin/bash
# A/B the variant libraries (_lib/libofdm_hip_<v>.so) on bench configs. Usage: bash tools/ab.sh "v1 v2 ..." "b c"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for cfg in $2; do for v in $1; do
  if [ "$v" = "default" ]; then unset OFDM_LIB_VARIANT; else export OFDM_LIB_VARIANT=$v; fi
  timeout -k 10 120 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${v}_${cfg}.json 2> gpurun_out/ab_${v}_${cfg}.err
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v cfg $cfg rc=$rc"; tail -3 gpurun_out/ab_${v}_${cfg}.err; exit $rc; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_${v}_${cfg}.json')); print('$v', '$cfg', '%.4g sym/s'%d['value'], {k:round(x,3) for k,x in d['roofline']['avg_launch_ms'].items()})"
done; done
