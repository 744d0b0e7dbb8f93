#!/bin/bash
# Every bench config on one GPU (GPU box): bash tools/bench_all.sh [tag]
# plus a 2-rank rehearsal of the multi-rank bench path on the same GPU (gloo).
export PYTHONUNBUFFERED=1
tag=${1:-r02}
mkdir -p gpurun_out
for cfg in ${BENCH_CONFIGS:-b c d e}; do
  timeout -k 10 240 python bench.py --config $cfg --steps ${BENCH_STEPS:-20} --warmup 5 \
      > gpurun_out/bench_${tag}_$cfg.json 2> gpurun_out/bench_${tag}_$cfg.err
  rc=$?; [ $rc -eq 0 ] || { echo "config $cfg rc=$rc"; tail -5 gpurun_out/bench_${tag}_$cfg.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${tag}_$cfg.json')); print('$cfg', '%.4g sym/s'%d['value'], d['roofline']['avg_launch_ms'], 'frac %.3f'%d['roofline']['frac'], 'dB', d.get('ber_vs_reference',{}).get('delta_db'), 'cpu', d.get('cpu_baseline',{}).get('value'))"
done
if [ -n "$RANKS2" ]; then
  OFDM_BENCH_DEVICE=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --backend gloo \
      --no-cpu-baseline --symbols 200000 > gpurun_out/bench_${tag}_2rank.json 2> gpurun_out/bench_${tag}_2rank.err
  rc=$?; tail -c 600 gpurun_out/bench_${tag}_2rank.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${tag}_2rank.err; exit $rc; }
fi
