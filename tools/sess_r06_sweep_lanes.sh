#!/bin/bash
# The config-c sweep line at 1..4 lanes (streams overlapping one point's TX with another's RX), twice
# each, interleaved: does a third lane fill the short launches' start/drain bubbles?
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in ${REPS:-1 2}; do for ln in ${LANES:-1 2 3 4}; do
  timeout -k 10 240 python bench.py --sweep --config c --steps 3 --warmup 1 --lanes $ln --no-cpu-baseline --no-ber-check \
      > gpurun_out/sl_${ln}_${rep}.json 2> gpurun_out/sl_${ln}_${rep}.err
  rc=$?; [ $rc -eq 0 ] || { echo "lanes $ln rc=$rc"; tail -3 gpurun_out/sl_${ln}_${rep}.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/sl_${ln}_${rep}.json')); print('$rep lanes $ln', '%.4g sym/s'%d['value'], '%.2f ms/step'%d['ms_per_step'])"
done; done
