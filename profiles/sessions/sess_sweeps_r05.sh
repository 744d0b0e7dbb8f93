#!/bin/bash
# the three BASELINE sweeps: configs c (default), d and e (the reference settings' SNR lists)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
T=${T:-r05s}
for c in c d e; do
  timeout -k 10 400 python bench.py --sweep --config $c > gpurun_out/${T}_sweep_$c.json 2> gpurun_out/${T}_sweep_$c.err
  rc=$?; echo "sweep $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_sweep_$c.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_sweep_$c.json')); print('$c', '%.4g'%d['value'], d['roofline'] and round(d['roofline']['frac'],3), d['roofline'] and {k:round(v,3) for k,v in d['roofline']['avg_launch_ms'].items()}, [(p['qam_order'], p['snr_db'], '%.3g'%p['ber']) for p in d['sweep']['per_point']][:15] if '$c' != 'c' else d.get('delta_db_at_1e-4'), '%.3g'%d['cpu_baseline']['value'])"
done
