#!/bin/bash
# steady-state traces + PMC of the final build (30 timed steps after the bench's clock ramp)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for c in b c d e; do
  PROF_STEPS=30 bash tools/profile.sh r04j_${c}_f64 --config $c --precision f64 --warmup 2 --ramp-seconds 0.25 > gpurun_out/r04j_prof_$c.txt 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04j_prof_$c.txt; exit $rc; }
  grep -h "k_tx\|k_rx" gpurun_out/prof_r04j_${c}_f64/trace/*kernel_stats.csv | cut -c1-120
done
