#!/bin/bash
# Profiles of the final build (TAG names them): for each bench config in complex128, a rocprofv3
# kernel trace (--kernel-trace --stats) and separate FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh),
# condensed into profiles/ by tools/pmc_summary.py on the CPU side afterwards.
export PYTHONUNBUFFERED=1
TAG=${TAG:-r04p}
for cfg in ${PROF_CONFIGS:-b c d e}; do
    syms=1000000; [ $cfg = d ] && syms=500000; [ $cfg = e ] && syms=250000
    bash tools/profile.sh ${TAG}_${cfg}_f64 --config $cfg --precision f64 || exit $?
done
if [ -n "$CTR_CONFIGS" ]; then
  for cfg in $CTR_CONFIGS; do bash tools/counters.sh ${TAG}_${cfg}_f64 --config $cfg --precision f64 || exit $?; done
fi
