# round-3 session: rocprofv3 kernel trace + FETCH/WRITE of the complex128 configs on the current
# build, and the pipe counters of configs b d e (complex128)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in b c d e; do
  PROF_STEPS=10 timeout -k 10 400 bash tools/profile.sh r03q_${c}_f64 --config $c --precision f64 > gpurun_out/r03q_prof_$c.txt 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/r03q_prof_$c.txt; exit 1; }
  echo "profile $c ok"
done
for c in b d e; do
  timeout -k 10 400 bash tools/counters.sh r03q_${c}_f64 --config $c --precision f64 > gpurun_out/r03q_ctr_$c.txt 2>&1 || { echo "counters $c failed"; tail -5 gpurun_out/r03q_ctr_$c.txt; exit 1; }
  echo "counters $c ok"
done
