# round-3 session (final build): full GPU suite and smoke, bench lines b-e, rocprofv3 kernel trace +
# FETCH/WRITE of configs c, d, e (their TX changed: symbol groups of 32)
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03aj_gpu_tests.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03aj_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03aj_smoke.txt 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03aj_smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r03aj_bench_b.json 2> gpurun_out/r03aj_bench_b.err || { tail -3 gpurun_out/r03aj_bench_b.err; exit 1; }
echo "bench b ok"
for c in c d e; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03aj_bench_$c.json 2> gpurun_out/r03aj_bench_$c.err || { tail -3 gpurun_out/r03aj_bench_$c.err; exit 1; }
  echo "bench $c ok"
done
for c in c d e; do
  PROF_STEPS=10 timeout -k 10 400 bash tools/profile.sh r03aj_${c}_f64 --config $c --precision f64 > gpurun_out/r03aj_prof_$c.txt 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/r03aj_prof_$c.txt; exit 1; }
  echo "profile $c ok"
done
