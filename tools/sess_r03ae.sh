# round-3 session: full GPU suite and smoke on the product library (config d RX one symbol per
# workgroup), bench lines b-e, rocprofv3 kernel trace + FETCH/WRITE of configs d and e, pipe counters of d/e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ae_gpu_tests.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03ae_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ae_smoke.txt 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03ae_smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r03ae_bench_b.json 2> gpurun_out/r03ae_bench_b.err || { tail -3 gpurun_out/r03ae_bench_b.err; exit 1; }
echo "bench b ok"
for c in c d e; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03ae_bench_$c.json 2> gpurun_out/r03ae_bench_$c.err || { tail -3 gpurun_out/r03ae_bench_$c.err; exit 1; }
  echo "bench $c ok"
done
for c in d e; do
  PROF_STEPS=10 timeout -k 10 400 bash tools/profile.sh r03ae_${c}_f64 --config $c --precision f64 > gpurun_out/r03ae_prof_$c.txt 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/r03ae_prof_$c.txt; exit 1; }
  echo "profile $c ok"
done
for c in b d e; do
  timeout -k 10 500 bash tools/counters.sh r03ae_${c} --config $c --precision f64 > gpurun_out/r03ae_ctr_$c.txt 2>&1 || { echo "counters $c failed"; tail -5 gpurun_out/r03ae_ctr_$c.txt; exit 1; }
  echo "counters $c ok"
done
