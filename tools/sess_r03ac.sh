# round-3 session: full GPU suite on the product library (buffer-loaded RX samples, 4-wave no-eq
# RX at N = 1024, separable-LUT multipath TX), bench lines b-e and the config b / c profiles
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ac_gpu_tests.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03ac_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r03ac_bench_b.json 2> gpurun_out/r03ac_bench_b.err || { tail -3 gpurun_out/r03ac_bench_b.err; exit 1; }
echo "bench b ok"
for c in c d e; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03ac_bench_$c.json 2> gpurun_out/r03ac_bench_$c.err || { tail -3 gpurun_out/r03ac_bench_$c.err; exit 1; }
  echo "bench $c ok"
done
for c in b c; do
  PROF_STEPS=10 timeout -k 10 400 bash tools/profile.sh r03ac_${c}_f64 --config $c --precision f64 > gpurun_out/r03ac_prof_$c.txt 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/r03ac_prof_$c.txt; exit 1; }
  echo "profile $c ok"
done
