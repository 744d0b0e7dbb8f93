# round-3 session: bench lines b-e, rocprofv3 kernel trace + FETCH/WRITE of the complex128 configs
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in b c d e; do
  PROF_STEPS=10 timeout -k 10 400 bash tools/profile.sh r03w_${c}_f64 --config $c --precision f64 > gpurun_out/r03w_prof_$c.txt 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/r03w_prof_$c.txt; exit 1; }
  echo "profile $c ok"
done
timeout -k 10 300 python -u bench.py > gpurun_out/r03w_bench_b.json 2> gpurun_out/r03w_bench_b.err || { tail -3 gpurun_out/r03w_bench_b.err; exit 1; }
for c in c d e; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03w_bench_$c.json 2> gpurun_out/r03w_bench_$c.err || { tail -3 gpurun_out/r03w_bench_$c.err; exit 1; }
  echo "bench $c ok"
done
