# round-3 session: whole GPU suite + smoke on the current build, default bench line (with the
# CPU baseline) and the bench lines of configs c d e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03l_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r03l_t.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03l_bench_default.json 2> gpurun_out/r03l_bench_default.err; rc=$?
echo "bench default rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/r03l_bench_default.err; exit $rc; }
for c in c d e; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03l_bench_$c.json 2> gpurun_out/r03l_bench_$c.err; rc=$?
  echo "bench $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/r03l_bench_$c.err; exit $rc; }
done
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base default" "c e" 2>&1 | grep -v amdgpu.ids
