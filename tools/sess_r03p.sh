# round-3 session: whole GPU suite + smoke, bench lines of b (default) c d e after the real-row FIR TX
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03p_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r03p_t.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03p_bench_default.json 2> gpurun_out/r03p_bench_default.err; rc=$?
echo "bench default rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/r03p_bench_default.err; exit $rc; }
for c in c d e; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03p_bench_$c.json 2> gpurun_out/r03p_bench_$c.err; rc=$?
  echo "bench $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/r03p_bench_$c.err; exit $rc; }
done
