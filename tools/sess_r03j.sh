# round-3 session: philox parity incl. complex128 adaptive, bench lines of configs c d e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_philox_parity.py tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03j_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r03j_t.txt; [ $rc -eq 0 ] || exit $rc
for c in d e c b; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03j_bench_$c.json 2> gpurun_out/r03j_bench_$c.err; rc=$?
  echo "bench $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/r03j_bench_$c.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03j_bench_$c.json')); v=d['c64_variant']; print('$c', '%.4g'%d['value'], d['dtype'], {k: round(x,3) for k,x in d['roofline']['avg_launch_ms'].items()}, 'frac %.3f'%d['roofline']['frac'], '| c64 %.4g'%v['value'], {k: round(x,3) for k,x in v['roofline']['avg_launch_ms'].items()}, 'frac %.3f'%v['roofline']['frac'], '| dB', d.get('ber_vs_reference',{}).get('delta_db'))"
done
