# round-3 session: GPU tests, bench lines of every config (complex128 headline + complex64
# companion), power / clock samples under the headline load
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03i_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r03i_t.txt; [ $rc -eq 0 ] || exit $rc
for c in b c d e; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > gpurun_out/r03i_bench_$c.json 2> gpurun_out/r03i_bench_$c.err; rc=$?
  echo "bench $c rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/r03i_bench_$c.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03i_bench_$c.json')); v=d['c64_variant']; print('$c', '%.4g'%d['value'], d['dtype'], {k: round(x,3) for k,x in d['roofline']['avg_launch_ms'].items()}, 'frac %.3f'%d['roofline']['frac'], '| c64 %.4g'%v['value'], {k: round(x,3) for k,x in v['roofline']['avg_launch_ms'].items()}, 'frac %.3f'%v['roofline']['frac'], '| dB', d.get('ber_vs_reference',{}).get('delta_db'), '| cpu', round(d['cpu_baseline']['value']))"
done
timeout -k 10 150 python bench.py --steps 8000 --warmup 5 --no-cpu-baseline --no-ber-check --no-variant --ramp-seconds 0 > gpurun_out/r03i_pw.json 2>/dev/null &
for i in 1 2 3 4 5 6 7 8; do sleep 8; rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Package Power|sclk clock level|mclk" | tr '\n' ' '; echo; done
wait
