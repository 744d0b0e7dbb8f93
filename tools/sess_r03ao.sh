# round-3 session (final product build): full GPU suite, smoke, default bench line
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ao_gpu_tests.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03ao_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ao_smoke.txt 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03ao_smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03ao_bench_b.json 2> gpurun_out/r03ao_bench_b.err || { tail -3 gpurun_out/r03ao_bench_b.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r03ao_bench_b.json')); r=d['roofline']; print(d['dtype'], '%.4g'%d['value'], 'frac %.3f'%r['frac'], {k:round(x,3) for k,x in r['avg_launch_ms'].items()}, 'c64 %.4g'%d['c64_variant']['value'], 'cpu %.4g'%d['cpu_baseline']['value'])"
