# round-3 session: the complex64 line of config b on its own (headline precision f32), to compare
# with the c64_variant measured after the complex128 run in the same process
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --precision f32 --steps 20 --warmup 5 --no-variant --no-cpu-baseline > gpurun_out/r03am_bench_b_f32.json 2> gpurun_out/r03am_bench_b_f32.err || { tail -3 gpurun_out/r03am_bench_b_f32.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03am_bench_b.json 2> gpurun_out/r03am_bench_b.err || { tail -3 gpurun_out/r03am_bench_b.err; exit 1; }
python -c "
import json
for f in ('gpurun_out/r03am_bench_b_f32.json','gpurun_out/r03am_bench_b.json'):
    d=json.load(open(f)); print(f, d['dtype'], '%.4g'%d['value'], {k:round(x,3) for k,x in d['roofline']['avg_launch_ms'].items()})
    v=d.get('c64_variant')
    if v: print('  c64_variant', '%.4g'%v['value'], {k:round(x,3) for k,x in v['roofline']['avg_launch_ms'].items()})
"
