set -o pipefail
TAG=r04d NO_BENCH=1 tools/gpu_session.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/r04d_bench_b.json 2> gpurun_out/r04d_bench_b.err; echo bench-b rc=$?; tail -c 1500 gpurun_out/r04d_bench_b.json
for cfg in c d e; do timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/r04d_bench_$cfg.json 2> gpurun_out/r04d_bench_$cfg.err; echo bench-$cfg rc=$?; python -c "import json; d=json.load(open('gpurun_out/r04d_bench_$cfg.json')); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d.get('ber_vs_reference',{}).get('delta_db'))"; done
timeout -k 10 400 python bench.py --config c --sweep > gpurun_out/r04d_sweep.json 2> gpurun_out/r04d_sweep.err; echo sweep rc=$?; python -c "import json; d=json.load(open('gpurun_out/r04d_sweep.json')); print('sweep', d['value'], d['ms_per_step'], d.get('delta_db_at_1e-4'), d.get('cpu_baseline',{}).get('value'))"
