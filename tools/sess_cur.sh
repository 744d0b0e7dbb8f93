set -o pipefail
TAG=r04c NO_BENCH=1 tools/gpu_session.sh || exit $?
timeout -k 10 400 python bench.py --config c --sweep --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04c_sweep.json 2> gpurun_out/r04c_sweep.err; echo sweep rc=$?; tail -c 300 gpurun_out/r04c_sweep.json
timeout -k 10 300 python tools/bench_variants.py --precision f64 --steps 10 > gpurun_out/r04c_variants_f64.json 2> gpurun_out/r04c_variants_f64.err; echo variants rc=$?; tail -9 gpurun_out/r04c_variants_f64.err
CTR_CONFIGS="c e" PROF_CONFIGS="" TAG=r04c bash tools/sess_prof.sh 2>&1 | tail -12
timeout -k 10 400 python bench.py --config c --sweep --steps 3 --warmup 1 --no-cpu-baseline --no-ber-check --lanes 2 > gpurun_out/r04c_sweep_l2.json 2> gpurun_out/r04c_sweep_l2.err; echo sweep-l2 rc=$?; python -c "import json; d=json.load(open('gpurun_out/r04c_sweep_l2.json')); print('sweep lanes2', d['value'], d['ms_per_step'])"
for L in 1 2; do timeout -k 10 200 python bench.py --config c --steps 30 --no-cpu-baseline --no-ber-check --no-variant --lanes $L > gpurun_out/r04c_c_l$L.json 2>/dev/null; python -c "import json; d=json.load(open('gpurun_out/r04c_c_l$L.json')); print('c lanes $L', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
AB_REPS=2 AB_STEPS=30 timeout -k 10 400 bash tools/ab.sh "default cr wq" "c e" 2>&1 | tee gpurun_out/r04c_ab_cr.txt
OFDM_LIB_VARIANT=cr timeout -k 10 300 python -m pytest tests/test_gpu_philox_parity.py -q -p no:cacheprovider -k "f64 and (N1024-M64-severe_multipath-MMSE-f64 or N4096-M256)" 2>&1 | tail -3
