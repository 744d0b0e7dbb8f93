set -o pipefail
TAG=r04b NO_BENCH=1 tools/gpu_session.sh || exit $?
AB_REPS=2 AB_STEPS=30 timeout -k 10 600 bash tools/ab.sh "old default h3" "c d e" 2>&1 | tee gpurun_out/r04b_ab.txt
timeout -k 10 400 python bench.py --config c --sweep --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04b_sweep.json 2> gpurun_out/r04b_sweep.err; echo sweep rc=$?; tail -c 600 gpurun_out/r04b_sweep.json
timeout -k 10 300 python tools/bench_variants.py --precision f64 --steps 10 > gpurun_out/r04b_variants_f64.json 2> gpurun_out/r04b_variants_f64.err; echo variants rc=$?; tail -9 gpurun_out/r04b_variants_f64.err
