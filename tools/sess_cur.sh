set -o pipefail
TAG=r04c NO_BENCH=1 tools/gpu_session.sh || exit $?
timeout -k 10 400 python bench.py --config c --sweep --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04c_sweep.json 2> gpurun_out/r04c_sweep.err; echo sweep rc=$?; tail -c 300 gpurun_out/r04c_sweep.json
timeout -k 10 300 python tools/bench_variants.py --precision f64 --steps 10 > gpurun_out/r04c_variants_f64.json 2> gpurun_out/r04c_variants_f64.err; echo variants rc=$?; tail -9 gpurun_out/r04c_variants_f64.err
CTR_CONFIGS="c e" PROF_CONFIGS="" TAG=r04c bash tools/sess_prof.sh 2>&1 | tail -12
