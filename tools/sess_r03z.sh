# round-3 session: the full GPU suite on the product library (complex128 RX at N = 4096 one symbol
# per workgroup, batched MMSE reciprocals), then config e's bench line and rocprofv3 profile
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03z_gpu_tests.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03z_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config e --steps 20 --warmup 5 > gpurun_out/r03z_bench_e.json 2> gpurun_out/r03z_bench_e.err || { tail -3 gpurun_out/r03z_bench_e.err; exit 1; }
echo "bench e ok"
PROF_STEPS=10 timeout -k 10 400 bash tools/profile.sh r03z_e_f64 --config e --precision f64 > gpurun_out/r03z_prof_e.txt 2>&1 || { echo "profile e failed"; tail -5 gpurun_out/r03z_prof_e.txt; exit 1; }
echo "profile e ok"
