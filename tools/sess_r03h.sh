export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_philox_parity.py tests/test_gpu_fullsize.py tests/test_gpu_edges.py tests/test_gpu_throughput.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/r03h_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "default rx1024" "b" 2>&1 | grep -v amdgpu.ids || exit 1
AB_REPS=2 AB_STEPS=20 AB_ARGS="--precision f32 --no-variant --ramp-seconds 0" bash tools/ab.sh "base ew3 e768" "e d" 2>&1 | grep -v amdgpu.ids || exit 1
(timeout -k 10 120 python bench.py --steps 3000 --warmup 5 --no-cpu-baseline --no-ber-check --no-variant --ramp-seconds 0 > gpurun_out/r03h_pw.json 2>/dev/null &)
sleep 25; rocm-smi --showpower --showclocks > gpurun_out/r03h_smi1.txt 2>&1; sleep 2; rocm-smi --showpower --showclocks > gpurun_out/r03h_smi2.txt 2>&1
grep -ihE "power|sclk|mclk|fclk" gpurun_out/r03h_smi1.txt gpurun_out/r03h_smi2.txt
sleep 20
