export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_variants.py --only d,b > gpurun_out/variants_d.json 2> gpurun_out/variants_d.err; rc=$?; grep -v amdgpu.ids gpurun_out/variants_d.err | tail; exit $rc
