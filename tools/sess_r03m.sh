# round-3 session: A/B of the complex128 Gauss-form window FIR + ordered RX loads (norep) + the
# replicated noise table (default)
# against the build before them (base), configs b c d e, plus the complex64 variants
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03m_t.txt 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/r03m_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base norep default" "b c d e" 2>&1 | grep -v amdgpu.ids
AB_REPS=1 AB_STEPS=40 AB_ARGS="--precision f32 --no-variant --ramp-seconds 0" bash tools/ab.sh "base default" "b e" 2>&1 | grep -v amdgpu.ids
