# round-3 session: grid-stride grids cut to whole rounds of resident workgroups (gr) against the
# 4096-workgroup cap (base); parity first
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OFDM_LIB_VARIANT=gr timeout -k 10 300 python -u -m pytest tests/test_gpu_philox_parity.py -k "(N4096-M256 or N1024-M64 or N2048-M0) and f64" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ah_t.txt 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03ah_t.txt; [ $rc -eq 0 ] || exit $rc
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "base gr" "b c d e" 2>&1 | grep -v amdgpu.ids
