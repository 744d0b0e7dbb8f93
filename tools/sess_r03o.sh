# round-3 session: complex128 window FIR -- complex rows (cplx), rows of reals at 512 threads
# (default) and at 256 threads (r256); configs d e, then c
export TMPDIR=/tmp PYTHONUNBUFFERED=1
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "cplx default r256" "${AB_CFGS:-d e}" 2>&1 | grep -v amdgpu.ids
