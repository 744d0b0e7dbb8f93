# round-3 session: complex128 config (b) A/B -- nontemporal TX stores (txnt), plain RX loads
# (rxnt0), 768-thread TX (tx768), 512-thread RX (rx512) against the default build
export TMPDIR=/tmp PYTHONUNBUFFERED=1
AB_REPS=2 AB_STEPS=40 AB_ARGS="--precision f64 --no-variant --ramp-seconds 0" bash tools/ab.sh "default txnt rxnt0 tx768 rx512" "b" 2>&1 | grep -v amdgpu.ids
