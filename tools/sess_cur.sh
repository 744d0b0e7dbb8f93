set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for cfg in b c d e; do
  out=gpurun_out/prof_r04f_${cfg}_f64; mkdir -p $out
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv -- python3 bench.py --config $cfg --precision f64 --steps 30 --warmup 2 --no-cpu-baseline --no-ber-check --no-variant > $out/trace.log 2>&1
  rc=$?; echo "$cfg trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
