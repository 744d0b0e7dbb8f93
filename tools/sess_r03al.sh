# round-3 session: BER curves of configs b, c, e with the throughput path in complex128 (the
# headline precision) against the reference-stream path
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for c in b c e; do
  timeout -k 10 400 python -u tools/ber_curve.py --config $c --precision f64 > gpurun_out/r03al_ber_curve_$c.json 2> gpurun_out/r03al_ber_curve_$c.err; rc=$?; echo "curve $c rc=$rc"; tail -1 gpurun_out/r03al_ber_curve_$c.err; [ $rc -eq 0 ] || exit $rc
done
