# round-3 session: BER curve of config d (adaptive loading, orders re-derived per SNR) with the
# complex128 throughput path against the reference-stream path
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/ber_curve.py --config d --precision f64 > gpurun_out/r03aq_ber_curve_d.json 2> gpurun_out/r03aq_ber_curve_d.err; rc=$?; echo "curve d rc=$rc"; tail -3 gpurun_out/r03aq_ber_curve_d.err; [ $rc -eq 0 ] || exit $rc
