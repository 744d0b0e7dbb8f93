#!/bin/bash
# final build: modem-variant throughput table (complex128) and the deep-tail BER of config (b)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_variants.py --precision f64 > gpurun_out/r04s_variants_f64.json 2> gpurun_out/r04s_variants_f64.err
rc=$?; echo "variants rc=$rc"; tail -9 gpurun_out/r04s_variants_f64.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ber_curve.py --config b --precision f64 --grid 26,26.5,27 --symbols 20000000 --ref-symbols 300000 > gpurun_out/r04s_ber_tail_b.json 2> gpurun_out/r04s_ber_tail_b.err
rc=$?; echo "ber tail rc=$rc"; tail -5 gpurun_out/r04s_ber_tail_b.err
exit $rc
