#!/bin/bash
# Final check of the committed build (TAG names the outputs): smoke, the whole GPU suite (incl. the
# one-rank RCCL group test), and the driver-shaped bench line.  Every GPU step has its own time limit.
export PYTHONUNBUFFERED=1
TAG=${TAG:-r06e}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke rc=$?"; tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log; grep -E "rccl|FAILED" gpurun_out/${TAG}_gpu_tests.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_b.json 2> gpurun_out/${TAG}_bench_b.err || { echo "bench rc=$?"; tail -3 gpurun_out/${TAG}_bench_b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_b.json')); r=d['roofline']; print('%.4g'%d['value'], r['bound'], round(r['frac'],3), r.get('issue',{}).get('valu'), r['traffic'], d['build_id'])"
exit 0
