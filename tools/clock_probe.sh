#!/bin/bash
# Samples the GPU clock and power while the bench kernels run back to back (GPU box):
#   bash tools/clock_probe.sh [bench args...]
# A long bench in the background (~15 s), rocm-smi sampled every second alongside.
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --steps ${PROBE_STEPS:-3000} --warmup 2 --no-cpu-baseline --no-ber-check "$@" \
    > gpurun_out/clock_probe_bench.json 2> gpurun_out/clock_probe_bench.err &
pid=$!
sleep ${PROBE_DELAY:-12}
for i in 1 2 3 4 5 6; do
    timeout -k 5 20 rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|fclk|Power|Temperature" \
        >> gpurun_out/clock_probe_smi.txt
    echo "--" >> gpurun_out/clock_probe_smi.txt
    sleep 1
done
wait $pid
rc=$?
cat gpurun_out/clock_probe_smi.txt
exit $rc
