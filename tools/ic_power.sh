#!/bin/bash
# Package power and clock of write-then-read batch streaming, Infinity-Cache-sized vs HBM-sized
# batches (GPU box): bash tools/ic_power.sh
mkdir -p gpurun_out
for mb in ${IC_SIZES:-128 2048}; do
    timeout -k 10 60 tools/hbm_probe loop $mb 6 > gpurun_out/ic_loop_$mb.json &
    pid=$!
    sleep 2.5
    for i in 1 2 3; do
        timeout -k 5 20 rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|Package Power" | sed "s/^/$mb MiB: /"
        sleep 0.7
    done
    wait $pid || exit $?
    cat gpurun_out/ic_loop_$mb.json
done
