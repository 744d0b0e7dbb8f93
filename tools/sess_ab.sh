#!/bin/bash
# final build: steady-state clock / package power of the full step and its ablations (configs b, c),
# stall counters of config d (its receiver is the dominant kernel)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/power_probe.py --config b --precision f64 --seconds 4 --only full,tx_only,rx_only,hbm_only,compute_only > gpurun_out/r04w_power_b.txt 2>&1; echo "b rc=$?"; grep -v amdgpu.ids gpurun_out/r04w_power_b.txt | head -5
timeout -k 10 200 python tools/power_probe.py --config c --precision f64 --seconds 4 --only full,tx_only,rx_only,hbm_only,compute_only > gpurun_out/r04w_power_c.txt 2>&1; echo "c rc=$?"; grep -v amdgpu.ids gpurun_out/r04w_power_c.txt | head -5
COUNTER_GROUPS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
  bash tools/counters.sh r04w_d --config d --precision f64 > gpurun_out/r04w_ctr_d.txt 2>&1
rc=$?; echo "ctr rc=$rc"
exit $rc
