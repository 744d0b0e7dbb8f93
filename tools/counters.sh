#!/bin/bash
# Pipe-utilisation counters of the fused kernels, one rocprofv3 --pmc pass per group (no trace
# domains).  Usage (GPU box): bash tools/counters.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/ctr_$tag
mkdir -p $out
args="--steps 2 --warmup 1 --no-cpu-baseline --no-ber-check --no-variant --ramp-seconds 0 $*"
timeout -k 10 60 rocprofv3 -L > $out/avail.txt 2>&1 || true
i=0
IFS=';' read -ra GROUPS_ <<< "${COUNTER_GROUPS:-SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES;SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE}"
for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp -d $out/g$i -o g$i --output-format csv -- python3 bench.py $args \
        > $out/g$i.log 2>&1
    rc=$?; echo "group $i ($grp) rc=$rc"; tail -2 $out/g$i.log
    [ $rc -eq 0 ] || exit $rc
done
