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
# every pass also counts GRBM_GUI_ACTIVE (its own block): the kernel's duration in the same pass, from
# which tools/pmc_summary.py --counters turns the SQ issue cycles into fractions of the SIMDs' time
IFS=';' read -ra GROUPS_ <<< "${COUNTER_GROUPS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE}"
for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $grp -d $out/g$i -o g$i --output-format csv -- python3 bench.py $args \
        > $out/g$i.log 2>&1
    rc=$?; echo "group $i ($grp) rc=$rc"; tail -2 $out/g$i.log
    [ $rc -eq 0 ] || exit $rc
done
