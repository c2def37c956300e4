#!/bin/bash
# Counter sweep of the RoIAlign forward variants (one rocprofv3 pass per counter group).
#   bash tools/pmc_sweep.sh <outdir> <variants>
set -e
OUT=${1:-gpurun_out/sweep}; V=${2:-8,9}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "GRBM_GUI_ACTIVE TA_BUSY_avr" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- python tools/bench_roi_align.py --variants $V --iters 5 > $OUT/p$i.log 2>&1
done
python tools/pmc_table.py $OUT roi_align > $OUT/table.txt
