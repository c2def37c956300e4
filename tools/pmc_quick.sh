#!/bin/bash
# A few counter passes over chosen RoIAlign variants (one rocprofv3 pass per group).
#   bash tools/pmc_quick.sh <outdir> <variants> [extra bench_roi_align args]
set -e
OUT=${1:-gpurun_out/pq}; V=${2:-10}; shift 2 || true
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
           "TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum" \
           "TA_BUFFER_READ_WAVEFRONTS_sum TA_BUFFER_WRITE_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -k 10 90 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- python tools/bench_roi_align.py --variants $V --iters 5 "$@" > $OUT/p$i.log 2>&1
done
python tools/pmc_table.py $OUT roi_align > $OUT/table.txt
