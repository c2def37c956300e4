#!/bin/bash
# GPU-box profiling recipe for one round: bench line, kernel stats (+ timed-step breakdown),
# the per-dispatch RoIAlign table (rocprofv3 / event pair / in-kernel span / tracer on the same
# dispatches), PMC traffic of the RoIAlign forward (separate FETCH / WRITE passes + known-byte
# FETCH calibration on the same kernel) and wave occupancy of the hot-path kernels.
#   bash tools/profile_round.sh <outdir under gpurun_out> [kernel] [calib variant]
set -e
OUT=${1:-gpurun_out/prof}
K=${2:-roi_align_fwd_quad_kernel}
CV=${3:-10}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/stats.log 2>&1
python tools/step_breakdown.py $OUT/stats --warmup 3 --steps 10 > $OUT/step_breakdown.json
rm -f $OUT/stats/run_kernel_trace.csv  # large; the summary and the breakdown are kept
mkdir -p $OUT/disp $OUT/disp_tracer
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/disp/trace -o run --output-format csv -- python tools/roi_dispatch_table.py --out $OUT/disp/launches.json > $OUT/disp.log 2>&1
python tools/roi_dispatch_table.py --join $OUT/disp --out $OUT/roi_dispatch_table.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/disp_tracer/trace -o run --output-format csv -- python tools/roi_dispatch_table.py --tracer --out $OUT/disp_tracer/launches.json > $OUT/disp_tracer.log 2>&1 && \
  python tools/roi_dispatch_table.py --join $OUT/disp_tracer --out $OUT/roi_dispatch_table_tracer.json || echo "tracer pass failed" >> $OUT/disp_tracer.log
rm -rf $OUT/disp/trace $OUT/disp_tracer/trace
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --trace-steps 0 > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --trace-steps 0 > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_calib_small -o run --output-format csv -- python tools/bench_roi_align.py --calib --calib-small --variants $CV > $OUT/pmc_calib_small.log 2>&1
timeout -k 10 300 rocprofv3 --pmc OccupancyPercent MeanOccupancyPerCU --kernel-trace -d $OUT/pmc_occ -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --trace-steps 0 > $OUT/pmc_occ.log 2>&1
python tools/pmc_summary.py --fetch $OUT/pmc_fetch --write $OUT/pmc_write --kernel $K \
  --calib-fetch $OUT/pmc_calib_small --calib-bytes 150994944 --out $OUT/roi_align_pmc.json
python tools/pmc_table.py $OUT/pmc_occ frh:: > $OUT/occupancy.txt
rm -rf $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_calib_small $OUT/pmc_occ
