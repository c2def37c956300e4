#!/bin/bash
# GPU-box profiling recipe for one round: bench line, kernel stats (+ timed-step breakdown),
# PMC traffic of the RoIAlign forward (separate FETCH / WRITE passes + known-byte FETCH
# calibration) and wave occupancy of the hot-path kernels.
#   bash tools/profile_round.sh <outdir under gpurun_out>
set -e
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/stats.log 2>&1
python tools/step_breakdown.py $OUT/stats --warmup 3 --steps 10 > $OUT/step_breakdown.json
rm -f $OUT/stats/run_kernel_trace.csv  # large; the summary and the breakdown are kept
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_calib -o run --output-format csv -- python tools/bench_roi_align.py --calib --variants 0 > $OUT/pmc_calib.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_calib_small -o run --output-format csv -- python tools/bench_roi_align.py --calib --calib-small --variants 0 > $OUT/pmc_calib_small.log 2>&1
timeout -k 10 300 rocprofv3 --pmc OccupancyPercent MeanOccupancyPerCU --kernel-trace -d $OUT/pmc_occ -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/pmc_occ.log 2>&1
python tools/pmc_summary.py --fetch $OUT/pmc_fetch --write $OUT/pmc_write --kernel roi_align_fwd_pair_kernel \
  --calib-fetch $OUT/pmc_calib $OUT/pmc_calib_small --calib-bytes 220463104 150994944 --out $OUT/roi_align_pmc.json
python tools/pmc_table.py $OUT/pmc_occ frh:: > $OUT/occupancy.txt
