#!/bin/bash
# Round-6 profiling recipe (GPU box): bench line, rocprofv3 kernel stats + timed-step breakdown
# (with the bench line the profiled process printed itself), PMC traffic of the RoIAlign forward
# in the fwd AND the train step (separate FETCH / WRITE passes + known-byte FETCH calibration of
# the same kernel), wave occupancy, stall counters of the RoIAlign forward, and L2 request / hit
# counters on the three RoI sets.
#   bash tools/profile_r06.sh <outdir under gpurun_out>
set -o pipefail
OUT=${1:-gpurun_out/r6_prof}
PART=${2:-all}   # a: bench / kernel stats / PMC traffic / occupancy;  b: per-set counters + RCCL trace
K=roi_align_fwd_cg_kernel
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 "$@"; }
if [ "$PART" != b ]; then
run 300 python bench.py --no-cpu-baseline > $OUT/bench_plain.json 2> $OUT/bench_plain.err || exit 1
run 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/stats.log || exit 1
# the timed steps start after the warmup AND the graph-capture steps: the bench line says where
W=$(python -c "import json; print(json.loads(open('$OUT/bench_under_rocprof.json').read().strip().splitlines()[-1])['roofline']['launches_before_timed_region'])")
python tools/step_breakdown.py $OUT/stats --warmup $W --steps 10 > $OUT/step_breakdown.json || exit 1
rm -f $OUT/stats/run_kernel_trace.csv
for m in fwd train; do
  A="--steps 3 --warmup 2 --no-cpu-baseline --trace-steps 0 --mode $m"
  run 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch_$m -o run --output-format csv -- python bench.py $A > $OUT/pmc_fetch_$m.log 2>&1 || exit 1
  run 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write_$m -o run --output-format csv -- python bench.py $A > $OUT/pmc_write_$m.log 2>&1 || exit 1
done
run 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_calib_small -o run --output-format csv -- python tools/bench_roi_align.py --calib --calib-small --variants 80 > $OUT/pmc_calib_small.log 2>&1 || exit 1
run 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_calib_band -o run --output-format csv -- python tools/bench_roi_align.py --calib --variants 80 > $OUT/pmc_calib_band.log 2>&1 || exit 1
python tools/pmc_summary.py --fetch $OUT/pmc_fetch_fwd --write $OUT/pmc_write_fwd --kernel $K --calib-kernel roi_align_fwd_cg_kernel \
  --calib-fetch $OUT/pmc_calib_small --calib-bytes 150994944 --out $OUT/roi_align_pmc.json || exit 1
python tools/pmc_summary.py --fetch $OUT/pmc_fetch_train --write $OUT/pmc_write_train --kernel $K --calib-kernel roi_align_fwd_cg_kernel \
  --calib-fetch $OUT/pmc_calib_band --calib-bytes 205520896 --out $OUT/roi_align_pmc_train.json || exit 1
run 300 rocprofv3 --pmc OccupancyPercent MeanOccupancyPerCU --kernel-trace -d $OUT/pmc_occ -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --trace-steps 0 > $OUT/pmc_occ.log 2>&1 || exit 1
python tools/pmc_table.py $OUT/pmc_occ frh:: > $OUT/occupancy.txt
rm -rf $OUT/pmc_fetch_* $OUT/pmc_write_* $OUT/pmc_calib_* $OUT/pmc_occ
fi
[ "$PART" = a ] && { echo profile part a done; exit 0; }
for set in bench voc train; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    mkdir -p $OUT/stall_$set
    run 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/stall_$set/p$i -o run --output-format csv -- python tools/bench_roi_sets.py --sets $set --variants 65 --rounds 1 --iters 3 > $OUT/stall_$set/p$i.log 2>&1 || { echo "stall pass $set $i failed"; exit 1; }
  done
  python tools/pmc_table.py $OUT/stall_$set roi_align_fwd > $OUT/roi_align_counters_$set.txt || true
  rm -rf $OUT/stall_$set
done
# RCCL readiness: the train step with DDP forced on over a world-size-1 nccl group, kernel trace
run 400 rocprofv3 --kernel-trace --stats -d $OUT/rccl -o run --output-format csv -- python bench.py --mode train --force-ddp --steps 5 --warmup 2 --no-cpu-baseline --trace-steps 0 > $OUT/rccl_train.json 2> $OUT/rccl_train.log || exit 1
python - <<PY > $OUT/rccl_kernels.txt
import csv, glob
rows = []
for p in glob.glob('$OUT/rccl/**/*kernel_stats.csv', recursive=True):
    rows += list(csv.DictReader(open(p)))
hit = [r for r in rows if any(k in r['Name'].lower() for k in ('nccl', 'rccl', 'allreduce', 'all_reduce', 'onerank'))]
print('kernels matching nccl/rccl/allreduce:', len(hit))
for r in hit:
    print(r['Name'][:160], r['Calls'], r['AverageNs'])
PY
cat $OUT/rccl_kernels.txt
# every RCCL collective on a world-1 communicator, kernel trace + RCCL's init log
NCCL_DEBUG=INFO run 200 rocprofv3 --kernel-trace --stats -d $OUT/rccl_diag -o run --output-format csv -- python tools/diag_rccl.py > $OUT/rccl_diag.out 2> $OUT/rccl_diag.log || exit 1
grep "^{" $OUT/rccl_diag.out > $OUT/rccl_diag.json; cat $OUT/rccl_diag.json
python - <<PY > $OUT/rccl_diag_kernels.txt
import csv, glob
for p in glob.glob('$OUT/rccl_diag/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        print(r['Name'][:160], r['Calls'], r['AverageNs'])
PY
cat $OUT/rccl_diag_kernels.txt
grep -i -E "NCCL INFO (RCCL version|Init|comm 0x|Channel 00|.*nranks)" $OUT/rccl_diag.out | head -20 > $OUT/rccl_diag_init.txt || true
rm -f $OUT/rccl_diag/*/run_kernel_trace.csv $OUT/rccl_diag/run_kernel_trace.csv
rm -f $OUT/rccl/*/run_kernel_trace.csv $OUT/rccl/run_kernel_trace.csv
rm -rf $OUT/pmc_fetch_* $OUT/pmc_write_* $OUT/pmc_calib_* $OUT/pmc_occ
echo profile done
