#!/bin/bash
# Round-6 RCCL evidence: every collective on a world-1 RCCL communicator under rocprofv3's kernel trace.
set -o pipefail
OUT=${1:-gpurun_out/r6_rccl}; mkdir -p $OUT; export TMPDIR=/tmp
NCCL_DEBUG=INFO timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/rccl_diag -o run --output-format csv -- python tools/diag_rccl.py > $OUT/rccl_diag.out 2> $OUT/rccl_diag.log || { tail -30 $OUT/rccl_diag.log; exit 1; }
grep "^{" $OUT/rccl_diag.out > $OUT/rccl_diag.json; cat $OUT/rccl_diag.json
python - <<PY > $OUT/rccl_diag_kernels.txt
import csv, glob
for p in glob.glob('$OUT/rccl_diag/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        print(r['Name'][:160], r['Calls'], r['AverageNs'])
PY
cat $OUT/rccl_diag_kernels.txt
grep -i "NCCL INFO" $OUT/rccl_diag.out | head -40 > $OUT/rccl_diag_init.txt || true
rm -f $OUT/rccl_diag/*/run_kernel_trace.csv $OUT/rccl_diag/run_kernel_trace.csv
