#!/bin/bash
# Round-6: kernel-level durations of the RoIAlign backward forms (rocprofv3 kernel trace of tools/bench_roi_bwd.py).
set -o pipefail
O=${1:-gpurun_out/r6_bwdprof}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/bench_roi_bwd.py --sets ${3:-bench,voc} --variants ${2:-0,4,6} --iters 5 > $O/bwd.log 2>&1 || { tail -30 $O/bwd.log; exit 1; }
grep -v amdgpu.ids $O/bwd.log | grep -v "^W2026\|^E2026"
python - <<PY
import csv, glob
for p in glob.glob('$O/prof/**/*kernel_stats.csv', recursive=True):
    rows = list(csv.DictReader(open(p)))
    rows.sort(key=lambda r: -float(r['TotalDurationNs']))
    for r in rows[:14]:
        print(r['Name'][:110], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us avg', round(float(r['MinNs'])/1e3,1), round(float(r['MaxNs'])/1e3,1))
PY
rm -f $O/prof/*/run_kernel_trace.csv $O/prof/run_kernel_trace.csv
