#!/bin/bash
# Round-6 RoIAlign backward variants (tools 0/2: product forms, 4/5: readlane tap lists) on the three RoI sets,
# and optionally the stamped channel-group forward (variant 94).
set -o pipefail
O=${1:-gpurun_out/r6_bwd}; mkdir -p $O; export TMPDIR=/tmp
if [ -n "$3" ]; then
timeout -k 10 300 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants $3 --rounds 3 > $O/roi_sets.log 2>&1 || { tail -30 $O/roi_sets.log; exit 1; }
grep -v amdgpu.ids $O/roi_sets.log
fi
timeout -k 10 300 python -u tools/bench_roi_bwd.py --variants ${2:-0,4,2,5} --iters 10 --json $O/roi_bwd.json > $O/roi_bwd.log 2>&1 || { tail -30 $O/roi_bwd.log; exit 1; }
grep -v amdgpu.ids $O/roi_bwd.log
