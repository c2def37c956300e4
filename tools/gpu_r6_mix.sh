#!/bin/bash
# Round-6 combined lab run: forward variants on the three RoI sets, then backward variants.
set -o pipefail
O=${1:-gpurun_out/r6_mix}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants $2 --rounds 5 > $O/roi_sets.log 2>&1 || { tail -30 $O/roi_sets.log; exit 1; }
grep -v "amdgpu.ids\|alive\|bands=[3-7]" $O/roi_sets.log
timeout -k 10 300 python -u tools/bench_roi_bwd.py --variants $3 --iters 10 --json $O/roi_bwd.json > $O/roi_bwd.log 2>&1 || { tail -30 $O/roi_bwd.log; exit 1; }
grep -v amdgpu.ids $O/roi_bwd.log
