#!/bin/bash
# Round 5 (d): hybrid quad/band RoIAlign variants on the three RoI sets.
set -uo pipefail
O=gpurun_out/r5_d
mkdir -p $O
timeout -k 10 400 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants ${1:-26,28,35,36,37} --rounds 3 --json $O/sets.json > $O/sets.log 2>&1 || { echo "sets failed"; tail -30 $O/sets.log; exit 1; }
grep -v "waves alive" $O/sets.log
