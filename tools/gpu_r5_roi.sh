#!/bin/bash
# Round 5: RoIAlign forward on the three RoI sets (product vs round-4 library vs variants),
# the train step's RoIs dumped, and the RoIAlign parity tests.
set -uo pipefail
O=gpurun_out/r5_roi
mkdir -p $O
timeout -k 10 300 python -u tools/bench_roi_sets.py --sets bench,voc --variants 25 --rounds 3 --json $O/sets.json > $O/sets.log 2>&1 || { echo "sets failed"; tail -30 $O/sets.log; exit 1; }
cat $O/sets.log
timeout -k 10 600 python -u bench.py --mode train --steps 10 --warmup 3 --trace-steps 0 --no-cpu-baseline --dump-rois $O/cfg2_rois_train.npz > $O/train.json 2> $O/train.err || { echo "train failed"; tail -30 $O/train.err; exit 1; }
cp $O/cfg2_rois_train.npz tests/golden/
timeout -k 10 300 python -u tools/bench_roi_sets.py --sets train --variants 25 --rounds 3 --json $O/sets_train.json > $O/sets_train.log 2>&1 || { echo "sets train failed"; tail -30 $O/sets_train.log; exit 1; }
cat $O/sets_train.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k roi_align > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
