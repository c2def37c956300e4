#!/bin/bash
# Round 5 (c): band kernel -- RoIAlign parity tests, then the RoI sets with the variants.
set -uo pipefail
O=gpurun_out/r5_c
mkdir -p $O
export TMPDIR=/tmp
cp gpurun_out/r5_roi/cfg2_rois_train.npz tests/golden/ 2>/dev/null || true
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "roi_align" tests/test_hand_derived.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants 10,26,28,33,31,29 --rounds 3 --json $O/sets.json > $O/sets.log 2>&1 || { echo "sets failed"; tail -30 $O/sets.log; exit 1; }
grep -v "waves alive" $O/sets.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "deterministic" > $O/pytest_det.log 2>&1 || { echo "pytest det failed"; tail -40 $O/pytest_det.log; exit 1; }
tail -3 $O/pytest_det.log
timeout -k 10 300 python -u tools/bench_roi_bwd.py --json $O/bwd.json > $O/bwd.log 2>&1 || { echo "bwd failed"; tail -20 $O/bwd.log; exit 1; }
cat $O/bwd.log
