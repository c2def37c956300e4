#!/bin/bash
# Round 5 (b): status word / launcher / fused tests, then the RoIAlign item-order variants.
set -uo pipefail
O=gpurun_out/r5_b
mkdir -p $O
export TMPDIR=/tmp
cp gpurun_out/r5_roi/cfg2_rois_train.npz tests/golden/ 2>/dev/null || true
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_status.py tests/test_gpu_fused.py tests/test_gpu_bench.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/gpu_r5_roi2.sh
