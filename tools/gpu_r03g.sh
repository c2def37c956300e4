# NMS scan timeline + NMS parity
set -o pipefail
O=${1:-gpurun_out/r03g}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_hand_derived.py \
  -k "nms" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_nms.py > $O/nms_lab.log 2>&1
