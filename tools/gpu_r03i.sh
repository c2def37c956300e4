# NMS resolver + merge changes: NMS / proposal / mcnms parity, NMS timeline, bench line
set -o pipefail
O=${1:-gpurun_out/r03i}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_hand_derived.py tests/test_gpu_whole.py \
  -k "nms or rpn or proposal or mcnms or multiclass or whole" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_nms.py > $O/nms_lab.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
