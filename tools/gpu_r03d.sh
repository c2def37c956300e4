# RoIAlign descriptor path: parity, lab A/B (+ stamps), bench line
set -o pipefail
O=${1:-gpurun_out/r03d}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_hand_derived.py \
  -k "roi_align or merge or proposals or rpn" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_roi_align.py --variants 0,2,1,3 --iters 20 --rounds 3 --after-write > $O/lab.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
