# round-3 check: changed-kernel parity tests, the bench line, the RoIAlign timeline cold and after a feature rewrite
set -o pipefail
O=${1:-gpurun_out/r03b}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_losses.py \
  tests/test_gpu_whole.py tests/test_gpu_parity.py -k "loss or whole or assign or roi_rows or level or anchor_target or bbox_target or forward_train or baseline_config" > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -u tools/bench_roi_align.py --variants 0,1 --iters 20 --cold --after-write > $O/lab.log 2>&1
