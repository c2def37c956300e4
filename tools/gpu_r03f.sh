# sampler keys / RPN merge changes: parity tests, bench line
set -o pipefail
O=${1:-gpurun_out/r03f}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_whole.py \
  -k "sampler or rpn or proposal or whole or forward_train or baseline_config or anchor_target or bbox_target" > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
