# quick check: selected GPU tests (pytest -k expression) then the bench line: bash tools/gpu_check.sh <outdir> "<k expr>"
set -o pipefail
O=${1:-gpurun_out/check}; K=${2:-sampler}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "$K" > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
