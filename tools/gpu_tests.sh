# GPU test suite: bash tools/gpu_tests.sh <outdir> [pytest -k expr]
set -o pipefail
O=${1:-gpurun_out/tests}; K=${2:-}
mkdir -p $O; export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
fi
