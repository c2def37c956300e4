# GPU tests then (unless the test step crashed / timed out) the bench: bash tools/gpu_tb.sh <outdir>
O=${1:-gpurun_out/tb}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
  echo "bench rc=$?" >> $O/bench.err
fi
exit $rc
