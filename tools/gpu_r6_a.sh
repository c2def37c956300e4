#!/bin/bash
# Round-6 first GPU check: the tests the ABI-3 changes touch, smoke(), the RCCL world-1 test,
# a train-mode bench with DDP forced on over RCCL.   bash tools/gpu_r6_a.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r6_a}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 "$@"; }
run 600 python -u -m pytest tests/test_gpu_status.py tests/test_gpu_losses.py tests/test_gpu_rccl.py \
  "tests/test_gpu_parity.py::test_roi_align_backward_deterministic" \
  "tests/test_gpu_parity.py::test_roi_align_backward_deterministic_nonfinite_and_unsupported" \
  tests/test_gpu_ddp.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
run 400 python bench.py --mode train --force-ddp --steps 10 --warmup 3 --trace-steps 0 --no-cpu-baseline > $OUT/bench_train_ddp.json 2> $OUT/bench_train_ddp.err || { tail -20 $OUT/bench_train_ddp.err; exit 1; }
run 400 python bench.py --mode train --steps 10 --warmup 3 --trace-steps 0 --no-cpu-baseline > $OUT/bench_train.json 2> $OUT/bench_train.err || { tail -20 $OUT/bench_train.err; exit 1; }
echo done
