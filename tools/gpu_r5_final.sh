#!/bin/bash
# Round-5 final GPU check (GPU box): the whole GPU suite, smoke(), the bench line, the RoIAlign
# forward on the three RoI sets, the RoIAlign backward forms, the proposals chain timing.
#   bash tools/gpu_r5_final.sh <outdir under gpurun_out>
set -o pipefail
OUT=${1:-gpurun_out/r5_final}
mkdir -p $OUT
run() { timeout -k 10 "$@"; }
run 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
run 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
run 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
run 300 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants "" --rounds 3 --json $OUT/roi_sets.json > $OUT/roi_sets.log 2>&1 || exit 1
run 200 python -u tools/bench_roi_bwd.py --json $OUT/roi_bwd.json > $OUT/roi_bwd.log 2>&1 || exit 1
run 200 python -u tools/bench_select.py --iters 100 > $OUT/select.json 2> $OUT/select.err || exit 1
echo final done
