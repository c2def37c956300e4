#!/bin/bash
# Round-6 RoIAlign forward variants (trim, interleaved rotation) on the three RoI sets, and the
# train step with / without the per-step status check.   bash tools/gpu_r6_b.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r6_b}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 "$@"; }
run 300 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants 62,63,64,65 --rounds 5 --json $OUT/roi_sets.json > $OUT/roi_sets.log 2>&1 || { tail -20 $OUT/roi_sets.log; exit 1; }
cat $OUT/roi_sets.log
for se in 1 0 1 0; do
  run 300 python bench.py --mode train --status-every $se --steps 20 --warmup 3 --trace-steps 0 --no-cpu-baseline >> $OUT/train_status.jsonl 2> $OUT/train_status.err || { tail -20 $OUT/train_status.err; exit 1; }
done
python -c "
import json
for l in open('$OUT/train_status.jsonl'):
    d=json.loads(l); print(d['config']['status_every'], round(d['value'],2), round(d['ms_per_step'],3))
"
