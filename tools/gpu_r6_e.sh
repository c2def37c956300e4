#!/bin/bash
set -o pipefail
OUT=${1:-gpurun_out/r6_e}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 "$@"; }
run 300 python bench.py --mode train --steps 10 --warmup 3 --trace-steps 2 --no-cpu-baseline > $OUT/train_plain.json 2> $OUT/train_plain.err || { tail -30 $OUT/train_plain.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/train_plain.json').read().strip().splitlines()[-1]); print('train', round(d['value'],2), round(d['ms_per_step'],1)); print(d['kernels'].get('device_timeline'))"
run 400 python -m cProfile -o $OUT/train.prof bench.py --mode train --steps 5 --warmup 2 --trace-steps 0 --no-cpu-baseline > $OUT/train.json 2> $OUT/train.err || { tail -30 $OUT/train.err; exit 1; }
python -c "
import pstats; p=pstats.Stats('$OUT/train.prof'); p.sort_stats('tottime').print_stats(20)
" > $OUT/summary.txt 2>&1
head -60 $OUT/summary.txt
run 300 python -u tools/bench_roi_bwd.py --variants 0,1,2,3 --iters 10 --json $OUT/roi_bwd.json > $OUT/roi_bwd.log 2>&1 || { tail -20 $OUT/roi_bwd.log; exit 1; }
grep -v amdgpu.ids $OUT/roi_bwd.log
