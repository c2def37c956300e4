#!/bin/bash
set -o pipefail
OUT=${1:-gpurun_out/r6_d}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 "$@"; }
run 400 python -u tools/diag_train_step.py > $OUT/diag_train.log 2>&1 || { tail -30 $OUT/diag_train.log; exit 1; }
grep -v amdgpu.ids $OUT/diag_train.log
run 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_fwd.json 2> $OUT/bench_fwd.err || { tail -20 $OUT/bench_fwd.err; exit 1; }
python -c "
import json; d=json.loads(open('$OUT/bench_fwd.json').read().strip().splitlines()[-1]); print('fwd', round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['avg_launch_us'], d['roofline']['traffic_source'])
print(d['kernels']['detection_path_kernels_us_per_step'])"
