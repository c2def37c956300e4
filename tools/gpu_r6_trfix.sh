#!/bin/bash
# Round-6: forward bench, then the train-mode bench in the same box (MIOpen user-db isolation).
set -o pipefail
O=${1:-gpurun_out/r6_trfix}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 600 python bench.py --mode train --no-cpu-baseline > $O/bench_train.json 2> $O/bench_train.err || { tail -20 $O/bench_train.err; exit 1; }
python -c "
import json
for f in ('bench', 'bench_train'):
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'])"
