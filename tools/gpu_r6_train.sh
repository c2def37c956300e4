#!/bin/bash
# Round-6: the train-mode bench line alone on a fresh box (the final check's train line ran
# MIOpen's naive convolutions in its timed steps), then the rocprofv3 kernel stats of it.
set -o pipefail
O=${1:-gpurun_out/r6_tr}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --mode train --no-cpu-baseline --steps 5 --warmup 3 > $O/train.json 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/train.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
mkdir -p $O/prof && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --mode train --no-cpu-baseline --steps 5 --warmup 3 > $O/train_rocprof.json 2> $O/rocprof.err || { tail -20 $O/rocprof.err; exit 1; }
echo done
