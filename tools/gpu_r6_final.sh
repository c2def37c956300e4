#!/bin/bash
# Round-6 final check: full GPU suite, smoke, the default bench line, the train-mode line, the
# selection / sampler timeline, and a rocprofv3 kernel-stats pass over the bench.
set -o pipefail
O=${1:-gpurun_out/r6_final}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ms_per_step'], d['roofline'])"
timeout -k 10 400 python bench.py --mode train --no-cpu-baseline > $O/bench_train.json 2> $O/bench_train.err || { tail -20 $O/bench_train.err; exit 1; }
timeout -k 10 300 python -u tools/bench_select.py --iters 50 > $O/select.json 2> $O/select.err || { tail -20 $O/select.err; exit 1; }
python -c "
import json;d=json.load(open('$O/select.json'));s=d['sampler'];print('sampler us/call', s['us_per_call_one_launch'], 'two-launch', s['us_per_call_two_launches'])"
mkdir -p $O/prof && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_rocprof.json 2> $O/rocprof.err || { tail -20 $O/rocprof.err; exit 1; }
echo profile done
