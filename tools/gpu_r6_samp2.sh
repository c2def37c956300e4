#!/bin/bash
# Round-6: the one-launch sampler's window-record path -- sampler / status / whole-detector
# tests, the selection timeline (tools/bench_select.py) and the bench line.
set -o pipefail
O=${1:-gpurun_out/r6_samp2}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "(sampl or fused or whole or target) and not timed_out_wait" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_select.py --iters 50 > $O/select.json 2> $O/select.err || { tail -20 $O/select.err; exit 1; }
python -c "
import json;d=json.load(open('$O/select.json'));s=d['sampler'];print('sampler us/call', s['us_per_call_one_launch'], 'two-launch', s['us_per_call_two_launches'])
[print(' ', k, v['rel_wg_start_us'], v['rel_launch_us_median'], v['rel_launch_us_max']) for k, v in s['timeline_one_launch'].items()]
print('proposals us/call', d['rpn_proposals']['us_per_call_one_launch_select'])"
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ms_per_step'], d['kernels']['detection_path_kernels_us_per_step'])"
# last: the subset whose order exposed the unranked repeated-selection rows (round 6)
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sampl or fused or whole or status" > $O/pytest_status.log 2>&1 || { tail -30 $O/pytest_status.log; exit 1; }
tail -1 $O/pytest_status.log
