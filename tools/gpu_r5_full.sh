#!/bin/bash
# Round 5: full GPU suite, smoke, bench line, then the round-5 profiling recipe.
set -o pipefail
O=${1:-gpurun_out/r5_full}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_tests.sh $O/tests; rc=$?
tail -5 $O/tests/pytest.log
grep -E "FAILED|ERROR" $O/tests/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step']); r=d['roofline']; print('roi', r['avg_launch_us'], r['frac'], 'in-step', r['in_step_span_us_median'], r['frac_in_step'])
for k in ('roofline_voc_rois','roofline_train_rois'): v=d.get(k) or {}; print(k, v.get('avg_launch_us'), v.get('frac'))
print('nms', d['kernels']['per_step']['nms']); print('det', d['kernels']['detection_path_us_per_step'])"
bash tools/profile_r05.sh $O/prof
