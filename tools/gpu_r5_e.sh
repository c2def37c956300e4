#!/bin/bash
set -o pipefail
O=gpurun_out/r5_e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_whole.py -k "device_sampler" tests/test_gpu_parity.py -k "device_sampler or roi_align or assign or prepend or bbox_target" > $O/pytest.log 2>&1; rc=$?
tail -40 $O/pytest.log | grep -v "^tests.*PASSED"
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step']); r=d['roofline']; print('roi', r['avg_launch_us'], r['frac'], 'in-step', r['in_step_span_us_median'], r['frac_in_step'])
for k in ('roofline_voc_rois','roofline_train_rois'): v=d.get(k) or {}; print(k, v.get('avg_launch_us'), v.get('frac'))
print('det', d['kernels']['detection_path_us_per_step'])"
