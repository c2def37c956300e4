#!/bin/bash
# Round-6: the RoIAlign GPU tests (forward, backward, deterministic, DDP) + smoke + bench line.
set -o pipefail
O=${1:-gpurun_out/r6_tests}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${2:-roi_align or roi or ddp or rccl or train or status}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value'],1), d['ms_per_step'], 'roi', round(r['avg_launch_us'],2), round(r['frac'],3), 'span', r['in_step_span_us_median'], 'traffic', r['traffic'], d['roofline_voc_rois']['avg_launch_us'], d['roofline_train_rois']['avg_launch_us'])"
