#!/bin/bash
# Round-6 restart check: full GPU suite, smoke, the default bench line, RoI-set lines.
set -o pipefail
O=${1:-gpurun_out/r6_start}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ms_per_step'], d['roofline'])"
timeout -k 10 300 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants 62 --rounds 5 > $O/roi_sets.log 2>&1 || { tail -20 $O/roi_sets.log; exit 1; }
grep -v amdgpu.ids $O/roi_sets.log
