#!/bin/bash
# Round-6: sampler tests + bench line (detection-path kernels), then the per-set RoIAlign counters.
set -o pipefail
O=${1:-gpurun_out/r6_samp}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sampl or fused or whole" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ms_per_step'], d['kernels']['detection_path_kernels_us_per_step'])"
timeout -k 10 300 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants 94 --rounds 5 > $O/roi_sets.log 2>&1 || { tail -20 $O/roi_sets.log; exit 1; }
grep -v "amdgpu.ids\|alive\|bands=[3-7]" $O/roi_sets.log
bash tools/profile_r06.sh $O/prof b
