#!/bin/bash
# Round-6: the sync-free train guard (fused SGD found_inf), the adopted RoIAlign trim + rotation,
# the atomic-free sampler slots, RoI processing-order experiment.
set -o pipefail
OUT=${1:-gpurun_out/r6_c}
mkdir -p $OUT
export TMPDIR=/tmp
run() { timeout -k 10 "$@"; }
run 700 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_status.py tests/test_gpu_rccl.py tests/test_gpu_fused.py \
  tests/test_gpu_whole.py "tests/test_gpu_parity.py::test_roi_align_forward_bench_config_bit_exact" \
  "tests/test_gpu_parity.py::test_roi_align_multilevel_vs_oracle" -k "not rpn_one_launch_selection" \
  -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run 200 python -u -m pytest tests/test_gpu_parity.py -k "sampler or device_sampler or sample" -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_sampler.log 2>&1 || { tail -40 $OUT/tests_sampler.log; exit 1; }
tail -1 $OUT/tests_sampler.log
run 200 python -u tools/bench_select.py --iters 100 > $OUT/select.json 2> $OUT/select.err || { tail -20 $OUT/select.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/select.json')); s=d['sampler']; print('sampler one-launch', s['us_per_call_one_launch'], 'two', s['us_per_call_two_launches'])
for k,v in s['timeline_one_launch'].items(): print('  ', k, v['rel_launch_us_median'], v['rel_launch_us_max'])
"
run 300 python -u tools/bench_roi_order.py --sets bench,voc,train --rounds 5 > $OUT/roi_order.log 2>&1 || { tail -20 $OUT/roi_order.log; exit 1; }
grep -v amdgpu.ids $OUT/roi_order.log
run 300 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants 62,66,67 --rounds 7 --json $OUT/roi_sets.json > $OUT/roi_sets.log 2>&1 || { tail -20 $OUT/roi_sets.log; exit 1; }
grep -v amdgpu.ids $OUT/roi_sets.log
for se in 0 1 0; do
  run 300 python bench.py --mode train --status-every $se --steps 20 --warmup 3 --trace-steps 0 --no-cpu-baseline >> $OUT/train_status.jsonl 2> $OUT/train_status.err || { tail -20 $OUT/train_status.err; exit 1; }
done
python -c "
import json
for l in open('$OUT/train_status.jsonl'):
    d=json.loads(l); print(d['config']['status_every'], round(d['value'],2), round(d['ms_per_step'],3))
"
