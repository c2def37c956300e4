# assign parity, two bench lines, kernel stats + timed-step breakdown, RoIAlign timeline (cold / after a rewrite)
set -o pipefail
O=${1:-gpurun_out/r03c}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "assign or roi_rows or anchor_target or bbox_target or forward_train" > $O/pytest.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err &&
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --trace-steps 0 > $O/stats.log 2>&1 &&
python tools/step_breakdown.py $O/stats --warmup 3 --steps 10 > $O/step_breakdown.json &&
rm -f $O/stats/run_kernel_trace.csv &&
timeout -k 10 300 python -u tools/bench_roi_align.py --variants 0,1 --iters 20 --cold --after-write > $O/lab.log 2>&1
