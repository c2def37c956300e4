set -o pipefail
O=gpurun_out/r03a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 240 python -u tools/bench_roi_align.py --variants 0,1 --iters 20 --rounds 2 --cold > $O/lab.log 2>&1 && \
bash tools/pmc_roi.sh $O/pmc 0 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --trace-steps 0 --no-cpu-baseline > $O/stats.log 2>&1 && \
python tools/step_breakdown.py $O/stats --warmup 5 --steps 10 > $O/step_breakdown.json; rm -f $O/stats/run_kernel_trace.csv
