set -e
mkdir -p gpurun_out/s24
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_hand_derived.py -m gpu -x -q --timeout 120 --timeout-method thread -k "nms or mcnms or multiclass or proposals or retina_predict or forward_train or degenerate" > gpurun_out/s24/t.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s24/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/s24/stats.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/s24/bench.json 2> gpurun_out/s24/bench.err
rm -f gpurun_out/s24/stats/run_kernel_trace.csv
