set -e
mkdir -p gpurun_out/s16
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_hand_derived.py -m gpu -x -q --timeout 120 --timeout-method thread -k "nms or mcnms or multiclass or proposals or retina_predict or forward_train or eval" > gpurun_out/s16/t.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/s16/nmsprof -o run --output-format csv -- python tools/bench_nms.py --ab > gpurun_out/s16/nms.log 2>&1
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/s16/bench.json 2> gpurun_out/s16/bench.err
