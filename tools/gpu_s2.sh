set -e
mkdir -p gpurun_out/s11
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s11/gputest.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/s11/nmsprof -o run --output-format csv -- python tools/bench_nms.py --ab > gpurun_out/s11/nms.log 2>&1
bash tools/profile_round.sh gpurun_out/s11/prof
