set -e
mkdir -p gpurun_out/s18
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tools_variants.py tests/test_hand_derived.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s18/t.log 2>&1
timeout -k 10 300 python tools/bench_roi_align.py --variants 21,47,29 --iters 100 --rounds 5 > gpurun_out/s18/roi.log 2>&1
