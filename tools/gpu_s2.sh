set -e
mkdir -p gpurun_out/s29
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tools_variants.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s29/t.log 2>&1
timeout -k 10 300 python tools/bench_roi_align.py --variants 47,55 --iters 100 --rounds 7 > gpurun_out/s29/roi.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s29/gputest.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/s29/bench.json 2> gpurun_out/s29/bench.err
