# RoIAlign laboratory run: bash tools/gpu_lab.sh <outdir> <variants> [extra args]
set -o pipefail
O=${1:-gpurun_out/lab}; V=${2:-0}; shift 2
mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_roi_align.py --variants $V --iters 20 --rounds 3 --cold "$@" > $O/lab.log 2>&1
