# round-3 profile set: bench line, kernel stats + timed-step breakdown, RoIAlign PMC traffic +
# occupancy (tools/profile_round.sh), RoIAlign per-wave timeline, NMS scan timeline
set -o pipefail
O=${1:-gpurun_out/r03p}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "rpn or proposal" > $O/pytest.log 2>&1 &&
bash tools/profile_round.sh $O &&
timeout -k 10 300 python -u tools/bench_roi_align.py --variants 0,1 --iters 20 --rounds 3 --after-write > $O/roi_align_timeline.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_nms.py > $O/nms_timeline.log 2>&1
