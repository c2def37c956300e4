# round-3 final profile set: bash tools/gpu_profile_r03b.sh <outdir>
#  two plain bench runs (process-to-process spread of the in-step RoIAlign duration), the
#  profile_round.sh set (bench line, rocprofv3 kernel stats + timed-step breakdown, RoIAlign
#  PMC traffic, occupancy), the NMS scan timeline and the RoIAlign per-wave timeline
set -o pipefail
O=${1:-gpurun_out/r03b}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_a.json 2> $O/bench_a.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err &&
bash tools/profile_round.sh $O &&
timeout -k 10 300 python -u tools/bench_nms.py > $O/nms_timeline.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_roi_align.py --variants 0,1 --iters 20 --rounds 3 --after-write > $O/roi_align_timeline.log 2>&1
