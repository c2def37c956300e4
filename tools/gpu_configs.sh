# per-config bench lines (extra lines; the BASELINE metric is cfg2 fwd): bash tools/gpu_configs.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/configs}; mkdir -p $O; export TMPDIR=/tmp
for cfg in faster_rcnn_r50 retinanet_r50_fpn cascade_rcnn_r50_fpn fcos_r50_fpn_atss; do
  timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --steps 10 > $O/$cfg.json 2> $O/$cfg.err || exit $?
done
timeout -k 10 400 python -u bench.py --config retinanet_r50_fpn --batch 8 --no-cpu-baseline --steps 10 > $O/retinanet_r50_fpn_b8.json 2> $O/retinanet_r50_fpn_b8.err || exit $?
timeout -k 10 600 python -u bench.py --mode train --no-cpu-baseline --steps 5 --warmup 3 > $O/train_cfg2.json 2> $O/train_cfg2.err
