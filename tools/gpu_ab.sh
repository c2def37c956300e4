# bench A/B of the schedule knobs on one box: bash tools/gpu_ab.sh <outdir>
O=${1:-gpurun_out/ab}; mkdir -p $O; export TMPDIR=/tmp
for cfg in "--proposal-stream off --rpn-order reference" "--proposal-stream on --rpn-order reference" \
           "--proposal-stream off --rpn-order finest-last" "--proposal-stream on --rpn-order finest-last" \
           "--proposal-stream off --rpn-order reference"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 $cfg > $O/$tag.json 2> $O/$tag.err || exit $?
done
