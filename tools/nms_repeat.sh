mkdir -p gpurun_out/r24
for i in 1 2 3 4 5 6; do timeout -k 10 100 python tools/bench_nms.py --segs 10 --n 5000 --thr 0.3 --no-timeline --variants 0,1 --iters 5 >> gpurun_out/r24/a.log 2>&1 || exit 1; done
timeout -k 10 100 python tools/bench_nms.py --segs 10 --n 2000 --thr 0.7 --variants 0,1,2 >> gpurun_out/r24/b.log 2>&1
