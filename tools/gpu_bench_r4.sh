# bench line + per-dispatch RoIAlign table: bash tools/gpu_bench_r4.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/r4_bench}; mkdir -p $O/disp $O/disp_tracer; export TMPDIR=/tmp
timeout -k 10 420 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/disp/trace -o run --output-format csv -- python tools/roi_dispatch_table.py --out $O/disp/launches.json > $O/disp.log 2>&1 && \
python tools/roi_dispatch_table.py --join $O/disp --out $O/roi_dispatch_table.json && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/disp_tracer/trace -o run --output-format csv -- python tools/roi_dispatch_table.py --tracer --out $O/disp_tracer/launches.json > $O/disp_tracer.log 2>&1 && \
python tools/roi_dispatch_table.py --join $O/disp_tracer --out $O/roi_dispatch_table_tracer.json
rc=$?
rm -rf $O/disp/trace $O/disp_tracer/trace
exit $rc
