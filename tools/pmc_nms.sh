# Issue / stall counters of the NMS kernels (the RPN call replayed by tools/bench_nms.py: the
# two-launch mask + scan and the one-launch nms_fused_kernel), one rocprofv3 --pmc pass per
# counter group: bash tools/pmc_nms.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/pmc_nms}; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace -d $O/a -o run --output-format csv -- python tools/bench_nms.py --iters 5 > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_CYCLES SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU --kernel-trace -d $O/c -o run --output-format csv -- python tools/bench_nms.py --iters 5 > $O/c.log 2>&1
rc=$?
python tools/pmc_table.py $O/a nms_ > $O/table_a.txt; python tools/pmc_table.py $O/c nms_ > $O/table_c.txt
rm -rf $O/a $O/c
exit $rc
