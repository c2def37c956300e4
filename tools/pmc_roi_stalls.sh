# Stall breakdown of the RoIAlign forward candidates (one rocprofv3 --pmc pass per counter
# group, tools/bench_roi_align.py launches only): bash tools/pmc_roi_stalls.sh <outdir> <variants>
set -o pipefail
O=${1:-gpurun_out/pmc_roi}; V=${2:-10}; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace -d $O/a -o run --output-format csv -- python tools/bench_roi_align.py --variants $V --iters 5 > $O/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCC_WRITE_REQ_LATENCY --kernel-trace -d $O/b -o run --output-format csv -- python tools/bench_roi_align.py --variants $V --iters 5 > $O/b.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES SQ_CYCLES SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU --kernel-trace -d $O/c -o run --output-format csv -- python tools/bench_roi_align.py --variants $V --iters 5 > $O/c.log 2>&1
rc=$?
python tools/pmc_table.py $O/a roi_align_fwd > $O/table_a.txt; python tools/pmc_table.py $O/b roi_align_fwd > $O/table_b.txt; python tools/pmc_table.py $O/c roi_align_fwd > $O/table_c.txt
rm -rf $O/a $O/b $O/c
exit $rc
