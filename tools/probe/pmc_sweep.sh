set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export SETS=all VARIANTS=${VARIANTS:-60} ITERS=2 WARM=1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcs1 -o p -- python3 tools/probe/probe_roi_sets.py > gpurun_out/pmcs1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/pmcs2 -o p -- python3 tools/probe/probe_roi_sets.py > gpurun_out/pmcs2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA TA_BUSY_avr TD_BUSY_avr --output-format csv -d gpurun_out/pmcs3 -o p -- python3 tools/probe/probe_roi_sets.py > gpurun_out/pmcs3.log 2>&1
echo done
