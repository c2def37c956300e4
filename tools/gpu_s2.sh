set -e
mkdir -p gpurun_out/s30
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s30/stats -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/s30/stats.log 2>&1
python tools/step_breakdown.py gpurun_out/s30/stats --warmup 3 --steps 10 > gpurun_out/s30/step_breakdown.json
rm -f gpurun_out/s30/stats/run_kernel_trace.csv
timeout -k 10 300 rocprofv3 --pmc OccupancyPercent MeanOccupancyPerCU --kernel-trace -d gpurun_out/s30/pmc_occ -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/s30/pmc_occ.log 2>&1
python tools/pmc_table.py gpurun_out/s30/pmc_occ frh:: > gpurun_out/s30/occupancy.txt
