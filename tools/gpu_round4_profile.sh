# round-4 GPU session: full GPU suite, then the profiling recipe and a counter list
set -o pipefail
O=${1:-gpurun_out/r4_full}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_tests.sh $O/tests && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
bash tools/profile_round.sh $O/prof && \
timeout -k 10 120 rocprofv3 --list-avail > $O/counters.txt 2>&1
