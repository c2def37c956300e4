# end-of-round GPU check: full GPU suite, smoke, bench line, profiling recipe
set -o pipefail
O=${1:-gpurun_out/final}; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_tests.sh $O/tests && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
bash tools/profile_round.sh $O/prof && \
timeout -k 10 300 python tools/bench_nms.py --iters 30 > $O/nms_timeline.log 2>&1 && \
timeout -k 10 300 python tools/bench_select.py --iters 50 > $O/select_timeline.json 2>&1
