set -e
mkdir -p gpurun_out/s25
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s25/gputest.log 2>&1
bash tools/profile_round.sh gpurun_out/s25/prof
