#!/bin/bash
# Round 5: RoIAlign item order / channels per wave on the three RoI sets, stamps, L2 hit PMC.
set -uo pipefail
O=gpurun_out/r5_roi2
mkdir -p $O
export TMPDIR=/tmp
cp gpurun_out/r5_roi/cfg2_rois_train.npz tests/golden/ 2>/dev/null || true
timeout -k 10 400 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants 26,12,9,27 --rounds 3 --json $O/sets.json > $O/sets.log 2>&1 || { echo "sets failed"; tail -30 $O/sets.log; exit 1; }
grep -v "waves alive" $O/sets.log
for grp in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  n=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $O/pmc_$n -o run --output-format csv -- python tools/bench_roi_sets.py --sets voc,bench --variants 26,12 --rounds 1 --iters 3 > $O/pmc_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
done
echo done
