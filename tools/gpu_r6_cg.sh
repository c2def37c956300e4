#!/bin/bash
# Round-6: channel-group RoIAlign forward candidates (tools variants 80-85) vs the product on the three RoI sets.
set -o pipefail
O=${1:-gpurun_out/r6_cg}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_roi_sets.py --sets bench,voc,train --variants ${2:-80,81,82,83,84,85} --rounds 5 --json $O/roi_sets.json > $O/roi_sets.log 2>&1 || { tail -30 $O/roi_sets.log; exit 1; }
grep -v amdgpu.ids $O/roi_sets.log
