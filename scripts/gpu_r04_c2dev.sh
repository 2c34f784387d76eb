#!/bin/bash
# Round 4: config 2's late window (iterations 1500..1564, a basis with a
# dense ~1500-column kernel) with the triangular solves on the device
# (the auto rule keeps m < 16 384 on the host): default, min rows 4096,
# forced; schedule shapes printed.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c2dev
mkdir -p $OUT
cd $R
MILP_TRI_SCHED=1 timeout -k 10 500 python3 -u scripts/probe.py --config c2 --warmup 1500 --steps 64 \
  --variants "" MILP_DEVICE_SOLVE_MIN_ROWS=4096 MILP_DEVICE_SOLVE=force \
  > $OUT/c2_late.json 2> $OUT/c2_late.err || exit 1
grep "it/s\|variant" $OUT/c2_late.err
