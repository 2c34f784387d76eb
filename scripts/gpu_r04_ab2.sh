#!/bin/bash
# Round 4: config-5 window A/B of the triangular-solve switches on the final
# tree (zero-copy staging kernels vs copy engine, two-vector U launch,
# device BTRAN loops, chain min levels).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_ab2
mkdir -p $OUT
cd $R
timeout -k 10 700 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 \
  --steps 1000 --variants "" MILP_TRI_BTRAN=0 MILP_TRI_BTRAN=0,MILP_TRI_PAIR=0 "" MILP_TRI_BTRAN=0 \
  MILP_TRI_BTRAN=0,MILP_TRI_PAIR=0 MILP_TRI_PAIR=0 > $OUT/c5.json 2> $OUT/c5.err || exit 1
grep -h "variant\|it/s" $OUT/c5.err
