#!/bin/bash
# Round 4: wall-clock host profile of config 2's late window (1 500..1 564).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c2sample
mkdir -p $OUT
cd $R
MILP_SAMPLE_PROFILE=100 MILP_SAMPLE_STACK=1 MILP_SAMPLE_WALL=1 timeout -k 10 300 python3 -u scripts/probe.py \
  --config c2 --warmup 1500 --steps 64 > $OUT/c2.json 2> $OUT/c2.err || exit 1
grep -h "it/s" $OUT/c2.err
grep -A45 "sampler\] inclusive" $OUT/c2.err
