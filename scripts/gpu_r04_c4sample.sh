#!/bin/bash
# Round 4: wall-clock host profile of one config-4 batch worker thread
# (fibers of many LPs), 1 024 LPs in flight.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c4sample
mkdir -p $OUT
cd $R
MILP_SAMPLE_PROFILE=100 MILP_SAMPLE_STACK=1 MILP_SAMPLE_WALL=batch MILP_SDUAL_PROFILE=1 timeout -k 10 200 \
  python3 -u scripts/probe_batch.py --node --lps 1024 --workers 1024 > $OUT/c4.json 2> $OUT/c4.err || exit 1
grep "LPs/s" $OUT/c4.err; grep "enqueued\|done at" $OUT/c4.err
grep -A45 "sampler\] inclusive" $OUT/c4.err
