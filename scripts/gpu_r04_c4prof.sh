#!/bin/bash
# Round 4: config 4 at 1 024 LPs in flight with the segment profile (device
# phase split, host ramp: when segments were enqueued and seen done).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c4prof
mkdir -p $OUT
cd $R
MILP_SDUAL_PROFILE=1 timeout -k 10 200 python3 -u scripts/probe_batch.py --node --lps 1024 \
  --workers 1024 > $OUT/c4.json 2> $OUT/c4.err || exit 1
timeout -k 10 200 python3 -u scripts/probe_batch.py --node --lps 1024 --workers 1024 --cpu \
  > $OUT/c4_cpu.json 2> $OUT/c4_cpu.err || exit 1
tail -45 $OUT/c4.err; tail -3 $OUT/c4_cpu.err
