#!/bin/bash
# Round 4: config-5 window vs the host pool's parts per loop (the pool is
# created with 16 threads; MILP_HOST_THREADS caps the parts per call).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_threads
mkdir -p $OUT
cd $R
MILP_HOST_THREADS=16 timeout -k 10 500 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20020 --steps 1000 --variants MILP_HOST_THREADS=8 MILP_HOST_THREADS=4 MILP_HOST_THREADS=12 \
  MILP_HOST_THREADS=16 > $OUT/c5.json 2> $OUT/c5.err || exit 1
grep -h "variant\|it/s" $OUT/c5.err
