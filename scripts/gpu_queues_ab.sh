#!/bin/bash
# C4 rate vs hardware queues per process, with fibers (MILP_BATCH_THREADS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for Q in 4 8 16; do
  for W in 16 64; do
    GPU_MAX_HW_QUEUES=$Q MILP_BATCH_THREADS=16 timeout -k 10 200 python -u scripts/probe_batch.py --lps 512 --workers $W > $OUT/q${Q}_w${W}.json 2> $OUT/q${Q}_w${W}.err || { echo "probe failed"; tail -20 $OUT/q${Q}_w${W}.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/q${Q}_w${W}.json')); print('Q=$Q W=$W', [round(v['lps_per_s'],1) for v in d['gpu'].values()])"
  done
done
echo done
