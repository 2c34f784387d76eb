#!/bin/bash
# Config-3 suite: fibers per thread (MILP_BATCH_FIBERS) and threads (--c3-workers).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for cfg in "4 16" "8 16" "2 16" "4 32" "4 16"; do
  set -- $cfg
  MILP_BATCH_FIBERS=$1 timeout -k 10 240 python -u bench.py --no-cpu --no-c2 --c5-window 200 --steps 50 --warmup 5 --batch-lps 16 --batch-workers 16 --c3-workers $2 > $OUT/c3ab.json 2> $OUT/c3ab.err || { echo "$cfg failed"; tail -20 $OUT/c3ab.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/c3ab.json').read().strip().splitlines()[-1]);c=d['c3'];print('fibers $1 threads $2', round(c['value'],1), c['seconds'])"
done
echo done
