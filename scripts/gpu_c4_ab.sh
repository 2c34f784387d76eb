#!/bin/bash
# Config-4 batch (15x10 family, 512 children, 128 in flight): default against
# MILP_STREAM_PRIORITY=0, twice each (box noise).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for cfg in default MILP_STREAM_PRIORITY=0; do
    if [ $cfg = default ]; then E=""; else E=$cfg; fi
    env $E timeout -k 10 120 python -u scripts/probe_batch.py --lps 512 --workers 128 > $OUT/c4ab.json 2> $OUT/c4ab.err || { echo "$cfg failed"; tail -20 $OUT/c4ab.err; exit 1; }
    python -c "import json,sys;d=json.load(open('$OUT/c4ab.json'));print('$cfg', round(d['gpu_w128']['lps_per_s']))"
  done
done
echo done
