#!/bin/bash
# Round 4: config 2 at iteration 300 with and without the device triangular
# solves (per-kernel device time in the JSON).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c2dev
mkdir -p $OUT
cd $R
timeout -k 10 400 python3 -u scripts/probe.py --config c2 --warmup 300 --steps 16 \
  --variants "" MILP_DEVICE_SOLVE_MIN_ROWS=4096 > $OUT/c2_300.json 2> $OUT/c2_300.err || exit 1
python3 -c "
import json
for k, d in json.load(open('$OUT/c2_300.json'))['gpu'].items():
    print(k, 'it/s', round(d['gpu_it_per_s'], 2))
    for n, v in d['kernels'].items():
        if v.get('call_ms', 0) > 1: print('   ', n, v)"
