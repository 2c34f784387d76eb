#!/bin/bash
# C5 U-solve plan A/B and the sharded-window divergence variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 \
  --variants "" "MILP_TRI_SYNCFREE=0" "MILP_TRI_SYNCFREE=0,MILP_TRI_WIDE=4096" \
  > $OUT/probe_plan.json 2> $OUT/probe_plan.err || { echo "plan probe failed"; tail -20 $OUT/probe_plan.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/probe_plan.json'))
for k,v in d['gpu'].items(): print(k, round(v['gpu_it_per_s'],1), {n:(s['launches'],s['device_ms'],s['call_ms']) for n,s in v['kernels'].items() if n.startswith('tri')})"
timeout -k 10 400 python -u scripts/probe_divergence.py --m 20000 --n 200000 --per-col 10 --seed 97 --caps 3000 \
  --variants MILP_SHARDS=8,MILP_DUAL_TIGHTEN_MIN=100000000 MILP_SHARDS=8,MILP_DEVICE_DUAL=off MILP_SHARDS=2 \
  MILP_SHARDS=8,MILP_FULL_ROWS=off MILP_SHARDS=8,MILP_DENSE_BLOCK=off \
  > $OUT/divergence2.log 2>&1 || { echo "divergence probe failed"; tail -20 $OUT/divergence2.log; exit 1; }
cat $OUT/divergence2.log
timeout -k 10 400 python -u scripts/probe_divergence.py --m 2000 --n 20000 --per-col 10 --seed 97 --caps 1000 \
  --variants MILP_SHARDS=8 MILP_SHARDS=8,MILP_DEVICE_DUAL=force > $OUT/divergence3.log 2>&1 || { echo "divergence probe 3 failed"; tail -20 $OUT/divergence3.log; exit 1; }
cat $OUT/divergence3.log
echo done
