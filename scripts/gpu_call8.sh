#!/bin/bash
# Sync-free U solve with write-through init (A/B vs the level plan), tests,
# and the shard bisect on the small-path switch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u -m pytest tests/test_device_solve_gpu.py -m gpu -q -x --timeout 100 --timeout-method thread \
  > $OUT/tri_tests.log 2>&1 || { echo "tri tests failed"; tail -30 $OUT/tri_tests.log; exit 1; }
tail -1 $OUT/tri_tests.log
timeout -k 10 300 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 \
  --variants "" "MILP_TRI_GRAPH=0" "MILP_TRI_SYNCFREE=0" \
  > $OUT/probe_plan.json 2> $OUT/probe_plan.err || { echo "plan probe failed"; tail -20 $OUT/probe_plan.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/probe_plan.json'))
for k,v in d['gpu'].items(): print(k, round(v['gpu_it_per_s'],1), {n:(s['launches'],s['device_ms'],s['call_ms']) for n,s in v['kernels'].items() if n.startswith('tri')})"
timeout -k 10 300 python -u scripts/probe_divergence.py --m 2000 --n 20000 --per-col 10 --seed 97 --caps 1000 \
  --variants MILP_SHARDS=8,MILP_SMALL_FUSED=off MILP_SHARDS=2,MILP_SMALL_FUSED=off > $OUT/divergence6.log 2>&1 || { echo "div6 failed"; tail -20 $OUT/divergence6.log; exit 1; }
cat $OUT/divergence6.log
echo done
