#!/bin/bash
# U-solve plans (fused level plan vs sync-free), their kernel split, and the
# sharded-window size/async variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 \
  --variants "" "MILP_TRI_GRAPH=0" "MILP_TRI_GRAPH=0,MILP_TRI_SYNCFREE_MIN_LEVELS=64" "MILP_TRI_GRAPH=0,MILP_TRI_SYNCFREE_MIN_LEVELS=64,MILP_TRI_MAPPED=0" \
  > $OUT/probe_plan.json 2> $OUT/probe_plan.err || { echo "plan probe failed"; tail -20 $OUT/probe_plan.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/probe_plan.json'))
for k,v in d['gpu'].items(): print(k, round(v['gpu_it_per_s'],1), {n:(s['launches'],s['device_ms'],s['call_ms']) for n,s in v['kernels'].items() if n.startswith('tri')})"
cd /tmp && export TMPDIR=/tmp
MILP_TRI_GRAPH=0 MILP_TRI_SYNCFREE_MIN_LEVELS=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_lv -o run -- python3 $R/scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 300 > $OUT/prof_lv.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_lv.log; }
find $OUT/prof_lv -name "*kernel_stats.csv" -exec cp {} $OUT/kstats_levels.csv \;
rm -rf $OUT/prof_lv
grep -i "tri_\|Name" $OUT/kstats_levels.csv | cut -c 1-200
cd $R
timeout -k 10 400 python -u scripts/probe_divergence.py --m 20000 --n 200000 --per-col 10 --seed 97 --caps 3000 \
  --variants MILP_SHARDS=8,MILP_ASYNC_SOLVES=off MILP_SHARDS=8,MILP_INLINE_TAU=off > $OUT/divergence4.log 2>&1 || { echo "div4 failed"; tail -20 $OUT/divergence4.log; exit 1; }
cat $OUT/divergence4.log
timeout -k 10 400 python -u scripts/probe_divergence.py --m 12000 --n 120000 --per-col 10 --seed 97 --caps 3000 \
  --variants MILP_SHARDS=8 MILP_SHARDS=1 > $OUT/divergence5.log 2>&1 || { echo "div5 failed"; tail -20 $OUT/divergence5.log; exit 1; }
cat $OUT/divergence5.log
echo done
