#!/bin/bash
# LPSolver tests, shard-window divergence probe, U-solve level timing, C5 profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_lp_solver.py tests/test_linear_solver.py -m gpu -q -x \
  --timeout 120 --timeout-method thread > $OUT/lp_solver_tests.log 2>&1 || { echo "lp solver tests failed"; tail -30 $OUT/lp_solver_tests.log; }
tail -2 $OUT/lp_solver_tests.log
timeout -k 10 400 python -u scripts/probe_divergence.py --m 20000 --n 200000 --per-col 10 --seed 97 --caps 3000 \
  --variants MILP_SHARDS=8 MILP_SHARDS=8,MILP_DEVICE_SOLVE=off MILP_SHARDS=1 MILP_SHARDS=1,MILP_TRI_LOWER=0 MILP_SHARDS=1,MILP_DEVICE_SOLVE=off \
  > $OUT/divergence.log 2>&1 || { echo "divergence probe failed"; tail -20 $OUT/divergence.log; exit 1; }
cat $OUT/divergence.log
MILP_TRI_DEBUG=2 MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=500 timeout -k 10 200 python -u scripts/probe.py --config c5 \
  --m 100000 --n 1000000 --warmup 20000 --steps 500 > $OUT/probe_dbg.json 2> $OUT/probe_dbg.err || { echo "dbg probe failed"; tail -20 $OUT/probe_dbg.err; exit 1; }
WORKLOADS=c5 TAG=r02 bash scripts/gpu_profile.sh > $OUT/profile.log 2>&1 || { echo "profile failed"; tail -20 $OUT/profile.log; exit 1; }
tail -3 $OUT/profile.log
echo done
