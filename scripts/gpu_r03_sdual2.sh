#!/bin/bash
# Round 3: device dual segments (tests/test_sdual_gpu.py) with per-LP launches
# and with the persistent pool kernel, config-4 children with segments on vs
# off, then the config-2 dump at iteration 454.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_sdual2
mkdir -p $OUT
for P in ${POOLS:-0 1}; do
  MILP_SDUAL_POOL=$P timeout -k 10 240 python3 -u -m pytest $R/tests/test_sdual_gpu.py -x -v \
    --timeout 120 --timeout-method thread -m gpu > $OUT/tests_pool$P.log 2>&1
  rc=$?
  echo "== tests pool=$P rc=$rc"; tail -3 $OUT/tests_pool$P.log
  if [ $rc -ne 0 ]; then grep -E "Error|assert|Timeout" $OUT/tests_pool$P.log | head -20; exit $rc; fi
done
for V in off device; do
  MILP_SDUAL=$V timeout -k 10 300 python3 -u $R/scripts/probe_batch.py --node --lps 512 \
    --workers 64 256 > $OUT/c4_$V.json 2> $OUT/c4_$V.err || { tail -20 $OUT/c4_$V.err; exit 1; }
  echo "== c4 $V"; cat $OUT/c4_$V.json | head -c 1500; echo
done
bash $R/scripts/gpu_r03_c2dump.sh
