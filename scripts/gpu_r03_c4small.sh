#!/bin/bash
# Round 3: config-4 children, small batch, device segments with and without
# the pool kernel, with the device phase profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_c4small
mkdir -p $OUT
for P in ${POOLS:-0 1}; do
  echo "== pool=$P $(date +%T)"
  MILP_SDUAL=device MILP_SDUAL_POOL=$P MILP_SDUAL_PROFILE=1 timeout -k 10 150 python3 -u \
    $R/scripts/probe_batch.py --node --lps ${LPS:-32} --workers ${W:-16} > $OUT/c4_pool$P.json \
    2> $OUT/c4_pool$P.err
  echo "rc=$?"; head -c 400 $OUT/c4_pool$P.json; echo; grep -A12 "sdual profile" $OUT/c4_pool$P.err
done
