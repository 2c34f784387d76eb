#!/bin/bash
# Round 3: device dual segments with the mailbox factorization service
# (tests/test_sdual_gpu.py), the config-2 dump at iteration 454, and config-4
# children with segments on vs off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_sdual2
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest $R/tests/test_sdual_gpu.py -x -v --timeout 300 \
  --timeout-method thread -m gpu > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; fi
for V in off device; do
  MILP_SDUAL=$V timeout -k 10 300 python3 -u $R/scripts/probe_batch.py --node --lps 512 \
    --workers 64 256 > $OUT/c4_$V.json 2> $OUT/c4_$V.err || { tail -20 $OUT/c4_$V.err; exit 1; }
  echo "== c4 $V"; cat $OUT/c4_$V.json | head -c 1500; echo
done
bash $R/scripts/gpu_r03_c2dump.sh
