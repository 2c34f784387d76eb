#!/bin/bash
# A/B of the small row-wise kernel's workgroup size on the config-4 probe,
# after the small-LP parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k small_lp > $OUT/gpu_small_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/gpu_small_tests.log; exit 1; }
tail -1 $OUT/gpu_small_tests.log
for T in 1024 256; do
  MILP_SMALL_THREADS=$T timeout -k 10 200 python -u $R/scripts/probe_batch.py --lps 512 --workers 1 8 16 > $OUT/probe_t$T.json 2> $OUT/probe_t$T.err || { echo "probe $T failed"; tail -20 $OUT/probe_t$T.err; exit 1; }
  echo "threads $T"; cat $OUT/probe_t$T.err
done
