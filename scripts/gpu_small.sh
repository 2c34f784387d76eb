#!/bin/bash
# Parity tests, then the config-4 probe with the small-LP fused update row on/off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python -u $R/scripts/probe_batch.py --lps 512 --workers 1 8 16 > $OUT/probe_on.json 2> $OUT/probe_on.err || { echo "probe failed"; tail -20 $OUT/probe_on.err; exit 1; }
MILP_SMALL_FUSED=off timeout -k 10 200 python -u $R/scripts/probe_batch.py --lps 512 --workers 1 8 16 > $OUT/probe_off.json 2> $OUT/probe_off.err || { echo "probe off failed"; tail -20 $OUT/probe_off.err; exit 1; }
cat $OUT/probe_on.err $OUT/probe_off.err
timeout -k 10 300 python -u $R/scripts/probe_c3.py --workers 1 8 16 > $OUT/probe_c3.json 2> $OUT/probe_c3.err || { echo "c3 probe failed"; tail -20 $OUT/probe_c3.err; exit 1; }
cat $OUT/probe_c3.err
