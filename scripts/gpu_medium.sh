#!/bin/bash
# Medium batched row-wise update row (kMediumRowWise): parity of the
# ta041-shaped batch against the oracle with the path on, then off (A/B).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u scripts/probe_batch.py --jobs 50 --machines 10 --lps 64 --workers 16 --cpu \
  > $OUT/medium_on.json 2> $OUT/medium_on.err || { echo "medium on failed"; tail -30 $OUT/medium_on.err; exit 1; }
cat $OUT/medium_on.json | cut -c1-300
MILP_MEDIUM=off timeout -k 10 300 python -u scripts/probe_batch.py --jobs 50 --machines 10 --lps 64 --workers 16 \
  > $OUT/medium_off.json 2> $OUT/medium_off.err || { echo "medium off failed"; tail -30 $OUT/medium_off.err; exit 1; }
cat $OUT/medium_off.json | cut -c1-300
MILP_TEST_TIMES=$OUT/test_times.txt timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $OUT/gpu_tests.log | head; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
echo done
