#!/bin/bash
# Round 4: engine trace of config 2 up to iteration 456 (per-iteration hashes
# incl. FTRAN stages, raw dumps at 453/454) to compare with the oracle's
# trace made on the CPU (scripts/c2_trace.py --oracle).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c2tr
mkdir -p $OUT
rm -f $OUT/c2*
MILP_TRACE=$OUT/c2 MILP_TRACE_DUMP=454 timeout -k 10 300 python3 -u scripts/c2_trace.py 456 > $OUT/run.log 2>&1
echo "rc=$?"
tail -3 $OUT/run.log
ls -la $OUT
