#!/bin/bash
# Host/device phase split of the C2 and C5 loops in steady-state windows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=${C2_EVERY:-20} timeout -k 10 300 python -u $R/scripts/probe.py --config c2 --warmup 3 --steps ${C2_STEPS:-64} > $OUT/phase_c2.json 2> $OUT/phase_c2.err || { echo "c2 failed"; tail -30 $OUT/phase_c2.err; exit 1; }
cat $OUT/phase_c2.json
if [ -z "$SKIP_C5" ]; then
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=500 timeout -k 10 300 python -u $R/scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 > $OUT/phase_c5.json 2> $OUT/phase_c5.err || { echo "c5 failed"; tail -30 $OUT/phase_c5.err; exit 1; }
cat $OUT/phase_c5.json
fi
