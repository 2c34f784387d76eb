#!/bin/bash
# Round-2 evidence: bench (N=1 defaults) and the C5 rocprofv3 passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
WORKLOADS=c5 TAG=r02 bash scripts/gpu_profile.sh > $OUT/profile.log 2>&1 || { echo "profile failed"; tail -20 $OUT/profile.log; exit 1; }
tail -3 $OUT/profile.log
echo done
