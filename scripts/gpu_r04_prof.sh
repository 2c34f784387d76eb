#!/bin/bash
# Round 4 rocprofv3 evidence: config 5 and config 2 (kernel trace + stats,
# FETCH_SIZE and WRITE_SIZE passes each in a run of its own; summaries and
# traffic_c5/c2.json via scripts/profile_summary.py), then a kernel trace of
# the config-4 pool batch (the persistent sdual kernel), last.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
WORKLOADS="c5 c2" TAG=${TAG:-r04} bash $R/scripts/gpu_profile.sh || exit 1
OUT=$R/gpurun_out/profiles/${TAG:-r04}_c4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- \
  python3 $R/scripts/probe_batch.py --node --lps 1024 --workers 1024 > $OUT/probe.log 2>&1
rc=$?; echo "c4 trace rc=$rc"
cp $OUT/trace/run_kernel_stats.csv $OUT/kernel_stats.csv 2>/dev/null
rm -rf $OUT/trace
exit $rc
