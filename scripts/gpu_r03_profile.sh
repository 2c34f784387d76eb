#!/bin/bash
# Round 3: rocprofv3 kernel trace + stats of the bench's config-5 section (the
# headline and its roofline kernel) and of a config-4 batch through the device
# dual segments.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/c5 -o c5 -- \
  python3 $R/bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu > $OUT/c5_bench.json 2> $OUT/c5_bench.log
rc=$?; echo "c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
MILP_SDUAL=device timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4 -o c4 -- \
  python3 $R/scripts/probe_batch.py --node --lps 1024 --workers 1024 > $OUT/c4_probe.json 2> $OUT/c4_probe.log
rc=$?; echo "c4 rc=$rc"
find $OUT -name "*stats*" | head
exit $rc
