#!/bin/bash
# Round 4: the config-3 stand-in extended to m = 16 000, engine
# (16 workers) then the 16-thread oracle. A heartbeat file shows progress.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c3big
mkdir -p $OUT
cd $R
( while true; do sleep 50; date +%T >> $OUT/heartbeat; done ) &
HB=$!
timeout -k 10 1000 python3 -u scripts/probe_c3.py --max-rows 16000 --workers 16 --cpu \
  > $OUT/c3_16k.json 2> $OUT/c3_16k.err
rc=$?
kill $HB
grep -h "LPs/s" $OUT/c3_16k.err | tail -5
exit $rc
