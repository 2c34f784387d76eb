#!/bin/bash
# Round 4: host transpose solves over independent runs (MILP_HOST_TRI_PAR):
# parity (full-size windows, host-loop parity), then config 2's late window
# with and without, and the config-5 window.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_tripar
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_fullsize_gpu.py tests/test_parity_gpu.py -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
MILP_HOST_TRI_PAR_DEBUG=1 timeout -k 10 500 python3 -u scripts/probe.py --config c2 --warmup 1500 --steps 64 \
  --variants "" MILP_HOST_TRI_PAR=0 > $OUT/c2_late.json 2> $OUT/c2_late.err || exit 1
grep -h "variant\|it/s" $OUT/c2_late.err
grep -h "tri par" $OUT/c2_late.err | sort | uniq -c | sort -rn | head -4; grep -h "tri par\] forward" $OUT/c2_late.err | tail -3
timeout -k 10 300 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 \
  --steps 1000 --variants "" MILP_HOST_TRI_PAR=0 > $OUT/c5.json 2> $OUT/c5.err || exit 1
grep -h "variant\|it/s" $OUT/c5.err
