#!/bin/bash
# Round 4: the device primal segment (MILP_SPRIMAL=on): GPU parity tests, the
# dual-segment tests again (same kernels), then config 3 with and without
# primal segments (whole suite, 16 workers; its three longest LPs alone).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_sprimal
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_sprimal_gpu.py -m gpu > $OUT/tests_sprimal.log 2>&1
rc=$?; echo "sprimal tests rc=$rc"; tail -3 $OUT/tests_sprimal.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_sdual_gpu.py -m gpu > $OUT/tests_sdual.log 2>&1
rc=$?; echo "sdual tests rc=$rc"; tail -3 $OUT/tests_sdual.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/probe_c3.py --workers 16 > $OUT/c3_off.json 2> $OUT/c3_off.err || exit 1
MILP_SPRIMAL=on timeout -k 10 300 python3 -u scripts/probe_c3.py --workers 16 > $OUT/c3_on.json 2> $OUT/c3_on.err || exit 1
MILP_SPRIMAL=on timeout -k 10 300 python3 -u scripts/probe_c3.py --single 89 93 86 --workers \
  > $OUT/c3_single_on.json 2> $OUT/c3_single_on.err || exit 1
tail -c 600 $OUT/c3_off.json; echo; tail -c 600 $OUT/c3_on.json; echo; tail -c 800 $OUT/c3_single_on.json
# Config 5: chain kernel width (levels of at most this many outputs go to the
# one-workgroup chain kernel; 1024 is the default).
timeout -k 10 600 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 \
  --steps 1000 --variants "" MILP_TRI_CHAIN_WIDTH=256 MILP_TRI_CHAIN_WIDTH=512 \
  MILP_TRI_CHAIN_WIDTH=2048 MILP_TRI_CHAIN_WIDTH=16384 > $OUT/c5_width.json 2> $OUT/c5_width.err || exit 1
grep "it/s" $OUT/c5_width.err
