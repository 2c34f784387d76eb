#!/bin/bash
# Round 4: the right-pool append overlapped with the device U solve: parity
# (device-solve tests, config-5 full-size golden windows), then the config-5
# window rate and its host profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_overlap
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_device_solve_gpu.py tests/test_fullsize_gpu.py -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
MILP_SAMPLE_PROFILE=100 MILP_SAMPLE_STACK=1 MILP_SAMPLE_WALL=1 timeout -k 10 300 python3 -u scripts/probe.py \
  --config c5 --m 100000 --n 1000000 --warmup 20020 --steps 1000 > $OUT/c5.json 2> $OUT/c5.err || exit 1
timeout -k 10 300 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 \
  --steps 1000 > $OUT/c5_plain.json 2> $OUT/c5_plain.err || exit 1
grep "it/s" $OUT/c5.err $OUT/c5_plain.err
grep -A40 "inclusive" $OUT/c5.err | head -42
