#!/bin/bash
# Round 3: device dual segment parity (tests/test_sdual_gpu.py), then the
# config-2 late-window bisection.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_sdual
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest $R/tests/test_sdual_gpu.py -x -v --timeout 300 \
  --timeout-method thread -m gpu > $OUT/tests.log 2>&1
rc=$?
tail -15 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash $R/scripts/gpu_r03_c2bisect.sh
