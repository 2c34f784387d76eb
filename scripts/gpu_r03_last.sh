#!/bin/bash
# Round 3: sdual GPU tests, the config-4 probe through the device segments, and
# the default bench (bench2.json).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r03_final
timeout -k 10 300 python3 -u -m pytest $R/tests/test_sdual_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $R/gpurun_out/r03_final/sdual_tests.log 2>&1
rc=$?; tail -1 $R/gpurun_out/r03_final/sdual_tests.log; [ $rc -eq 0 ] || exit $rc
WS=1024 bash $R/scripts/gpu_r03_c4scale.sh || exit 1
timeout -k 10 800 python3 -u $R/bench.py > $R/gpurun_out/r03_final/bench2.json \
  2> $R/gpurun_out/r03_final/bench2.log
echo "bench rc=$?"
