#!/bin/bash
# Round 3: batch-path GPU tests with the device segments as the default, then
# the default bench (bench3.json).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r03_final
timeout -k 10 600 python3 -u -m pytest $R/tests/test_sdual_gpu.py $R/tests/test_parity_gpu.py \
  $R/tests/test_cpsat.py $R/tests/test_fullsize_gpu.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -k "sdual or batched or batch or node or config3" \
  > $R/gpurun_out/r03_final/verify_tests.log 2>&1
rc=$?; tail -1 $R/gpurun_out/r03_final/verify_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python3 -u $R/bench.py > $R/gpurun_out/r03_final/bench3.json \
  2> $R/gpurun_out/r03_final/bench3.log
echo "bench rc=$?"
