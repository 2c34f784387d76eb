#!/bin/bash
# Round 3: the batch-path GPU tests and the bench with the device dual segments
# switched on for every batch call (MILP_SDUAL=device) and 1 024 LPs in flight.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r03_final
export MILP_SDUAL=device
timeout -k 10 600 python3 -u -m pytest $R/tests/test_parity_gpu.py $R/tests/test_cpsat.py \
  $R/tests/test_fullsize_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "batched or batch or node or config3" > $R/gpurun_out/r03_final/verify_sdual_tests.log 2>&1
rc=$?; tail -1 $R/gpurun_out/r03_final/verify_sdual_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python3 -u $R/bench.py --batch-workers 1024 > $R/gpurun_out/r03_final/bench4.json \
  2> $R/gpurun_out/r03_final/bench4.log
echo "bench rc=$?"
