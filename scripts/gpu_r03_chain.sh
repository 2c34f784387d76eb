#!/bin/bash
# Round 3: the single-workgroup tail of the sync-free U solve (tri_chain_kernel):
# device-solve parity with it, then C5 with and without it.
set -o pipefail
mkdir -p gpurun_out/r03_chain
timeout -k 10 600 python3 -u -m pytest tests/test_device_solve_gpu.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/r03_chain/tests.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_fullsize_gpu.py -x -q --timeout 280 \
  --timeout-method thread -m gpu -k config5 > gpurun_out/r03_chain/c5_window.log 2>&1 &&
MILP_TRI_SCHED=1 timeout -k 10 400 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20000 --steps 320 --variants MILP_TRI_CHAIN=1 MILP_TRI_CHAIN=0 \
  > gpurun_out/r03_chain/c5.json 2> gpurun_out/r03_chain/c5.err
