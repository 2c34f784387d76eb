#!/bin/bash
# Round 3: narrow segments anywhere in the sync-free schedule (one workgroup
# each): device-solve parity, C5 with and without them, and config 2's late
# window with its U and L solves on the device.
set -o pipefail
mkdir -p gpurun_out/r03_chain2
timeout -k 10 600 python3 -u -m pytest tests/test_device_solve_gpu.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/r03_chain2/tests.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_fullsize_gpu.py -x -q --timeout 280 \
  --timeout-method thread -m gpu -k config5 > gpurun_out/r03_chain2/c5_window.log 2>&1 &&
timeout -k 10 400 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20000 --steps 320 --variants MILP_TRI_CHAIN=1 MILP_TRI_CHAIN=0 MILP_TRI_CHAIN=1 \
  > gpurun_out/r03_chain2/c5.json 2> gpurun_out/r03_chain2/c5.err &&
MILP_TRI_SCHED=1 timeout -k 10 500 python3 -u scripts/probe.py --config c2 --warmup 1500 --steps 64 \
  --variants MILP_DEVICE_SOLVE=force,MILP_TRI_BTRAN=0 > gpurun_out/r03_chain2/c2.json \
  2> gpurun_out/r03_chain2/c2.err
