#!/bin/bash
# Round 3: U-solve variants on C5 (rate + kernel split) and their parity tests.
set -o pipefail
mkdir -p gpurun_out/r03_tri
timeout -k 10 240 python3 -u -m pytest tests/test_device_solve_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "c5_71 or dense_dual" > gpurun_out/r03_tri/tests.log 2>&1 &&
timeout -k 10 400 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20000 --steps 192 --variants "" MILP_TRI_POLL_MAX=8 MILP_TRI_POLL_MAX=32 \
  MILP_TRI_PERSIST=32,MILP_TRI_XCD=1,MILP_TRI_POLL_MAX=8 MILP_TRI_PERSIST=32,MILP_TRI_XCD=1 \
  MILP_TRI_PERSIST=64,MILP_TRI_POLL_MAX=4 MILP_TRI_PERSIST=128,MILP_TRI_POLL_MAX=4 \
  MILP_TRI_MAPPED=0 > gpurun_out/r03_tri/probe.json 2> gpurun_out/r03_tri/probe.err
