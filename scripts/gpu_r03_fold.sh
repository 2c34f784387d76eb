#!/bin/bash
# Round 3: long outputs fold as their inputs arrive (device solve parity, deep
# dense chains); the deferred tau's L and etas back on the worker (pair A/B);
# config 2's schedule shapes and its late window with every solve forced on
# the device.
set -o pipefail
mkdir -p gpurun_out/r03_fold
timeout -k 10 600 python3 -u -m pytest tests/test_device_solve_gpu.py tests/test_parity_gpu.py \
  -x -q --timeout 300 --timeout-method thread -m gpu -k "device or async" \
  > gpurun_out/r03_fold/tests.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_fullsize_gpu.py -x -q --timeout 280 \
  --timeout-method thread -m gpu -k config5 > gpurun_out/r03_fold/c5_window.log 2>&1 &&
timeout -k 10 400 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20000 --steps 320 --variants MILP_TRI_PAIR=1 MILP_TRI_PAIR=0 \
  > gpurun_out/r03_fold/c5_pair.json 2> gpurun_out/r03_fold/c5_pair.err &&
MILP_TRI_SCHED=1 MILP_DEVICE_SOLVE_MIN_ROWS=1000 timeout -k 10 300 python3 -u scripts/probe.py \
  --config c2 --warmup 1500 --steps 8 > gpurun_out/r03_fold/c2_sched.json \
  2> gpurun_out/r03_fold/c2_sched.err &&
timeout -k 10 500 python3 -u scripts/probe.py --config c2 --warmup 1500 --steps 64 \
  --variants MILP_DEVICE_SOLVE=force > gpurun_out/r03_fold/c2_force.json \
  2> gpurun_out/r03_fold/c2_force.err
