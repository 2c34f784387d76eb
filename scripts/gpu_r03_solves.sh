#!/bin/bash
# Round 3: parity of the device triangular-solve family, then config 2's late
# window with and without device solves (phase split on the default run).
set -o pipefail
mkdir -p gpurun_out/r03_solves
timeout -k 10 400 python3 -u -m pytest tests/test_device_solve_gpu.py tests/test_boundary.py -x -q \
  --timeout 120 --timeout-method thread -m gpu > gpurun_out/r03_solves/tests.log 2>&1 &&
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=64 timeout -k 10 300 python3 -u scripts/probe.py \
  --config c2 --warmup 1500 --steps 64 > gpurun_out/r03_solves/c2_phase.json \
  2> gpurun_out/r03_solves/c2_phase.err &&
timeout -k 10 400 python3 -u scripts/probe.py --config c2 --warmup 1500 --steps 64 \
  --variants MILP_DEVICE_SOLVE=force MILP_DEVICE_SOLVE=force,MILP_TRI_BTRAN=0 \
  > gpurun_out/r03_solves/c2_variants.json 2> gpurun_out/r03_solves/c2_variants.err
