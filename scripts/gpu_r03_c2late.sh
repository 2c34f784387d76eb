#!/bin/bash
# Round 3: where config 2's late window (iteration 1500) spends its time, and
# whether the device triangular solves help there.
set -o pipefail
mkdir -p gpurun_out/r03_c2late
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=64 timeout -k 10 300 python3 -u scripts/probe.py \
  --config c2 --warmup 1500 --steps 64 > gpurun_out/r03_c2late/phase.json \
  2> gpurun_out/r03_c2late/phase.err &&
timeout -k 10 400 python3 -u scripts/probe.py --config c2 --warmup 1500 --steps 64 \
  --variants MILP_DEVICE_SOLVE=force MILP_DEVICE_SOLVE_MIN_ROWS=8192 \
  > gpurun_out/r03_c2late/variants.json 2> gpurun_out/r03_c2late/variants.err
