#!/bin/bash
# Round 3: parity of the new paths (counters, cross-process split, shards),
# then config 2's late window with and without device solves, then C5 host
# thread counts.
set -o pipefail
mkdir -p gpurun_out/r03_solves
timeout -k 10 500 python3 -u -m pytest tests/test_boundary.py tests/test_split_gpu.py \
  tests/test_shards_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu \
  > gpurun_out/r03_solves/tests2.log 2>&1 &&
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=64 timeout -k 10 300 python3 -u scripts/probe.py \
  --config c2 --warmup 1500 --steps 64 > gpurun_out/r03_solves/c2_phase.json \
  2> gpurun_out/r03_solves/c2_phase.err &&
timeout -k 10 400 python3 -u scripts/probe.py --config c2 --warmup 1500 --steps 64 \
  --variants MILP_DEVICE_SOLVE=force MILP_DEVICE_SOLVE=force,MILP_TRI_BTRAN=0 \
  > gpurun_out/r03_solves/c2_variants.json 2> gpurun_out/r03_solves/c2_variants.err &&
timeout -k 10 300 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20000 --steps 192 --variants "" MILP_HOST_THREADS=16 \
  > gpurun_out/r03_solves/c5_threads.json 2> gpurun_out/r03_solves/c5_threads.err
