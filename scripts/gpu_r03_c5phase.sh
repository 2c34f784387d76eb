#!/bin/bash
# C5 phase split around the bench window (round 3 study).
set -o pipefail
mkdir -p gpurun_out/r03_c5phase
export MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=64
timeout -k 10 300 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20000 --steps 192 > gpurun_out/r03_c5phase/probe.json 2> gpurun_out/r03_c5phase/probe.err &&
MILP_TRI_DEBUG=1 timeout -k 10 300 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20000 --steps 64 > gpurun_out/r03_c5phase/probe_dbg.json 2> gpurun_out/r03_c5phase/probe_dbg.err
