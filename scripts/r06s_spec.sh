#!/bin/bash
# Speculative flip FTRAN: its parity tests, the device-dual parity files,
# then config 5 with it on (with the oracle check) and off.
out=${1:-gpurun_out/r06s_a}
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
bash scripts/gpu_run.sh "$out" \
  "spec@300=$T tests/test_device_solve_gpu.py -k 'speculative or async_tau'" \
  "dual@400=$T tests/test_parity_gpu.py -k 'device_dual or async_tau'" \
  "c5on@330=MILP_SPEC_FLIP_STATS=1 python -u bench.py --no-c2 --no-c3 --batch-lps 0" \
  "c5off@240=MILP_SPEC_FLIP=0 python -u bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu"
