#!/bin/bash
# The speculative u column reused by the MPF update: parity, then config 5.
out=${1:-gpurun_out/r06s_d}
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
bash scripts/gpu_run.sh "$out" \
  "spec@300=$T tests/test_device_solve_gpu.py" \
  "dual@400=$T tests/test_parity_gpu.py -k 'device_dual or async_tau or mps'" \
  "c5on@330=MILP_SPEC_FLIP_STATS=1 python -u bench.py --no-c2 --no-c3 --batch-lps 0" \
  "c5on2@200=python -u bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu"
