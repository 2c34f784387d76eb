#!/bin/bash
# Early boxed-flip flags: parity, then config 5 on/off (oracle check on the first).
out=${1:-gpurun_out/r06s_g}
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
bash scripts/gpu_run.sh "$out" \
  "spec@300=$T tests/test_device_solve_gpu.py -k 'early or speculative or async_tau'" \
  "dual@400=$T tests/test_parity_gpu.py -k 'device_dual or async_tau or mps'" \
  "split@300=$T tests/test_split_gpu.py tests/test_shards_gpu.py" \
  "c5on@330=python -u bench.py --no-c2 --no-c3 --batch-lps 0" \
  "c5off@200=MILP_EARLY_FLIPS=0 python -u bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu" \
  "c5on2@200=python -u bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu" \
  "c5off2@200=MILP_EARLY_FLIPS=0 python -u bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu"
