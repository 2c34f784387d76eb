#!/bin/bash
# Round 3: direction + tau U solves in one launch -- parity and rate; the
# multi-GPU batch entry; config-4 node workload by LPs in flight.
set -o pipefail
mkdir -p gpurun_out/r03_pair
timeout -k 10 500 python3 -u -m pytest tests/test_device_solve_gpu.py tests/test_parity_gpu.py \
  tests/test_boundary.py -x -q --timeout 200 --timeout-method thread -m gpu \
  -k "async or device_u_solve or device_dual or btran or batch_solve_gpus" \
  > gpurun_out/r03_pair/tests.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_fullsize_gpu.py -x -q --timeout 280 \
  --timeout-method thread -m gpu -k config5 > gpurun_out/r03_pair/c5_window.log 2>&1 &&
timeout -k 10 400 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20000 --steps 320 --variants MILP_TRI_PAIR=1 MILP_TRI_PAIR=0 \
  > gpurun_out/r03_pair/probe.json 2> gpurun_out/r03_pair/probe.err &&
timeout -k 10 400 python3 -u scripts/probe_batch.py --node --lps 1024 --workers 128 256 512 \
  > gpurun_out/r03_pair/c4_workers.json 2> gpurun_out/r03_pair/c4_workers.err
