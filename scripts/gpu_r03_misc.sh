#!/bin/bash
# Round 3: medium-kind batch parity after the hash change, the config-2 early
# window's phase split, and a two-rank rehearsal of bench.py's multi-GPU path
# (both ranks on the one GPU, small sizes).
set -o pipefail
mkdir -p gpurun_out/r03_misc
timeout -k 10 300 python3 -u -m pytest tests/test_parity_gpu.py -x -q --timeout 200 \
  --timeout-method thread -m gpu -k "batched_children or small_lp_one_launch" \
  > gpurun_out/r03_misc/tests.log 2>&1 &&
MILP_PHASE_TIMING=1 timeout -k 10 300 python3 -u scripts/probe.py --config c2 --warmup 3 \
  --steps 64 > gpurun_out/r03_misc/c2_early.json 2> gpurun_out/r03_misc/c2_early.err &&
MILP_BENCH_ONE_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
  --steps 20 --warmup 5 --c5-m 20000 --c5-n 200000 --c5-window 3000 --no-c2 --c3-max-rows 300 \
  --batch-lps 64 --batch-workers 16 > gpurun_out/r03_misc/bench_n2.json \
  2> gpurun_out/r03_misc/bench_n2.err
