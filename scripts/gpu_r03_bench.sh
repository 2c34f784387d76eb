#!/bin/bash
# Round 3: the driver's bench command (N=1), then a longer C5 window.
set -o pipefail
mkdir -p gpurun_out/r03_bench
timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 \
  > gpurun_out/r03_bench/bench.json 2> gpurun_out/r03_bench/bench.err &&
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 1000 --warmup 20 --no-c2 --no-c3 \
  --batch-lps 0 > gpurun_out/r03_bench/bench_c5_1000.json 2> gpurun_out/r03_bench/bench_c5_1000.err
