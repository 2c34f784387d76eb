#!/bin/bash
# One GPU session: parity tests, smoke, bench. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py --m 2000 --n 10000 --steps 20 --no-cpu > gpurun_out/bench_small.log 2>&1 || { echo "small bench failed"; cat gpurun_out/bench_small.log; exit 1; }
cat gpurun_out/bench_small.log
