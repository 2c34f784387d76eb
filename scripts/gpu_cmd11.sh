set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "device_dual" > gpurun_out/gpu_tests_dd.log 2>&1 || { echo "device dual tests failed"; tail -60 gpurun_out/gpu_tests_dd.log; exit 1; }
tail -1 gpurun_out/gpu_tests_dd.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=1000 timeout -k 10 600 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 > gpurun_out/probe_c5.json 2> gpurun_out/probe_c5.err || { echo "c5 probe failed"; tail -30 gpurun_out/probe_c5.err; exit 1; }
cat gpurun_out/probe_c5.json
