set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "async_tau" > gpurun_out/gpu_tests_at.log 2>&1 || { echo "async tau tests failed"; tail -60 gpurun_out/gpu_tests_at.log; exit 1; }
tail -1 gpurun_out/gpu_tests_at.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=1000 timeout -k 10 600 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 --variants "MILP_ASYNC_TAU=off" "MILP_ASYNC_TAU=on" > gpurun_out/probe_c5a.json 2> gpurun_out/probe_c5a.err || { echo "c5 failed"; tail -30 gpurun_out/probe_c5a.err; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/probe_c5a.json'))
for k,v in d['gpu'].items(): print(k, v['gpu_it_per_s'])
"
