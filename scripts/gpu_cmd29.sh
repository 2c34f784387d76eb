set -o pipefail
mkdir -p gpurun_out
MILP_CHECK_SCRATCH=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('C2', d['value'], d['cpu_baseline']['value']); c5=d['c5']; print('C5', c5['value'], c5['cpu_baseline']['value']); print('C3', d['c3']['value'], d['c3']['cpu_baseline']['value']); print('C4', d['batched']['value'], d['batched']['cpu_baseline']['value'])"
