set -o pipefail
mkdir -p gpurun_out
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=1000 timeout -k 10 600 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 --variants "MILP_HOST_THREADS=1" "MILP_HOST_THREADS=4" "MILP_HOST_THREADS=1" > gpurun_out/probe_c5t.json 2> gpurun_out/probe_c5t.err || { echo "c5 failed"; tail -30 gpurun_out/probe_c5t.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/probe_c5t.json'))
for k,v in d['gpu'].items(): print(k, v['gpu_it_per_s'])
"
