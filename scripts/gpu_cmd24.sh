set -o pipefail
mkdir -p gpurun_out




MILP_PHASE_TIMING=1 timeout -k 10 600 python -u scripts/probe.py --config c2 --warmup 3 --steps 100 --variants "MILP_ASYNC_SOLVES=off" "MILP_ASYNC_SOLVES=force" "MILP_ASYNC_SOLVES=off2" > gpurun_out/probe_c2a.json 2> gpurun_out/probe_c2a.err || { echo "c2 failed"; tail -30 gpurun_out/probe_c2a.err; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/probe_c2a.json'))
for k,v in d['gpu'].items(): print(k, v['gpu_it_per_s'])
"
