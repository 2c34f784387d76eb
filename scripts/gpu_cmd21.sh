set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 --variants "MILP_HOST_THREADS=4" "MILP_HOST_THREADS=1" > gpurun_out/probe_c5t.json 2> gpurun_out/probe_c5t.err || { echo "c5 failed"; tail -30 gpurun_out/probe_c5t.err; exit 1; }
timeout -k 10 600 python -u scripts/probe.py --config c2 --warmup 3 --steps 100 --variants "MILP_HOST_THREADS=4" "MILP_HOST_THREADS=1" > gpurun_out/probe_c2t.json 2> gpurun_out/probe_c2t.err || { echo "c2 failed"; tail -30 gpurun_out/probe_c2t.err; exit 1; }
python -c "
import json
for f in ['gpurun_out/probe_c5t.json','gpurun_out/probe_c2t.json']:
  d=json.load(open(f))
  for k,v in d['gpu'].items(): print(f, k, v['gpu_it_per_s'])
"
