#!/bin/bash
# Round 3: config-4 children through the device dual segments at growing
# numbers of LPs in flight (W), phase profile for each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_c4scale
mkdir -p $OUT
for W in ${WS:-64 256 1024}; do
  echo "== W=$W $(date +%T)"
  MILP_SDUAL=${SDUAL:-device} MILP_SDUAL_PROFILE=1 timeout -k 10 150 python3 -u \
    $R/scripts/probe_batch.py --node --lps ${LPS:-1024} --workers $W > $OUT/c4_w$W.json \
    2> $OUT/c4_w$W.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); g=[v for k,v in d.items() if k.startswith('gpu_')][0]; print({k: g[k] for k in ('lps_per_s','iterations','wall_s','host_cpu_s')})" $OUT/c4_w$W.json
  grep -A13 "sdual profile" $OUT/c4_w$W.err
done
