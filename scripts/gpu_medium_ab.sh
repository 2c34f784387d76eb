#!/bin/bash
# ta041-shaped batch: device triangular solves (default, m >= 16384) against
# host solves (MILP_DEVICE_SOLVE=off), 16 and 64 LPs in flight.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u scripts/probe_batch.py --jobs 50 --machines 10 --lps 64 --workers 16 64 \
  > $OUT/mab_dev.json 2> $OUT/mab_dev.err || { echo "dev failed"; tail -30 $OUT/mab_dev.err; exit 1; }
cut -c1-200 $OUT/mab_dev.json
MILP_DEVICE_SOLVE=off timeout -k 10 300 python -u scripts/probe_batch.py --jobs 50 --machines 10 --lps 64 --workers 16 64 --cpu \
  > $OUT/mab_host.json 2> $OUT/mab_host.err || { echo "host failed"; tail -30 $OUT/mab_host.err; exit 1; }
cut -c1-200 $OUT/mab_host.json
echo done
