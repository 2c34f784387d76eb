#!/bin/bash
# Round 4: config 3 with primal segments after sizing the pool grid to the
# LPs in flight: whole suite on/off, the three longest LPs alone with
# segments (MILP_SDUAL=device turns them on outside batch calls), and the
# config-4 probe as a check that the 1 024-LP pool is unchanged.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c3seg
mkdir -p $OUT
cd $R
MILP_SPRIMAL=on timeout -k 10 300 python3 -u scripts/probe_c3.py --workers 16 > $OUT/c3_on.json 2> $OUT/c3_on.err || exit 1
timeout -k 10 300 python3 -u scripts/probe_c3.py --workers 16 > $OUT/c3_off.json 2> $OUT/c3_off.err || exit 1
MILP_SPRIMAL=on MILP_SDUAL=device MILP_SDUAL_PROFILE=1 timeout -k 10 300 python3 -u scripts/probe_c3.py \
  --single 89 93 86 --workers > $OUT/c3_single_on.json 2> $OUT/c3_single_on.err || exit 1
timeout -k 10 200 python3 -u scripts/probe_batch.py --node --lps 1024 --workers 1024 \
  > $OUT/c4.json 2> $OUT/c4.err || exit 1
# Config 2's late window (iterations 1500..1564): primal loop phase split.
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=64 timeout -k 10 300 python3 -u scripts/probe.py \
  --config c2 --warmup 1500 --steps 64 > $OUT/c2_late.json 2> $OUT/c2_late.err || exit 1
grep -h "LPs/s\|us/it\|gpu_us" $OUT/*.err | head -20
