#!/bin/bash
# Round 4: host sampling profiles (MILP_SAMPLE_PROFILE, engine/sampler.cc):
# config 5's 1 000-iteration window and the config-4 batch (whole run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_sample
mkdir -p $OUT
cd $R
MILP_SAMPLE_PROFILE=100 MILP_SAMPLE_STACK=1 MILP_SAMPLE_WALL=1 timeout -k 10 300 python3 -u scripts/probe.py --config c5 \
  --m 100000 --n 1000000 --warmup 20020 --steps 1000 > $OUT/c5.json 2> $OUT/c5.err || exit 1
MILP_SAMPLE_PROFILE=100 MILP_SAMPLE_STACK=1 timeout -k 10 200 python3 -u scripts/probe_batch.py --node \
  --lps 1024 --workers 1024 > $OUT/c4.json 2> $OUT/c4.err || exit 1
grep -A50 "sampler" $OUT/c5.err | head -100
