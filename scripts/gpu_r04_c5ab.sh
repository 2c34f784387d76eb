#!/bin/bash
# Round 4 config-5 study: schedule shapes of the factor triangles
# (MILP_TRI_SCHED), the host phase split (MILP_PHASE_TIMING) and an A/B of
# the round-3 switches (two-vector U launch, chain kernel, device BTRAN loops)
# on the bench window, one process per variant set.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c5ab
mkdir -p $OUT
# Config 3's critical path: its three longest LPs alone, engine and oracle,
# with the primal loop's host phase split.
MILP_PHASE_TIMING=1 timeout -k 10 300 python3 -u $R/scripts/probe_c3.py --single 89 93 86 \
  --workers --cpu > $OUT/c3_single.json 2> $OUT/c3_single.err || exit 1
# Config 4 at 128 LPs in flight (the per-GPU share over 8 GPUs): device phase
# profile of the segments.
MILP_SDUAL_PROFILE=1 timeout -k 10 200 python3 -u $R/scripts/probe_batch.py --node --lps 1024 \
  --workers 128 > $OUT/c4_w128.json 2> $OUT/c4_w128.err || exit 1
MILP_TRI_SCHED=1 MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=500 timeout -k 10 300 \
  python3 -u $R/scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 --steps 1000 \
  > $OUT/phase.json 2> $OUT/phase.err || exit 1
timeout -k 10 600 python3 -u $R/scripts/probe.py --config c5 --m 100000 --n 1000000 \
  --warmup 20020 --steps 1000 --variants "" MILP_TRI_PAIR=0 MILP_TRI_CHAIN=0 MILP_TRI_BTRAN=0 \
  > $OUT/ab.json 2> $OUT/ab.err
