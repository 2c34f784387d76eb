#!/bin/bash
# Config-5 profile of the final round-6 tree (after the tightening change).
set -u
cd $GRAFT_REPO_ROOT
scripts/gpu_run.sh gpurun_out/r06_prof3 \
 "c5@900=bash scripts/profile_bench.sh r06_c5 c5 --no-c2 --no-c3 --batch-lps 0 --steps 20 --warmup 5 --no-cpu"
