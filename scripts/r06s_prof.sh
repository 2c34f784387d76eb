#!/bin/bash
# Round-6 (last session) config-5 profile of the committed tree (scripts/profile_bench.sh),
# copied into gpurun_out/profiles/r06s_c5/ for profiles/.
set -u
cd $GRAFT_REPO_ROOT
scripts/gpu_run.sh gpurun_out/r06s_prof \
 "c5@900=bash scripts/profile_bench.sh r06s_c5 c5 --no-c2 --no-c3 --batch-lps 0 --steps 20 --warmup 5 --no-cpu"
