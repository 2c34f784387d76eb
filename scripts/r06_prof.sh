#!/bin/bash
# Round-6 profiles of the committed tree (scripts/profile_bench.sh per
# section), copied into gpurun_out/profiles/r06_<section>/ for profiles/.
set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
scripts/gpu_run.sh gpurun_out/r06_prof \
 "c4@600=PROFILE_LPS=1025 bash scripts/profile_bench.sh r06_c4 c4 --no-c5 --no-c2 --no-c3 --profile-batch --no-cpu --batch-share-lps 0" \
 "c5@900=bash scripts/profile_bench.sh r06_c5 c5 --no-c2 --no-c3 --batch-lps 0 --steps 20 --warmup 5 --no-cpu" \
 "c2@600=bash scripts/profile_bench.sh r06_c2 c2 --no-c5 --no-c3 --batch-lps 0 --no-cpu --c2-late 0"
