#!/bin/bash
# Round-6 config-3 profile of the committed tree for profiles/r06_c3. With
# HIP's default 4 hardware queues the kernel trace of this batch faults inside
# rocprofiler-sdk (profiles/r06_c3trace); with 16 it completes. The counter
# passes serialize dispatches, so all passes run the batch on 2 host threads.
set -u
cd $GRAFT_REPO_ROOT
scripts/gpu_run.sh gpurun_out/r06_prof2 \
 "c3@1100=GPU_MAX_HW_QUEUES=16 bash scripts/profile_bench.sh r06_c3 c3 --no-c5 --no-c2 --batch-lps 0 --no-cpu --profile-batch --c3-workers 2"
