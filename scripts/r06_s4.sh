set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
B="python3 -u bench.py --no-c5 --no-c2 --no-c3"
scripts/gpu_run.sh gpurun_out/r06_d \
 "shared@400=$T tests/test_sdual_gpu.py -k shared_caches" \
 "c4base@300=$B" \
 "c4sh@300=MILP_BATCH_SHARED_LU=1 MILP_BATCH_SHARED_NORMS=1 $B" \
 "c3trace@400=cd /tmp && export TMPDIR=/tmp && MILP_CRASH_REPORT=1 MILP_DEVICE_RESET_AT_EXIT=1 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r06_d/c3t -o run --output-format csv -- python3 $R/bench.py --no-c5 --no-c2 --batch-lps 0 --profile-batch --no-cpu"
