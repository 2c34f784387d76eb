set -u
cd $GRAFT_REPO_ROOT
P="python3 -u scripts/probe_batch.py --node --lps 1024"
scripts/gpu_run.sh gpurun_out/r06_a \
 "shared@300=MILP_TEST_SHARED_CACHES=1 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_sdual_gpu.py -k shared_caches" \
 "base@200=MILP_SDUAL_PROFILE=1 $P --workers 1024" \
 "sh@200=MILP_SDUAL_PROFILE=1 MILP_BATCH_SHARED_LU=1 MILP_BATCH_SHARED_NORMS=1 $P --workers 1024" \
 "srv8@200=MILP_SDUAL_PROFILE=1 MILP_SDUAL_SERVERS=8 $P --workers 1024" \
 "w128@200=MILP_SDUAL_PROFILE=1 $P --workers 128" \
 "w128sh@200=MILP_SDUAL_PROFILE=1 MILP_BATCH_SHARED_LU=1 MILP_BATCH_SHARED_NORMS=1 $P --workers 128"
