set -u
cd $GRAFT_REPO_ROOT
B="python3 -u bench.py --no-c5 --no-c2 --batch-lps 0 --no-cpu --profile-batch"
scripts/gpu_run.sh gpurun_out/r06_k \
 "p8@200=MILP_BATCH_PRIORITY_LPS=8 $B" \
 "p12@200=MILP_BATCH_PRIORITY_LPS=12 $B" \
 "p16@200=MILP_BATCH_PRIORITY_LPS=16 $B" \
 "p24@200=MILP_BATCH_PRIORITY_LPS=24 $B" \
 "p12f2@200=MILP_BATCH_PRIORITY_LPS=12 MILP_BATCH_FIBERS=2 $B" \
 "p8b@200=MILP_BATCH_PRIORITY_LPS=8 $B"
