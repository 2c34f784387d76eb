set -u
cd $GRAFT_REPO_ROOT
B="python3 -u bench.py --no-c5 --no-c2 --batch-lps 0 --no-cpu --profile-batch"
scripts/gpu_run.sh gpurun_out/r06_j \
 "base@200=$B" \
 "hpool@200=MILP_BATCH_HOST_POOL=1 $B" \
 "prio8@200=MILP_BATCH_PRIORITY_LPS=8 $B" \
 "prio2@200=MILP_BATCH_PRIORITY_LPS=2 $B" \
 "fib2@200=MILP_BATCH_FIBERS=2 $B" \
 "base2@200=$B"
