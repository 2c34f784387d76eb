set -u
cd $GRAFT_REPO_ROOT
B="python3 -u bench.py --no-c5 --no-c2 --batch-lps 0 --no-cpu --profile-batch"
scripts/gpu_run.sh gpurun_out/r06_l \
 "base@200=$B" \
 "d4@200=MILP_BATCH_DEDICATED=4 $B" \
 "d8@200=MILP_BATCH_DEDICATED=8 $B" \
 "d8hp@200=MILP_BATCH_DEDICATED=8 MILP_BATCH_HOST_POOL=1 $B" \
 "d4b@200=MILP_BATCH_DEDICATED=4 $B" \
 "base2@200=$B"
