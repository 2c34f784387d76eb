set -u
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
P="python3 -u scripts/probe_batch.py --node"
scripts/gpu_run.sh gpurun_out/r06_e \
 "seg128@200=$P --lps 128 --workers 128" \
 "off128@200=MILP_SDUAL=off $P --lps 128 --workers 128" \
 "off1024@200=MILP_SDUAL=off $P --lps 1024 --workers 128 256" \
 "seg256@200=$P --lps 256 --workers 256" \
 "c3trace1@400=cd /tmp && export TMPDIR=/tmp && MILP_BATCH_FIBERS=1 MILP_CRASH_REPORT=1 MILP_DEVICE_RESET_AT_EXIT=1 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r06_e/c3t -o run --output-format csv -- python3 $R/bench.py --no-c5 --no-c2 --batch-lps 0 --profile-batch --no-cpu"
