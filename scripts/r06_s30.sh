set -u
cd $GRAFT_REPO_ROOT
scripts/gpu_run.sh gpurun_out/r06_dd \
 "solo@300=python3 -u scripts/probe_c3.py --max-rows 16000 --workers --single 93 91 88"
