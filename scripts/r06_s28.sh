set -u
cd $GRAFT_REPO_ROOT
C2="python3 -u scripts/probe.py --config c2 --warmup 3 --steps 64"
scripts/gpu_run.sh gpurun_out/r06_bb \
 "ph@300=MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=64 $C2" \
 "wall@300=MILP_SAMPLE_PROFILE=50 MILP_SAMPLE_WALL=1 $C2"
