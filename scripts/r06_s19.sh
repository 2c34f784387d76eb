set -u
cd $GRAFT_REPO_ROOT
C5="python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
steps=()
for r in 1 2 3 4; do
  steps+=("a$r@200=$C5" "s$r@200=MILP_SYNC_SPIN=1 $C5")
done
steps+=("ph@200=MILP_SYNC_SPIN=1 MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=1000 $C5")
scripts/gpu_run.sh gpurun_out/r06_s "${steps[@]}"
