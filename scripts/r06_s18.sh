set -u
cd $GRAFT_REPO_ROOT
C5="python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
steps=()
for r in 1 2 3 4; do
  steps+=("a$r@200=$C5" "b$r@200=MILP_HOST_THREADS=8 $C5" "c$r@200=MILP_HUGEPAGES=0 $C5" "d$r@200=MILP_HOST_THREADS=8 MILP_HUGEPAGES=0 $C5")
done
scripts/gpu_run.sh gpurun_out/r06_r "${steps[@]}"
