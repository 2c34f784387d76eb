set -u
cd $GRAFT_REPO_ROOT
C5="python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
scripts/gpu_run.sh gpurun_out/r06_z "lu@200=MILP_LU_TIMING=1 $C5"
