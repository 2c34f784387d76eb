set -u
cd $GRAFT_REPO_ROOT
C5="python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
scripts/gpu_run.sh gpurun_out/r06_q \
 "def@200=$C5" \
 "nohuge@200=MILP_HUGEPAGES=0 $C5" \
 "def2@200=$C5" \
 "nohuge2@200=MILP_HUGEPAGES=0 $C5" \
 "t8@200=MILP_HOST_THREADS=8 $C5" \
 "ph@200=MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=1000 $C5"
grep -h AnonHugePages /proc/meminfo > gpurun_out/r06_q/meminfo.txt || true
