set -u
cd $GRAFT_REPO_ROOT
C5="python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > gpurun_out/thp.txt 2>&1 || true
nproc >> gpurun_out/thp.txt; lscpu | head -20 >> gpurun_out/thp.txt || true
scripts/gpu_run.sh gpurun_out/r06_p \
 "t8@200=$C5" \
 "t16@200=MILP_HOST_THREADS=16 $C5" \
 "t8b@200=$C5" \
 "t16b@200=MILP_HOST_THREADS=16 $C5" \
 "t12@200=MILP_HOST_THREADS=12 $C5" \
 "ph16@200=MILP_HOST_THREADS=16 MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=1000 $C5"
