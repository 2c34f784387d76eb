set -u
cd $GRAFT_REPO_ROOT
export MILP_SDUAL=device
P="python3 -u scripts/probe_batch.py --node --lps 1024"
T="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
scripts/gpu_run.sh gpurun_out/r06_b \
 "comm@200=$T tests/test_comm_gpu.py" \
 "shp@200=python3 -u scripts/probe_shared.py 6,6" \
 "shp2@200=python3 -u scripts/probe_shared.py 15,10" \
 "base@200=MILP_SDUAL_PROFILE=1 $P --workers 1024" \
 "sh@200=MILP_SDUAL_PROFILE=1 MILP_BATCH_SHARED_LU=1 MILP_BATCH_SHARED_NORMS=1 $P --workers 1024" \
 "srv8@200=MILP_SDUAL_PROFILE=1 MILP_SDUAL_SERVERS=8 $P --workers 1024" \
 "w128@200=MILP_SDUAL_PROFILE=1 $P --workers 128" \
 "c5ph@300=MILP_PHASE_TIMING=1 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
