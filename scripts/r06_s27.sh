set -u
cd $GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
C5="python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
scripts/gpu_run.sh gpurun_out/r06_aa \
 "tests@600=$T tests/test_device_solve_gpu.py tests/test_fullsize_gpu.py tests/test_parity_gpu.py" \
 "lu@200=MILP_LU_TIMING=1 $C5" \
 "bench@400=python3 -u bench.py --no-c2 --no-c3 --batch-lps 0 --batch-share-lps 0 --steps 20 --warmup 5"
