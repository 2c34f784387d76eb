set -u
cd $GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider"
B="python3 -u bench.py --no-c5 --no-c2 --no-c3 --no-cpu --batch-share-lps 0"
scripts/gpu_run.sh gpurun_out/r06_n \
 "tests@600=$T tests/test_batch_policy_gpu.py tests/test_sdual_gpu.py tests/test_independent_gpu.py tests/test_comm_gpu.py" \
 "t0@200=MILP_SDUAL_TAIL=0 $B" \
 "t32@200=$B" \
 "t0b@200=MILP_SDUAL_TAIL=0 $B" \
 "t32b@200=$B" \
 "t16@200=MILP_SDUAL_TAIL=16 $B" \
 "t64@200=MILP_SDUAL_TAIL=64 $B"
