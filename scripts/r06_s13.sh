set -u
cd $GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
scripts/gpu_run.sh gpurun_out/r06_m \
 "tests@600=$T tests/test_batch_policy_gpu.py tests/test_independent_gpu.py tests/test_comm_gpu.py"
