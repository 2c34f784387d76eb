set -u
cd $GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
scripts/gpu_run.sh gpurun_out/r06_x \
 "par@600=$T tests/test_parity_gpu.py -k 'device_dual'" \
 "bench@400=python3 -u bench.py --no-c2 --no-c3 --batch-lps 0 --batch-share-lps 0 --steps 20 --warmup 5"
