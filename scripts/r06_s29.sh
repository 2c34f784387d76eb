set -u
cd $GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
B3="python3 -u bench.py --no-c5 --no-c2 --batch-lps 0 --no-cpu --profile-batch"
scripts/gpu_run.sh gpurun_out/r06_cc \
 "tests@700=$T tests/test_fullsize_gpu.py tests/test_parity_gpu.py -k 'config3 or medium or batch'" \
 "c3a@200=$B3" "c3b@200=$B3" \
 "c3full@400=python3 -u bench.py --no-c5 --no-c2 --batch-lps 0"
