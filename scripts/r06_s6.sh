set -u
cd $GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
scripts/gpu_run.sh gpurun_out/r06_f \
 "sdual@400=$T tests/test_sdual_gpu.py" \
 "prof@200=MILP_SDUAL_PROFILE=1 python3 -u scripts/probe_batch.py --node --lps 1024 --workers 1024" \
 "c4@300=python3 -u bench.py --no-c5 --no-c2 --no-c3" \
 "suite@900=$T tests -m gpu"
