set -u
cd $GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
scripts/gpu_run.sh gpurun_out/r06_g \
 "tests@900=$T tests/test_fullsize_gpu.py tests/test_shards_gpu.py tests/test_split_gpu.py tests/test_parity_gpu.py" \
 "bench@600=python3 -u bench.py --steps 20 --warmup 5 --no-c2 --no-c3 --batch-lps 0" \
 "probe@300=python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
