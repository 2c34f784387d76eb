set -u
cd $GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
scripts/gpu_run.sh gpurun_out/r06_h \
 "probe@300=python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000" \
 "tests@600=$T tests/test_fullsize_gpu.py tests/test_shards_gpu.py" \
 "bench@600=python3 -u bench.py --steps 20 --warmup 5 --no-c2 --no-c3 --batch-lps 0" \
 "w1000@300=python3 -u scripts/whole_solve.py --configs c5 --c5-m 1000 --c5-n 10000 --limit-s 250" \
 "w2000@300=python3 -u scripts/whole_solve.py --configs c5 --c5-m 2000 --c5-n 20000 --limit-s 250"
