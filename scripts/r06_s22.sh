set -u
cd $GRAFT_REPO_ROOT
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
C5="python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
steps=("par@600=$T tests/test_parity_gpu.py -k 'device_dual'")
steps+=("ts@200=MILP_TIGHTEN_STATS=1 $C5")
for r in 1 2 3; do
  steps+=("new$r@200=$C5" "old$r@200=MILP_DUAL_TIGHTEN_SORT=1 $C5")
done
steps+=("bench@400=python3 -u bench.py --no-c2 --no-c3 --batch-lps 0 --batch-share-lps 0 --steps 20 --warmup 5")
scripts/gpu_run.sh gpurun_out/r06_v "${steps[@]}"
