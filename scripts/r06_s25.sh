set -u
cd $GRAFT_REPO_ROOT
B3="python3 -u bench.py --no-c5 --no-c2 --batch-lps 0 --no-cpu --profile-batch"
B4="python3 -u bench.py --no-c5 --no-c2 --no-c3 --no-cpu"
C5="python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
steps=()
for r in 1 2 3; do
  steps+=("c4q4_$r@200=$B4" "c4q8_$r@200=GPU_MAX_HW_QUEUES=8 $B4")
done
for r in 1 2; do
  steps+=("c3q4_$r@200=$B3" "c3q8_$r@200=GPU_MAX_HW_QUEUES=8 $B3" "c5q4_$r@200=$C5" "c5q8_$r@200=GPU_MAX_HW_QUEUES=8 $C5")
done
scripts/gpu_run.sh gpurun_out/r06_y "${steps[@]}"
