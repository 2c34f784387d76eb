set -u
cd $GRAFT_REPO_ROOT
B3="python3 -u bench.py --no-c5 --no-c2 --batch-lps 0 --no-cpu --profile-batch"
B4="python3 -u bench.py --no-c5 --no-c2 --no-c3 --no-cpu --batch-share-lps 0"
C5="python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000"
scripts/gpu_run.sh gpurun_out/r06_w \
 "c3q4@200=$B3" "c3q16@200=GPU_MAX_HW_QUEUES=16 $B3" \
 "c4q4@200=$B4" "c4q16@200=GPU_MAX_HW_QUEUES=16 $B4" \
 "c5q4@200=$C5" "c5q16@200=GPU_MAX_HW_QUEUES=16 $C5" \
 "c3q8@200=GPU_MAX_HW_QUEUES=8 $B3" "c4q8@200=GPU_MAX_HW_QUEUES=8 $B4"
