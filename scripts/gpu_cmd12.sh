set -o pipefail
mkdir -p gpurun_out
MILP_PHASE_TIMING=1 MILP_PHASE_TIMING_EVERY=1000 timeout -k 10 600 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 > gpurun_out/probe_c5.json 2> gpurun_out/probe_c5.err || { echo "c5 probe failed"; tail -30 gpurun_out/probe_c5.err; exit 1; }
cat gpurun_out/probe_c5.json
grep "device ratio test" gpurun_out/probe_c5.err | tail -25
