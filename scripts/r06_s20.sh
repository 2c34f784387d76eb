set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_t
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o run -- python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 300 > gpurun_out/r06_t/probe.out 2> gpurun_out/r06_t/probe.err && \
f=$(find /tmp/kt -name "*kernel_trace.csv" | head -1) && python3 scripts/kt_tail.py "$f" gpurun_out/r06_t/kt_tail.csv 3000
