#!/bin/bash
# rocprofv3 passes of one bench.py command, each its own run (kernel trace
# with --stats, FETCH_SIZE, WRITE_SIZE: the TCC slots cannot hold both),
# summarised into profiles/<tag>/ by scripts/profile_summary.py.
#   scripts/profile_bench.sh <tag> <c2|c3|c4|c5> <bench.py arguments...>
# For c3/c4 set PROFILE_LPS to the LPs the profiled process solves (bench.py
# --profile-batch prints it): the traffic is then also given per LP.
# Runs from the repo root on the GPU box; a failing pass ends the script.
set -o pipefail
tag=$1
workload=$2
shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$tag
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# A profiled run releases every HIP resource at exit (mi_lp_shutdown), so
# that rocprofiler-sdk's own teardown finds nothing left.
export MILP_DEVICE_RESET_AT_EXIT=1 MILP_CRASH_REPORT=1
# TRACE_EXTRA: arguments appended to the trace pass only (argparse keeps the
# last occurrence), e.g. "--c3-workers 2": the kernel trace of the 16-thread
# config-3 batch faults inside rocprofiler-sdk (profiles/r06_c3trace), the
# counter passes below run the benched arguments. trace.log (with the engine's
# MILP_CRASH_REPORT frames) stays in $OUT on failure.
# The per-dispatch traces and counter rows (hundreds of MB over a config-5
# solve) stay on the box, also when a pass fails: gpurun copies back at most
# 64 MiB.
cleanup() { rm -f $OUT/trace/run_kernel_trace.csv $OUT/*/run_counter_collection.csv $OUT/*/*.db; }
trap cleanup EXIT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py "$@" ${TRACE_EXTRA:-} > $OUT/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  p=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -k 10 600 rocprofv3 --pmc $c -d $OUT/$p -o run --output-format csv -- \
    python3 $R/bench.py "$@" > $OUT/$p.log 2>&1 || { echo "$c pass failed"; exit 1; }
done
cd $R && PROFILE_OUT_ROOT=$R/gpurun_out/profiles python3 scripts/profile_summary.py $OUT $tag $workload ${PROFILE_LPS:-0}
