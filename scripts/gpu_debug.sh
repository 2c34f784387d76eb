#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/trace_diff.py > gpurun_out/trace_diff.log 2>&1; rc=$?
cat gpurun_out/trace_diff.log; exit $rc
