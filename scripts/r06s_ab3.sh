#!/bin/bash
# Interleaved same-box A/B of the speculative flip FTRAN on config 5's window.
out=${1:-gpurun_out/r06s_ab}
B="python -u bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu"
bash scripts/gpu_run.sh "$out" \
  "on1@200=$B" "off1@200=MILP_SPEC_FLIP=0 $B" \
  "on2@200=$B" "off2@200=MILP_SPEC_FLIP=0 $B" \
  "on3@200=$B" "off3@200=MILP_SPEC_FLIP=0 $B"
