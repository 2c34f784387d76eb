#!/bin/bash
# Config 5 with the speculative flip FTRAN on (oracle check) and off, twice.
out=${1:-gpurun_out/r06s_b}
bash scripts/gpu_run.sh "$out" \
  "c5on@330=MILP_SPEC_FLIP_STATS=1 python -u bench.py --no-c2 --no-c3 --batch-lps 0" \
  "c5off@200=MILP_SPEC_FLIP=0 python -u bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu" \
  "c5on2@200=python -u bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu" \
  "c5off2@200=MILP_SPEC_FLIP=0 python -u bench.py --no-c2 --no-c3 --batch-lps 0 --no-cpu"
