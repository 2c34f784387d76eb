#!/bin/bash
# Round validation on one GPU box: the whole GPU suite, smoke(), the default
# bench, then two short probes. Each step under its own time limit; the
# session stops at the first failing step (scripts/gpu_run.sh).
#   scripts/gpu_final.sh OUT_DIR
out=${1:-gpurun_out/final}
B3="python -u bench.py --no-c5 --no-c2 --batch-lps 0 --no-cpu --profile-batch"
exec_steps=(
  "tests@780=python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider"
  "smoke@120=python -u -c 'import __graft_entry__ as g; g.smoke()'"
  "bench@330=python -u bench.py"
  "c3s1@100=MILP_SMALL_BATCH_STREAMS=1 $B3"
)
bash scripts/gpu_run.sh "$out" "${exec_steps[@]}"
