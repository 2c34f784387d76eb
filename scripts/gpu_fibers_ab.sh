#!/bin/bash
# Batched small LPs with several LPs per host thread on fibers (engine/fibers.h):
# parity of the batched paths with fibers on, then C4 / C3 rates per setting.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
MILP_BATCH_FIBERS=3 MILP_BATCH_THREADS=2 timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x -k "batch" --timeout 250 --timeout-method thread \
  > $OUT/fiber_tests.log 2>&1 || { echo "fiber tests failed"; grep -E "FAILED|Error" $OUT/fiber_tests.log | head; tail -30 $OUT/fiber_tests.log; exit 1; }
tail -1 $OUT/fiber_tests.log
for T in 16; do
  for W in 16 32 48 64; do
    MILP_BATCH_THREADS=$T timeout -k 10 200 python -u scripts/probe_batch.py --lps 512 --workers $W > $OUT/c4_t${T}_w${W}.json 2> $OUT/c4_t${T}_w${W}.err || { echo "c4 probe failed"; tail -20 $OUT/c4_t${T}_w${W}.err; exit 1; }
    echo "C4 threads=$T workers=$W: $(tail -c 400 $OUT/c4_t${T}_w${W}.json)"
  done
done
for F in 1 2 3 4; do
  MILP_BATCH_FIBERS=$F timeout -k 10 200 python -u scripts/probe_c3.py --workers 16 > $OUT/c3_f$F.json 2> $OUT/c3_f$F.err || { echo "c3 probe failed"; tail -20 $OUT/c3_f$F.err; exit 1; }
  echo "C3 fibers=$F: $(tail -c 300 $OUT/c3_f$F.json)"
done
echo done
