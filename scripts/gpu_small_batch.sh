#!/bin/bash
# Batched small-LP launches (MILP_SMALL_BATCH=1): parity, then C4 / C3 rates.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ -n "$RUN_TESTS" ]; then
MILP_SMALL_BATCH=1 MILP_BATCH_FIBERS=2 MILP_BATCH_THREADS=2 timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_fullsize_gpu.py -k "small or batch or config3 or random or jobshop or known" -m gpu -q -x -n 4 --timeout 250 --timeout-method thread \
  > $OUT/sb_tests.log 2>&1 || { echo "small-batch tests failed"; grep -E "FAILED|Error" $OUT/sb_tests.log | head; tail -30 $OUT/sb_tests.log; exit 1; }
tail -1 $OUT/sb_tests.log
fi
for W in 64 128 192; do
  MILP_SMALL_BATCH=1 MILP_BATCH_THREADS=16 timeout -k 10 200 python -u scripts/probe_batch.py --lps 512 --workers $W > $OUT/sb_c4_w$W.json 2> $OUT/sb_c4_w$W.err || { echo "c4 probe failed"; tail -20 $OUT/sb_c4_w$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/sb_c4_w$W.json')); print('C4 batch W=$W', [round(v['lps_per_s'],1) for k,v in d.items() if k.startswith('gpu_')])"
done
for F in 4 8; do
  MILP_SMALL_BATCH=1 MILP_BATCH_FIBERS=$F timeout -k 10 200 python -u scripts/probe_c3.py --workers 16 > $OUT/sb_c3_f$F.json 2> $OUT/sb_c3_f$F.err || { echo "c3 probe failed"; tail -20 $OUT/sb_c3_f$F.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/sb_c3_f$F.json')); print('C3 batch F=$F', [round(v['lps_per_s'],1) for k,v in d.items() if k.startswith('gpu_')])"
done
echo done
