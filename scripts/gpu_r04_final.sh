#!/bin/bash
# Round 4 close: the whole GPU suite, smoke, the default bench line, and the
# two-rank one-GPU rehearsal of the split config-5 path (shared-memory
# exchange; gloo for the barrier/max, every rank on GPU 0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUTDIR:-r04_final}
mkdir -p $OUT
cd $R
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests -m gpu > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $OUT/bench.json; echo
[ $rc -eq 0 ] || exit $rc
MILP_BENCH_ONE_GPU=1 timeout -k 10 600 python3 -u bench.py --gpus 2 --no-c2 --no-c3 --batch-lps 0 \
  --no-cpu > $OUT/rehearsal_2rank.json 2> $OUT/rehearsal_2rank.err
rc=$?; echo "rehearsal rc=$rc"; tail -c 600 $OUT/rehearsal_2rank.json; echo
exit $rc
