#!/bin/bash
# Round 4: rank-one products with the next chunk prefetched, parallel
# zeroing of long vectors: segment parity (dual and primal), config 4 with
# the segment profile, config 5's window.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_r1pf
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_sdual_gpu.py tests/test_sprimal_gpu.py -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
MILP_SDUAL_PROFILE=1 timeout -k 10 200 python3 -u scripts/probe_batch.py --node --lps 1024 \
  --workers 1024 > $OUT/c4.json 2> $OUT/c4.err || exit 1
timeout -k 10 200 python3 -u scripts/probe_batch.py --node --lps 1024 --workers 1024 \
  > $OUT/c4b.json 2> $OUT/c4b.err || exit 1
timeout -k 10 300 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 \
  --steps 1000 > $OUT/c5.json 2> $OUT/c5.err || exit 1
grep -h "LPs/s\|it/s" $OUT/*.err
grep "rank-one\|btran  \|ftran  \|tau solve\|rc+norms" $OUT/c4.err
