#!/bin/bash
# Round 4: chain kernel with the next output's structure prefetched: the
# device-solve parity tests and the config-5 full-size window parity, then
# the config-5 window rate (twice, to see the noise).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_chainpf
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_device_solve_gpu.py tests/test_fullsize_gpu.py::test_config5_window_parity -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 \
  --steps 1000 --variants "" MILP_TRI_CHAIN_WIDTH=512 "" > $OUT/c5.json 2> $OUT/c5.err || exit 1
grep -h "it/s" $OUT/c5.err
python3 -c "
import json
for k, d in json.load(open('$OUT/c5.json'))['gpu'].items():
    for n, v in d['kernels'].items():
        if n == 'tri_solve': print('   ', k, n, v)"
