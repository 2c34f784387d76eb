#!/bin/bash
# Round 4: chain kernel with LDS inputs and ready words, records one output
# ahead: the device-solve parity tests, then the config-5 window rate and
# kernel split (probe), then the sdual instruction-fetch counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_chain
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_device_solve_gpu.py -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 \
  --steps 1000 --variants "" MILP_TRI_CHAIN=0 MILP_TRI_CHAIN_WIDTH=4096 MILP_TRI_CHAIN_WIDTH=16384 > $OUT/c5.json 2> $OUT/c5.err || exit 1
python3 -c "
import json
for k, d in json.load(open('$OUT/c5.json'))['gpu'].items():
    print(k, 'c5 it/s', d['gpu_it_per_s'], {n: (v['launches'], v['device_ms']) for n, v in d['kernels'].items()})"
