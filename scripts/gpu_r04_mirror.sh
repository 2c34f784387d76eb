#!/bin/bash
# Round 4: dual device mode without the host mirror of the update-row list:
# the dual-device parity tests, then the config-5 window.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_mirror
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_fullsize_gpu.py tests/test_parity_gpu.py -m gpu > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 \
  --steps 1000 > $OUT/c5.json 2> $OUT/c5.err || exit 1
grep -h "it/s" $OUT/c5.err
python3 -c "
import json
for k, d in json.load(open('$OUT/c5.json'))['gpu'].items():
    for n, v in d['kernels'].items():
        if v.get('device_ms', 0) > 20: print('   ', n, v)"
