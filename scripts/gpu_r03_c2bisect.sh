#!/bin/bash
# Round 3: the config-2 late-window golden (iteration 1564) differs from the
# oracle's. Run it under switches that move the device triangular solves back
# to the host, one variant per pytest process, plus a traced engine run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_c2bisect
mkdir -p $OUT
for V in "MILP_TRI_BTRAN=0" "MILP_TRI_CHAIN=0" "MILP_TRI_LOWER=0" "MILP_TRI_PAIR=0" "MILP_DEVICE_SOLVE=off"; do
  echo "== $V $(date +%T)"
  env $V timeout -k 10 150 python3 -u -m pytest $R/tests/test_fullsize_gpu.py -x -q --timeout 140 \
    --timeout-method thread -m gpu -k "windows_golden and 1564" > $OUT/$(echo $V | tr '=' '_').log 2>&1
  rc=$?
  echo "rc=$rc"; tail -3 $OUT/$(echo $V | tr '=' '_').log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo "== trace $(date +%T)"
MILP_TRACE=$OUT/c2tr timeout -k 10 150 python3 -u - <<'PY' > $OUT/trace.log 2>&1
import sys
sys.path[:0] = ['tests', 'or-tools_amd']
from mi_glop import abi, engine
import lp_gen
lp = lp_gen.dense_box_lp(10000, 50000, 20261015)
g = engine.LpHandle(abi.default_params(max_number_of_iterations=1564))
g.load(lp)
r = g.solve()
print("done", r.iterations, float(r.objective).hex())
PY
echo "trace rc=$?"
