#!/bin/bash
# Round 3: the engine's primal-residual checks (CorrectErrorsOnVariableValues)
# on config 2 up to iteration 456, to compare with the oracle's.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_c2res
mkdir -p $OUT
rm -f $OUT/res.device
MILP_TRACE_RESIDUAL=$OUT/res.device timeout -k 10 200 python3 -u - <<'PY' > $OUT/run.log 2>&1
import sys
sys.path[:0] = ['tests', 'or-tools_amd']
from mi_glop import abi, engine
import lp_gen
lp = lp_gen.dense_box_lp(10000, 50000, 20261015)
g = engine.LpHandle(abi.default_params(max_number_of_iterations=456))
g.load(lp)
r = g.solve()
print("done", r.iterations, float(r.objective).hex())
PY
echo "rc=$?"; cat $OUT/res.device
