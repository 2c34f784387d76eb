#!/bin/bash
# Round 3: one LP through the sdual pool kernel with progress reports.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_pooldebug
mkdir -p $OUT
MILP_SDUAL=device MILP_SDUAL_POOL=1 MILP_SDUAL_DEBUG=1 timeout -k 5 25 python3 -u - <<'PY' > $OUT/run.log 2>&1
import sys
sys.path[:0] = ['tests', 'or-tools_amd']
from mi_glop import abi, engine
import lp_gen
lp = lp_gen.random_sparse_lp(60, 240, 0.05, 900)
g = engine.LpHandle(abi.default_params(use_dual_simplex=1), 0)
g.load(lp)
r = g.solve()
print("done", r.iterations, r.problem_status, g.run_counters())
PY
echo "rc=$?"; tail -30 $OUT/run.log
