#!/usr/bin/env python3
"""Debug aid: config-2 LP (dense 10k x 50k, seed 20261015, primal) solved up
to an iteration cap under MILP_TRACE (per-iteration hashes incl. the FTRAN
stages) with MILP_TRACE_DUMP at the given iteration, by the oracle (--oracle,
on the CPU) or by the engine (on the GPU). Usage:
  MILP_TRACE=<prefix> MILP_TRACE_DUMP=<k> c2_trace.py [--oracle] <cap>"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "or-tools_amd"), os.path.join(REPO, "tests")]
from mi_glop import abi  # noqa: E402
import lp_gen  # noqa: E402

use_oracle = "--oracle" in sys.argv
cap = int([a for a in sys.argv[1:] if not a.startswith("--")][0])
lp = lp_gen.dense_box_lp(10000, 50000, 20261015)
p = abi.default_params(max_number_of_iterations=cap)
if use_oracle:
    import oracle_lib
    h = oracle_lib.OracleLp(p)
else:
    from mi_glop import engine
    h = engine.LpHandle(p)
h.load(lp)
t = time.time()
r = h.solve()
print("done", r.iterations, float(r.objective).hex(), f"{time.time() - t:.1f}s", flush=True)
