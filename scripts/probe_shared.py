#!/usr/bin/env python3
"""Bisect the shared batch caches (development aid): a node's children
through mi_lp_batch_solve_bounds with MILP_BATCH_SHARED_LU / _NORMS set per
combination; each child's deterministic time against the oracle's."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "or-tools_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from mi_glop import abi, engine  # noqa: E402
import oracle_lib  # noqa: E402
import test_sdual_gpu as T  # noqa: E402

shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "6,6").split(","))
lp, state, lbs, ubs = T._children(shape, 24)
p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
o = oracle_lib.OracleLp(p)
o.load(lp)
ref = []
for i in range(len(lbs)):
    o.set_variable_bounds(lbs[i], ubs[i])
    o.load_basis_state(state)
    ref.append(o.solve())
for combo in ("00", "10", "01", "11"):
    os.environ["MILP_BATCH_SHARED_LU"] = combo[0]
    os.environ["MILP_BATCH_SHARED_NORMS"] = combo[1]
    ws = [engine.LpHandle(p) for _ in range(8)]
    for w in ws:
        w.load(lp)
    res = engine.batch_solve_bounds(ws, lbs, ubs, state)
    diffs = [(i, (r.deterministic_time - q.deterministic_time) / 2e-9)
             for i, (r, q) in enumerate(zip(res, ref))
             if r.deterministic_time != q.deterministic_time]
    same = all(r.iterations == q.iterations and r.objective == q.objective
               for r, q in zip(res, ref))
    print(f"lu={combo[0]} norms={combo[1]} parity={same} dtime diffs (ops): {diffs[:12]}",
          flush=True)
