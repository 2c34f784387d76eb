#!/usr/bin/env python3
"""Generates tests/golden/c2_windows.json: the CPU oracle's state on the
config-2 LP (bench.py: dense 10k x 50k, seed 20261015, primal simplex, Glop
defaults) at the iteration caps bench.py's two windows end at (67: the early
window 3..67; 1564: the late window 1500..1564).

The oracle needs ~0.5 s per iteration on this LP late in the solve, too slow
for a GPU test, so it runs here once and the test compares the engine with
these digests (sha256 of the exact bytes of basis, state, statuses, primal,
duals and reduced costs; status, iteration count and objective as values).
Test infrastructure only: the oracle is the checker."""
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "or-tools_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
from mi_glop import abi  # noqa: E402
import lp_gen  # noqa: E402
import oracle_lib  # noqa: E402


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def lp_digest(lp):
    """The LP the digests describe (the GPU test checks it builds the same)."""
    return {k: digest(getattr(lp, k)) for k in ("row_lb", "row_ub", "obj", "vals")}


def state_digests(o, r):
    var, cons = o.statuses()
    return {"iterations": int(r.iterations), "problem_status": int(r.problem_status),
            "error_code": int(r.error_code), "objective": float(r.objective).hex(),
            "basis": digest(o.basis()), "state": digest(o.state()),
            "var_status": digest(var), "cons_status": digest(cons),
            "primal": digest(o.primal()), "duals": digest(o.duals()),
            "reduced_costs": digest(o.reduced_costs())}


def main():
    caps = [int(c) for c in (sys.argv[1:] or ["67", "1564"])]
    seed = 20261015
    t = time.time()
    lp = lp_gen.dense_box_lp(10000, 50000, seed)
    print(f"generated in {time.time() - t:.1f}s", flush=True)
    out = {"lp": "lp_gen.dense_box_lp(10000, 50000, 20261015)",
           "lp_digest": lp_digest(lp),
           "params": "abi.default_params(max_number_of_iterations=cap)",
           "generator": "scripts/make_c2_window_golden.py", "caps": {}}
    path = os.path.join(REPO, "tests", "golden", "c2_windows.json")
    for cap in caps:
        o = oracle_lib.OracleLp(abi.default_params(max_number_of_iterations=cap))
        o.load(lp)
        t = time.time()
        r = o.solve()
        out["caps"][str(cap)] = state_digests(o, r)
        out["caps"][str(cap)]["oracle_seconds"] = round(time.time() - t, 1)
        print(cap, out["caps"][str(cap)], flush=True)
        json.dump(out, open(path, "w"), indent=1)
        del o


if __name__ == "__main__":
    main()
