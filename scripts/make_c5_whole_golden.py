#!/usr/bin/env python3
"""Generates tests/golden/c5_whole_<m>.json: the CPU oracle's final state on
the config-5 generator's LP with m rows and 10 m columns (bench.py's config 5
is m = 100 000: sparse, 10 per column, seed 20261015, dual simplex, Glop
defaults) solved to its final status with no iteration cap,
plus the oracle's whole-solve rate (iterations / wall of the simplex solve,
SURVEY 8(d)) on this container's host (one core).

The full size needs ~13 iterations per row (measured: 13 045 at m = 1 000,
34 201 at m = 2 000), so its whole solve is hours for the oracle; smaller
shapes run here once and scripts/whole_solve.py compares the engine's final
state with these digests. Test infrastructure only: the oracle is the
checker."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "or-tools_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "scripts"))

from mi_glop import abi  # noqa: E402
import lp_gen  # noqa: E402
import oracle_lib  # noqa: E402
from make_c2_window_golden import lp_digest, state_digests  # noqa: E402


def main():
    seed = 20261015
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    n = 10 * m
    t = time.time()
    lp = lp_gen.sparse_c5_lp(m, n, 10, seed)
    gen_s = time.time() - t
    p = abi.default_params(use_dual_simplex=1)
    o = oracle_lib.OracleLp(p)
    o.record_iteration_times(True)
    o.load(lp)
    t = time.time()
    r = o.solve()
    wall = time.time() - t
    out = {"lp": lp_digest(lp), "seed": seed, "m": m, "n": n, "per_col": 10,
           "final": state_digests(o, r), "objective": float(r.objective),
           "oracle_solve_s": round(wall, 2), "oracle_it_per_s": r.iterations / wall,
           "oracle_host": os.uname().nodename, "gen_s": round(gen_s, 1)}
    ts = o.iteration_times()
    if len(ts) > 0:
        out["oracle_iteration_time_at"] = {str(k): round(ts[k - 1], 3) for k in
                                           (1000, 5000, 10000, 20000, 40000, 80000)
                                           if k <= len(ts)}
    path = os.path.join(REPO, "tests", "golden", f"c5_whole_{m}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
