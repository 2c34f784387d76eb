#!/usr/bin/env python3
"""Whole solves on the MI355X (GetNumberOfIterations() / wall
time of the simplex solve): config 5 (sparse 100k x 1M, dual simplex) and
config 2 (dense 10k x 50k, primal simplex) run from the loaded LP to their
final status with no iteration cap, timed from the first iteration to the
last (load to HBM excluded, as bench.py's windows exclude it).

Checks, per LP:
  - KKT of the returned basic solution, computed here in numpy from the LP
    and the engine's primal values, duals and reduced costs (a property of
    the answer, no oracle): bound and row violations, rc = c - A^T y, the
    sign of every reduced cost and dual against its variable's status;
  - config 5 only: the final state's digests against tests/golden/
    c5_whole.json (the CPU oracle's own whole solve, scripts/
    make_c5_whole_golden.py), when that file is present.
Prints one JSON line per config. Development aid: the driver's bench.py
keeps its windows; this is the whole-solve leg the windows are judged by."""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "or-tools_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from mi_glop import abi, engine  # noqa: E402
import lp_gen  # noqa: E402

from kkt import kkt  # noqa: E402  (tests/kkt.py)


def log(msg):
    print(f"[whole {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def whole(name, lp, params, golden=None, limit_s=900.0):
    h = engine.LpHandle(params)
    h.load(lp)
    h.record_iteration_times(True)
    t0 = time.perf_counter()
    h.begin(1)  # upload, first factorization, iteration 1
    setup = time.perf_counter() - t0
    t1 = time.perf_counter()
    fin, it = False, 1
    next_log = t1 + 30.0
    while not fin and time.perf_counter() - t1 < limit_s:
        fin, it = h.run_until(it + 500)
        if time.perf_counter() > next_log:
            log(f"{name}: {it} iterations after {time.perf_counter() - t1:.0f}s")
            next_log += 30.0
    capped = not fin
    if capped:
        h.stop()
    r = h.finish()
    wall = time.perf_counter() - t1
    ts = h.iteration_times()
    var, cons = h.statuses()
    x, y, rc = h.primal(), h.duals(), h.reduced_costs()
    out = {"config": name, "m": lp.m, "n": lp.n, "nnz": int(lp.nnz),
           "status": int(r.problem_status), "iterations": int(r.iterations),
           "objective": float(r.objective), "setup_s": round(setup, 2),
           "solve_s": round(setup + wall, 2),
           "it_per_s_whole": r.iterations / (setup + wall), "capped_at_s": limit_s if capped else None,
           "kkt": kkt(lp, x, y, rc, var, cons, bool(lp.maximize))}
    if len(ts) >= 10:
        marks = {}
        for k in (1000, 5000, 10000, 20000, 40000, 80000, 160000):
            if k <= len(ts):
                marks[str(k)] = round(ts[k - 1], 3)
        out["engine_iteration_time_at"] = marks
    digests = {"iterations": int(r.iterations), "problem_status": int(r.problem_status),
               "error_code": int(r.error_code), "objective": float(r.objective).hex(),
               "basis": digest(h.basis()), "state": digest(h.state()),
               "var_status": digest(var), "cons_status": digest(cons),
               "primal": digest(x), "duals": digest(y), "reduced_costs": digest(rc)}
    if golden is not None:
        g = golden["final"]
        bad = sorted(k for k in g if g[k] != digests[k])
        out["oracle_check"] = {"fields": sorted(g), "mismatches": len(bad), "differing": bad,
                               "oracle_it_per_s": golden.get("oracle_it_per_s"),
                               "oracle_solve_s": golden.get("oracle_solve_s"),
                               "oracle_host": golden.get("oracle_host")}
    out["digests"] = digests
    h.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="*", default=["c5", "c2"])
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--limit-s", type=float, default=900.0,
                    help="wall-clock cap per solve (the result then says capped_at_s)")
    ap.add_argument("--c5-m", type=int, default=100000)
    ap.add_argument("--c5-n", type=int, default=1000000)
    a = ap.parse_args()
    for c in a.configs:
        if c == "c5":
            lp = lp_gen.sparse_c5_lp(a.c5_m, a.c5_n, 10, a.seed)
            gp = os.path.join(REPO, "tests", "golden", f"c5_whole_{a.c5_m}.json")
            golden = json.load(open(gp)) if os.path.exists(gp) else None
            log(f"c5: {a.c5_m}x{a.c5_n} solving to the end")
            out = whole(f"config 5 shape {a.c5_m}x{a.c5_n}", lp,
                        abi.default_params(use_dual_simplex=1), golden, a.limit_s)
        else:
            lp = lp_gen.dense_box_lp(10000, 50000, a.seed)
            log("c2: solving to the end")
            out = whole("config 2", lp, abi.default_params(), None, a.limit_s)
        log(f"{c}: {out['iterations']} iterations, status {out['status']}, "
            f"{out['it_per_s_whole']:.1f} it/s")
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
