"""Finds the first iteration cap at which the engine and the oracle differ
on one LP, for several engine switch settings (one handle per setting).
Diagnostic for parity failures; prints one line per (variant, cap)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "or-tools_amd"))

import numpy as np  # noqa: E402

from mi_glop import abi, engine  # noqa: E402

import lp_gen  # noqa: E402
import oracle_lib  # noqa: E402
import parity_util  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=600)
    ap.add_argument("--n", type=int, default=6000)
    ap.add_argument("--per-col", type=int, default=6)
    ap.add_argument("--seed", type=int, default=78)
    ap.add_argument("--dual", type=int, default=1)
    ap.add_argument("--caps", type=int, nargs="*", default=[50, 100, 200, 400, 800, 1600, 3200])
    ap.add_argument("--variants", nargs="*", default=["X=1"])
    a = ap.parse_args()
    lp = lp_gen.sparse_c5_lp(a.m, a.n, a.per_col, a.seed)
    for var in a.variants:
        saved = dict(os.environ)
        for kv in var.split(","):
            k, v = kv.split("=", 1)
            os.environ[k] = v
        for cap in a.caps:
            p = abi.default_params(use_dual_simplex=a.dual, max_number_of_iterations=cap)
            o = oracle_lib.OracleLp(p)
            o.load(lp)
            ro = o.solve()
            g = engine.LpHandle(p)
            g.load(lp)
            t = time.time()
            rg = g.solve()
            try:
                parity_util.compare(o, ro, g, rg, lp)
                ok = "equal"
            except AssertionError as e:
                ok = "DIFFER " + str(e).splitlines()[0][:160]
            st = g.kernel_stats()
            print(f"{var} cap={cap} it={rg.iterations}/{ro.iterations} "
                  f"status={rg.problem_status}/{ro.problem_status} {ok} "
                  f"tri={st['tri_solve']['launches']} triL={st['tri_solve_l']['launches']} "
                  f"tau={st['tri_solve_tau']['launches']} ratio={st['dual_ratio']['launches']} "
                  f"{time.time() - t:.2f}s", flush=True)
            del g
            if ok != "equal":
                break
        os.environ.clear()
        os.environ.update(saved)


if __name__ == "__main__":
    main()
