"""Debug aid: solve LPs with the oracle and the device engine under
MILP_TRACE and report the first iteration whose hashed iterate differs."""
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "or-tools_amd"), os.path.join(REPO, "tests")]
prefix = os.path.join(tempfile.mkdtemp(), "trace")
os.environ["MILP_TRACE"] = prefix

from mi_glop import abi, engine  # noqa: E402
import kat_lps  # noqa: E402
import lp_gen  # noqa: E402
import parity_util  # noqa: E402

cases = [(b.__name__, b()[0]) for b in kat_lps.ALL]
cases += [(f"sparse{s}", lp_gen.random_sparse_lp(40, 120, 0.08, s)) for s in range(4)]
cases += [("dense", lp_gen.dense_box_lp(48, 192, 1))]
for name, lp in cases:
    for dual in (0, 1):
        for suf in (".oracle", ".device"):
            if os.path.exists(prefix + suf):
                os.remove(prefix + suf)
        p = abi.default_params(use_dual_simplex=dual)
        o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q, 0))
        a = open(prefix + ".oracle").read().splitlines() if os.path.exists(prefix + ".oracle") else []
        b = open(prefix + ".device").read().splitlines() if os.path.exists(prefix + ".device") else []
        first = next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), None)
        ok = first is None and len(a) == len(b) and ro.iterations == rg.iterations
        print(f"{name:28s} dual={dual} st={ro.problem_status}/{rg.problem_status} "
              f"err={ro.error_code}/{rg.error_code} oracle_it={ro.iterations} dev_it={rg.iterations} "
              f"obj {ro.objective!r} {rg.objective!r} {'OK' if ok else 'DIFF'}")
        if first is not None:
            print("   oracle:", a[first]); print("   device:", b[first])
            if first > 0:
                print("   prev  :", a[first - 1])
            k = first + 1
            while k < len(a) and a[k].startswith("  "):
                print("   o", a[k]); print("   d", b[k] if k < len(b) else None); k += 1
        if rg.error_code:
            print("   device error:", g.last_error() if hasattr(g, "last_error") else "?")
