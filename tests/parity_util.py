"""Shared helpers: run one LP through the oracle and through the MI355X
engine and compare everything the drop-in contract promises:
status, iteration count, basis and statuses bit-exact; objective within 1e-6
relative (observed: bit-identical)."""
import numpy as np

from mi_glop import abi

import oracle_lib


def solve_both(lp, params, handle_factory):
    o = oracle_lib.OracleLp(params)
    o.load(lp)
    ro = o.solve()
    g = handle_factory(params)
    g.load(lp)
    rg = g.solve()
    return o, ro, g, rg


def compare(o, ro, g, rg, lp, rel_tol=1e-6):
    assert rg.error_code == ro.error_code, (rg.error_code, ro.error_code)
    assert rg.problem_status == ro.problem_status, (
        abi.PROBLEM_STATUS[rg.problem_status], abi.PROBLEM_STATUS[ro.problem_status])
    assert rg.iterations == ro.iterations, (rg.iterations, ro.iterations)
    if ro.error_code != 0 or ro.problem_status == abi.INVALID_PROBLEM:
        return
    if np.isfinite(ro.objective):
        assert abs(rg.objective - ro.objective) <= rel_tol * max(1.0, abs(ro.objective)), (
            rg.objective, ro.objective)
    else:
        assert rg.objective == ro.objective
    np.testing.assert_array_equal(g.basis(), o.basis())
    np.testing.assert_array_equal(g.state(), o.state())
    gv, gc = g.statuses()
    ov, oc = o.statuses()
    np.testing.assert_array_equal(gv, ov)
    np.testing.assert_array_equal(gc, oc)
    # Same pivots and same arithmetic: values agree to the last bit.
    np.testing.assert_array_equal(g.primal(), o.primal())
    np.testing.assert_array_equal(g.duals(), o.duals())
    np.testing.assert_array_equal(g.reduced_costs(), o.reduced_costs())
