"""CPU tests of the oracle: pinned by the reference's own known answers
(tests/kat_lps.py cites the upstream test lines) and by HiGHS objectives on
seeded synthetic LPs."""
import numpy as np
import pytest

from mi_glop import abi

import kat_lps
import lp_gen
import oracle_lib


@pytest.mark.parametrize("builder", kat_lps.ALL, ids=lambda f: f.__name__)
@pytest.mark.parametrize("dual", [0, 1])
def test_known_answers(builder, dual):
    lp, exp = builder()
    o = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=dual))
    o.load(lp)
    r = o.solve()
    if "status_in" in exp:
        assert abi.PROBLEM_STATUS[r.problem_status] in exp["status_in"]
        return
    assert r.problem_status == exp["status"]
    assert r.objective == pytest.approx(exp["objective"], rel=1e-9, abs=1e-9)
    for key, getter in (("primal", o.primal), ("duals", o.duals),
                        ("reduced_costs", o.reduced_costs),
                        ("activities", o.activities)):
        if key in exp:
            np.testing.assert_allclose(getter(), exp[key], rtol=1e-7, atol=1e-7)


@pytest.mark.parametrize("seed", range(24))
@pytest.mark.parametrize("dual", [0, 1])
def test_against_highs(seed, dual):
    m = [6, 12, 40, 90][seed % 4]
    n = [9, 30, 70, 250][seed % 4]
    lp = lp_gen.random_sparse_lp(m, n, 0.3 if m < 30 else 0.06, seed,
                                 maximize=bool(seed % 2))
    st, ref = lp_gen.to_scipy(lp)
    o = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=dual))
    o.load(lp)
    r = o.solve()
    if st != 0:
        assert r.problem_status != abi.OPTIMAL
        return
    assert r.problem_status == abi.OPTIMAL
    assert abs(r.objective - ref) <= 1e-6 * max(1.0, abs(ref))


def test_dense_box_against_highs():
    lp = lp_gen.dense_box_lp(60, 240, 7)
    st, ref = lp_gen.to_scipy(lp)
    o = oracle_lib.OracleLp()
    o.load(lp)
    r = o.solve()
    assert st == 0 and r.problem_status == abi.OPTIMAL
    assert abs(r.objective - ref) <= 1e-9 * max(1.0, abs(ref))


def test_warm_start_bound_change_dual():
    """CP-SAT style re-solve: same matrix, one bound tightened, warm-started
    dual simplex (linear_programming_constraint.cc:443-464, 709-760)."""
    lp = lp_gen.random_sparse_lp(40, 120, 0.08, 5)
    p = abi.default_params(use_dual_simplex=1)
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    r0 = o.solve()
    assert r0.problem_status == abi.OPTIMAL
    x = o.primal()
    j = int(np.argmax(np.abs(x - np.round(x))))
    lp.col_ub = lp.col_ub.copy()
    lp.col_ub[j] = np.floor(x[j])
    o.load(lp)
    r1 = o.solve()
    st, ref = lp_gen.to_scipy(lp)
    if st == 0:
        assert r1.problem_status == abi.OPTIMAL
        assert abs(r1.objective - ref) <= 1e-6 * max(1, abs(ref))
    # Warm start is cheaper than a cold solve of the same LP.
    cold = oracle_lib.OracleLp(p)
    cold.load(lp)
    rc = cold.solve()
    assert r1.iterations <= rc.iterations


def _invalid_variants():
    """LinearProgram::IsValid / IsCleanedUp failures (lp_solver.cc:185-202);
    pdlp/test_util.cc also ships an invalid / inconsistent-bounds LP."""
    import copy
    base, _ = kat_lps.tiny_lp()
    out = []
    lp = copy.deepcopy(base); lp.row_lb[0], lp.row_ub[0] = 5.0, 1.0; out.append(("row lb>ub", lp))
    lp = copy.deepcopy(base); lp.col_lb[1] = np.inf; out.append(("col lb=+inf", lp))
    lp = copy.deepcopy(base); lp.vals[0] = 0.0; out.append(("explicit zero", lp))
    lp = copy.deepcopy(base); lp.vals[1] = np.nan; out.append(("nan coefficient", lp))
    lp = copy.deepcopy(base); lp.obj[2] = np.inf; out.append(("inf objective", lp))
    lp = copy.deepcopy(base)
    lp.row_idx[0], lp.row_idx[1] = lp.row_idx[1], lp.row_idx[0]
    out.append(("unsorted rows", lp))
    return out


@pytest.mark.parametrize("case", _invalid_variants(), ids=lambda c: c[0])
def test_oracle_invalid_problem(case):
    _, lp = case
    o = oracle_lib.OracleLp(abi.default_params())
    o.load(lp)
    r = o.solve()
    assert r.problem_status == abi.INVALID_PROBLEM


def test_oracle_batched_children_match_sequential():
    """The batch scheduler (shared counter, 4 worker handles) gives every
    child the same result as a fresh sequential solve (C4 workload)."""
    import jobshop
    lp, ycols = jobshop.relaxation(jobshop.FT06)
    root = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=1))
    root.load(lp)
    assert root.solve().problem_status == abi.OPTIMAL
    st = root.state()
    lbs, ubs = jobshop.child_bounds(lp, ycols, 32, 5)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    ws = [oracle_lib.OracleLp(p) for _ in range(4)]
    for w in ws:
        w.load(lp)
    res = oracle_lib.batch_solve_bounds(ws, lbs, ubs, st)
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    for i in range(32):
        o.set_variable_bounds(lbs[i], ubs[i])
        o.load_basis_state(st)
        r = o.solve()
        assert (res[i].problem_status, res[i].iterations, res[i].objective) == \
            (r.problem_status, r.iterations, r.objective)


def test_netlib_suite_shapes_and_oracle_on_smallest():
    """Config-3 stand-in suite: 94 deterministic LPs from 27 rows up; the
    smallest members solve to OPTIMAL on the oracle and agree with HiGHS."""
    import netlib_suite
    shapes = netlib_suite.suite_shapes(max_rows=1000)
    assert len(shapes) == 94
    assert shapes[0][0] == 27 and shapes[-1][0] == 1000
    assert shapes == netlib_suite.suite_shapes(max_rows=1000)  # deterministic
    lps = netlib_suite.suite(count=94, max_rows=1000)[:6]
    for lp in lps:
        o = oracle_lib.OracleLp(abi.default_params())
        o.load(lp)
        r = o.solve()
        assert r.problem_status == abi.OPTIMAL
        st, val = lp_gen.to_scipy(lp)
        assert st == 0 and abs(r.objective - val) <= 1e-6 * max(1.0, abs(val))


@pytest.mark.parametrize("builder", kat_lps.ALL, ids=lambda f: f.__name__)
@pytest.mark.parametrize("dual", [0, 1])
def test_product_form_known_answers(builder, dual):
    """use_middle_product_form_update=false: Glop's product-form (eta)
    updates, basis_representation.cc:25-176, on the
    reference's known-answer LPs.

    Upstream quirk, restated as is: in this mode LeftSolveForUnitRow
    (basis_representation.cc:403-411) keeps as rho's non-zero list only the
    positions the eta solves touched, and the dense LU solve that follows
    fills in others; UpdateRow::ComputeUpdateRow (update_row.cc:90-104)
    iterates that list, so the update row can miss entries. The dual simplex
    can then end ABNORMAL or IMPRECISE where the middle-product form is exact (two of the
    known-answer LPs here; clearing the list makes them pass, which confirms
    the cause). Not pinned against a running Glop (it cannot be built here)."""
    lp, exp = builder()
    o = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=dual,
                                               use_middle_product_form_update=0))
    o.load(lp)
    r = o.solve()
    if dual and abi.PROBLEM_STATUS[r.problem_status] in ("ABNORMAL", "IMPRECISE"):
        return
    if "status_in" in exp:
        assert abi.PROBLEM_STATUS[r.problem_status] in exp["status_in"]
        return
    assert r.problem_status == exp["status"]
    assert r.objective == pytest.approx(exp["objective"], rel=1e-9, abs=1e-9)


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("dual", [0, 1])
def test_product_form_against_highs(seed, dual):
    m = [12, 40, 90, 150][seed % 4]
    n = [30, 70, 250, 400][seed % 4]
    lp = lp_gen.random_sparse_lp(m, n, 0.3 if m < 30 else 0.06, 500 + seed,
                                 maximize=bool(seed % 2))
    st, ref = lp_gen.to_scipy(lp)
    o = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=dual,
                                               use_middle_product_form_update=0))
    o.load(lp)
    r = o.solve()
    if st != 0:
        assert r.problem_status != abi.OPTIMAL
        return
    assert r.problem_status == abi.OPTIMAL
    assert abs(r.objective - ref) <= 1e-6 * max(1.0, abs(ref))


@pytest.mark.parametrize("basis", [1, 3])  # BIXBY, MAROS
@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("dual", [0, 1])
def test_crash_bases_against_highs(basis, seed, dual):
    """initial_basis BIXBY and MAROS (initial_basis.cc:43-103, 208-356;
    revised_simplex.cc:1197-1275), SURVEY 8(a) a26: optimal objective
    unchanged. LPs with equality rows (fixed slacks) and all bound types,
    so both crash procedures replace slacks."""
    m = [12, 40, 90, 150][seed % 4]
    n = [30, 70, 250, 400][seed % 4]
    lp = lp_gen.random_sparse_lp(m, n, 0.3 if m < 30 else 0.06, 900 + seed,
                                 eq_frac=0.5, maximize=bool(seed % 2))
    # Columns scaled to infinity norm 1 (what BIXBY expects of a scaled LP).
    for j in range(lp.n):
        s0, s1 = lp.col_starts[j], lp.col_starts[j + 1]
        if s1 > s0:
            scale = np.abs(lp.vals[s0:s1]).max()
            lp.vals[s0:s1] /= scale
            lp.obj[j] /= scale
            lp.col_lb[j] *= scale
            lp.col_ub[j] *= scale
    st, ref = lp_gen.to_scipy(lp)
    o = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=dual, initial_basis=basis))
    o.load(lp)
    r = o.solve()
    if st != 0:
        assert r.problem_status != abi.OPTIMAL
        return
    assert r.problem_status == abi.OPTIMAL
    assert abs(r.objective - ref) <= 1e-6 * max(1.0, abs(ref))


@pytest.mark.parametrize("basis", [1, 3])
@pytest.mark.parametrize("builder", kat_lps.ALL, ids=lambda f: f.__name__)
def test_crash_bases_known_answers(builder, basis):
    lp, exp = builder()
    o = oracle_lib.OracleLp(abi.default_params(initial_basis=basis))
    o.load(lp)
    r = o.solve()
    if "status_in" in exp:
        assert abi.PROBLEM_STATUS[r.problem_status] in exp["status_in"]
        return
    assert r.problem_status == exp["status"]
    assert r.objective == pytest.approx(exp["objective"], rel=1e-9, abs=1e-9)
