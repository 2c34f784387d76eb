"""CP-SAT boundary entry points (include/mi_lp.h, revised_simplex.h:161-237).

CPU part: the oracle's restatements are checked against what the reference
promises of them (GetUnitRowLeftInverse is e_r^T B^-1, ComputeDictionary is
B^-1 A, SetIntegralityScale + Polish keeps an optimal basis, the objective
limit stops the dual simplex, SetStartingVariableValuesForNextSolve is
honoured). GPU part: the engine answers every call bit for bit like the
oracle (revised_simplex.cc:126-137, 2588-2734, 3785-3806;
sat/linear_programming_constraint.cc:319, 430, 1247, 1264)."""
import numpy as np
import pytest

from mi_glop import abi

import kat_lps
import lp_gen
import oracle_lib


def _dense_a_with_slacks(lp):
    a = np.zeros((lp.m, lp.n + lp.m))
    for j in range(lp.n):
        for k in range(lp.col_starts[j], lp.col_starts[j + 1]):
            a[lp.row_idx[k], j] = lp.vals[k]
    a[:, lp.n:] = np.eye(lp.m)  # slack columns (sparse.cc:462-487)
    return a


def _solved_oracle(lp, **kw):
    o = oracle_lib.OracleLp(abi.default_params(**kw))
    o.load(lp)
    r = o.solve()
    return o, r


def test_unit_row_left_inverse_is_a_row_of_b_inverse():
    lp = lp_gen.random_sparse_lp(30, 90, 0.15, 7)
    o, r = _solved_oracle(lp)
    assert r.problem_status == abi.OPTIMAL
    a = _dense_a_with_slacks(lp)
    b = a[:, o.basis()]
    for row in range(lp.m):
        rho, nz = o.unit_row_left_inverse(row)
        e = np.zeros(lp.m)
        e[row] = 1.0
        np.testing.assert_allclose(rho @ b, e, atol=1e-9)
        if len(nz):
            assert set(np.nonzero(rho)[0]) <= set(nz)


def test_dictionary_is_b_inverse_a():
    lp = lp_gen.random_sparse_lp(20, 50, 0.2, 8)
    o, r = _solved_oracle(lp)
    a = _dense_a_with_slacks(lp)
    b = a[:, o.basis()]
    starts, cols, vals = o.dictionary()
    d = np.zeros_like(a)
    for row in range(lp.m):
        for k in range(starts[row], starts[row + 1]):
            d[row, cols[k]] = vals[k]
    np.testing.assert_allclose(d, np.linalg.solve(b, a), atol=1e-9)
    scales = np.linspace(0.5, 2.0, lp.n + lp.m)
    s2, c2, v2 = o.dictionary(scales)
    np.testing.assert_array_equal(s2, starts)
    basis = o.basis()
    for row in range(lp.m):
        for k in range(starts[row], starts[row + 1]):
            assert v2[k] == vals[k] * (scales[c2[k]] / scales[basis[row]])


def test_polish_keeps_optimality():
    lp, expect = kat_lps.ALL[0]()
    o, r = _solved_oracle(lp)
    for col in range(lp.n):
        o.set_integrality_scale(col, 1.0)
    r2 = o.solve()
    assert r2.problem_status == abi.OPTIMAL
    assert abs(r2.objective - r.objective) <= 1e-9 * max(1.0, abs(r.objective))


def test_objective_limit_reached_in_dual_simplex():
    lp = lp_gen.random_sparse_lp(40, 120, 0.1, 9)
    o, r = _solved_oracle(lp, use_dual_simplex=1)
    assert not o.objective_limit_reached()
    # A limit the dual objective crosses before optimality (minimization:
    # objective_upper_limit; revised_simplex.cc:1107-1125).
    o2, r2 = _solved_oracle(lp, use_dual_simplex=1, objective_upper_limit=r.objective - 1.0)
    if lp.maximize:
        o2, r2 = _solved_oracle(lp, use_dual_simplex=1,
                                objective_lower_limit=r.objective + 1.0)
    assert o2.objective_limit_reached()
    assert r2.problem_status == abi.DUAL_FEASIBLE


def test_matrix_changed_and_starting_values_accepted():
    lp = lp_gen.random_sparse_lp(20, 60, 0.2, 10)
    o, r = _solved_oracle(lp)
    o.notify_matrix_unchanged()
    o.notify_matrix_changed()
    o.set_starting_variable_values(np.zeros(lp.n + lp.m))
    r2 = o.solve()
    assert r2.problem_status == abi.OPTIMAL
    assert abs(r2.objective - r.objective) <= 1e-9 * max(1.0, abs(r.objective))


# --- engine vs oracle (GPU) ---------------------------------------------------

def _both(lp, **kw):
    from mi_glop import engine
    import parity_util
    p = abi.default_params(**kw)
    return parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q))


@pytest.mark.gpu
@pytest.mark.parametrize("dual", [0, 1])
def test_unit_row_and_dictionary_parity(dual):
    import parity_util
    lp = lp_gen.random_sparse_lp(60, 200, 0.08, 11)
    o, ro, g, rg = _both(lp, use_dual_simplex=dual)
    parity_util.compare(o, ro, g, rg, lp)
    for row in range(0, lp.m, 7):
        ov, onz = o.unit_row_left_inverse(row)
        gv, gnz = g.unit_row_left_inverse(row)
        np.testing.assert_array_equal(gv, ov)
        np.testing.assert_array_equal(gnz, onz)
    for a, b in zip(g.dictionary(), o.dictionary()):
        np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [12, 13, 14])
def test_polish_parity(seed):
    """Integrality scales set: the OPTIMAL solve runs Polish (RNG-driven
    degenerate pivots); the engine must make the same pivots."""
    import parity_util
    from mi_glop import engine
    lp = lp_gen.random_sparse_lp(50, 160, 0.1, seed)
    p = abi.default_params()
    o = oracle_lib.OracleLp(p)
    g = engine.LpHandle(p)
    for h in (o, g):
        h.load(lp)
        for col in range(lp.n):
            h.set_integrality_scale(col, 1.0 + (col % 3))
    ro = o.solve()
    rg = g.solve()
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.gpu
def test_objective_limit_and_starting_values_parity():
    import parity_util
    from mi_glop import engine
    lp = lp_gen.random_sparse_lp(40, 120, 0.1, 15)
    _, r = _solved_oracle(lp, use_dual_simplex=1)
    kw = dict(use_dual_simplex=1)
    if lp.maximize:
        kw["objective_lower_limit"] = r.objective + 1.0
    else:
        kw["objective_upper_limit"] = r.objective - 1.0
    o, ro, g, rg = _both(lp, **kw)
    parity_util.compare(o, ro, g, rg, lp)
    assert g.objective_limit_reached() == o.objective_limit_reached() is True
    start = np.linspace(0.0, 1.0, lp.n + lp.m)
    p = abi.default_params()
    o2 = oracle_lib.OracleLp(p)
    g2 = engine.LpHandle(p)
    for h in (o2, g2):
        h.load(lp)
        h.set_starting_variable_values(start)
        h.notify_matrix_changed()
    ro2 = o2.solve()
    rg2 = g2.solve()
    parity_util.compare(o2, ro2, g2, rg2, lp)


def test_clear_integrality_scales_drops_polish():
    """ClearIntegralityScales (revised_simplex.h:236): after the clear, a solve
    is the plain solve (no Polish), as CP-SAT relies on when it resets the
    scales (sat/linear_programming_constraint.cc:424-433)."""
    lp = lp_gen.random_sparse_lp(50, 160, 0.1, 12)
    plain, rp = _solved_oracle(lp)
    o = oracle_lib.OracleLp(abi.default_params())
    o.load(lp)
    for col in range(lp.n):
        o.set_integrality_scale(col, 1.0 + (col % 3))
    o.clear_integrality_scales()
    r = o.solve()
    assert r.iterations == rp.iterations
    np.testing.assert_array_equal(o.basis(), plain.basis())
    np.testing.assert_array_equal(o.primal(), plain.primal())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [12, 13])
def test_clear_integrality_scales_parity(seed):
    """mi_lp_clear_integrality_scales: scales set, cleared, then a subset set
    again (the CP-SAT sequence of linear_programming_constraint.cc:424-433);
    the engine's solve equals the oracle's bit for bit."""
    import parity_util
    from mi_glop import engine
    lp = lp_gen.random_sparse_lp(50, 160, 0.1, seed)
    p = abi.default_params()
    o = oracle_lib.OracleLp(p)
    g = engine.LpHandle(p)
    for h in (o, g):
        h.load(lp)
        for col in range(lp.n):
            h.set_integrality_scale(col, 2.0)
        h.clear_integrality_scales()
        for col in range(0, lp.n, 2):
            h.set_integrality_scale(col, 1.0 + (col % 3))
    ro = o.solve()
    rg = g.solve()
    parity_util.compare(o, ro, g, rg, lp)
    for h in (o, g):
        h.clear_integrality_scales()
    ro2 = o.solve()
    rg2 = g.solve()
    parity_util.compare(o, ro2, g, rg2, lp)


@pytest.mark.gpu
def test_iteration_times_and_run_counters():
    """mi_lp_record_iteration_times / mi_lp_get_run_counters (bench.py's window
    statistics): one timestamp per iteration, non-decreasing, readable while a
    begun solve is parked; the factorization count grows across a window with
    refactorizations and matches the oracle-independent bookkeeping."""
    from mi_glop import engine
    lp = lp_gen.random_sparse_lp(120, 400, 0.05, 16)
    g = engine.LpHandle(abi.default_params(use_dual_simplex=1))
    g.load(lp)
    g.record_iteration_times(True)
    g.begin(20)
    c0 = g.run_counters()
    assert c0["iterations"] == 20
    ts = g.iteration_times()
    assert len(ts) == 20 and np.all(np.diff(ts) >= 0.0)
    fin, it = g.run_until(150)
    c1 = g.run_counters()
    assert c1["iterations"] == it
    # The slack basis needs no factorization; 64 updates later one is made.
    assert c1["factorizations"] >= c0["factorizations"]
    if it > 70:
        assert c1["factorizations"] >= 1
    assert c1["factorization_seconds"] >= c0["factorization_seconds"]
    g.stop()
    r = g.finish()
    assert len(g.iteration_times()) == r.iterations


@pytest.mark.gpu
def test_batch_solve_gpus_parity():
    """mi_lp_batch_solve_gpus (SURVEY 8(b)'s batch entry with num_gpus): each
    device's handles on a thread pool of their own; every LP equals the
    oracle's solve bit for bit. A device outside [0, num_gpus) is refused."""
    import parity_util
    from mi_glop import engine
    lps = [lp_gen.random_sparse_lp(40 + 7 * k, 120 + 20 * k, 0.08, 30 + k) for k in range(6)]
    p = abi.default_params(use_dual_simplex=1)
    hs = []
    for lp in lps:
        h = engine.LpHandle(p)
        h.load(lp)
        hs.append(h)
    res = engine.batch_solve_gpus(hs, num_gpus=engine.device_count(), threads_per_gpu=2)
    for lp, h, r in zip(lps, hs, res):
        o = oracle_lib.OracleLp(p)
        o.load(lp)
        parity_util.compare(o, o.solve(), h, r, lp)
    with pytest.raises(RuntimeError):
        engine.batch_solve_gpus(hs, num_gpus=0)
