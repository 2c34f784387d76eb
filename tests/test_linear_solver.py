"""MPSolver-shaped front end (mi_glop.linear_solver), config 1 plumbing.

The models are the reference's own MPSolver examples with their stated
answers: examples/tests/lp_test.cc:55-85 (34 at (6, 4)),
glop/samples/simple_glop_program.cc (4), linear_solver/python/
model_builder_test.py:49-135 (733.3333 - 5.5). The CPU part checks the
model extraction (GLOPInterface::ExtractModel + LinearProgram::CleanUp)
against the known-answer LPs and solves it with the oracle; the GPU part
solves through the engine and checks the answers, the status maps of
glop_utils.cc:18-125 and bit-equality with the oracle."""
import math

import numpy as np
import pytest

from mi_glop import abi, engine, linear_solver

import os
import sys

from mi_glop.lp import LinearProgram

import kat_lps
import oracle_lib

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "oracle"))
import oracle_scaling  # noqa: E402

INF = math.inf


def lp_test_model():
    solver = linear_solver.Solver("LinearProgrammingExample",
                                  linear_solver.GLOP_LINEAR_PROGRAMMING)
    x = solver.MakeNumVar(0.0, INF, "x")
    y = solver.MakeNumVar(0.0, INF, "y")
    obj = solver.MutableObjective()
    obj.SetCoefficient(x, 3)
    obj.SetCoefficient(y, 4)
    obj.SetMaximization()
    c0 = solver.MakeRowConstraint(-INF, 14.0, "c0")
    c0.SetCoefficient(x, 1)
    c0.SetCoefficient(y, 2)
    c1 = solver.MakeRowConstraint(0.0, INF, "c1")
    c1.SetCoefficient(x, 3)
    c1.SetCoefficient(y, -1)
    c2 = solver.MakeRowConstraint(-INF, 2.0, "c2")
    c2.SetCoefficient(x, 1)
    c2.SetCoefficient(y, -1)
    return solver, (x, y), (c0, c1, c2)


def simple_glop_model():
    solver = linear_solver.Solver.CreateSolver("GLOP")
    x = solver.NumVar(0, 1, "x")
    y = solver.NumVar(0, 2, "y")
    ct = solver.Constraint(-solver.infinity(), 2, "ct")
    ct.SetCoefficient(x, 1)
    ct.SetCoefficient(y, 1)
    solver.Objective().SetCoefficient(x, 3)
    solver.Objective().SetCoefficient(y, 1)
    solver.Objective().SetMaximization()
    return solver, (x, y), (ct,)


def model_builder_model():
    solver = linear_solver.Solver.CreateSolver("glop")
    xs = [solver.NumVar(1 if i == 0 else 0, INF, f"x{i + 1}") for i in range(3)]
    rows = [([1, 1, 1], 100), ([10, 4, 5], 600), ([2, 2, 6], 300)]
    cons = []
    for coefs, ub in rows:
        c = solver.Constraint(-INF, ub)
        for v, a in zip(xs, coefs):
            c.SetCoefficient(v, a)
        cons.append(c)
    solver.Maximize({xs[0]: 10, xs[1]: 6, xs[2]: 4})
    solver.Objective().SetOffset(-5.5)
    return solver, tuple(xs), tuple(cons)


def _same_lp(a, b):
    for f in ("col_starts", "row_idx", "vals", "col_lb", "col_ub", "row_lb", "row_ub", "obj"):
        np.testing.assert_array_equal(np.asarray(getattr(a, f), float),
                                      np.asarray(getattr(b, f), float), err_msg=f)
    assert (a.m, a.n, a.maximize, a.obj_offset) == (b.m, b.n, b.maximize, b.obj_offset)


@pytest.mark.parametrize("model,kat", [(lp_test_model, kat_lps.lp_test_cc),
                                       (simple_glop_model, kat_lps.mutable_objective_lp),
                                       (model_builder_model, kat_lps.model_builder_lp)])
def test_extraction_matches_known_answer_lp(model, kat):
    solver, _, _ = model()
    lp = solver.to_linear_program()
    ref, expect = kat()
    _same_lp(lp, ref)
    o = oracle_lib.OracleLp(abi.default_params())
    o.load(lp)
    r = o.solve()
    assert r.problem_status == abi.OPTIMAL
    assert abs(r.objective - expect["objective"]) <= 1e-6 * max(1.0, abs(expect["objective"]))


def test_cleanup_merges_and_drops():
    solver = linear_solver.Solver.CreateSolver("GLOP")
    x = solver.NumVar(0, 1)
    y = solver.NumVar(0, 1)
    c = solver.Constraint(0, 1)
    c.SetCoefficient(y, 2.0)
    c.SetCoefficient(x, 0.0)   # explicit zero: dropped
    c2 = solver.Constraint(0, 1)
    c2.SetCoefficient(x, 1.0)
    c2.SetCoefficient(x, 3.0)  # last write wins, as MPConstraint::SetCoefficient
    lp = solver.to_linear_program()
    assert list(lp.col_starts) == [0, 1, 2]
    assert list(lp.row_idx) == [1, 0] and list(lp.vals) == [3.0, 2.0]
    assert solver.CreateSolver("SCIP") is None
    with pytest.raises(ValueError):
        solver.IntVar(0, 1, "b")


@pytest.mark.gpu
@pytest.mark.parametrize("presolve", [True, False])
@pytest.mark.parametrize("model,expect", [
    (lp_test_model, dict(objective=34.0, primal=[6, 4])),
    (simple_glop_model, dict(objective=4.0, primal=[1, 1])),
    (model_builder_model, dict(objective=733.3333333333334 - 5.5,
                               primal=[100.0 / 3, 200.0 / 3, 0.0]))])
def test_solve_through_engine(model, expect, presolve):
    _check_solve(model, expect, presolve)


def _check_solve(model, expect, presolve):
    solver, xs, cons = model()
    if not presolve:
        assert solver.SetSolverSpecificParametersAsString("use_preprocessing: false")
    assert solver.Solve() == linear_solver.Solver.OPTIMAL
    assert abs(solver.Objective().Value() - expect["objective"]) <= 1e-6 * abs(expect["objective"])
    np.testing.assert_allclose([v.solution_value() for v in xs], expect["primal"], atol=1e-7)
    lp = solver.to_linear_program()
    p = abi.default_params()
    if presolve:
        # Glop's default LPSolver flow (presolve on): the same flow with the
        # oracle simplex behind it (mi_lp_solver_solve_with) is the check.
        def simplex(inner):
            o = oracle_lib.OracleLp(p)
            o.load(inner)
            r = o.solve()
            v, c = o.statuses()
            return r, o.primal(), o.duals(), v, c

        rw, sol = engine.solve_lp_with(lp, simplex)
        want = {"x": sol["x"], "rc": sol["rc"], "y": sol["y"], "objective": rw.objective}
        ov, oc = sol["vstat"], sol["cstat"]
    else:
        # Presolve off: the simplex restatement on the scaling restatement's
        # LP, then the restated recovery (lp_solver.cc:150-367).
        arr, fac = oracle_scaling.scale_lp(lp)
        slp = LinearProgram(lp.m, lp.n, lp.col_starts, lp.row_idx, arr["vals"], arr["col_lb"],
                            arr["col_ub"], arr["row_lb"], arr["row_ub"], arr["obj"],
                            arr["obj_offset"], arr["obj_scale"], lp.maximize)
        o = oracle_lib.OracleLp(p)
        o.load(slp)
        ro = o.solve()
        ov, oc = o.statuses()
        want = oracle_scaling.recover_and_verify(lp, fac, o.primal(), o.duals(), ov,
                                                 ro.problem_status == abi.OPTIMAL)
    np.testing.assert_array_equal([v.solution_value() for v in xs], want["x"])
    np.testing.assert_array_equal([v.reduced_cost() for v in xs], want["rc"])
    np.testing.assert_array_equal([c.dual_value() for c in cons], want["y"])
    assert solver.Objective().Value() == want["objective"]
    bmap = linear_solver.Solver._BASIS
    assert [v.basis_status() for v in xs] == [bmap[int(s)] for s in ov]
    assert [c.basis_status() for c in cons] == [bmap[int(s)] for s in oc]
    assert solver.iterations() >= 0


@pytest.mark.gpu
def test_infeasible_and_unbounded_status_maps():
    s = linear_solver.Solver.CreateSolver("GLOP")
    x = s.NumVar(0, 1, "x")
    c = s.Constraint(2, INF)
    c.SetCoefficient(x, 1)
    assert s.Solve() == linear_solver.Solver.INFEASIBLE
    for presolve in (False, True):
        s2 = linear_solver.Solver.CreateSolver("GLOP")
        if not presolve:
            assert s2.SetSolverSpecificParametersAsString("use_preprocessing: false")
        y = s2.NumVar(0, INF, "y")
        s2.Objective().SetCoefficient(y, 1)
        s2.Objective().SetMaximization()
        c2 = s2.Constraint(0, INF)
        c2.SetCoefficient(y, 1)
        # The simplex proves the ray (DUAL_INFEASIBLE -> UNBOUNDED); Glop's
        # default presolve stops first at the empty column with an infinite
        # target (INFEASIBLE_OR_UNBOUNDED), which MPSolver reports as
        # INFEASIBLE (glop_utils.cc:25-38).
        want = linear_solver.Solver.INFEASIBLE if presolve else linear_solver.Solver.UNBOUNDED
        assert s2.Solve() == want


def test_solver_specific_parameters_text():
    """GLOPInterface::SetSolverSpecificParametersAsString (glop_interface.cc:
    397-411): GlopParameters text, enum values by name, LPSolver and presolve
    fields included."""
    s = linear_solver.Solver("p")
    assert s.SetSolverSpecificParametersAsString(
        "use_preprocessing: true solve_dual_problem: ALWAYS_DO "
        "feasibility_rule: DANTZIG initial_basis: MAROS cost_scaling: MEAN_COST_SCALING "
        "preprocessor_zero_tolerance: 1e-10 use_dual_simplex: true")
    assert s._solver_params.use_preprocessing == 1
    assert s._solver_params.solve_dual_problem == 0
    assert s._solver_params.cost_scaling == 2
    assert s._solver_params.preprocessor_zero_tolerance == 1e-10
    assert s._params.feasibility_rule == 0 and s._params.initial_basis == 3
    assert s._params.use_dual_simplex == 1
    assert not s.SetSolverSpecificParametersAsString("no_such_field: 3")
    assert not s.SetSolverSpecificParametersAsString("solve_dual_problem: SOMETIMES")


def test_mpsolver_path_with_oracle_simplex(monkeypatch):
    """The GPU tests above, with the engine handle replaced by the same
    LPSolver flow over the CPU oracle (test_solve_cli._OracleHandle): the
    MPSolver mirror's extraction, parameters, status map and solution
    accessors on CPU."""
    import test_solve_cli
    monkeypatch.setattr(linear_solver.engine, "LpHandle", test_solve_cli._OracleHandle)
    for presolve in (True, False):
        _check_solve(lp_test_model, dict(objective=34.0, primal=[6, 4]), presolve)
        _check_solve(simple_glop_model, dict(objective=4.0, primal=[1, 1]), presolve)
        _check_solve(model_builder_model, dict(objective=733.3333333333334 - 5.5,
                                               primal=[100.0 / 3, 200.0 / 3, 0.0]), presolve)
    test_infeasible_and_unbounded_status_maps()
