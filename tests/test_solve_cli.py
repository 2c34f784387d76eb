"""The `solve` command line (or-tools_amd/mi_glop/solve.py), restating
linear_solver/solve.cc:261-398 for --solver=glop."""
import os

import numpy as np
import pytest

from mi_glop import mps, solve

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden", "mps")


def test_flags_follow_the_reference():
    a = solve.parse_args(["--input", "x.mps", "--params", "use_preprocessing: true"])
    assert a.solver == "glop" and a.time_limit == float("inf")
    for bad in (["--input", "x", "--solver", "scip"],
                ["--input", "x", "--params", "a: 1", "--params_file", "f"],
                ["--input", "x", "--time_limit", "0"], []):
        with pytest.raises(SystemExit):
            solve.parse_args(bad)


def test_model_extraction_is_the_mps_lp():
    lp = mps.read_mps(os.path.join(GOLDEN, "test2.mps"), with_names=True)
    s, xs = solve.build_solver(lp, device=0)
    got = s.to_linear_program()
    for k in ("col_starts", "row_idx", "vals", "col_lb", "col_ub", "row_lb", "row_ub", "obj"):
        np.testing.assert_array_equal(getattr(got, k), getattr(lp, k), err_msg=k)
    assert got.obj_offset == lp.obj_offset and got.maximize == lp.maximize
    assert [x.name() for x in xs] == lp.col_names


class _OracleHandle:
    """Test double for engine.LpHandle: the same LPSolver flow
    (mi_lp_solver_solve_with) with the CPU oracle as the simplex."""

    def __init__(self, params, device=0):
        self.params = params

    def set_params(self, p):
        self.params = p

    def solve_lp(self, model, sp):
        import oracle_lib
        from mi_glop import engine

        def simplex(inner):
            o = oracle_lib.OracleLp(self.params)
            o.load(inner)
            r = o.solve()
            v, c = o.statuses()
            return r, o.primal(), o.duals(), v, c
        return engine.solve_lp_with(model, simplex, sp)


@pytest.mark.parametrize("params", ["", "use_preprocessing: true",
                                    "use_preprocessing: true solve_dual_problem: ALWAYS_DO"])
def test_solve_cli_with_oracle_simplex(tmp_path, capsys, monkeypatch, params):
    from mi_glop import linear_solver
    monkeypatch.setattr(linear_solver.engine, "LpHandle", _OracleHandle)
    sol = tmp_path / "out.sol"
    csv = tmp_path / "out.csv"
    rc = solve.main(["--input", os.path.join(GOLDEN, "test2.mps"), "--params", params,
                     "--sol_file", str(sol), "--output_csv", str(csv)])
    out = capsys.readouterr().out
    assert rc == 0, out
    assert "Status      : MPSOLVER_OPTIMAL" in out and "Dimension   : 5 x 8" in out
    value = float(out.split("Objective   :")[1].split()[0])
    assert abs(value - 3.236842105263158) <= 1e-9
    lines = sol.read_text().splitlines()
    assert lines[0].startswith("=obj= ") and len(lines) == 9
    assert len(csv.read_text().splitlines()) == 8
