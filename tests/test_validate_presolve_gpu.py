"""GPU runs of the round-5 LPSolver additions (collected after the rest of
the GPU suite): the presolve path of mi_lp_solver_solve (presolve, scaling,
the engine on the reduced LP, postsolve) against the same flow with the
oracle as the simplex, bit for bit, and the `solve` command line. Their CPU
counterparts are tests/test_presolve.py and tests/test_solve_cli.py."""
import os

import numpy as np
import pytest

from mi_glop import abi, engine, solve

import kat_lps
import lp_gen
from test_presolve import oracle_simplex

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden", "mps")


def _gpu_cases():
    cases = [(f"presolve_{s}_{'tall' if t else 'wide'}",
              lambda s=s, t=t: lp_gen.presolve_lp(40 + 3 * s, 90 + 5 * s, 500 + s,
                                                  maximize=bool(s % 2), tall=t))
             for s in range(4) for t in (False, True)]
    cases += [(f.__name__, lambda f=f: f()[0]) for f in kat_lps.ALL]
    return cases


@pytest.mark.gpu
@pytest.mark.parametrize("case", _gpu_cases(), ids=lambda c: c[0])
def test_presolve_engine_parity(case):
    """mi_lp_solver_solve with use_preprocessing = 1: presolve, scaling, the
    engine on the reduced LP, postsolve. Bit-equal to the same flow with the
    oracle as the simplex (mi_lp_solver_solve_with)."""
    lp = case[1]()
    p = abi.default_params(use_dual_simplex=1)
    sp = abi.default_solver_params(use_preprocessing=1)
    rg, sg = engine.LpHandle(p).solve_lp(lp, sp)
    ro, so = engine.solve_lp_with(lp, oracle_simplex(p), sp)
    assert (rg.error_code, rg.problem_status, rg.iterations) == \
        (ro.error_code, ro.problem_status, ro.iterations)
    assert rg.objective == ro.objective
    for k in ("x", "y", "rc", "act", "vstat", "cstat"):
        np.testing.assert_array_equal(sg[k], so[k], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("params", ["", "use_preprocessing: true"])
def test_solve_cli_on_gpu(tmp_path, capsys, params):
    sol = tmp_path / "out.sol"
    csv = tmp_path / "out.csv"
    rc = solve.main(["--input", os.path.join(GOLDEN, "test2.mps"), "--params", params,
                     "--sol_file", str(sol), "--output_csv", str(csv)])
    out = capsys.readouterr().out
    assert rc == 0
    assert "Status      : MPSOLVER_OPTIMAL" in out
    value = float(out.split("Objective   :")[1].split()[0])
    assert abs(value - 3.236842105263158) <= 1e-9
    assert sol.read_text().startswith("=obj= ")
    assert len(csv.read_text().splitlines()) == 8
