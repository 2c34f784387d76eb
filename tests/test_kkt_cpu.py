"""The KKT checker (tests/kkt.py) pinned on CPU: every OPTIMAL answer of the
oracle passes it, and a perturbed answer does not (the checker can fail)."""
import numpy as np
import pytest

from mi_glop import abi

import kkt
import lp_gen
import oracle_lib


def _solve(lp, dual):
    o = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=dual))
    o.load(lp)
    r = o.solve()
    v, c = o.statuses()
    return r, o.primal(), o.duals(), o.reduced_costs(), v, c


@pytest.mark.parametrize("dual", [0, 1])
@pytest.mark.parametrize("make", [
    lambda: lp_gen.random_sparse_lp(60, 200, 0.06, 1),
    lambda: lp_gen.random_sparse_lp(80, 260, 0.05, 2, maximize=True),
    lambda: lp_gen.dense_box_lp(48, 192, 3),
    lambda: lp_gen.sparse_c5_lp(300, 3000, 10, 4),
    lambda: lp_gen.dual_phase1_lp(90, 330, 5),
], ids=["sparse", "sparse_max", "dense_box", "c5_shape", "dual_phase1"])
def test_oracle_answers_pass_kkt(make, dual):
    lp = make()
    r, x, y, rc, v, c = _solve(lp, dual)
    assert r.problem_status == abi.OPTIMAL
    k = kkt.assert_optimal(lp, x, y, rc, v, c)
    assert abs(k["primal_objective"] + lp.obj_offset - r.objective) <= \
        1e-9 * max(1.0, abs(r.objective))


def test_checker_rejects_a_wrong_answer():
    lp = lp_gen.random_sparse_lp(60, 200, 0.06, 1)
    r, x, y, rc, v, c = _solve(lp, 1)
    bad_y = y.copy()
    i = int(np.argmax(np.abs(y)))
    bad_y[i] = -bad_y[i] if bad_y[i] != 0 else 1.0
    with pytest.raises(AssertionError):
        kkt.assert_optimal(lp, x, bad_y, rc, v, c)
