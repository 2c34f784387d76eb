"""The batch call's choice of loop (simplex.cc SetBatchMode): with MILP_SDUAL
unset, device segments run only when at least MILP_SDUAL_MIN_LPS (512) LPs
are in flight, the batched-launch path below that; both give the oracle's
answer for every child."""
import pytest

from mi_glop import abi, engine

import oracle_lib
import test_sdual_gpu as T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("min_lps,segments", [(None, False), ("1", True)])
def test_children_mode_by_lps_in_flight(min_lps, segments, monkeypatch):
    monkeypatch.delenv("MILP_SDUAL", raising=False)
    if min_lps is None:
        monkeypatch.delenv("MILP_SDUAL_MIN_LPS", raising=False)
    else:
        monkeypatch.setenv("MILP_SDUAL_MIN_LPS", min_lps)
    lp, state, lbs, ubs = T._children((6, 6), 24)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    workers = [engine.LpHandle(p) for _ in range(8)]
    for w in workers:
        w.load(lp)
    res = engine.batch_solve_bounds(workers, lbs, ubs, state)
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    for i, r in enumerate(res):
        o.set_variable_bounds(lbs[i], ubs[i])
        o.load_basis_state(state)
        ro = o.solve()
        assert (r.error_code, r.problem_status, r.iterations, r.objective) == \
            (ro.error_code, ro.problem_status, ro.iterations, ro.objective), i
    segs = sum(w.run_counters()["sdual_segments"] for w in workers)
    assert (segs > 0) == segments, segs
