"""The device primal simplex segment on the MI355X (or-tools_amd/csrc/sdual/
sprimal_core.h, Glop's PrimalMinimize loop, revised_simplex.cc:2751-3045):
phase-I and phase-II primal iterations run whole on one workgroup, the host
engine keeps the factorizations and the loop's other branches. Enabled with
MILP_SPRIMAL=on. Every result must equal the oracle's bit for bit, and the
segments must have run (on the device when MILP_SDUAL=device)."""
import numpy as np
import pytest

from mi_glop import abi, engine
import kat_lps
import lp_gen
import oracle_lib
import parity_util

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["device", "host"])
def sprimal_mode(request, monkeypatch):
    monkeypatch.setenv("MILP_SDUAL", request.param)
    monkeypatch.setenv("MILP_SPRIMAL", "on")
    return request.param


def _check_ran(g, mode):
    c = g.run_counters()
    assert c["sdual_segments"] > 0 and c["sdual_iterations"] > 0, c
    if mode == "device":
        assert g.kernel_stats()["sdual"]["launches"] == c["sdual_segments"]


@pytest.mark.parametrize("seed", range(4))
def test_sprimal_single_lp_parity(seed, sprimal_mode):
    m, n = 50 + 40 * seed, 160 + 120 * seed
    lp = lp_gen.random_sparse_lp(m, n, 0.05 if seed % 2 else 0.03, 910 + seed,
                                 maximize=bool(seed % 2))
    p = abi.default_params()
    o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q, 0))
    parity_util.compare(o, ro, g, rg, lp)
    _check_ran(g, sprimal_mode)


def test_sprimal_pfi_parity(sprimal_mode):
    """The primal loop with product-form (eta) updates,
    use_middle_product_form_update = false (basis_representation.cc:25-176)."""
    lp = lp_gen.random_sparse_lp(150, 500, 0.04, 733)
    p = abi.default_params(use_middle_product_form_update=0)
    o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q, 0))
    parity_util.compare(o, ro, g, rg, lp)
    _check_ran(g, sprimal_mode)


def test_sprimal_kats(sprimal_mode):
    """Known-answer LPs (optimal, infeasible, unbounded) through the primal
    loop with segments on."""
    for builder in kat_lps.ALL:
        lp, _ = builder()
        p = abi.default_params()
        o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q, 0))
        parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("cap", [1, 7, 60])
def test_sprimal_iteration_cap(cap, sprimal_mode):
    lp = lp_gen.random_sparse_lp(120, 300, 0.04, 77)
    p = abi.default_params(max_number_of_iterations=cap)
    o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q, 0))
    parity_util.compare(o, ro, g, rg, lp)


def test_sprimal_netlib_batch(monkeypatch):
    """The config-3 stand-in suite (LPs up to 300 rows) through the batch API
    (4 threads of fibers, the device pool) with primal segments on; each LP
    equals the oracle solving it alone."""
    import netlib_suite
    monkeypatch.setenv("MILP_SDUAL", "device")
    monkeypatch.setenv("MILP_SPRIMAL", "on")
    suite = netlib_suite.suite(max_rows=300)
    p = abi.default_params()
    handles = []
    for lp in suite:
        h = engine.LpHandle(p)
        h.load(lp)
        handles.append(h)
    got = engine.batch_solve(handles, num_threads=4)
    for i, (lp, r) in enumerate(zip(suite, got)):
        o = oracle_lib.OracleLp(p)
        o.load(lp)
        ro = o.solve()
        assert (r.error_code, r.problem_status, r.iterations) == \
            (ro.error_code, ro.problem_status, ro.iterations), i
        assert r.objective == ro.objective or (
            np.isnan(r.objective) and np.isnan(ro.objective)), (i, r.objective, ro.objective)
        np.testing.assert_array_equal(handles[i].primal(), o.primal())
    assert sum(h.run_counters()["sdual_segments"] for h in handles) > 0
    for h in handles:
        h.close()
