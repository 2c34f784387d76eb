"""Dense U solves of FTRAN on the device (engine/device_solve.hip,
kernels/tri_solve.hip) vs the CPU oracle, which runs Glop's host loop
TriangularMatrix::TransposeLowerSolve (sparse.cc:899-955).

MILP_DEVICE_SOLVE=force sends every dense U solve (the solver's thread and
the tau worker) to the device at test size; the engine must still reproduce
the oracle bit for bit (basis, statuses, values, iterations) and its
deterministic time must not move. Three device variants: the default
readiness-driven single launch (tri_syncfree_kernel) with zero-copy staging,
the level-scheduled plan (MILP_TRI_SYNCFREE=0), and the level plan with
copy-engine staging (MILP_TRI_MAPPED=0)."""
import pytest

from mi_glop import abi, engine

import kat_lps
import lp_gen
import parity_util

pytestmark = pytest.mark.gpu


def _handle(params):
    return engine.LpHandle(params)


def _cases():
    cases = []
    for seed in (71, 72, 73):
        cases.append((f"c5_{seed}", lambda s=seed: lp_gen.sparse_c5_lp(400 + 40 * (s % 3),
                                                                      4000, 6, s), 1))
    # Its U fills in (a hundred entries per row, depth ~250 by iteration
    # 4000): long outputs go through the batched-entries path.
    cases.append(("c5_wide", lambda: lp_gen.sparse_c5_lp(1500, 12000, 8, 74), 1))
    cases.append(("sparse_primal", lambda: lp_gen.random_sparse_lp(200, 900, 0.04, 75), 0))
    cases.append(("dense_primal", lambda: lp_gen.dense_box_lp(97, 400, 76), 0))
    cases.append(("dense_dual", lambda: lp_gen.dense_box_lp(120, 600, 77), 1))
    # A deep chain of long outputs (a dense bump of a few hundred columns):
    # each output folds its groups as its inputs arrive.
    cases.append(("dense_deep", lambda: lp_gen.dense_box_lp(320, 1280, 78), 1))
    return cases


VARIANTS = {
    "syncfree": {},
    "levels": {"MILP_TRI_SYNCFREE": "0"},
    "levels_copies": {"MILP_TRI_SYNCFREE": "0", "MILP_TRI_MAPPED": "0"},
    "syncfree_copies": {"MILP_TRI_MAPPED": "0"},
    "persistent_xcd": {"MILP_TRI_PERSIST": "32", "MILP_TRI_XCD": "1", "MILP_TRI_POLL_MAX": "8"},
    "persistent_chip": {"MILP_TRI_PERSIST": "64", "MILP_TRI_POLL_MAX": "4"},
    # Single-workgroup narrow segments (off by default since round 5), and
    # narrow segments of any width (long runs cut at the LDS capacity).
    "chain": {"MILP_TRI_CHAIN": "1"},
    "wide_chain": {"MILP_TRI_CHAIN": "1", "MILP_TRI_CHAIN_WIDTH": "100000",
                   "MILP_TRI_CHAIN_MIN_LEVELS": "1"},
    # Levels padded to wave boundaries (off by default since round 5).
    "padded": {"MILP_TRI_PAD": "1"},
    # The two U solves as separate launches (the two-vector launch is the
    # default since round 5), and the device BTRAN loops (off by default).
    "no_pair_btran": {"MILP_TRI_PAIR": "0", "MILP_TRI_BTRAN": "1"},
}


# The default single-launch kernel on every case; the level-plan variants on
# two (their kernels are shared, only the schedule walk differs).
_PARAMS = [(c, "syncfree") for c in _cases()] + [
    (c, v) for c in _cases() if c[0] in ("c5_71", "dense_dual")
    for v in ("levels", "levels_copies", "syncfree_copies", "persistent_xcd",
              "persistent_chip", "chain", "wide_chain", "padded", "no_pair_btran")]


@pytest.mark.parametrize("case,variant", _PARAMS, ids=lambda x: x if isinstance(x, str) else x[0])
def test_device_u_solve_parity(case, variant, monkeypatch):
    name, build, dual = case
    lp = build()
    # Capped: forced onto the device at test size every solve pays a
    # dependency hop per level; the window covers many refactorizations.
    p = abi.default_params(use_dual_simplex=dual, max_number_of_iterations=1500)
    monkeypatch.setenv("MILP_DEVICE_SOLVE", "off")
    _, _, _, r_host = parity_util.solve_both(lp, p, _handle)
    for k, v in VARIANTS[variant].items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("MILP_DEVICE_SOLVE", "force")
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    assert rg.deterministic_time == r_host.deterministic_time
    stats = g.kernel_stats()
    st = stats["tri_solve"]
    if name.startswith("c5") or name.startswith("dense"):
        assert st["launches"] > 0, f"{name}: no dense U solve reached the device"
    if name.startswith("dense"):
        # Dense bases make every FTRAN's L solve dense too: the device L solve
        # (LowerSolveStartingAt restated as a gather, MILP_TRI_LOWER) ran.
        assert stats["tri_solve_l"]["launches"] > 0, f"{name}: no dense L solve on the device"


@pytest.mark.parametrize("device_dual", ["off", "force"])
@pytest.mark.parametrize("async_solves", ["off", "force"])
def test_device_u_solve_with_async_tau_and_device_dual(device_dual, async_solves, monkeypatch):
    """The tau FTRAN's dense U solves run on the device from the
    factorization's worker (own stream, own graph) while the solver's thread
    sends its own; with the dual device mode on or off, the results are the
    oracle's."""
    monkeypatch.setenv("MILP_DEVICE_SOLVE", "force")
    monkeypatch.setenv("MILP_DEVICE_DUAL", device_dual)
    monkeypatch.setenv("MILP_ASYNC_SOLVES", async_solves)
    monkeypatch.setenv("MILP_TRI_PAIR", "1")  # the two-vector launch where it applies
    lp = lp_gen.sparse_c5_lp(600, 6000, 6, 78)
    # Capped: forced onto the device, the deep L and U of this small LP take
    # a dependency hop per level (milliseconds per solve, where the host loop
    # takes microseconds); the window is what the parity check needs.
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1200)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    assert g.kernel_stats()["tri_solve"]["launches"] > 0


def _spec_flip_stats():
    import ctypes
    out = (ctypes.c_int64 * 3)()
    engine.lib().milp_spec_flip_stats(out)
    return list(out)


@pytest.mark.parametrize("seed", [78, 81])
@pytest.mark.parametrize("early", ["0", "1"])
def test_early_boxed_flips_parity(seed, early, monkeypatch):
    """The next loop top's boxed-flip decisions launched right after the
    reduced-cost update (DeviceLp::DualBoxedFlipsEarly) and taken only when
    nothing changed the reduced costs or those columns' bits since: the
    oracle's results either way."""
    monkeypatch.setenv("MILP_DEVICE_SOLVE", "force")
    monkeypatch.setenv("MILP_DEVICE_DUAL", "force")
    monkeypatch.setenv("MILP_EARLY_FLIPS", early)
    lp = lp_gen.sparse_c5_lp(500, 5000, 6, seed)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1500)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("seed", [78, 79, 80])
@pytest.mark.parametrize("spec", ["0", "1"])
def test_speculative_flip_ftran_parity(seed, spec, monkeypatch):
    """The next iteration's bound-flip FTRAN (MakeBoxedVariableDualFeasible,
    revised_simplex.cc:2391-2437) computed ahead: L and the etas after the
    ratio test, the pivot's MPF update applied inside the direction's FTRAN,
    the U solve on its own stream (engine/lu.cc SpecFlipBegin/Launch/Take).
    Used or dropped, the results and the deterministic time are the
    oracle's bit for bit; with it on, the next iterations use most of them."""
    monkeypatch.setenv("MILP_DEVICE_SOLVE", "force")
    monkeypatch.setenv("MILP_DEVICE_DUAL", "force")
    monkeypatch.setenv("MILP_SPEC_FLIP", spec)
    lp = lp_gen.sparse_c5_lp(600, 6000, 6, seed)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1500)
    before = _spec_flip_stats()
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    after = _spec_flip_stats()
    started, used = after[0] - before[0], after[1] - before[1]
    if spec == "1":
        assert started > 0 and used > 0, (started, used, after[2] - before[2])
    else:
        assert started == 0


@pytest.mark.parametrize("builder", kat_lps.ALL, ids=lambda f: f.__name__)
@pytest.mark.parametrize("dual", [0, 1])
def test_device_u_solve_known_answers(builder, dual, monkeypatch):
    monkeypatch.setenv("MILP_DEVICE_SOLVE", "force")
    lp, _ = builder()
    p = abi.default_params(use_dual_simplex=dual)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


def test_device_u_solve_warm_started_children(monkeypatch):
    """CP-SAT-style re-solves: each child refactorizes, so the device schedule
    is rebuilt for every factorization key."""
    monkeypatch.setenv("MILP_DEVICE_SOLVE", "force")
    import jobshop
    lp, ycols = jobshop.relaxation(jobshop.FT06)
    p = abi.default_params(use_dual_simplex=1)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    state = o.state()
    lbs, ubs = jobshop.child_bounds(lp, ycols, 6, 5)
    for i in range(len(lbs)):
        for h in (o, g):
            h.set_variable_bounds(lbs[i], ubs[i])
            h.load_basis_state(state)
        ro2 = o.solve()
        rg2 = g.solve()
        parity_util.compare(o, ro2, g, rg2, lp)


@pytest.mark.parametrize("pfi", [0, 1], ids=["mpf", "product_form"])
@pytest.mark.parametrize("dual", [0, 1])
def test_device_btran_and_upper_solve_parity(pfi, dual, monkeypatch):
    """Every dense loop of the factorization's solves on the device:
    BTRAN's U^T (TransposeUpperSolve, sparse.cc:848-897), L^T
    (TransposeLowerSolve), the unit-row U^T (LowerSolveStartingAt,
    lu_factorization.cc:405-436), and with product-form etas the FTRAN's
    UpperSolve (sparse.cc:814-846, a scatter restated as a gather with the
    loop's zero skip and division). Forced onto the device at test size, the
    engine must equal the oracle bit for bit and the device solves must run."""
    monkeypatch.setenv("MILP_DEVICE_SOLVE", "force")
    monkeypatch.setenv("MILP_TRI_BTRAN", "1")
    lp = lp_gen.dense_box_lp(90, 300, 81 + dual)
    p = abi.default_params(use_dual_simplex=dual, use_middle_product_form_update=1 - pfi,
                           max_number_of_iterations=600)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    st = g.kernel_stats()
    assert st["tri_solve_t"]["launches"] > 0, "no dense BTRAN solve reached the device"
    if pfi:
        assert st["tri_solve_upper"]["launches"] > 0, "no dense UpperSolve on the device"


def test_device_btran_sparse_dual_parity(monkeypatch):
    """A sparse dual LP whose BTRANs turn dense late: forced device solves of
    every kind against the oracle."""
    monkeypatch.setenv("MILP_DEVICE_SOLVE", "force")
    monkeypatch.setenv("MILP_TRI_BTRAN", "1")
    lp = lp_gen.sparse_c5_lp(700, 7000, 7, 83)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1500)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
