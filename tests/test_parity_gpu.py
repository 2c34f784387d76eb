"""MI355X engine vs CPU oracle on the same inputs (runs on the GPU box).

The engine executes the pricing SpMV, the update-row kernels, the primal
edge-norm dots, and the residual/basic-value SpMVs on the GPU; everything
must come out bit-identical to the oracle (basis, statuses, iteration count,
values), which is stronger than the 1e-6 objective contract."""
import numpy as np
import pytest

from mi_glop import abi, engine

import kat_lps
import lp_gen
import oracle_lib
import parity_util

pytestmark = pytest.mark.gpu


def _handle(params):
    return engine.LpHandle(params)


@pytest.mark.parametrize("builder", kat_lps.ALL, ids=lambda f: f.__name__)
@pytest.mark.parametrize("dual", [0, 1])
def test_known_answer_parity(builder, dual):
    lp, _ = builder()
    p = abi.default_params(use_dual_simplex=dual)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("seed", range(16))
@pytest.mark.parametrize("dual", [0, 1])
def test_random_sparse_parity(seed, dual):
    m = [8, 30, 90, 200][seed % 4]
    n = [20, 90, 300, 900][seed % 4]
    lp = lp_gen.random_sparse_lp(m, n, 0.25 if m < 40 else 0.04, 100 + seed,
                                 maximize=bool(seed % 2))
    p = abi.default_params(use_dual_simplex=dual)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("block", ["off", "force"])
@pytest.mark.parametrize("shape", [(40, 160), (97, 400), (202, 900), (259, 1100)])
def test_dense_primal_parity(shape, block, monkeypatch):
    """Config-2 family at test size: dense rows make rho dense, so the
    column-wise update row and the column dots are exercised, both through
    the CSC kernels (block=off) and the value-only dense block (force);
    odd m covers the ColumnScalarProduct tail terms."""
    monkeypatch.setenv("MILP_DENSE_BLOCK", block)
    lp = lp_gen.dense_box_lp(shape[0], shape[1], 3)
    o, ro, g, rg = parity_util.solve_both(lp, abi.default_params(), _handle)
    parity_util.compare(o, ro, g, rg, lp)
    st = g.kernel_stats()
    assert st["update_row"]["launches"] > 0
    assert st["primal_norms"]["launches"] > 0
    assert st["pricing"]["launches"] > 0
    per_launch = st["pricing"]["bytes"] / st["pricing"]["launches"]
    structural = shape[0] * shape[1]
    if block == "force":  # dense block streams 8 B per entry, CSC 12 B
        assert per_launch < 12.0 * structural
    else:
        assert per_launch > 12.0 * structural


@pytest.mark.parametrize("block", ["off", "force"])
@pytest.mark.parametrize("shape", [(97, 400), (259, 1100)])
def test_parked_edge_norm_update_parity(shape, block, monkeypatch):
    """The edge-norm dots parked after a row-wise update row ride on the next
    pricing pass (phase I resets the costs every iteration). With and without
    parking, every result must equal the oracle's, and parking must remove
    standalone dots passes."""
    monkeypatch.setenv("MILP_DENSE_BLOCK", block)
    lp = lp_gen.dense_box_lp(shape[0], shape[1], 7)
    launches = {}
    for defer in ("0", "1"):
        monkeypatch.setenv("MILP_DEFER_NORMS", defer)
        o, ro, g, rg = parity_util.solve_both(lp, abi.default_params(), _handle)
        parity_util.compare(o, ro, g, rg, lp)
        launches[defer] = g.kernel_stats()["primal_norms"]["launches"]
    assert launches["1"] < launches["0"], launches


@pytest.mark.parametrize("chunk_max", ["0", "1000000"])
@pytest.mark.parametrize("seed", [21, 22, 23])
def test_row_wise_kernel_choice_parity(seed, chunk_max, monkeypatch):
    """Row-wise update rows through the column-order kernel (every filtered
    rho, chunk_max=0) or the row-chunk kernel (always): both must reproduce
    the host scatter order, so the dual simplex matches the oracle bit for bit
    either way. Config-5-shaped LPs (a few entries per column)."""
    monkeypatch.setenv("MILP_ROWWISE_CHUNK_MAX_ROWS", chunk_max)
    monkeypatch.setenv("MILP_SMALL_FUSED", "off")  # these N would take the one-launch kernel
    lp = lp_gen.sparse_c5_lp(300 + 50 * (seed % 3), 3000, 6, seed)
    p = abi.default_params(use_dual_simplex=1)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    st = g.kernel_stats()
    assert st["update_row"]["launches"] > 0


@pytest.mark.parametrize("full_rows", ["on", "off"])
@pytest.mark.parametrize("dual", [0, 1])
@pytest.mark.parametrize("shape", [(97, 500, 31), (160, 1200, 32)])
def test_full_row_kernel_parity(shape, dual, full_rows, monkeypatch):
    """Dense A: every CSR row holds all structural columns, so row-wise
    update rows go through the full-row kernel (direct entry addressing, list
    order k, slack outputs through the row tags) unless disabled. Both ways
    must match the oracle bit for bit, in primal and dual simplex."""
    monkeypatch.setenv("MILP_FULL_ROWS", full_rows)
    monkeypatch.setenv("MILP_SMALL_FUSED", "off")
    m, n, seed = shape
    lp = lp_gen.dense_box_lp(m, n, seed)
    p = abi.default_params(use_dual_simplex=dual)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    st = g.kernel_stats()
    assert st["update_row"]["launches"] + st["single_row"]["launches"] > 0


def test_full_and_partial_rows_parity(monkeypatch):
    """Some rows full, some not: a filtered list that mixes them takes the
    general row-wise kernels, an all-full list the full-row kernel."""
    monkeypatch.setenv("MILP_SMALL_FUSED", "off")
    rng = np.random.default_rng(9)
    m, n = 70, 400
    dense = rng.uniform(-1, 1, size=(m, n))
    holes = rng.random(size=(m, n)) < 0.3
    holes[: m // 2] = False  # the first half of the rows stays full
    dense[holes] = 0.0
    lp = lp_gen.from_dense_box(dense, rng)
    for dual in (0, 1):
        p = abi.default_params(use_dual_simplex=dual)
        o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
        parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("unroll", ["8", "32"])
def test_dense_block_unroll_parity(unroll, monkeypatch):
    """The dense-block kernel's load depth does not change any result."""
    monkeypatch.setenv("MILP_DENSE_BLOCK", "force")
    monkeypatch.setenv("MILP_DENSE_UNROLL", unroll)
    lp = lp_gen.dense_box_lp(131, 700, 4)
    o, ro, g, rg = parity_util.solve_both(lp, abi.default_params(), _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("block", ["off", "force"])
@pytest.mark.parametrize("seed", [11, 12])
def test_dense_dual_parity(seed, block, monkeypatch):
    monkeypatch.setenv("MILP_DENSE_BLOCK", block)
    lp = lp_gen.dense_box_lp(81 + seed, 300, seed)
    p = abi.default_params(use_dual_simplex=1)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


def test_mixed_dense_sparse_columns(monkeypatch):
    """Some full columns next to sparse ones: both kernels share one launch
    set (dense block + CSC over the remaining columns)."""
    monkeypatch.setenv("MILP_DENSE_BLOCK", "force")
    rng = np.random.default_rng(5)
    m, n = 60, 240
    dense = rng.uniform(-1, 1, size=(m, n))
    dense[:, 80:] *= rng.uniform(size=(m, n - 80)) < 0.08
    lp = lp_gen.from_dense_box(dense, rng)
    for dual in (0, 1):
        p = abi.default_params(use_dual_simplex=dual)
        o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
        parity_util.compare(o, ro, g, rg, lp)


def test_warm_start_parity():
    """Bound tightened + LoadStateForNextSolve, dual simplex (CP-SAT call-out)."""
    lp = lp_gen.random_sparse_lp(60, 200, 0.06, 9)
    p = abi.default_params(use_dual_simplex=1)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    x = o.primal()
    j = int(np.argmax(np.abs(x - np.round(x))))
    lp.col_ub = lp.col_ub.copy()
    lp.col_ub[j] = np.floor(x[j])
    o.load(lp)
    g.load(lp)
    ro2 = o.solve()
    rg2 = g.solve()
    parity_util.compare(o, ro2, g, rg2, lp)
    state = o.state()
    o.load_basis_state(state)
    g.load_basis_state(state)
    ro3 = o.solve()
    rg3 = g.solve()
    parity_util.compare(o, ro3, g, rg3, lp)


def test_iteration_limit_and_resume_slicing():
    """mi_lp_begin/run_until (bench slicing) must not change the result."""
    lp = lp_gen.dense_box_lp(64, 256, 5)
    p = abi.default_params()
    g = engine.LpHandle(p)
    g.load(lp)
    full = g.solve()
    g2 = engine.LpHandle(p)
    g2.load(lp)
    g2.begin(3)
    fin, it = g2.run_until(7)
    assert fin or it == 7
    r = g2.finish()
    assert r.iterations == full.iterations and r.objective == full.objective
    np.testing.assert_array_equal(g2.basis(), g.basis())


def test_invalid_problem_status():
    lp, _ = kat_lps.small_primal_infeasible_lp()
    lp.row_lb = lp.row_lb.copy()
    lp.row_lb[0] = 5.0  # lb > ub: LinearProgram::IsValid fails
    lp.row_ub = lp.row_ub.copy()
    lp.row_ub[0] = 1.0
    g = engine.LpHandle()
    g.load(lp)
    r = g.solve()
    assert r.problem_status == abi.INVALID_PROBLEM
    o, ro, g, rg = parity_util.solve_both(lp, abi.default_params(), _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("fused", ["auto", "serial", "serial256", "by_column", "off"])
@pytest.mark.parametrize("dual", [0, 1])
@pytest.mark.parametrize("case", ["sparse", "c5", "dense", "jobshop"])
def test_small_lp_one_launch_update_row_parity(case, dual, fused, monkeypatch):
    """Small LPs (N <= 8192): every update row is one launch with its inputs,
    the relevant mask and the list in mapped host memory: row-wise rows
    applied in turn out of LDS (few rows) or column by column (many rows),
    and the column-wise row with the edge-norm dots. The dense case (a dense
    block) mixes them with the generic kernels within one solve (deferred
    mask uploads). The
    dual simplex computes tau while that launch runs (MILP_INLINE_TAU). Bit
    for bit equal to the oracle (deterministic time included), either way."""
    monkeypatch.setenv("MILP_SMALL_FUSED", "off" if fused == "off" else "on")
    monkeypatch.setenv("MILP_INLINE_TAU", "off" if fused == "off" else "on")
    if fused != "auto":  # row-wise rows applied in turn, or column by column
        serial = fused.startswith("serial")
        monkeypatch.setenv("MILP_SMALL_SERIAL_ROWS", "1000000" if serial else "0")
    if fused == "serial256":  # the 4-wave workgroup variant
        monkeypatch.setenv("MILP_SMALL_THREADS", "256")
    if case == "sparse":
        lp = lp_gen.random_sparse_lp(200, 900, 0.04, 7, maximize=True)
    elif case == "c5":
        lp = lp_gen.sparse_c5_lp(400, 4000, 6, 41)
    elif case == "dense":
        lp = lp_gen.dense_box_lp(120, 900, 5)
    else:
        import jobshop
        lp, _ = jobshop.relaxation(jobshop.random_instance(8, 6, 5))
    p = abi.default_params(use_dual_simplex=dual)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    st = g.kernel_stats()
    assert st["update_row"]["launches"] + st["single_row"]["launches"] > 0


@pytest.mark.parametrize("shape", [(6, 6), (10, 10), (25, 10)])
def test_batched_children_parity(shape):
    """Config-4 batch: children of one search node (bounds of two order
    variables fixed), warm-started from the root basis, solved by 4 GPU
    workers; each child must match the oracle solving it alone. 25x10 has
    N > 8192: the mid-size batched update row (kMediumRowWise) and the host
    triangular solves of a batch."""
    import jobshop
    jobs = jobshop.FT06 if shape == (6, 6) else jobshop.random_instance(*shape, 3)
    lp, ycols = jobshop.relaxation(jobs)
    if shape == (25, 10):
        assert 8192 < lp.m + lp.n <= 65536
    root = engine.LpHandle(abi.default_params(use_dual_simplex=1))
    root.load(lp)
    assert root.solve().problem_status == abi.OPTIMAL
    state = root.state()
    lbs, ubs = jobshop.child_bounds(lp, ycols, 24, 11)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    workers = [engine.LpHandle(p) for _ in range(4)]
    for w in workers:
        w.load(lp)
    res = engine.batch_solve_bounds(workers, lbs, ubs, state)
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    for i, r in enumerate(res):
        o.set_variable_bounds(lbs[i], ubs[i])
        o.load_basis_state(state)
        ro = o.solve()
        assert (r.error_code, r.problem_status, r.iterations) == \
            (ro.error_code, ro.problem_status, ro.iterations), i
        assert r.objective == ro.objective, (i, r.objective, ro.objective)


def _device_dual_cases():
    cases = []
    for seed in range(6):
        m = [30, 90, 200][seed % 3]
        n = [90, 300, 900][seed % 3]
        cases.append(("sparse", lambda m=m, n=n, s=seed: lp_gen.random_sparse_lp(
            m, n, 0.25 if m < 40 else 0.04, 300 + s, maximize=bool(s % 2))))
    for seed in (31, 32):
        cases.append(("c5", lambda s=seed: lp_gen.sparse_c5_lp(400, 4000, 6, s)))
    cases.append(("dense", lambda: lp_gen.dense_box_lp(93, 300, 13)))
    for builder in kat_lps.ALL:
        cases.append((builder.__name__, lambda b=builder: b()[0]))
    return cases


@pytest.mark.parametrize("tighten", ["0", "100000000"])
@pytest.mark.parametrize("case", _device_dual_cases(), ids=lambda c: c[0])
def test_device_dual_mode_parity(case, tighten, monkeypatch):
    """Dual phase II with the reduced costs and the update row kept on the
    device (device-filtered bound-flipping ratio test, device rc update,
    device boxed dual-feasibility decisions), forced on small LPs: every
    result must equal the oracle's, which runs Glop's host loops."""
    monkeypatch.setenv("MILP_DEVICE_DUAL", "force")
    monkeypatch.setenv("MILP_DUAL_TIGHTEN_MIN", tighten)  # 0: always tighten
    lp = case[1]()
    p = abi.default_params(use_dual_simplex=1)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("target", ["1", "3"])
@pytest.mark.parametrize("case", _device_dual_cases(), ids=lambda c: c[0])
def test_device_dual_mode_parity_small_selection(case, target, monkeypatch):
    """The tightening walk over the smallest keys only (simplex_kernels.hip
    dual_tighten) with the selection cut to 1 or 3 keys, so that its walks
    leave the gathered prefix or accept its last key: the bound must then
    stay B (the host gets every candidate) and every result equal the
    oracle's."""
    monkeypatch.setenv("MILP_DEVICE_DUAL", "force")
    monkeypatch.setenv("MILP_DUAL_TIGHTEN_MIN", "0")
    monkeypatch.setenv("MILP_TIGHTEN_TARGET", target)
    lp = case[1]()
    p = abi.default_params(use_dual_simplex=1)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


def test_device_dual_mode_warm_start_and_children(monkeypatch):
    """CP-SAT-style re-solves in dual device mode: bound change + warm start."""
    monkeypatch.setenv("MILP_DEVICE_DUAL", "force")
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


@pytest.mark.parametrize("dual", [0, 1])
@pytest.mark.parametrize("case", ["dense", "sparse"])
def test_host_parallel_loops_parity(case, dual, monkeypatch):
    """The engine's O(N) host loops (price rebuild and updates, edge-norm
    update, reduced-cost update, dual prices, update-row fetch) split over the
    host pool at every size: results must not change."""
    monkeypatch.setenv("MILP_HOST_PARALLEL_MIN", "1")
    if case == "dense":
        lp = lp_gen.dense_box_lp(120, 900, 41)
    else:
        lp = lp_gen.sparse_c5_lp(400, 4000, 6, 42)
    p = abi.default_params(use_dual_simplex=dual)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("seed", [51, 52, 53])
@pytest.mark.parametrize("device_dual", ["off", "force"])
def test_async_tau_parity(seed, device_dual, monkeypatch):
    """The dual loop's tau FTRAN runs on the factorization's worker thread
    (MILP_ASYNC_SOLVES=force at test size) while the update row, ratio test and
    direction FTRAN run: same results and iteration count as the oracle, and the
    same deterministic time as the serial engine (the worker's bumps are
    applied in serial order)."""
    monkeypatch.setenv("MILP_DEVICE_DUAL", device_dual)
    lp = lp_gen.sparse_c5_lp(500 + 40 * (seed % 3), 5000, 6, seed)
    p = abi.default_params(use_dual_simplex=1)
    dtime = {}
    for mode in ("off", "force"):
        monkeypatch.setenv("MILP_ASYNC_SOLVES", mode)
        o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
        parity_util.compare(o, ro, g, rg, lp)
        dtime[mode] = rg.deterministic_time
    assert dtime["force"] == dtime["off"]


@pytest.mark.parametrize("shape", [(97, 500, 61), (160, 1200, 62)])
@pytest.mark.parametrize("block", ["off", "force"])
def test_async_direction_left_inverse_parity(shape, block, monkeypatch):
    """Primal steepest edge: B^-T d runs on the factorization's worker while
    the entering tests, ratio test and update row run, and is taken by the
    edge-norm update (or dropped when the iteration restarts). Dense LPs
    (phase I every iteration): results and deterministic time unchanged."""
    monkeypatch.setenv("MILP_DENSE_BLOCK", block)
    m, n, seed = shape
    lp = lp_gen.dense_box_lp(m, n, seed)
    dtime = {}
    for mode in ("off", "force"):
        monkeypatch.setenv("MILP_ASYNC_SOLVES", mode)
        o, ro, g, rg = parity_util.solve_both(lp, abi.default_params(), _handle)
        parity_util.compare(o, ro, g, rg, lp)
        dtime[mode] = rg.deterministic_time
    assert dtime["force"] == dtime["off"]


@pytest.mark.parametrize("name", ["test2.mps", "maximization.mps", "solomon_bp_c101.mps"])
@pytest.mark.parametrize("dual", [0, 1])
def test_mps_file_parity(name, dual):
    """LPs read from the reference's MPS fixtures (mi_mps_read_file) solve on
    the GPU exactly as on the oracle (solomon_bp_c101: its LP relaxation)."""
    import os
    from mi_glop import mps
    lp = mps.read_mps(os.path.join(os.path.dirname(__file__), "golden", "mps", name))
    p = abi.default_params(use_dual_simplex=dual)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("builder", kat_lps.ALL, ids=lambda f: f.__name__)
@pytest.mark.parametrize("dual", [0, 1])
def test_product_form_known_answer_parity(builder, dual):
    """use_middle_product_form_update=false (product-form etas, SURVEY 8(a)
    a14): engine and oracle agree bit for bit, including where upstream's
    eta path ends ABNORMAL/IMPRECISE (see test_oracle.py)."""
    lp, _ = builder()
    p = abi.default_params(use_dual_simplex=dual, use_middle_product_form_update=0)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("dual", [0, 1])
def test_product_form_random_parity(seed, dual):
    m = [30, 90, 200][seed % 3]
    n = [90, 300, 900][seed % 3]
    lp = lp_gen.random_sparse_lp(m, n, 0.25 if m < 40 else 0.04, 700 + seed,
                                 maximize=bool(seed % 2))
    p = abi.default_params(use_dual_simplex=dual, use_middle_product_form_update=0)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


def test_product_form_dense_parity():
    lp = lp_gen.dense_box_lp(97, 400, 3)
    p = abi.default_params(use_middle_product_form_update=0)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


@pytest.mark.parametrize("basis", [1, 3])  # BIXBY, MAROS
@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("dual", [0, 1])
def test_crash_basis_parity(basis, seed, dual):
    """initial_basis BIXBY / MAROS: engine == oracle."""
    m = [40, 90, 150, 200][seed % 4]
    n = [70, 250, 400, 900][seed % 4]
    lp = lp_gen.random_sparse_lp(m, n, 0.06, 900 + seed, eq_frac=0.5, maximize=bool(seed % 2))
    for j in range(lp.n):
        s0, s1 = lp.col_starts[j], lp.col_starts[j + 1]
        if s1 > s0:
            scale = np.abs(lp.vals[s0:s1]).max()
            lp.vals[s0:s1] /= scale
            lp.obj[j] /= scale
            lp.col_lb[j] *= scale
            lp.col_ub[j] *= scale
    p = abi.default_params(use_dual_simplex=dual, initial_basis=basis)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
