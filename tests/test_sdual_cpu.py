"""CPU checks of the device simplex segments' restatement
(or-tools_amd/csrc/sdual/sdual_core.h, sprimal_core.h). The oracle's test
build liboracle_sdual.so runs the same restatement, compiled for the host,
inside the oracle's own loops -- the dual loop (revised_simplex.cc:3058-3367
from the leaving-row choice on) and the primal loop (:2751-3045 from the
entering-column choice on, phases I and II); every result must equal the
plain oracle's bit for bit, and the segments must actually have run."""
import ctypes
import math

import numpy as np
import pytest

from mi_glop import abi, cpsat
import jobshop
import kat_lps
import lp_gen
import oracle_lib


def _counters(primal=False):
    L = oracle_lib.lib("sdual")
    L.oracle_sdual_counter.restype = ctypes.c_int64
    k = 2 if primal else 0
    return L.oracle_sdual_counter(k), L.oracle_sdual_counter(k + 1)


def _full(o, r):
    var, cons = o.statuses()
    return dict(err=r.error_code, status=r.problem_status, it=r.iterations,
                obj=float(r.objective).hex(), x=o.primal().tobytes(),
                rc=o.reduced_costs().tobytes(), y=o.duals().tobytes(),
                basis=o.basis().tobytes(), var=var.tobytes(), cons=cons.tobytes(),
                state=o.state().tobytes())


def _both(lp, p, state=None, bounds=None):
    out = []
    for variant in ("glop", "sdual"):
        o = oracle_lib.OracleLp(p, variant=variant)
        o.load(lp)
        if bounds is not None:
            o.set_variable_bounds(*bounds)
        if state is not None:
            o.load_basis_state(state)
        out.append(_full(o, o.solve()))
    return out


def _assert_same(a, b, tag):
    bad = [k for k in a if a[k] != b[k]]
    assert not bad, (tag, bad, a["it"], b["it"], a["obj"], b["obj"])


@pytest.mark.parametrize("seed", range(8))
def test_sdual_restatement_sparse(seed):
    seg0, it0 = _counters()
    m, n = 40 + 25 * seed, 150 + 60 * seed
    lp = lp_gen.random_sparse_lp(m, n, 0.06 if seed % 2 else 0.03, 700 + seed,
                                 maximize=bool(seed % 3 == 0))
    a, b = _both(lp, abi.default_params(use_dual_simplex=1))
    _assert_same(a, b, seed)
    seg1, it1 = _counters()
    assert seg1 > seg0 and it1 > it0


def test_sdual_restatement_kats():
    for lp, expect in (kat_lps.tiny_lp(),):
        a, b = _both(lp, abi.default_params(use_dual_simplex=1))
        _assert_same(a, b, "tiny")


@pytest.mark.parametrize("shape", [(6, 6), (10, 5)])
def test_sdual_restatement_children(shape):
    """Config-4 children (CP-SAT BranchOnVar LPs, warm-started dual simplex
    with an iteration cap, linear_programming_constraint.cc:485-584)."""
    jobs = jobshop.FT06 if shape == (6, 6) else jobshop.random_instance(*shape, 5)
    lp, ycols = jobshop.relaxation(jobs)
    root = oracle_lib.OracleLp(abi.default_params(use_dual_simplex=1))
    root.load(lp)
    rr = root.solve()
    state, x = root.state(), root.primal()
    node = cpsat.IntegerTrail(lp.col_lb, lp.col_ub,
                              obj_lb=math.ceil(rr.objective - cpsat.K_CP_EPSILON))
    cols = cpsat.fractional_columns(x, ycols, limit=12)
    lbs, ubs = cpsat.branch_lps(node, x, cols)
    seg0, _ = _counters()
    for cap in (1000, 7):
        p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=cap)
        for i in range(len(lbs)):
            a, b = _both(lp, p, state=state, bounds=(lbs[i], ubs[i]))
            _assert_same(a, b, (cap, i))
    seg1, _ = _counters()
    assert seg1 > seg0


def test_sdual_restatement_c5_shape():
    """A config-5-shaped LP (sparse, dual steepest edge) at small size."""
    lp = lp_gen.sparse_c5_lp(300, 3000, 6, 41)
    a, b = _both(lp, abi.default_params(use_dual_simplex=1))
    _assert_same(a, b, "c5")


def test_uniform_int_matches_libstdcxx():
    """The restatement's std::uniform_int_distribution<int> over mt19937_64
    (libstdc++ Lemire path) draws what the oracle draws: exercised through
    tie-heavy LPs (equal costs give equal prices and ratios)."""
    m, n = 60, 200
    rng = np.random.default_rng(5)
    lp = lp_gen.random_sparse_lp(m, n, 0.05, 77)
    lp.obj = np.round(rng.uniform(-1, 1, lp.n) * 2) / 2  # many ties
    a, b = _both(lp, abi.default_params(use_dual_simplex=1))
    _assert_same(a, b, "ties")


def test_sdual_restatement_resume_paths():
    """With almost no room for later factorizations in the arena
    (MILP_SDUAL_LU_SLACK), every refactorization inside a segment hands the
    LP back through the resume exits (kExitResumeTop / kExitResumePivot);
    results must not change. Runs in a child process (the cap is read once)."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path[:0] = %r\n"
        "import test_sdual_cpu as t, lp_gen\n"
        "from mi_glop import abi\n"
        "for seed in range(3):\n"
        "    lp = lp_gen.random_sparse_lp(80 + 30 * seed, 300, 0.05, 40 + seed)\n"
        "    a, b = t._both(lp, abi.default_params(use_dual_simplex=1))\n"
        "    t._assert_same(a, b, seed)\n"
        "lp = lp_gen.sparse_c5_lp(300, 3000, 6, 41)\n"
        "a, b = t._both(lp, abi.default_params(use_dual_simplex=1))\n"
        "t._assert_same(a, b, 'c5')\n"
        "print('ok')\n") % (sys.path[:6],)
    env = dict(os.environ, MILP_SDUAL_LU_SLACK="64")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def _segment_iterations(lp, p, phase1):
    """Iterations the oracle's sdual variant ran inside segments, with dual
    phase I in segments (MILP_SDUAL_PHASE1 unset) or on the host loop."""
    import os
    old = os.environ.pop("MILP_SDUAL_PHASE1", None)
    if not phase1:
        os.environ["MILP_SDUAL_PHASE1"] = "0"
    try:
        _, it0 = _counters()
        o = oracle_lib.OracleLp(p, variant="sdual")
        o.load(lp)
        out = _full(o, o.solve())
        _, it1 = _counters()
    finally:
        os.environ.pop("MILP_SDUAL_PHASE1", None)
        if old is not None:
            os.environ["MILP_SDUAL_PHASE1"] = old
    return out, it1 - it0


@pytest.mark.parametrize("seed", range(6))
def test_sdual_restatement_dual_phase1(seed):
    """Glop's dedicated dual phase I (revised_simplex.cc:2198-2388,
    entering_variable.cc:241-355) in segments: LPs whose slack basis is dual
    infeasible on unboxed columns, so that DualMinimize(feasibility_phase)
    runs many iterations; seed 5 is dual infeasible (phase I ends
    DUAL_INFEASIBLE). Equal to the plain oracle bit for bit, and the segments
    ran phase-I iterations (more than with phase I kept on the host)."""
    m, n = 60 + 40 * seed, 200 + 100 * seed
    lp = lp_gen.dual_phase1_lp(m, n, 900 + seed, unbounded_cols=2 if seed == 5 else 0)
    p = abi.default_params(use_dual_simplex=1)
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    plain = _full(o, o.solve())
    seg, it_on = _segment_iterations(lp, p, True)
    host_p1, it_off = _segment_iterations(lp, p, False)
    _assert_same(plain, seg, seed)
    _assert_same(plain, host_p1, seed)
    assert it_on > it_off, (it_on, it_off)
    if seed == 5:
        assert plain["status"] == seg["status"]


@pytest.mark.parametrize("cap", [1, 5, 37])
def test_sdual_restatement_dual_phase1_caps(cap):
    """Dual phase I stopped by an iteration cap inside a segment
    (kExitReturnOk in the phase-I loop) and the solve's status after it,
    for the MPF and the PFI updates; a minimization with the costs negated
    runs the same phase from the other side."""
    lp = lp_gen.dual_phase1_lp(120, 420, 977)
    flipped = lp_gen.dual_phase1_lp(120, 420, 977)
    flipped.obj = -flipped.obj
    flipped.maximize = False
    for case, q in (("max", lp), ("min", flipped)):
        for mpf in (1, 0):
            p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=cap,
                                   use_middle_product_form_update=mpf)
            a, b = _both(q, p)
            _assert_same(a, b, (case, mpf, cap))


@pytest.mark.parametrize("kind", ["sparse", "phase1", "suite", "primal"])
def test_sdual_restatement_pfi(kind):
    """The product-form updates (use_middle_product_form_update = false:
    EtaFactorization, basis_representation.cc:25-176, and the dense LU
    solves around it) in segments. The suite member runs hundreds of
    iterations, so segments also end at the eta room and repack the host's
    etas."""
    import netlib_suite
    if kind == "sparse":
        lps = [lp_gen.random_sparse_lp(60 + 30 * k, 240 + 80 * k, 0.05, 720 + k) for k in range(3)]
    elif kind == "phase1":
        lps = [lp_gen.dual_phase1_lp(80 + 40 * k, 300 + 100 * k, 960 + k) for k in range(3)]
    elif kind == "suite":
        lps = [netlib_suite.suite(max_rows=1500)[63]]
    else:  # the primal loop's segments (Glop's default algorithm)
        lps = [lp_gen.random_sparse_lp(90, 320, 0.05, 721), netlib_suite.suite(max_rows=1500)[45]]
    p = abi.default_params(use_dual_simplex=0 if kind == "primal" else 1,
                           use_middle_product_form_update=0)
    for k, lp in enumerate(lps):
        seg0, it0 = _counters(primal=kind == "primal")
        a, b = _both(lp, p)
        _assert_same(a, b, (kind, k))
        seg1, it1 = _counters(primal=kind == "primal")
        assert it1 - it0 > 0
    if kind == "suite":
        assert seg1 - seg0 > 8  # the eta room ended segments


def test_sdual_restatement_dual_phase1_resume_paths():
    """Dual phase I (and the PFI updates) through the resume exits (MILP_SDUAL_LU_SLACK: every
    refactorization inside a segment hands the LP back), in a child process."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path[:0] = %r\n"
        "import test_sdual_cpu as t, lp_gen\n"
        "from mi_glop import abi\n"
        "for seed in range(3):\n"
        "    lp = lp_gen.dual_phase1_lp(100 + 40 * seed, 400, 950 + seed)\n"
        "    a, b = t._both(lp, abi.default_params(use_dual_simplex=1))\n"
        "    t._assert_same(a, b, seed)\n"
        "    p = abi.default_params(use_dual_simplex=1, use_middle_product_form_update=0)\n"
        "    a, b = t._both(lp, p)\n"
        "    t._assert_same(a, b, ('pfi', seed))\n"
        "print('ok')\n") % (sys.path[:6],)
    env = dict(os.environ, MILP_SDUAL_LU_SLACK="64")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("seed", range(8))
def test_sprimal_restatement_sparse(seed):
    """Primal simplex (Glop's default), phase I and II in segments."""
    seg0, it0 = _counters(primal=True)
    m, n = 30 + 20 * seed, 90 + 50 * seed
    lp = lp_gen.random_sparse_lp(m, n, 0.06 if seed % 2 else 0.03, 900 + seed,
                                 maximize=bool(seed % 3 == 0))
    a, b = _both(lp, abi.default_params())
    _assert_same(a, b, seed)
    seg1, it1 = _counters(primal=True)
    assert seg1 > seg0 and it1 > it0


def test_sprimal_restatement_netlib_shaped():
    """The config-3 stand-in suite up to 300 rows, every LP bit-identical."""
    import netlib_suite
    seg0, it0 = _counters(primal=True)
    for i, lp in enumerate(netlib_suite.suite(max_rows=300)):
        a, b = _both(lp, abi.default_params())
        _assert_same(a, b, i)
    seg1, it1 = _counters(primal=True)
    assert it1 - it0 > 10000


def test_sprimal_restatement_kats():
    """Known-answer LPs (optimal, infeasible, unbounded) on both loops."""
    for builder in kat_lps.ALL:
        lp, _ = builder()
        for dual in (0, 1):
            a, b = _both(lp, abi.default_params(use_dual_simplex=dual))
            _assert_same(a, b, (builder.__name__, dual))


@pytest.mark.parametrize("cap", [1, 5, 40])
def test_sprimal_restatement_iteration_cap(cap):
    """An iteration cap ends a segment (kExitReturnOk) at the same point."""
    lp = lp_gen.random_sparse_lp(120, 300, 0.04, 77)
    a, b = _both(lp, abi.default_params(max_number_of_iterations=cap))
    _assert_same(a, b, cap)


def test_sprimal_restatement_resume_paths():
    """Primal segments with almost no room for later factorizations
    (MILP_SDUAL_LU_SLACK): every refactorization hands the LP back through the
    resume exits; results must not change. Runs in a child process (the cap
    is read once)."""
    import os
    import subprocess
    import sys
    code = (
        "import sys; sys.path[:0] = %r\n"
        "import test_sdual_cpu as t, lp_gen\n"
        "from mi_glop import abi\n"
        "s0 = t._counters(primal=True)\n"
        "for seed in range(3):\n"
        "    lp = lp_gen.random_sparse_lp(80 + 30 * seed, 300, 0.05, 60 + seed)\n"
        "    a, b = t._both(lp, abi.default_params())\n"
        "    t._assert_same(a, b, seed)\n"
        "assert t._counters(primal=True)[1] > s0[1]\n"
        "print('ok')\n") % (sys.path[:6],)
    env = dict(os.environ, MILP_SDUAL_LU_SLACK="64")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
