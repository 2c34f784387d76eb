"""BTRAN's forward U^T solve with a dense tail on the device (dense_tail.hip,
DeviceLp::DenseTailSolve): TriangularMatrix::TransposeUpperSolve
(sparse.cc:848-897) when U's last columns hold most of its entries -- config
2's late bases, whose ~1 500 dense columns each read ~8 500 slack rows. The
engine's result must be the oracle's bit for bit; the size thresholds are
lowered so that LPs of a few hundred rows take the device path."""
import numpy as np
import pytest

from mi_glop import abi, engine

import lp_gen
import parity_util

pytestmark = pytest.mark.gpu


def _cases():
    rng = np.random.default_rng(5)
    mixed = rng.uniform(-1, 1, size=(300, 900))
    mixed[:, ::3] *= rng.uniform(size=(300, 300)) < 0.05  # a third of the columns sparse
    return [
        ("dense_primal", lambda: lp_gen.dense_box_lp(400, 1600, 11), 0, 900),
        ("dense_dual", lambda: lp_gen.dense_box_lp(300, 1200, 12), 1, 700),
        ("mixed_primal", lambda: lp_gen.from_dense_box(mixed, np.random.default_rng(6)), 0, 800),
    ]


@pytest.mark.parametrize("case", _cases(), ids=lambda c: c[0])
def test_dense_tail_parity(case, monkeypatch):
    name, build, dual, cap = case
    monkeypatch.setenv("MILP_DENSE_TAIL", "1")
    monkeypatch.setenv("MILP_DENSE_TAIL_MIN_ENTRIES", "2000")
    monkeypatch.setenv("MILP_DENSE_TAIL_MIN_COLS", "8")
    lp = build()
    p = abi.default_params(use_dual_simplex=dual, max_number_of_iterations=cap)
    o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q))
    parity_util.compare(o, ro, g, rg, lp)
    assert g.kernel_stats()["tri_solve_t"]["launches"] > 0, "the dense-tail solve did not run"


def test_dense_tail_off_is_the_host_loop(monkeypatch):
    """MILP_DENSE_TAIL=0: the same solve on the host loop, same result."""
    monkeypatch.setenv("MILP_DENSE_TAIL", "0")
    lp = lp_gen.dense_box_lp(400, 1600, 11)
    p = abi.default_params(max_number_of_iterations=900)
    o, ro, g, rg = parity_util.solve_both(lp, p, lambda q: engine.LpHandle(q))
    parity_util.compare(o, ro, g, rg, lp)
    assert g.kernel_stats()["tri_solve_t"]["launches"] == 0
