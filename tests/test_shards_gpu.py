"""Column shards (DeviceLp MILP_SHARDS): the columns of [A | I]
split into S blocks, each on a DeviceLp of its own ("virtual" shards: all on
the one GPU of the test box), must reproduce the unsplit engine -- and so the
oracle -- bit for bit: the per-column work joins in column order, the dual
ratio test's filter keeps a superset per shard (engine/device_shards.hip).
The reference pattern is pdlp/sharder_test.cc:128-172 (sharded results
equal the unsharded ones)."""
import pytest

from mi_glop import abi, engine

import lp_gen
import parity_util

pytestmark = pytest.mark.gpu


def _handle(params):
    return engine.LpHandle(params)


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_sharded_dual_device_mode(shards, monkeypatch):
    """Dual simplex in the dual device mode (device reduced costs, ratio-test
    filter, boxed flips) over S column shards."""
    monkeypatch.setenv("MILP_SHARDS", str(shards))
    monkeypatch.setenv("MILP_DEVICE_DUAL", "force")
    lp = lp_gen.sparse_c5_lp(800, 8000, 6, 90 + shards)
    p = abi.default_params(use_dual_simplex=1)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    st = g.kernel_stats()
    assert st["dual_ratio"]["launches"] >= shards, "the shards' ratio filters did not run"


@pytest.mark.parametrize("shards", [2, 8])
def test_sharded_primal(shards, monkeypatch):
    """Primal simplex: pricing, update rows (row- and column-wise) and the
    edge-norm list dots over S column shards."""
    monkeypatch.setenv("MILP_SHARDS", str(shards))
    lp = lp_gen.random_sparse_lp(300, 1500, 0.03, 95 + shards)
    p = abi.default_params(use_dual_simplex=0)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    assert g.kernel_stats()["pricing"]["launches"] > 0


@pytest.mark.parametrize("small_fused", ["auto", "off"])
def test_sharded_generic_path_small_lp(small_fused, monkeypatch):
    """The per-shard generic path (MILP_SMALL_FUSED=off forces it at this
    size): a shard whose columns are all relevant at the start (slack basis)
    must still receive its relevant mask (regression: it once kept the
    device's uninitialized words and its update rows came back empty)."""
    monkeypatch.setenv("MILP_SHARDS", "2")
    monkeypatch.setenv("MILP_SMALL_FUSED", small_fused)
    lp = lp_gen.sparse_c5_lp(2000, 20000, 10, 97)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)


def test_sharded_c5_shaped_window(monkeypatch):
    """A 20k x 200k config-5-shaped LP, 8 virtual shards, dual device mode
    at its default size threshold, 3000 iterations against the oracle."""
    monkeypatch.setenv("MILP_SHARDS", "8")
    lp = lp_gen.sparse_c5_lp(20000, 200000, 10, 97)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=3000)
    o, ro, g, rg = parity_util.solve_both(lp, p, _handle)
    parity_util.compare(o, ro, g, rg, lp)
    assert g.kernel_stats()["dual_ratio"]["launches"] > 0
