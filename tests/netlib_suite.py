"""Config 3 workload: a seeded "Netlib-shaped" suite of 94 LPs.

The Netlib files are not in this container or in the reference (SURVEY.md
8(c)), so config 3 runs on a deterministic stand-in with Netlib's spread of
shapes: row counts log-spaced from 27 (afiro) to a few thousand, 1.5-4
columns per row, a handful of non-zeros per column, and every row/column
bound type (equality, ranged, one-sided rows; boxed, one-sided and free
columns), built by lp_gen.random_sparse_lp so that each LP is feasible and
bounded.
"""
import numpy as np

import lp_gen

SUITE_SIZE = 94
SUITE_SEED = 20261015


def suite_shapes(count=SUITE_SIZE, max_rows=3000, seed=SUITE_SEED):
    """(m, n, density, seed) per LP, smallest first."""
    rng = np.random.default_rng(seed)
    ms = np.unique(np.round(np.geomspace(27, max_rows, count)).astype(int))
    while len(ms) < count:  # geomspace rounds small sizes together
        ms = np.unique(np.concatenate([ms, rng.integers(27, max_rows, count - len(ms))]))
    ms = np.sort(ms[:count])
    shapes = []
    for i, m in enumerate(ms):
        n = int(m * rng.uniform(1.5, 4.0))
        per_col = rng.uniform(2.5, 8.0)
        density = min(0.5, per_col / m)
        shapes.append((int(m), n, float(density), int(seed + 17 * i)))
    return shapes


def suite(count=SUITE_SIZE, max_rows=3000, seed=SUITE_SEED):
    """The LPs of the suite (lp_gen.LinearProgram), smallest first."""
    return [lp_gen.random_sparse_lp(m, n, d, s, maximize=bool(s % 2))
            for (m, n, d, s) in suite_shapes(count, max_rows, seed)]
