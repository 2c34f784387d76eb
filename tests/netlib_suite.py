"""Config 3 workload: a seeded "Netlib-shaped" suite of 94 LPs.

The Netlib files are not in this container or in the reference (SURVEY.md
8(c)), so config 3 runs on a deterministic stand-in with Netlib's spread of
shapes: row counts log-spaced from 27 (afiro) to a few thousand, 1.5-4
columns per row, a handful of non-zeros per column, and every row/column
bound type (equality, ranged, one-sided rows; boxed, one-sided and free
columns), built by lp_gen.random_sparse_lp so that each LP is feasible and
bounded.

Netlib's large members (scfxm, sctap, stocfor3 at 16 675 rows, pilot) are
multi-period models whose bases factor with little fill; a uniformly random
matrix of that size factors densely and takes ~10 m iterations (6 554 rows:
65 k iterations, 330 s on the oracle). Members above STAIRCASE_MIN_ROWS rows
are therefore staircase LPs (lp_gen.staircase_lp: periods of 50 rows, 20 %
of the columns carrying into the next period, n = 1.2-2.0 m), which keep
the iteration count near 2 m as Netlib's do. bench.py's default suite runs
to 16 000 rows ("m from 27 to ~16k").
"""
import numpy as np

import lp_gen

SUITE_SIZE = 94
SUITE_SEED = 20261015
STAIRCASE_MIN_ROWS = 2000


def suite_shapes(count=SUITE_SIZE, max_rows=3000, seed=SUITE_SEED):
    """(m, n, density, seed) per LP, smallest first. For a staircase member
    (m > STAIRCASE_MIN_ROWS) density is unused and n = 1.2-2.0 m."""
    rng = np.random.default_rng(seed)
    ms = np.unique(np.round(np.geomspace(27, max_rows, count)).astype(int))
    while len(ms) < count:  # geomspace rounds small sizes together
        ms = np.unique(np.concatenate([ms, rng.integers(27, max_rows, count - len(ms))]))
    ms = np.sort(ms[:count])
    shapes = []
    for i, m in enumerate(ms):
        u = rng.uniform(1.5, 4.0)
        n = int(m * u) if m <= STAIRCASE_MIN_ROWS else int(m * (1.2 + 0.32 * (u - 1.5)))
        per_col = rng.uniform(2.5, 8.0)
        density = min(0.5, per_col / m)
        shapes.append((int(m), n, float(density), int(seed + 17 * i)))
    return shapes


def suite(count=SUITE_SIZE, max_rows=3000, seed=SUITE_SEED):
    """The LPs of the suite (lp_gen.LinearProgram), smallest first."""
    return [member(*shape) for shape in suite_shapes(count, max_rows, seed)]


def member(m, n, density, seed):
    """One suite LP from its shape tuple."""
    if m > STAIRCASE_MIN_ROWS:
        return lp_gen.staircase_lp(m, n, seed, block_rows=50, link_frac=0.2, eq_frac=0.1,
                                   maximize=bool(seed % 2))
    return lp_gen.random_sparse_lp(m, n, density, seed, maximize=bool(seed % 2))
