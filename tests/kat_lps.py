"""Known-answer LPs taken from the reference's own tests (golden vectors).

Each builder cites the reference test that states the expected answer:
  pdlp/test_util.h:25-110 + test_util.cc:35-265   (TestLp, TinyLp, ...)
  linear_solver/python/model_builder_test.py:49-135
  examples/tests/lp_test.cc:55-85, 136-170; glop/samples/simple_glop_program.cc
The expected values below are copied from those test files' assertions.
"""
import numpy as np

from mi_glop.lp import LinearProgram

INF = np.inf


def test_lp():
    # pdlp/test_util.cc:35-49; optimum -34 at [-1, 8, 1, 2.5] (test_util.h:43-47)
    trip = [(0, 0, 2), (0, 1, 1), (0, 2, 1), (0, 3, 2), (1, 0, 1), (1, 2, 1),
            (2, 0, 4), (3, 2, 1.5), (3, 3, -1)]
    lp = LinearProgram.from_triplets(
        4, 4, trip, [-INF, -2, -INF, 2.5], [INF, INF, 6, 3.5],
        [12, -INF, -4, -1], [12, 7, INF, 1], [5.5, -2, -1, 1], offset=-14,
        name="pdlp_TestLp")
    return lp, dict(objective=-34.0, primal=[-1, 8, 1, 2.5],
                    duals=[-2, 0, 2.375, 2.0 / 3], status=0)


def tiny_lp():
    # pdlp/test_util.cc:69-87; optimum -1 at [1,0,6,2], dual [0.5,4,0],
    # reduced costs [0,1.5,-3.5,0] (test_util.h:60-66)
    trip = [(0, 0, 2), (0, 1, 1), (0, 2, 1), (0, 3, 2), (1, 0, 1), (1, 2, 1),
            (2, 2, 1), (2, 3, -1)]
    lp = LinearProgram.from_triplets(
        3, 4, trip, [0, 0, 0, 0], [2, 4, 6, 3], [12, 7, 1], [12, INF, INF],
        [5, 2, 1, 1], offset=-14, name="pdlp_TinyLp")
    return lp, dict(objective=-1.0, primal=[1, 0, 6, 2], duals=[0.5, 4.0, 0.0],
                    reduced_costs=[0.0, 1.5, -3.5, 0.0], status=0)


def correlation_clustering_lp():
    # pdlp/test_util.cc:89-108; value 1, primal [1,1,0,1,0,0] (test_util.h:87-90)
    trip = [(0, 1, -1), (0, 2, 1), (0, 5, -1), (1, 3, -1), (1, 4, 1), (1, 5, -1),
            (2, 0, -1), (2, 1, -1), (2, 3, 1)]
    lp = LinearProgram.from_triplets(
        3, 6, trip, [0] * 6, [1] * 6, [-1, -1, -1], [INF] * 3,
        [-1, -1, 1, -1, 1, -1], offset=4, name="pdlp_CorrelationClusteringLp")
    return lp, dict(objective=1.0, status=0)


def correlation_clustering_star_lp():
    # pdlp/test_util.cc:110-129; value 1.5, primal [.5,.5,.5,0,0,0], dual [.5]*3
    trip = [(0, 0, -1), (0, 1, -1), (0, 3, 1), (1, 0, -1), (1, 2, -1), (1, 4, 1),
            (2, 1, -1), (2, 2, -1), (2, 5, 1)]
    lp = LinearProgram.from_triplets(
        3, 6, trip, [0] * 6, [1] * 6, [-1, -1, -1], [INF] * 3,
        [-1, -1, -1, 1, 1, 1], offset=3, name="pdlp_CorrelationClusteringStarLp")
    return lp, dict(objective=1.5, primal=[0.5, 0.5, 0.5, 0, 0, 0],
                    duals=[0.5, 0.5, 0.5], status=0)


def small_primal_infeasible_lp():
    # pdlp/test_util.cc:208-222
    trip = [(0, 0, 1), (0, 1, -1), (1, 0, -1), (1, 1, 1)]
    lp = LinearProgram.from_triplets(
        2, 2, trip, [0, 0], [INF, INF], [-INF, -INF], [1, -2], [1, 1],
        name="pdlp_SmallPrimalInfeasibleLp")
    return lp, dict(status_in=("PRIMAL_INFEASIBLE", "DUAL_UNBOUNDED"))


def small_dual_infeasible_lp():
    # pdlp/test_util.cc:224-229
    trip = [(0, 0, 1), (0, 1, -1), (1, 0, -1), (1, 1, 1)]
    lp = LinearProgram.from_triplets(
        2, 2, trip, [0, 0], [INF, INF], [-INF, -INF], [1, 2], [-1, -1],
        name="pdlp_SmallDualInfeasibleLp")
    return lp, dict(status_in=("PRIMAL_UNBOUNDED", "DUAL_INFEASIBLE"))


def small_initialization_lp():
    # pdlp/test_util.cc:238-251 (bounded, non-zero lower bounds)
    trip = [(0, 0, 1), (0, 1, 1), (1, 0, 1), (1, 1, 2)]
    lp = LinearProgram.from_triplets(
        2, 2, trip, [0.5, 0.5], [2, 2], [-INF, -INF], [2, 2], [-4, 0],
        name="pdlp_SmallInitializationLp")
    # No answer is stated upstream; hand-derived: x0 + 2 x1 <= 2 with
    # x1 >= 0.5 gives x0 <= 1, so min -4 x0 = -4 (cross-checked with HiGHS).
    return lp, dict(objective=-4.0, primal=[1.0, 0.5], status=0)


def model_builder_lp():
    # linear_solver/python/model_builder_test.py:49-135:
    # max 10x1+6x2+4x3-5.5, x1+x2+x3<=100, 10x1+4x2+5x3<=600, 2x1+2x2+6x3<=300,
    # x1>=1 -> 733.333333-5.5 at (33.333333, 66.666667, 0), activities (100,600,200)
    A = [[1, 1, 1], [10, 4, 5], [2, 2, 6]]
    lp = LinearProgram.from_dense(A, [1, 0, 0], [INF] * 3, [-INF] * 3,
                                  [100, 600, 300], [10, 6, 4], offset=-5.5,
                                  maximize=True, name="model_builder_test")
    return lp, dict(objective=733.3333333333334 - 5.5,
                    primal=[100.0 / 3, 200.0 / 3, 0.0],
                    activities=[100, 600, 200], status=0)


def lp_test_cc():
    # examples/tests/lp_test.cc:55-85: max 3x+4y, x+2y<=14, 3x-y>=0, x-y<=2
    # -> (6, 4), objective 34.
    A = [[1, 2], [3, -1], [1, -1]]
    lp = LinearProgram.from_dense(A, [0, 0], [INF, INF], [-INF, 0, -INF],
                                  [14, INF, 2], [3, 4], maximize=True,
                                  name="examples_lp_test")
    return lp, dict(objective=34.0, primal=[6, 4], status=0)


def mutable_objective_lp():
    # examples/tests/lp_test.cc:136-170 / glop/samples/simple_glop_program.cc:
    # max 3x+y, x<=1, y<=2, x+y<=2 -> 4.
    A = [[1, 1]]
    lp = LinearProgram.from_dense(A, [0, 0], [1, 2], [-INF], [2], [3, 1],
                                  maximize=True, name="simple_glop_program")
    return lp, dict(objective=4.0, primal=[1, 1], status=0)


def maximization_mps():
    # linear_solver/testdata/maximization.mps: max x s.t. x <= 4 (as a row) -> 4
    lp = LinearProgram.from_dense([[1.0]], [0], [INF], [-INF], [4], [1],
                                  maximize=True, name="maximization_mps")
    return lp, dict(objective=4.0, status=0)


ALL = [test_lp, tiny_lp, correlation_clustering_lp, correlation_clustering_star_lp,
       small_primal_infeasible_lp, small_dual_infeasible_lp, small_initialization_lp,
       model_builder_lp, lp_test_cc, mutable_objective_lp, maximization_mps]
