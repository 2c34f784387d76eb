"""ctypes view of the C ABI declared in include/mi_lp.h.

Only plain structs and pointers cross the boundary. The
struct layouts here must match include/mi_lp.h field for field.
"""
import ctypes
import math

INF = math.inf


class MiGlopParams(ctypes.Structure):
    """POD mirror of glop::GlopParameters (ortools/glop/parameters.proto)."""

    _fields_ = [
        ("use_dual_simplex", ctypes.c_int32),
        ("feasibility_rule", ctypes.c_int32),
        ("optimization_rule", ctypes.c_int32),
        ("initial_basis", ctypes.c_int32),
        ("use_transposed_matrix", ctypes.c_int32),
        ("basis_refactorization_period", ctypes.c_int32),
        ("dynamically_adjust_refactorization_period", ctypes.c_int32),
        ("change_status_to_imprecise", ctypes.c_int32),
        ("markowitz_zlatev_parameter", ctypes.c_int32),
        ("allow_simplex_algorithm_change", ctypes.c_int32),
        ("devex_weights_reset_period", ctypes.c_int32),
        ("use_middle_product_form_update", ctypes.c_int32),
        ("initialize_devex_with_column_norms", ctypes.c_int32),
        ("exploit_singleton_column_in_initial_basis", ctypes.c_int32),
        ("random_seed", ctypes.c_int32),
        ("perturb_costs_in_dual_simplex", ctypes.c_int32),
        ("use_dedicated_dual_feasibility_algorithm", ctypes.c_int32),
        ("push_to_vertex", ctypes.c_int32),
        ("dual_price_prioritize_norm", ctypes.c_int32),
        ("use_scaling", ctypes.c_int32),
        ("max_number_of_iterations", ctypes.c_int64),
        ("refactorization_threshold", ctypes.c_double),
        ("recompute_reduced_costs_threshold", ctypes.c_double),
        ("recompute_edges_norm_threshold", ctypes.c_double),
        ("primal_feasibility_tolerance", ctypes.c_double),
        ("dual_feasibility_tolerance", ctypes.c_double),
        ("ratio_test_zero_threshold", ctypes.c_double),
        ("harris_tolerance_ratio", ctypes.c_double),
        ("small_pivot_threshold", ctypes.c_double),
        ("minimum_acceptable_pivot", ctypes.c_double),
        ("drop_tolerance", ctypes.c_double),
        ("solution_feasibility_tolerance", ctypes.c_double),
        ("max_number_of_reoptimizations", ctypes.c_double),
        ("lu_factorization_pivot_threshold", ctypes.c_double),
        ("max_time_in_seconds", ctypes.c_double),
        ("max_deterministic_time", ctypes.c_double),
        ("markowitz_singularity_threshold", ctypes.c_double),
        ("dual_small_pivot_threshold", ctypes.c_double),
        ("objective_lower_limit", ctypes.c_double),
        ("objective_upper_limit", ctypes.c_double),
        ("degenerate_ministep_factor", ctypes.c_double),
        ("relative_cost_perturbation", ctypes.c_double),
        ("relative_max_cost_perturbation", ctypes.c_double),
        ("initial_condition_number_threshold", ctypes.c_double),
        ("crossover_bound_snapping_distance", ctypes.c_double),
    ]


# Proto defaults, ortools/glop/parameters.proto (field numbers in mi_lp.h).
_DEFAULTS = dict(
    use_dual_simplex=0, feasibility_rule=1, optimization_rule=1, initial_basis=2,
    use_transposed_matrix=1, basis_refactorization_period=64,
    dynamically_adjust_refactorization_period=1, change_status_to_imprecise=1,
    markowitz_zlatev_parameter=3, allow_simplex_algorithm_change=0,
    devex_weights_reset_period=150, use_middle_product_form_update=1,
    initialize_devex_with_column_norms=1,
    exploit_singleton_column_in_initial_basis=1, random_seed=1,
    perturb_costs_in_dual_simplex=0, use_dedicated_dual_feasibility_algorithm=1,
    push_to_vertex=1, dual_price_prioritize_norm=0, use_scaling=1,
    max_number_of_iterations=-1, refactorization_threshold=1e-9,
    recompute_reduced_costs_threshold=1e-8, recompute_edges_norm_threshold=100.0,
    primal_feasibility_tolerance=1e-8, dual_feasibility_tolerance=1e-8,
    ratio_test_zero_threshold=1e-9, harris_tolerance_ratio=0.5,
    small_pivot_threshold=1e-6, minimum_acceptable_pivot=1e-6,
    drop_tolerance=1e-14, solution_feasibility_tolerance=1e-6,
    max_number_of_reoptimizations=40.0, lu_factorization_pivot_threshold=0.01,
    max_time_in_seconds=INF, max_deterministic_time=INF,
    markowitz_singularity_threshold=1e-15, dual_small_pivot_threshold=1e-4,
    objective_lower_limit=-INF, objective_upper_limit=INF,
    degenerate_ministep_factor=0.01, relative_cost_perturbation=1e-5,
    relative_max_cost_perturbation=1e-7, initial_condition_number_threshold=1e50,
    crossover_bound_snapping_distance=INF,
)


def default_params(**overrides):
    p = MiGlopParams()
    for k, v in _DEFAULTS.items():
        setattr(p, k, v)
    for k, v in overrides.items():
        if k not in _DEFAULTS:
            raise KeyError(f"unknown GlopParameters field {k!r}")
        setattr(p, k, v)
    return p


class MiLpResult(ctypes.Structure):
    _fields_ = [
        ("problem_status", ctypes.c_int32),
        ("error_code", ctypes.c_int32),
        ("iterations", ctypes.c_int64),
        ("objective", ctypes.c_double),
        ("deterministic_time", ctypes.c_double),
        ("solve_seconds", ctypes.c_double),
    ]


class MiLpKernelStats(ctypes.Structure):
    _fields_ = [
        ("launches", ctypes.c_int64 * 16),
        ("algorithmic_bytes", ctypes.c_double * 16),
        ("device_ms", ctypes.c_double * 16),
        ("call_ms", ctypes.c_double * 16),
    ]


# glop::ProblemStatus (lp_data/lp_types.h:106-168)
PROBLEM_STATUS = [
    "OPTIMAL", "PRIMAL_INFEASIBLE", "DUAL_INFEASIBLE", "INFEASIBLE_OR_UNBOUNDED",
    "PRIMAL_UNBOUNDED", "DUAL_UNBOUNDED", "INIT", "PRIMAL_FEASIBLE",
    "DUAL_FEASIBLE", "ABNORMAL", "INVALID_PROBLEM", "IMPRECISE",
]
OPTIMAL = 0
PRIMAL_INFEASIBLE = 1
DUAL_INFEASIBLE = 2
INFEASIBLE_OR_UNBOUNDED = 3
PRIMAL_UNBOUNDED = 4
DUAL_UNBOUNDED = 5
INIT = 6
PRIMAL_FEASIBLE = 7
DUAL_FEASIBLE = 8
ABNORMAL = 9
INVALID_PROBLEM = 10
IMPRECISE = 11

# glop::VariableStatus / ConstraintStatus (lp_data/lp_types.h:188-219)
BASIC, FIXED_VALUE, AT_LOWER_BOUND, AT_UPPER_BOUND, FREE = 0, 1, 2, 3, 4

# Kernel ids (include/mi_lp.h MI_K_*)
class MiLpRunCounters(ctypes.Structure):
    """mi_lp_run_counters (include/mi_lp.h): window statistics."""
    _fields_ = [
        ("factorizations", ctypes.c_int64),
        ("factorization_seconds", ctypes.c_double),
        ("iterations", ctypes.c_int64),
        ("u_levels", ctypes.c_int64),
        ("u_outputs", ctypes.c_int64),
        ("u_entries", ctypes.c_int64),
        ("sdual_segments", ctypes.c_int64),
        ("sdual_iterations", ctypes.c_int64),
    ]


KERNEL_NAMES = ["pricing", "update_row", "primal_norms", "rc_update", "tri_solve",
                "col_norms", "spmv_rows", "single_row", "dual_ratio", "readback",
                "tri_solve_tau", "tri_solve_l", "tri_solve_t", "tri_solve_upper", "sdual",
                "exchange"]

# Names of every exported entry point of include/mi_lp.h (checked by tests).
EXPORTED_SYMBOLS = [
    "mi_glop_params_default", "mi_lp_device_count", "mi_lp_shutdown", "mi_lp_create",
    "mi_lp_destroy", "mi_lp_last_error", "mi_lp_set_params", "mi_lp_load",
    "mi_lp_load_basis_state", "mi_lp_clear_basis_state",
    "mi_lp_notify_matrix_unchanged", "mi_lp_solve", "mi_lp_get_primal",
    "mi_lp_get_reduced_costs", "mi_lp_get_duals", "mi_lp_get_activities",
    "mi_lp_get_statuses", "mi_lp_get_basis", "mi_lp_get_state",
    "mi_lp_get_primal_ray", "mi_lp_get_dual_ray",
    "mi_lp_get_dual_ray_row_combination", "mi_lp_begin", "mi_lp_run_until",
    "mi_lp_finish", "mi_lp_stop", "mi_lp_get_kernel_stats", "mi_lp_reset_kernel_stats",
    "mi_lp_set_kernel_timing", "mi_lp_set_kernel_timing_ids", "mi_lp_batch_solve", "mi_lp_set_variable_bounds",
    "mi_lp_batch_solve_bounds", "mi_lp_notify_matrix_changed",
    "mi_lp_set_starting_variable_values", "mi_lp_set_integrality_scale",
    "mi_lp_objective_limit_reached", "mi_lp_get_unit_row_left_inverse",
    "mi_lp_compute_dictionary", "mi_lp_get_dictionary",
    "mi_mps_read_file", "mi_mps_parse_string", "mi_mps_error", "mi_mps_dims", "mi_mps_get",
    "mi_mps_name", "mi_mps_col_name", "mi_mps_row_name", "mi_mps_free",
    "mi_lp_solver_params_default", "mi_lp_scale", "mi_lp_solver_solve",
    "mi_lp_clear_integrality_scales", "mi_lp_record_iteration_times",
    "mi_lp_get_iteration_times", "mi_lp_get_run_counters", "mi_lp_set_exchange",
    "mi_exchange_open", "mi_exchange_allgather", "mi_exchange_close",
    "mi_lp_batch_solve_gpus", "mi_lp_solver_solve_with",
    "mi_presolve_create", "mi_presolve_destroy", "mi_presolve_run", "mi_presolve_dims",
    "mi_presolve_get", "mi_presolve_recover", "mi_presolve_num_passes", "mi_presolve_pass_name",
    "mi_lp_comm_get_unique_id", "mi_lp_comm_create", "mi_lp_comm_rank", "mi_lp_comm_size",
    "mi_lp_share_bound", "mi_lp_comm_allreduce_device", "mi_lp_comm_allgather_device",
    "mi_lp_comm_last_error", "mi_lp_comm_destroy",
]


class MiLpSolverParams(ctypes.Structure):
    """include/mi_lp.h mi_lp_solver_params: the GlopParameters fields that
    glop::LPSolver and its presolve read around the simplex (parameters.proto
    field numbers 16, 57, 60, 24, 199; presolve 34, 67, 20, 21, 39, 22, 52)."""
    _fields_ = [
        ("use_scaling", ctypes.c_int32),
        ("scaling_method", ctypes.c_int32),
        ("cost_scaling", ctypes.c_int32),
        ("provide_strong_optimal_guarantee", ctypes.c_int32),
        ("max_valid_magnitude", ctypes.c_double),
        ("use_preprocessing", ctypes.c_int32),
        ("use_implied_free_preprocessor", ctypes.c_int32),
        ("solve_dual_problem", ctypes.c_int32),
        ("change_status_to_imprecise", ctypes.c_int32),
        ("dualizer_threshold", ctypes.c_double),
        ("preprocessor_zero_tolerance", ctypes.c_double),
        ("solution_feasibility_tolerance", ctypes.c_double),
        ("drop_tolerance", ctypes.c_double),
    ]


# GlopParameters::ScalingAlgorithm / CostScalingAlgorithm (parameters.proto:34-36, 194-210)
SCALING_DEFAULT, EQUILIBRATION, LINEAR_PROGRAM = 0, 1, 2
NO_COST_SCALING, CONTAIN_ONE_COST_SCALING, MEAN_COST_SCALING, MEDIAN_COST_SCALING = 0, 1, 2, 3
# GlopParameters::SolverBehavior (parameters.proto:42-46)
ALWAYS_DO, NEVER_DO, LET_SOLVER_DECIDE = 0, 1, 2


def default_solver_params(**overrides):
    p = MiLpSolverParams(use_scaling=1, scaling_method=EQUILIBRATION,
                         cost_scaling=CONTAIN_ONE_COST_SCALING,
                         provide_strong_optimal_guarantee=1, max_valid_magnitude=1e30,
                         use_preprocessing=1, use_implied_free_preprocessor=1,
                         solve_dual_problem=LET_SOLVER_DECIDE, dualizer_threshold=1.5,
                         preprocessor_zero_tolerance=1e-9, solution_feasibility_tolerance=1e-6,
                         drop_tolerance=1e-14, change_status_to_imprecise=1)
    for k, v in overrides.items():
        if k not in dict(MiLpSolverParams._fields_):
            raise KeyError(f"unknown LPSolver parameter {k!r}")
        setattr(p, k, v)
    return p
