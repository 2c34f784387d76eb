/*
 * mi_lp.h -- C ABI of the MI355X revised-simplex LP engine (drop-in for Glop).
 *
 * Plain pointers and sizes only; no C++ or torch types cross this boundary.
 * Every entry point below replaces one piece of the Glop / MPSolver interface
 * of OR-Tools 9.7 (paths relative to the reference checkout):
 *
 *   mi_lp_create / mi_lp_destroy     glop::RevisedSimplex ctor/dtor
 *                                    (ortools/glop/revised_simplex.h:125-129)
 *   mi_lp_set_params                 RevisedSimplex::SetParameters
 *                                    (revised_simplex.h:132, .cc:3586-3593)
 *   mi_lp_load                       the LinearProgram handed to Solve()
 *                                    (revised_simplex.cc:139, lp_data.h:56);
 *                                    CSC, rows sorted per column, no explicit
 *                                    zeros (LinearProgram::IsCleanedUp,
 *                                    lp_solver.cc:185-191)
 *   mi_lp_load_basis_state           RevisedSimplex::LoadStateForNextSolve
 *                                    (revised_simplex.h:153, .cc:120-124)
 *   mi_lp_clear_basis_state          RevisedSimplex::ClearStateForNextSolve (.cc:114)
 *   mi_lp_notify_matrix_unchanged    NotifyThatMatrixIsUnchangedForNextSolve (.cc:131)
 *   mi_lp_solve                      RevisedSimplex::Solve (revised_simplex.cc:139-635)
 *                                    + the ProblemStatus mapping of
 *                                    LPSolver::RunRevisedSimplexIfNeeded
 *                                    (lp_solver.cc:591-658)
 *   mi_lp_get_*                      GetVariableValue / GetReducedCost /
 *                                    GetDualValue / GetConstraintActivity /
 *                                    GetVariableStatus / GetConstraintStatus /
 *                                    GetBasis / GetState / GetPrimalRay /
 *                                    GetDualRay / GetDualRayRowCombination
 *                                    (revised_simplex.h:172-239, .cc:637-713)
 *   mi_lp_begin / mi_lp_run_until /  the PrimalMinimize/DualMinimize loops
 *   mi_lp_finish                     (revised_simplex.cc:2751-3367) driven in
 *                                    bounded slices (benchmark harness only)
 *   mi_lp_batch_solve                CP-SAT's per-worker LP call-out
 *                                    (sat/linear_programming_constraint.cc:709-760)
 *                                    for many independent LPs at once
 *
 * Error codes mirror glop::Status::ErrorCode (ortools/glop/status.h:29-44).
 * Threading: one handle = one host thread = one HIP stream (RevisedSimplex is
 * not thread safe either).
 */
#ifndef MI_LP_H_
#define MI_LP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Opaque solver handle (one glop::RevisedSimplex + its device state). */
typedef struct mi_lp mi_lp;

/* glop::Status::ErrorCode (status.h:29-44) + ABI-level codes. */
enum {
  MI_LP_OK = 0,
  MI_LP_ERROR_LU = 1,
  MI_LP_ERROR_BOUND = 2,
  MI_LP_ERROR_NULL = 3,
  MI_LP_ERROR_INVALID_PROBLEM = 4,
  MI_LP_ERROR_DEVICE = 100, /* HIP runtime failure or missing GPU */
  MI_LP_ERROR_STATE = 101,  /* call out of order (e.g. getter before solve) */
  MI_LP_ERROR_INTERNAL = 102 /* host exception inside the engine (e.g. out of
                                memory); the handle stays usable */
};

/* glop::ProblemStatus (ortools/lp_data/lp_types.h:106-168). */
enum {
  MI_LP_OPTIMAL = 0,
  MI_LP_PRIMAL_INFEASIBLE = 1,
  MI_LP_DUAL_INFEASIBLE = 2,
  MI_LP_INFEASIBLE_OR_UNBOUNDED = 3,
  MI_LP_PRIMAL_UNBOUNDED = 4,
  MI_LP_DUAL_UNBOUNDED = 5,
  MI_LP_INIT = 6,
  MI_LP_PRIMAL_FEASIBLE = 7,
  MI_LP_DUAL_FEASIBLE = 8,
  MI_LP_ABNORMAL = 9,
  MI_LP_INVALID_PROBLEM = 10,
  MI_LP_IMPRECISE = 11
};

/* glop::VariableStatus / ConstraintStatus (lp_types.h:188-219). */
enum {
  MI_LP_BASIC = 0,
  MI_LP_FIXED_VALUE = 1,
  MI_LP_AT_LOWER_BOUND = 2,
  MI_LP_AT_UPPER_BOUND = 3,
  MI_LP_FREE = 4
};

/* GlopParameters enums (ortools/glop/parameters.proto:49-92). */
enum { MI_LP_DANTZIG = 0, MI_LP_STEEPEST_EDGE = 1, MI_LP_DEVEX = 2 };
enum { MI_LP_BASIS_NONE = 0, MI_LP_BASIS_BIXBY = 1, MI_LP_BASIS_TRIANGULAR = 2,
       MI_LP_BASIS_MAROS = 3 };

/* POD mirror of the GlopParameters fields read by RevisedSimplex
 * (ortools/glop/parameters.proto, field numbers in comments). Fill with
 * mi_glop_params_default() first; defaults are the proto defaults. */
typedef struct mi_glop_params {
  int32_t use_dual_simplex;                          /* 31, false  */
  int32_t feasibility_rule;                          /* 1, STEEPEST_EDGE */
  int32_t optimization_rule;                         /* 2, STEEPEST_EDGE */
  int32_t initial_basis;                             /* 17, TRIANGULAR */
  int32_t use_transposed_matrix;                     /* 18, true */
  int32_t basis_refactorization_period;              /* 19, 64 */
  int32_t dynamically_adjust_refactorization_period; /* 63, true */
  int32_t change_status_to_imprecise;                /* 58, true */
  int32_t markowitz_zlatev_parameter;                /* 29, 3 */
  int32_t allow_simplex_algorithm_change;            /* 32, false */
  int32_t devex_weights_reset_period;                /* 33, 150 */
  int32_t use_middle_product_form_update;            /* 35, true; false = product-form etas
                                                        (async/inline tau off) */
  int32_t initialize_devex_with_column_norms;        /* 36, true */
  int32_t exploit_singleton_column_in_initial_basis; /* 37, true */
  int32_t random_seed;                               /* 43, 1 */
  int32_t perturb_costs_in_dual_simplex;             /* 53, false */
  int32_t use_dedicated_dual_feasibility_algorithm;  /* 62, true */
  int32_t push_to_vertex;                            /* 65, true */
  int32_t dual_price_prioritize_norm;                /* 69, false */
  int32_t use_scaling;                               /* 16, true (Bixby only) */
  int64_t max_number_of_iterations;                  /* 27, -1 */
  double refactorization_threshold;                  /* 6, 1e-9 */
  double recompute_reduced_costs_threshold;          /* 8, 1e-8 */
  double recompute_edges_norm_threshold;             /* 9, 100 */
  double primal_feasibility_tolerance;               /* 10, 1e-8 */
  double dual_feasibility_tolerance;                 /* 11, 1e-8 */
  double ratio_test_zero_threshold;                  /* 12, 1e-9 */
  double harris_tolerance_ratio;                     /* 13, 0.5 */
  double small_pivot_threshold;                      /* 14, 1e-6 */
  double minimum_acceptable_pivot;                   /* 15, 1e-6 */
  double drop_tolerance;                             /* 52, 1e-14 */
  double solution_feasibility_tolerance;             /* 22, 1e-6 */
  double max_number_of_reoptimizations;              /* 56, 40 */
  double lu_factorization_pivot_threshold;           /* 25, 0.01 */
  double max_time_in_seconds;                        /* 26, inf */
  double max_deterministic_time;                     /* 45, inf */
  double markowitz_singularity_threshold;            /* 30, 1e-15 */
  double dual_small_pivot_threshold;                 /* 38, 1e-4 */
  double objective_lower_limit;                      /* 40, -inf */
  double objective_upper_limit;                      /* 41, inf */
  double degenerate_ministep_factor;                 /* 42, 0.01 */
  double relative_cost_perturbation;                 /* 54, 1e-5 */
  double relative_max_cost_perturbation;             /* 55, 1e-7 */
  double initial_condition_number_threshold;         /* 59, 1e50 */
  double crossover_bound_snapping_distance;          /* 64, inf */
} mi_glop_params;

typedef struct mi_lp_result {
  int32_t problem_status; /* MI_LP_OPTIMAL ... */
  int32_t error_code;     /* MI_LP_OK ... (non-OK => problem_status ABNORMAL) */
  int64_t iterations;     /* RevisedSimplex::GetNumberOfIterations */
  double objective;       /* RevisedSimplex::GetObjectiveValue */
  double deterministic_time;
  double solve_seconds;   /* wall time of Solve() */
} mi_lp_result;

/* Per-kernel accounting kept by the engine (roofline bookkeeping). */
typedef struct mi_lp_kernel_stats {
  int64_t launches[16];
  double algorithmic_bytes[16];
  double device_ms[16]; /* HIP-event time, filled when timing is enabled */
  double call_ms[16];   /* host wall time of the whole device call: uploads,
                           launches, downloads, synchronization */
} mi_lp_kernel_stats;

enum {
  MI_K_PRICING = 0,     /* ComputeReducedCosts SpMV (reduced_costs.cc:352-423) */
  MI_K_UPDATE_ROW = 1,  /* UpdateRow column/row-wise (update_row.cc:196-306) */
  MI_K_PRIMAL_NORMS = 2,/* UpdateEdgeSquaredNorms (primal_edge_norms.cc:208-258) */
  MI_K_RC_UPDATE = 3,   /* UpdateReducedCosts (reduced_costs.cc:444-488) */
  MI_K_TRI_SOLVE = 4,   /* dense U solve of FTRAN, TriangularMatrix::TransposeLowerSolve
                           (sparse.cc:899-955, lu_factorization.cc:314-331) */
  MI_K_COL_NORMS = 5,   /* initial edge norms, identity basis (primal_edge_norms.cc:147-161) */
  MI_K_SPMV_ROWS = 6,   /* A x row sums: residual / basic values (variable_values.cc:101-133) */
  MI_K_SINGLE_ROW = 7,  /* ComputeUpdatesForSingleRow (update_row.cc:261-280) */
  MI_K_DUAL_RATIO = 8,  /* dual ratio-test candidate filter (entering_variable.cc:37-130) */
  MI_K_READBACK = 9,    /* update-row list download / single-coefficient reads */
  MI_K_TRI_SOLVE_TAU = 10, /* the same dense U solve for the tau FTRAN on the
                              factorization's worker thread (dual_edge_norms.cc:134-141) */
  MI_K_TRI_SOLVE_L = 11,   /* dense L solve of FTRAN (sparse.cc:793-812) on the device */
  MI_K_TRI_SOLVE_T = 12,   /* dense solves of BTRAN on the device: U^T (TransposeUpperSolve,
                              sparse.cc:848-897), L^T (TransposeLowerSolve), the unit-row U^T
                              (LowerSolveStartingAt, lu_factorization.cc:405-436) */
  MI_K_TRI_SOLVE_UPPER = 13, /* dense UpperSolve (sparse.cc:814-846): the product-form and
                                squared-norm FTRANs' U */
  MI_K_SDUAL = 14,      /* device dual simplex segment: whole phase-II dual iterations of one
                           LP on one workgroup (revised_simplex.cc:3058-3367); bytes = the
                           state arena moved in and out */
  MI_K_EXCHANGE = 15,   /* cross-process split joins (mi_lp_set_exchange): all-gathers, host
                           wall time, bytes gathered */
  MI_K_COUNT = 16
};

void mi_glop_params_default(mi_glop_params* p);

/* Returns the number of visible GPUs (0 on a host without one). */
int mi_lp_device_count(void);
/* Process teardown: drains the persistent batched-segment grids and joins the
 * engine's service threads (LU servers, batched-launch launchers) while the
 * HIP runtime is still up. Registered with atexit when the first such object
 * is created; hosts whose own teardown runs earlier (Python atexit, a plugin
 * unload) call it explicitly. Idempotent; later solves restart what they need.
 * (No Glop counterpart: Glop owns no threads or device state.) */
int mi_lp_shutdown(void);

int mi_lp_create(int device, mi_lp** out);
int mi_lp_destroy(mi_lp* h);
const char* mi_lp_last_error(const mi_lp* h);
int mi_lp_set_params(mi_lp* h, const mi_glop_params* p);

/* m constraints, n variables; A in CSC with n+1 col_starts. Bounds may be
 * +/-INFINITY. maximize != 0 => objective is maximized. */
int mi_lp_load(mi_lp* h, int32_t m, int32_t n, const int64_t* col_starts,
               const int32_t* row_idx, const double* vals, const double* col_lb,
               const double* col_ub, const double* row_lb, const double* row_ub,
               const double* obj, double obj_offset, double obj_scale,
               int32_t maximize);

/* statuses: n+m glop::VariableStatus values (structural then slacks). */
int mi_lp_load_basis_state(mi_lp* h, const int8_t* statuses, int32_t len);
int mi_lp_clear_basis_state(mi_lp* h);
/* Replaces the variable bounds of the loaded LP (n each); the matrix stays
 * resident in HBM. LinearProgram::SetVariableBounds as CP-SAT does before
 * each LP solve (sat/linear_programming_constraint.cc:412, 512, 535, 705). */
int mi_lp_set_variable_bounds(mi_lp* h, const double* col_lb, const double* col_ub);
int mi_lp_notify_matrix_unchanged(mi_lp* h);

/* CP-SAT's calls on the RevisedSimplex it keeps per LP constraint
 * (sat/linear_programming_constraint.cc:319,430,1247,1264):
 *   mi_lp_notify_matrix_changed          NotifyThatMatrixIsChangedForNextSolve
 *                                        (revised_simplex.h:169, .cc:135)
 *   mi_lp_set_starting_variable_values   SetStartingVariableValuesForNextSolve
 *                                        (revised_simplex.h:161, .cc:126); n+m values
 *   mi_lp_set_integrality_scale          SetIntegralityScale (revised_simplex.h:237,
 *                                        .cc:2588); a later OPTIMAL solve then runs
 *                                        Polish() (.cc:341-344, 2595-2734)
 *   mi_lp_objective_limit_reached        objective_limit_reached (revised_simplex.h:186)
 *   mi_lp_get_unit_row_left_inverse      GetUnitRowLeftInverse (revised_simplex.h:209):
 *                                        e_row^T B^-1 of the current basis, m dense
 *                                        values + its non-zero rows (non_zeros may be
 *                                        NULL; an empty list means "dense")
 *   mi_lp_compute_dictionary /           ComputeDictionary (revised_simplex.h:226,
 *   mi_lp_get_dictionary                 .cc:3785): B^-1 A row by row, scaled by
 *                                        column_scales (NULL: unscaled); the first call
 *                                        returns the entry count, the second copies
 *                                        row_starts (m+1), cols and values out. */
int mi_lp_notify_matrix_changed(mi_lp* h);
int mi_lp_set_starting_variable_values(mi_lp* h, const double* values, int32_t len);
int mi_lp_set_integrality_scale(mi_lp* h, int32_t col, double scale);
/* RevisedSimplex::ClearIntegralityScales (revised_simplex.h:236), called by
 * sat/linear_programming_constraint.cc:424 before it sets the scales again. */
int mi_lp_clear_integrality_scales(mi_lp* h);
int mi_lp_objective_limit_reached(const mi_lp* h, int32_t* reached);
int mi_lp_get_unit_row_left_inverse(mi_lp* h, int32_t row, double* values, int32_t* non_zeros,
                                    int32_t* num_non_zeros);
int mi_lp_compute_dictionary(mi_lp* h, const double* column_scales, int32_t scales_len,
                             int64_t* nnz);
int mi_lp_get_dictionary(const mi_lp* h, int64_t* row_starts, int32_t* cols, double* values);

/* interrupt may be NULL; a non-zero value stops the solve like a time limit
 * (glop_interface.cc:138-140). */
int mi_lp_solve(mi_lp* h, const volatile int32_t* interrupt, mi_lp_result* out);

int mi_lp_get_primal(const mi_lp* h, double* x);            /* n */
int mi_lp_get_reduced_costs(const mi_lp* h, double* rc);    /* n */
int mi_lp_get_duals(const mi_lp* h, double* y);             /* m */
int mi_lp_get_activities(const mi_lp* h, double* act);      /* m */
int mi_lp_get_statuses(const mi_lp* h, int8_t* var, int8_t* cons); /* n, m */
int mi_lp_get_basis(const mi_lp* h, int32_t* basis);        /* m, column ids */
int mi_lp_get_state(const mi_lp* h, int8_t* statuses);      /* n+m */
int mi_lp_get_primal_ray(const mi_lp* h, double* ray);      /* n+m */
int mi_lp_get_dual_ray(const mi_lp* h, double* ray);        /* m */
int mi_lp_get_dual_ray_row_combination(const mi_lp* h, double* v); /* n+m */

/* Benchmark slicing: mi_lp_begin starts Solve() on a worker thread that
 * parks when num_iterations reaches pause_at (negative = never).
 * mi_lp_run_until moves the pause point and blocks until the worker parks
 * again or finishes (*finished = 1); the device stream is synchronized
 * before it returns. mi_lp_finish joins and fills the result. */
int mi_lp_begin(mi_lp* h, int64_t pause_at);
int mi_lp_run_until(mi_lp* h, int64_t pause_at, int32_t* finished,
                    int64_t* iterations);
int mi_lp_finish(mi_lp* h, mi_lp_result* out);
/* Interrupts a begun solve at its next time-limit check (the interrupt flag
 * of glop_interface.cc:186-189); follow with mi_lp_finish. */
int mi_lp_stop(mi_lp* h);

int mi_lp_get_kernel_stats(const mi_lp* h, mi_lp_kernel_stats* s);
int mi_lp_reset_kernel_stats(mi_lp* h);
/* enable != 0: bracket every hot kernel with HIP events. The events are
 * read back when the stats are collected (or every 512 launches): timing adds
 * no synchronization to the iteration it measures. */
int mi_lp_set_kernel_timing(mi_lp* h, int32_t enable);
/* The same for the kernel ids whose bits are set in id_mask (bit k = id k of
 * mi_lp_kernel_stats; 0 = off): a benchmark times its dominant kernel
 * without paying two event records on every other launch. */
int mi_lp_set_kernel_timing_ids(mi_lp* h, uint32_t id_mask);

/* Window statistics for the benchmark harness (the reference keeps the same
 * numbers in RevisedSimplex's stats, revised_simplex.h:717-760, and
 * BasisFactorization's, basis_representation.h:359-373).
 * mi_lp_record_iteration_times: enable a timestamp (seconds since Solve()
 * started) per completed iteration; call before mi_lp_begin or while paused.
 * mi_lp_get_iteration_times copies min(cap, count) of them and returns count
 * (a negative error code when the solve is running). */
typedef struct mi_lp_run_counters {
  int64_t factorizations;       /* LU factorizations computed so far */
  double factorization_seconds; /* host wall time spent in them */
  int64_t iterations;           /* RevisedSimplex::GetNumberOfIterations */
  /* The device schedule of the current factorization's U (FTRAN's dense U
   * solve, 0 when none was built): dependency levels, computed outputs,
   * gather entries. A level is a dependency hop of the solve. */
  int64_t u_levels;
  int64_t u_outputs;
  int64_t u_entries;
  /* Device dual simplex segments (MILP_SDUAL; phase-II dual iterations run
   * whole on one workgroup) and the iterations they ran, since creation. */
  int64_t sdual_segments;
  int64_t sdual_iterations;
} mi_lp_run_counters;
int mi_lp_record_iteration_times(mi_lp* h, int32_t enable);
int64_t mi_lp_get_iteration_times(const mi_lp* h, double* out, int64_t cap);
int mi_lp_get_run_counters(const mi_lp* h, mi_lp_run_counters* c);

/* Cross-process split of ONE LP over `world` processes (the
 * reference's sharding pattern is pdlp/sharder.h:34-160): every process loads
 * the same LP into its handle and runs the same host control flow; process
 * `rank` keeps column block `rank` of [A | I] (64-aligned blocks balanced by
 * entries, as MILP_SHARDS cuts them) on its own GPU. Each per-column device
 * operation runs on the owned block, and its results are joined in block
 * order through `allgather`: the update row's list, the pricing reduced
 * costs, the dual ratio test's filtered breakpoints (the all-reduce(min) of
 * the bound is implicit: each block filters under its own bound, a superset
 * of the joint filter) and the entering column's coefficient. Results are
 * bit-identical to the unsplit engine. allgather(ctx, send, send_bytes, recv,
 * recv_bytes) must place every rank's bytes in rank order (recv_bytes[r]
 * bytes from rank r, all ranks' sizes known to the caller) and return 0.
 * Call before mi_lp_load; world <= 1 or allgather == NULL turns it off. */
typedef int (*mi_lp_allgather_fn)(void* ctx, const void* send, int64_t send_bytes, void* recv,
                                  const int64_t* recv_bytes);
int mi_lp_set_exchange(mi_lp* h, int32_t rank, int32_t world, void* ctx,
                       mi_lp_allgather_fn allgather);

/* Same-node exchange for mi_lp_set_exchange (engine/exchange.cc): an
 * all-gather of host bytes through one POSIX shared-memory segment, so the
 * split's per-iteration joins run in C++ with no Python and no socket on the
 * path (the joined messages are consumed by every rank's host control flow).
 * Rank 0 creates `name` (a fresh shm name, e.g. "/mi_lp_<uuid>", distributed
 * by the caller), the others attach; the name is unlinked once all `world`
 * ranks attached. Messages longer than slot_bytes go in several rounds.
 * Pass (ctx = the exchange, allgather = mi_exchange_allgather) to
 * mi_lp_set_exchange; close after the handle is done with it. */
typedef struct mi_exchange mi_exchange;
int mi_exchange_open(const char* name, int32_t rank, int32_t world, int64_t slot_bytes,
                     mi_exchange** out);
int mi_exchange_allgather(void* ctx, const void* send, int64_t send_bytes, void* recv,
                          const int64_t* recv_bytes);
void mi_exchange_close(mi_exchange* x);

/* Batch API: solves count independent LPs already loaded in handles (all on
 * the same device) on num_threads host threads; each thread drives several
 * LPs as fibers (MILP_BATCH_FIBERS, default 4) switching at device waits, and
 * their one-launch update rows go out in batched launches (one workgroup per
 * LP request; MILP_SMALL_BATCH=0 turns that off). Results are per LP and
 * identical to one-at-a-time solves.
 * Returns non-OK only for bad arguments; each LP's outcome (including its
 * error code) is in results[i]. No exception crosses this boundary. */
int mi_lp_batch_solve(mi_lp* const* handles, int32_t count, int32_t num_threads,
                      mi_lp_result* results);
/* mi_lp_batch_solve over several GPUs of one process (SURVEY 8(b)
 * mi_lp_batch_solve(hs, count, num_gpus, ...)): every handle's device must be
 * in [0, num_gpus); each device's handles run on a pool of threads_per_gpu
 * threads of their own, all devices at once. */
int mi_lp_batch_solve_gpus(mi_lp* const* handles, int32_t count, int32_t num_gpus,
                           int32_t threads_per_gpu, mi_lp_result* results);
/* Batched children of one search node: count LPs that share
 * the workers' loaded matrix and differ in variable bounds (lbs/ubs are
 * count x n, row-major), each warm-started from warm_state (n+m statuses,
 * may be NULL, else warm_len must be n+m) like LoadStateForNextSolve. The
 * workers may be on several GPUs; they run on at most 16 host threads
 * (MILP_BATCH_THREADS), dealt device by device, a thread's workers as fibers
 * with batched small-LP launches (as mi_lp_batch_solve), every worker pulling
 * the next child from one shared counter. A child whose bounds or state cannot be loaded is
 * not solved: results[i] = {ABNORMAL, that error code}. */
int mi_lp_batch_solve_bounds(mi_lp* const* workers, int32_t num_workers, int32_t count,
                             const double* lbs, const double* ubs, const int8_t* warm_state,
                             int32_t warm_len, mi_lp_result* results);

/* Multi-GPU bound sharing over RCCL: the batched LPs are
 * sharded across GPUs with no data-path collective; the one exchange is the
 * search's objective bound, an all-reduce(min) of one float64 over xGMI —
 * the cross-GPU analogue of SharedResponseManager::UpdateInnerObjectiveBounds
 * (ortools/sat/synchronization.h:306), which a CP-SAT worker thread calls
 * with its LP's bound. One communicator per rank (process or thread), bound
 * to a GPU; its unique id is created once (mi_lp_comm_get_unique_id, rank 0)
 * and handed to every rank out of band, as ncclGetUniqueId's. RCCL is ROCm's
 * librccl.so.1, opened privately (dlopen RTLD_LOCAL). Errors: MI_LP_ERROR_DEVICE
 * (message in mi_lp_comm_last_error; with c == NULL, why RCCL is unusable). */
typedef struct mi_lp_comm mi_lp_comm;
enum { MI_LP_COMM_ID_BYTES = 128 };
enum { MI_LP_BOUND_MIN = 0, MI_LP_BOUND_MAX = 1 };
int mi_lp_comm_get_unique_id(uint8_t* id /* MI_LP_COMM_ID_BYTES */);
/* Collective over the nranks ranks (ncclCommInitRank): blocks until all join. */
int mi_lp_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device,
                      mi_lp_comm** out);
int32_t mi_lp_comm_rank(const mi_lp_comm* c);
int32_t mi_lp_comm_size(const mi_lp_comm* c);
/* *bound <- min (MI_LP_BOUND_MIN) or max over the ranks of *bound: the value
 * goes through an 8-byte device buffer and one ncclAllReduce(ncclFloat64);
 * returns once the result is on the host. Every rank must call it. */
int mi_lp_share_bound(mi_lp_comm* c, double* bound, int32_t op);
/* The same reduction in place on a caller's device buffer of count doubles,
 * and an all-gather of bytes_per_rank bytes per rank between device buffers
 * (recv holds nranks blocks in rank order). Synchronous. */
int mi_lp_comm_allreduce_device(mi_lp_comm* c, double* d_values, int64_t count, int32_t op);
int mi_lp_comm_allgather_device(mi_lp_comm* c, const void* d_send, void* d_recv,
                                int64_t bytes_per_rank);
const char* mi_lp_comm_last_error(const mi_lp_comm* c);
void mi_lp_comm_destroy(mi_lp_comm* c);

/* MPS ingestion: the reader that fills the
 * LinearProgram handed to mi_lp_load, replacing
 *   glop::MPSReader::ParseFile / ParseString   (ortools/lp_data/mps_reader.h:39-60,
 *                                               mps_reader_template.h ParseFile)
 * with the LinearProgram data wrapper (mps_reader.cc:22-112). Formats as
 * MPSReaderFormat: auto-detection tries fixed, then free. On error the return
 * code is MI_LP_ERROR_INVALID_PROBLEM (absl::InvalidArgumentError upstream)
 * and mi_mps_error() holds the message; the model is always allocated and
 * must be released with mi_mps_free. The matrix comes back cleaned up (CSC,
 * rows sorted per column, no zeros), ready for mi_lp_load. */
typedef struct mi_mps_model mi_mps_model;
enum { MI_MPS_AUTO = 0, MI_MPS_FREE = 1, MI_MPS_FIXED = 2 };
int mi_mps_read_file(const char* path, int32_t format, mi_mps_model** out,
                     int32_t* format_used);
int mi_mps_parse_string(const char* text, int32_t format, mi_mps_model** out,
                        int32_t* format_used);
const char* mi_mps_error(const mi_mps_model* m);
int mi_mps_dims(const mi_mps_model* m, int32_t* num_rows, int32_t* num_cols, int64_t* nnz);
/* Any output pointer may be NULL. col_starts has num_cols + 1 entries. */
int mi_mps_get(const mi_mps_model* m, int64_t* col_starts, int32_t* row_idx, double* vals,
               double* col_lb, double* col_ub, double* row_lb, double* row_ub, double* obj,
               double* obj_offset, int32_t* maximize, int8_t* is_integer);
const char* mi_mps_name(const mi_mps_model* m);
const char* mi_mps_col_name(const mi_mps_model* m, int32_t col);
const char* mi_mps_row_name(const mi_mps_model* m, int32_t row);
void mi_mps_free(mi_mps_model* m);

/* LPSolver layer: what glop::LPSolver::SolveWithTimeLimit
 * (ortools/glop/lp_solver.cc:150-262) does around RevisedSimplex::Solve for
 * the MPSolver path (glop_interface.cc:104-169): IsCleanedUp / IsValid checks,
 * ScalingPreprocessor::Run (preprocessor.cc:3855-3876: SparseMatrixScaler
 * geometric + equilibration passes, matrix_scaler.cc; ScaleObjective /
 * ScaleBounds, lp_data.cc:1190-1258), the engine solve on handle h, then
 * ScalingPreprocessor::RecoverSolution (preprocessor.cc:3878-3912) and the
 * value part of LoadAndVerifySolution (lp_solver.cc:334-367: reduced costs,
 * Kahan objective, strong-optimal moves, activities). With use_preprocessing
 * (the default, as in Glop) MainLpPreprocessor's passes run before the
 * scaling and their postsolve after it (engine/presolve.cc),
 * and the postsolved solution goes through IsProblemSolutionConsistent
 * (lp_solver.cc:679-790; inconsistent = ABNORMAL). out->objective is the
 * unscaled problem objective; the arrays (n / m entries, any may be NULL)
 * are the unscaled solution. An invalid LP gives MI_LP_OK with
 * problem_status MI_LP_INVALID_PROBLEM, as LPSolver returns it. */
enum { MI_LP_SCALING_DEFAULT = 0, MI_LP_EQUILIBRATION = 1, MI_LP_LINEAR_PROGRAM = 2 };
enum { MI_LP_NO_COST_SCALING = 0, MI_LP_CONTAIN_ONE_COST_SCALING = 1,
       MI_LP_MEAN_COST_SCALING = 2, MI_LP_MEDIAN_COST_SCALING = 3 };
typedef struct mi_lp_solver_params {
  int32_t use_scaling;                      /* 16, true */
  int32_t scaling_method;                   /* 57, EQUILIBRATION (LINEAR_PROGRAM not built:
                                               geometric + equilibration, as upstream
                                               when its scaling LP fails) */
  int32_t cost_scaling;                     /* 60, CONTAIN_ONE_COST_SCALING */
  int32_t provide_strong_optimal_guarantee; /* 24, true */
  double max_valid_magnitude;               /* 199, 1e30 */
  /* Presolve: MainLpPreprocessor's passes (preprocessor.cc:76-147), on by
   * default as in Glop (parameters.proto:326); 0 = scaling only. DESIGN.md §6a. */
  int32_t use_preprocessing;                /* 34, true */
  int32_t use_implied_free_preprocessor;    /* 67, true */
  int32_t solve_dual_problem;               /* 20, LET_SOLVER_DECIDE (ALWAYS_DO 0,
                                               NEVER_DO 1, LET_SOLVER_DECIDE 2) */
  int32_t change_status_to_imprecise;       /* 58, true: LoadAndVerifySolution may
                                               report IMPRECISE */
  double dualizer_threshold;                /* 21, 1.5 */
  double preprocessor_zero_tolerance;       /* 39, 1e-9 */
  double solution_feasibility_tolerance;    /* 22, 1e-6 */
  double drop_tolerance;                    /* 52, 1e-14 */
} mi_lp_solver_params;
void mi_lp_solver_params_default(mi_lp_solver_params* p);
/* ScalingPreprocessor::Run alone, in place on the caller's arrays (no device
 * needed): row_scale (m) / col_scale (n) receive SparseMatrixScaler's
 * unscaling factors, *cost_factor / *bound_factor the divisors of
 * ScaleObjective / ScaleBounds. With use_scaling = 0 nothing changes and
 * every factor is 1. */
int mi_lp_scale(const mi_lp_solver_params* sp, int32_t m, int32_t n, const int64_t* col_starts,
                const int32_t* row_idx, double* vals, double* col_lb, double* col_ub,
                double* row_lb, double* row_ub, double* obj, double* obj_offset,
                double* obj_scale, double* row_scale, double* col_scale, double* cost_factor,
                double* bound_factor);
int mi_lp_solver_solve(mi_lp* h, const mi_lp_solver_params* sp, int32_t m, int32_t n,
                       const int64_t* col_starts, const int32_t* row_idx, const double* vals,
                       const double* col_lb, const double* col_ub, const double* row_lb,
                       const double* row_ub, const double* obj, double obj_offset,
                       double obj_scale, int32_t maximize, const volatile int32_t* interrupt,
                       mi_lp_result* out, double* primal, double* duals, double* reduced_costs,
                       double* activities, int8_t* var_status, int8_t* cons_status);

/* The same LPSolver flow with the simplex supplied by the caller
 * (LPSolver::RunRevisedSimplexIfNeeded, lp_solver.cc:591-658, is the call
 * site): fn receives the presolved and scaled LP, fills out (problem_status,
 * iterations, error_code) and the solution arrays (n primal values, m dual
 * values, n variable and m constraint statuses) and returns MI_LP_OK or an
 * error code, which is passed through. mi_lp_solver_solve is this with the
 * engine's handle behind fn. */
typedef int (*mi_lp_simplex_fn)(void* user, int32_t m, int32_t n, const int64_t* col_starts,
                                const int32_t* row_idx, const double* vals,
                                const double* col_lb, const double* col_ub,
                                const double* row_lb, const double* row_ub, const double* obj,
                                double obj_offset, double obj_scale, int32_t maximize,
                                mi_lp_result* out, double* primal, double* duals,
                                int8_t* var_status, int8_t* cons_status);
int mi_lp_solver_solve_with(mi_lp_simplex_fn fn, void* user, const mi_lp_solver_params* sp,
                            int32_t m, int32_t n, const int64_t* col_starts,
                            const int32_t* row_idx, const double* vals, const double* col_lb,
                            const double* col_ub, const double* row_lb, const double* row_ub,
                            const double* obj, double obj_offset, double obj_scale,
                            int32_t maximize, mi_lp_result* out, double* primal, double* duals,
                            double* reduced_costs, double* activities, int8_t* var_status,
                            int8_t* cons_status);

/* Presolve alone (host only, no device needed): MainLpPreprocessor's passes
 * (glop/preprocessor.cc:76-147, without the scaling) on a copy of the LP, and
 * DestructiveRecoverSolution (:203-209) for a solution of the presolved LP.
 *   mi_presolve_run       *status = Glop's status after presolve (MI_LP_INIT:
 *                         the simplex must run on the presolved LP;
 *                         MI_LP_INVALID_PROBLEM: IsValid failed, nothing ran)
 *   mi_presolve_dims      presolved sizes and direction (the dualizer turns
 *                         the LP into a maximization)
 *   mi_presolve_get       the presolved LP (any pointer may be NULL)
 *   mi_presolve_recover   solution of the presolved LP (its sizes) -> solution
 *                         of the original LP (original sizes); *status in/out
 *                         (the dualizer maps primal/dual statuses); once only
 *   mi_presolve_pass_name the passes that changed the LP, in order */
typedef struct mi_presolve mi_presolve;
mi_presolve* mi_presolve_create(void);
void mi_presolve_destroy(mi_presolve* ps);
int mi_presolve_run(mi_presolve* ps, const mi_lp_solver_params* sp, int32_t m, int32_t n,
                    const int64_t* col_starts, const int32_t* row_idx, const double* vals,
                    const double* col_lb, const double* col_ub, const double* row_lb,
                    const double* row_ub, const double* obj, double obj_offset, double obj_scale,
                    int32_t maximize, int32_t* status);
int mi_presolve_dims(const mi_presolve* ps, int32_t* m, int32_t* n, int64_t* nnz,
                     int32_t* maximize);
int mi_presolve_get(const mi_presolve* ps, int64_t* col_starts, int32_t* row_idx, double* vals,
                    double* col_lb, double* col_ub, double* row_lb, double* row_ub, double* obj,
                    double* obj_offset, double* obj_scale);
int mi_presolve_recover(mi_presolve* ps, int32_t* status, const double* primal,
                        const double* duals, const int8_t* var_status, const int8_t* cons_status,
                        double* primal_out, double* duals_out, int8_t* var_status_out,
                        int8_t* cons_status_out);
int32_t mi_presolve_num_passes(const mi_presolve* ps);
const char* mi_presolve_pass_name(const mi_presolve* ps, int32_t i);

#ifdef __cplusplus
}
#endif

#endif /* MI_LP_H_ */
