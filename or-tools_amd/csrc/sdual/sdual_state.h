// Device-resident dual simplex segment ("sdual"): the state of one LP.
//
// Glop's dual simplex iteration (revised_simplex.cc:3058-3367, the phase-II
// loop body and its helpers) runs as one workgroup per LP on the GPU. The host
// engine keeps everything that is not a plain iteration: Markowitz
// factorizations, the recomputations after them, phase changes, status
// decisions. At a segment boundary the host packs its state into this flat
// structure (sdual_bridge.inc), the device runs iterations until the loop needs
// the host again, and the host unpacks the state and continues at the
// matching point of its own loop (SdExit).
//
// Every array lives in one arena per LP (device memory on the GPU, host
// memory in the host build used by the CPU checks); the struct itself is the
// arena's header. Sizes: m rows, N = n + m columns. Glop's std::vector
// capacities become fixed capacities here; the host never starts a segment
// that could overflow them (sd_can_start).
#ifndef MILP_SDUAL_STATE_H_
#define MILP_SDUAL_STATE_H_

#include <stdint.h>

#if defined(__HIPCC__)
#define SD_HD __host__ __device__
#define SD_INLINE __host__ __device__ inline
#else
#define SD_HD
#define SD_INLINE inline
#endif

namespace sdual {

using f64 = double;

// ScatteredVector (lp_data/scattered_vector.h:61-177). `size` is
// values.size(); is_non_zero is all false between uses (as upstream).
struct Vec {
  f64* values;
  int size;
  int* nz;
  int nnz;
  int sorted;
  char* mask;
};

// DynamicMaximum<Index> (glop/pricing.h:58-345): values, the candidate
// bitset, the top-k cache with its threshold, and the equivalent-choices
// scratch (size + 1 entries).
struct DynMax {
  f64* values;
  uint64_t* cand;
  int size;  // values_.size()
  int ntops;
  f64 threshold;
  int32_t tops_idx[32];
  f64 tops_val[32];
  int32_t* equiv;
};

// CompactSparseMatrix read-only view (sparse.h:291-512).
struct Csc {
  const int64_t* starts;
  const int32_t* rows;
  const f64* coefs;
  int num_rows;
  int num_cols;
};

// TriangularMatrix (sparse.h:583-921): L, U and their transposes.
struct Tri {
  int64_t* starts;  // num_cols + 1
  int32_t* rows;
  f64* coefs;
  f64* diag;  // diagonal_coefficients_, size num_cols
  int num_rows;
  int num_cols;
  int first_non_identity;
  int all_ones;
  int64_t ncoefs;  // coefficients_.size() (num_entries() = num_cols + ncoefs)
  // Level schedule of the transposed (gather) solve over this matrix: the
  // columns of level k are lv_order[lv_starts[k] .. lv_starts[k + 1]) and
  // read only columns of earlier levels. num_levels < 0: no schedule.
  int32_t* lv_order;
  int32_t* lv_starts;
  int32_t num_levels;
  int32_t lv_pad;
};

// Growing CompactSparseMatrix (the MPF storages, basis_representation.h).
struct Store {
  int64_t* starts;  // cap_cols + 1
  int32_t* rows;
  f64* coefs;
  int num_rows;
  int num_cols;
  int cap_cols;
  int64_t cap_entries;
};

// Why the device handed the LP back, and where the host loop resumes
// (RevisedSimplex::DualMinimize, engine/simplex.cc).
enum SdExit : int32_t {
  kExitNone = 0,
  kExitLoopTop = 1,        // `refactorize = exit_refactorize; continue;`
  kExitNoLeaving = 2,      // leaving_row == kInvalidRow block
  kExitPrecision = 3,      // TestPrecision failed: UpdateDualPrices({row}); continue
  kExitNoEntering = 4,     // entering_col == kInvalidCol block
  kExitReturnOk = 5,       // iteration or deterministic limit: return OK
  kExitPivotRefactor = 6,  // UpdateAndPivot must refactorize (host Markowitz)
  kExitLuError = 7,        // degenerate rank-one update / LU failure: return error
  kExitCapacity = 8,       // a fixed capacity would overflow: resume at loop top
  kExitOptimal = 9,        // no leaving row on a fresh factorization: OPTIMAL
  kExitObjectiveLimit = 10,  // DUAL_FEASIBLE, objective limit reached
  // The host already refactorized (its LU did not fit the arena): resume
  // after RefactorizeBasisIfNeeded's factorization with old_refactorize =
  // exit_refactorize, or after UpdateAndPivot's.
  kExitResumeTop = 11,
  kExitResumePivot = 12,
  // Primal segment: a final status (exit_status: ProblemStatus), and an
  // unbounded ray (the host builds it from the direction).
  kExitStatus = 13,
  kExitUnbounded = 14,
};

// The factorization as the device stores it: a header followed by its arrays;
// array pointers are offsets from the header until installed (sd_install_lu).
struct LuImage {
  int64_t bytes;
  int32_t status;  // 0 OK, 1 LU error, 2 did not fit
  int32_t is_identity;
  int32_t col_perm_empty;
  int32_t pad;
  double last_fact_dtime;
  Tri lower, upper, tupper, tlower;
  int64_t off_col_perm, off_inv_col_perm, off_row_perm, off_inv_row_perm;
};

// Host <-> running kernel requests (pinned, mapped): the device asks for a
// Markowitz factorization of its basis; the host answers with an LuImage.
struct Mailbox {
  int32_t flag;  // 0 idle, 1 request, 2 answer ready
  int32_t bump;  // UpdateAndPivot raised the LU pivot threshold first
  int64_t image_cap;
};

struct Lp {
  // ---- problem (read-only during a segment) ----
  int m;  // rows
  int N;  // columns of [A | I]
  Csc A;  // compact_matrix_
  Csc At; // transposed_matrix_ (num_cols = m)
  f64* objective;  // objective_ (rewritten by the primal phase-I costs)

  // ---- parameters (GlopParameters subset) ----
  f64 drop_tolerance;
  f64 primal_feasibility_tolerance;
  f64 recompute_edges_norm_threshold;
  f64 minimum_acceptable_pivot;
  f64 ratio_test_zero_threshold;
  f64 harris_tolerance_ratio;
  f64 degenerate_ministep_factor;
  f64 dual_small_pivot_threshold;
  f64 small_pivot_threshold;
  f64 refactorization_threshold;
  f64 lu_factorization_pivot_threshold;
  int use_transposed_matrix;
  int put_more_importance_on_norm;  // VariableValues::put_more_importance_on_norm_
  int dual_price_prioritize_norm;   // GlopParameters
  int64_t max_number_of_iterations;

  // ---- VariablesInfo ----
  f64* lb;
  f64* ub;
  int8_t* vtype;
  int8_t* vstatus;
  uint64_t* can_inc;
  uint64_t* can_dec;
  uint64_t* relevant;
  uint64_t* is_basic;
  uint64_t* not_basic;
  uint64_t* boxed;
  int nwords;  // (N + 63) / 64
  int64_t num_entries_relevant;
  int boxed_relevant;

  int32_t* basis;
  f64* x;  // VariableValues::variable_values_

  // ---- ReducedCosts ----
  f64* rc;
  f64* cost_pert;
  f64* basic_obj;
  int must_refactorize;
  int recompute_bo_left_inverse;
  int recompute_bo;
  int recompute_rc;
  int rc_precise;
  int rc_recomputed;
  int has_cost_shift;
  f64 dual_tol;
  f64 rc_dtime;

  // ---- DualEdgeNorms ----
  f64* norms;
  int norms_recompute;

  // ---- DynamicMaximum dual_prices_ (pricing.h:58-345) over the rows ----
  DynMax dp;

  // ---- UpdateRow ----
  Vec rho;
  int32_t* rho_filtered;
  int n_rho_filtered;
  int32_t* nzpos;  // non_zero_position_list_
  int n_nzpos;
  uint64_t* nzset;  // non_zero_position_set_ (nwords)
  f64* coeff;       // coefficient_ (N)
  char* col_flag;   // column-wise pass scratch (N, zero between uses)
  int left_inv_for;
  int urow_for;
  int64_t ur_ops;
  int last_alg;

  // ---- EnteringVariable ----
  int64_t ent_ops;
  int32_t* bp_col;  // breakpoints_ heap (N)
  f64* bp_ratio;
  f64* bp_mag;
  int32_t* ent_equiv;  // equivalent_entering_choices_ (N + 1)

  // ---- RevisedSimplex ----
  Vec dir;
  f64 dir_inf_norm;
  int32_t* flips;  // bound_flip_candidates_ (N)
  int n_flips;
  int32_t* changed_cols;  // MakeBoxedVariableDualFeasible scratch (N)
  Vec ia0;                // VariableValues::initially_all_zero_scratchpad_
  int64_t num_iterations;
  int64_t num_update_price_ops;
  f64 primal_norms_dtime;  // PrimalEdgeNorms::DeterministicTime() (constant here)
  f64 last_det_update;     // last_deterministic_time_update_
  f64 tl_det_elapsed;      // TimeLimit deterministic elapsed
  f64 tl_det_max;          // max_deterministic_time

  // ---- LuFactorization ----
  Tri lower, upper, tupper, tlower;
  int32_t* col_perm;  // empty when col_perm_empty
  int32_t* inv_col_perm;
  int32_t* row_perm;
  int32_t* inv_row_perm;
  int col_perm_empty;
  int is_identity;
  f64* zero_scratch;  // dense_zero_scratchpad_ (zero between uses)
  char* stored;       // TriangularMatrix::stored_ (false between uses)
  int32_t* col_u_rows;  // column_of_upper_ (m + 1)
  f64* col_u_coefs;
  int n_col_u;

  // ---- BasisFactorization (MPF) ----
  int num_updates;
  int max_updates;
  int dynamic_period;
  int tau_is_computed;
  int tau_can_opt;
  Vec tau;
  f64 last_fact_dtime;
  f64 bf_dtime;
  int32_t* left_pool;   // left_pool_mapping_ (m, -1 = none)
  int32_t* right_pool;  // right_pool_mapping_ (N, -1 = none)
  Store storage;
  Store right_storage;
  f64* mpf_scratch;  // scratchpad_ (m, zero between uses)
  int32_t* mpf_scratch_nz;  // scratchpad_non_zeros_ (2m)
  int n_mpf_scratch_nz;

  // ---- EtaFactorization (basis_representation.cc:25-176): the product-form
  // updates used instead of the MPF when use_middle_product_form_update is
  // false (mpf == 0). Eta k: its column (the leaving row), the pivot, the
  // dense coefficients (m, eta column zeroed) and, when the direction was
  // sparse (< 0.5 m non-zeros), its entries in list order.
  int mpf;
  int eta_count;
  int eta_cap;
  int eta_pad;
  int32_t* eta_col;
  f64* eta_piv;
  f64* eta_dense;          // eta_cap x m
  int64_t* eta_sp_starts;  // eta_cap + 1; an empty range = the dense loops
  int32_t* eta_sp_rows;
  f64* eta_sp_coefs;
  int64_t eta_sp_cap;
  f64* pfi_scratch;        // LuFactorization::dense_column_scratchpad_ (m)

  // ---- RankOneUpdateFactorization ----
  int32_t* r1_u;
  int32_t* r1_v;
  f64* r1_mu;
  int r1_count;
  int r1_cap;
  int64_t r1_num_entries;
  f64 r1_dtime;

  // ---- std::mt19937_64 (libstdc++ layout: _M_x[312], _M_p) ----
  uint64_t mt[312];
  uint64_t mti;

  // ---- refactorization service ----
  char* lu_region;  // installed LuImage (arena)
  int64_t lu_cap;
  Mailbox* mb;       // mapped host memory (device mode)
  int32_t* mb_basis; // m entries
  char* mb_image;    // LuImage written by the host
  // Host mode: computes the factorization of s->basis into s->lu_region;
  // returns the LuImage status.
  int (*lu_service)(void* ctx, Lp* s, int bump);
  void* lu_ctx;
  // Host mode debugging aid: called at OnIterationDone.
  void (*trace)(const Lp* s);

  // ---- state the post-factorization block uses ----
  Vec bolinv;     // ReducedCosts::basic_objective_left_inverse_
  Vec vv_scratch; // VariableValues::scratchpad_
  f64 dual_feasibility_tolerance;
  int64_t a_num_entries;
  f64* dpv;  // dual_pricing_vector_ (the phase-I prices, permuted with the basis)
  int dpv_size;
  int phase_optimization;
  // ---- dual phase I (DualMinimize(feasibility_phase = true)) ----
  int dual_phase1;  // the segment runs the phase-I loop (revised_simplex.cc:2198-2388)
  int n_dual_inf;   // num_dual_infeasible_positions_
  int diid_size;    // dual_infeasibility_improvement_direction_.size(): 0 or N
  int dp1_pad;
  f64* diid;        // dual_infeasibility_improvement_direction_ (N)
  f64 dual_objective_limit;
  int objective_limit_reached;
  int rc_notify;  // SetRecomputeReducedCostsAndNotifyWatchers ran
  int64_t factorizations;  // served during the segment

  // ---- transfers of the pooled path (the workgroup moves its own arena) ----
  uint64_t arena_dev;    // device address of this header's arena
  uint64_t staging_dev;  // device view of the pinned staging image
  // Arena layout: [header][scratch][mutable][read-only][LU image][storages]:
  // the header and [mutable_begin, in_end) move in, the scratch is zeroed on
  // the device, the header and [mutable_begin, mutable_end) move out (plus
  // the storages' used prefixes both ways).
  int64_t scratch_begin;
  int64_t scratch_end;
  int64_t mutable_begin;
  int64_t fixed_end;     // in_end: the LU image's last used byte
  int64_t mutable_end;
  f64* coeff_out;        // DeviceLp's update-row coefficients (N), refreshed at the end
  // Device time per loop phase (wall_clock64 ticks, 100 MHz): see sd_run
  // (0-8 loop phases, 9-15 sub-phases and transfers, 16-31 finer
  // sub-phases, sdual_bridge.inc names them).
  uint64_t phase_ticks[32];
  // The workgroup's LDS scratch (set by the kernel before sd_run; null on the
  // host): dense vectors of the triangular sweeps are staged there.
  f64* lds;
  int32_t lds_doubles;
  int32_t lds_pad;
  f64* lds_scratch;  // SdScratch after the staging area (device only)
  int32_t lds_busy;  // a solve's working vector occupies the staging area
  int32_t lds_pad2;

  // ---- primal segment (PrimalMinimize, revised_simplex.cc:2751-3045) ----
  int primal;             // the segment runs the primal loop (sp_run)
  int phase_feasibility;  // phase_ == FEASIBILITY: phase-I costs
  f64 primal_objective_limit;
  f64 recompute_reduced_costs_threshold;
  // PrimalPrices (reduced_costs.cc:512-600): a DynamicMaximum over columns.
  DynMax pp;
  int pp_recompute;
  // PrimalEdgeNorms (primal_edge_norms.cc), steepest edge.
  int pen_recompute;  // recompute_edge_squared_norms_
  int pen_pad;
  f64* pen_norms;     // edge_squared_norms_ (N)
  int64_t pen_ops;    // num_operations_
  Vec dli;            // direction_left_inverse_
  // Ratio-test scratch: Harris leaving candidates (m), phase-I breakpoints
  // (2m + 2: row, ratio, magnitude, target bound).
  int32_t* lc_row;
  f64* lc_ratio;
  int32_t* bp1_row;
  f64* bp1_ratio;
  f64* bp1_mag;
  f64* bp1_target;
  int32_t exit_status;  // kExitStatus: the ProblemStatus
  int32_t exit_entering;
  f64 exit_reduced_cost;

  // ---- loop carry and exit ----
  int refactorize;  // the host loop's `refactorize` flag
  int32_t exit_code;
  int32_t exit_row;       // leaving_row at the exit
  int32_t exit_col;       // leaving_col (kExitPivotRefactor) / entering_col
  int32_t exit_lu_bump;   // UpdateAndPivot raised the LU pivot threshold
  f64 exit_cost_variation;
  f64 exit_target_bound;
  int64_t iterations_done;  // this segment
  int64_t iteration_cap;    // stop after this many (0 = no cap)
};

}  // namespace sdual

#endif  // MILP_SDUAL_STATE_H_
