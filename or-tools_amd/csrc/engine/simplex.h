// Types shared by the MI355X simplex engine (simplex.cc): GlopParameters
// mirror, LinearProgram input, TimeLimit, RNG helpers, DynamicMaximum and
// VariablesInfo, following OR-Tools 9.7 ortools/glop (file:line per class).
#ifndef MILP_SIMPLEX_H_
#define MILP_SIMPLEX_H_

#include <chrono>
#include <random>

#include "lu.h"

namespace milp {

// GlopParameters subset (parameters.proto); field meaning mirrors
// include/mi_lp.h mi_glop_params.
struct GlopParameters {
  bool use_dual_simplex = false;
  int feasibility_rule = 1;   // STEEPEST_EDGE
  int optimization_rule = 1;  // STEEPEST_EDGE
  int initial_basis = 2;      // TRIANGULAR
  bool use_transposed_matrix = true;
  int basis_refactorization_period = 64;
  bool dynamically_adjust_refactorization_period = true;
  bool change_status_to_imprecise = true;
  int markowitz_zlatev_parameter = 3;
  bool allow_simplex_algorithm_change = false;
  int devex_weights_reset_period = 150;
  bool use_middle_product_form_update = true;
  bool initialize_devex_with_column_norms = true;
  bool exploit_singleton_column_in_initial_basis = true;
  int random_seed = 1;
  bool perturb_costs_in_dual_simplex = false;
  bool use_dedicated_dual_feasibility_algorithm = true;
  bool push_to_vertex = true;
  bool dual_price_prioritize_norm = false;
  bool use_scaling = true;
  int64_t max_number_of_iterations = -1;
  double refactorization_threshold = 1e-9;
  double recompute_reduced_costs_threshold = 1e-8;
  double recompute_edges_norm_threshold = 100.0;
  double primal_feasibility_tolerance = 1e-8;
  double dual_feasibility_tolerance = 1e-8;
  double ratio_test_zero_threshold = 1e-9;
  double harris_tolerance_ratio = 0.5;
  double small_pivot_threshold = 1e-6;
  double minimum_acceptable_pivot = 1e-6;
  double drop_tolerance = 1e-14;
  double solution_feasibility_tolerance = 1e-6;
  double max_number_of_reoptimizations = 40;
  double lu_factorization_pivot_threshold = 0.01;
  double max_time_in_seconds = kInfinity;
  double max_deterministic_time = kInfinity;
  double markowitz_singularity_threshold = 1e-15;
  double dual_small_pivot_threshold = 1e-4;
  double objective_lower_limit = -kInfinity;
  double objective_upper_limit = kInfinity;
  double degenerate_ministep_factor = 0.01;
  double relative_cost_perturbation = 1e-5;
  double relative_max_cost_perturbation = 1e-7;
  double initial_condition_number_threshold = 1e50;
  double crossover_bound_snapping_distance = kInfinity;

  LuParameters lu() const {
    LuParameters p;
    p.markowitz_singularity_threshold = markowitz_singularity_threshold;
    p.markowitz_zlatev_parameter = markowitz_zlatev_parameter;
    p.lu_factorization_pivot_threshold = lu_factorization_pivot_threshold;
    return p;
  }
};

// The LinearProgram handed to Solve(): A (m x n, CSC, cleaned up), bounds,
// objective (lp_data/lp_data.h:56-529 subset).
struct LinearProgram {
  int m = 0, n = 0;
  std::vector<int64_t> col_starts;
  std::vector<int32_t> row_idx;
  std::vector<double> vals;
  std::vector<double> col_lb, col_ub, row_lb, row_ub, obj;
  double obj_offset = 0.0;
  double obj_scale = 1.0;
  bool maximize = false;
  // Hash of (m, n, col_starts, row_idx, vals) set at load: the batch caches
  // are shared only between handles whose matrices hash alike.
  uint64_t matrix_fingerprint = 0;
};

// util/time_limit.h subset: wall clock + deterministic time + interrupt.
struct TimeLimit {
  double max_seconds = kInfinity;
  double max_deterministic = kInfinity;
  const volatile int32_t* interrupt = nullptr;
  double deterministic_elapsed = 0.0;
  std::chrono::steady_clock::time_point start = std::chrono::steady_clock::now();
  double GetElapsedTime() const {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - start)
        .count();
  }
  void AdvanceDeterministicTime(double d) { deterministic_elapsed += d; }
  bool LimitReached() const {
    if (interrupt != nullptr && *interrupt != 0) return true;
    if (deterministic_elapsed > max_deterministic) return true;
    return max_seconds < kInfinity && GetElapsedTime() > max_seconds;
  }
};

using Rng = std::mt19937_64;  // util/random_engine.h:23

// absl::Bernoulli(gen, p) as published in abseil-cpp 20230125.3
// (absl/random/bernoulli_distribution.h): one 32-bit variate from
// FastUniformBits (= low 32 bits of one mt19937_64 draw), fast-path compare
// against p*2^32. No reference test pins this stream: PARITY UNPINNED here.
inline bool AbslBernoulli(Rng& g, double p) {
  const double kP32 = 4294967296.0;
  while (true) {
    const uint64_t c = static_cast<uint64_t>(static_cast<int64_t>(p * kP32));
    const uint32_t v = static_cast<uint32_t>(g());
    if (v != c) return v < c;
    const double q = static_cast<double>(c) / kP32;
    const double here = (p - q) * kP32;
    if (here == 0) return false;
    p = here;
  }
}
inline int UniformInt(Rng& g, int hi) {  // std::uniform_int_distribution<int>(0, hi)
  return std::uniform_int_distribution<int>(0, hi)(g);
}

// pricing.h:58-345 DynamicMaximum.
class DynamicMaximum {
  friend struct SdualBridge;

 public:
  explicit DynamicMaximum(Rng* random) : random_(random) {}
  void ClearAndResize(int n) {
    tops_.clear();
    threshold_ = -kInfinity;
    values_.resize(n);
    is_candidate_.ClearAndResize(n);
  }
  void Clear() { ClearAndResize(0); }
  int Size() const { return static_cast<int>(values_.size()); }
  void Remove(int position) { is_candidate_.Clear(position); }
  void StartDenseUpdates() {
    tops_.clear();
    threshold_ = kInfinity;
  }
  void DenseAddOrUpdate(int position, Fractional value) {
    is_candidate_.Set(position);
    values_[position] = value;
  }
  void AddOrUpdate(int position, Fractional value) {
    is_candidate_.Set(position);
    values_[position] = value;
    if (value >= threshold_) UpdateTopK(position, value);
  }
  // AddOrUpdate on a state that is cleared (ClearAndResize) before it is
  // read again: only the top-k bookkeeping, which may draw from the RNG
  // (pricing.h:303-307), has an effect that outlives the clear.
  void AddOrUpdateBeforeClear(int position, Fractional value) {
    if (value >= threshold_) UpdateTopK(position, value);
  }
  int GetMaximum();
  // Bulk access for the parallel host loops (host_pool.h): the values and
  // candidate bits are written element by element in parallel, then the
  // top-k bookkeeping of each AddOrUpdate is replayed serially, in order.
  Fractional* mutable_values() { return values_.data(); }
  uint64_t* mutable_candidate_words() { return is_candidate_.mutable_data(); }
  void ReplayTopK(int position, Fractional value) {
    if (value >= threshold_) UpdateTopK(position, value);
  }

 private:
  struct HeapElement {
    int index;
    Fractional value;
  };
  struct HeapLess {  // pricing.h:148-150: min-heap on value.
    bool operator()(const HeapElement& a, const HeapElement& b) const {
      return a.value > b.value;
    }
  };
  void UpdateTopK(int position, Fractional value);
  int RandomizeIfManyChoices(int best);
  // GetMaximum's full scan: the candidates it acts on, found by the host
  // pool (false: scan serially).
  bool ScanCandidatesInParallel(std::vector<int>* processed) const;

 public:
  // For k in [0, n): keep[k] ? AddOrUpdate(pos[k], value[k]) : Remove(pos[k]),
  // the positions distinct. Long lists on a full top-k run the writes in
  // parallel and replay only the AddOrUpdates that reach UpdateTopK, in
  // order (the same heap operations and RNG draws as the loop).
  void BulkAddOrUpdate(const int* pos, const Fractional* value, const uint8_t* keep, size_t n);

 private:

  Rng* random_;
  std::vector<int> equivalent_choices_;
  std::vector<Fractional> values_;
  Bitset is_candidate_;
  Fractional threshold_ = -kInfinity;
  std::vector<HeapElement> tops_;
};

// variables_info.{h,cc}
class VariablesInfo {
  friend struct SdualBridge;

 public:
  explicit VariablesInfo(const CompactSparseMatrix& m) : matrix_(m) {}
  bool LoadBoundsAndReturnTrueIfUnchanged(const std::vector<double>& vlb,
                                          const std::vector<double>& vub,
                                          const std::vector<double>& clb,
                                          const std::vector<double>& cub);
  void InitializeFromBasisState(int first_slack_col, int num_new_cols,
                                const std::vector<VariableStatus>& state);
  int ChangeUnusedBasicVariablesToFree(const std::vector<int>& basis);
  int SnapFreeVariablesToBound(Fractional distance,
                               const std::vector<Fractional>& starting_values);
  void InitializeToDefaultStatus();
  VariableStatus DefaultVariableStatus(int col) const;
  void MakeBoxedVariableRelevant(bool value);
  void UpdateToBasicStatus(int col);
  void UpdateToNonBasicStatus(int col, VariableStatus status);
  void TransformToDualPhaseIProblem(Fractional tol, const std::vector<Fractional>& rc);
  void EndDualPhaseI(Fractional tol, const std::vector<Fractional>& rc);

  const std::vector<VariableType>& GetTypeRow() const { return variable_type_; }
  const std::vector<VariableStatus>& GetStatusRow() const { return variable_status_; }
  const Bitset& GetCanIncreaseBitRow() const { return can_increase_; }
  const Bitset& GetCanDecreaseBitRow() const { return can_decrease_; }
  const Bitset& GetIsRelevantBitRow() const { return relevance_; }
  const Bitset& GetIsBasicBitRow() const { return is_basic_; }
  const Bitset& GetNotBasicBitRow() const { return not_basic_; }
  const Bitset& GetNonBasicBoxedVariables() const { return non_basic_boxed_variables_; }
  int64_t GetNumEntriesInRelevantColumns() const { return num_entries_in_relevant_columns_; }
  const std::vector<Fractional>& GetVariableLowerBounds() const { return lower_bounds_; }
  const std::vector<Fractional>& GetVariableUpperBounds() const { return upper_bounds_; }
  Fractional GetBoundDifference(int col) const {
    return upper_bounds_[col] - lower_bounds_[col];
  }
  // Status changes are appended to *log while set (dual device mode keeps a
  // device copy of the column bits in sync with it).
  void SetChangeLog(std::vector<int>* log) { change_log_ = log; }
  // can_decrease | can_increase << 1 | non-basic boxed << 2 | status << 3
  // (kernel_args.h kCol*).
  uint8_t ColumnBits(int col) const {
    return static_cast<uint8_t>((can_decrease_.IsSet(col) ? 1 : 0) |
                                (can_increase_.IsSet(col) ? 2 : 0) |
                                (non_basic_boxed_variables_.IsSet(col) ? 4 : 0) |
                                (static_cast<int>(variable_status_[col]) << 3));
  }

 private:
  void ResetStatusInfo();
  VariableType ComputeVariableType(int col) const;
  void SetRelevance(int col, bool relevance);
  void UpdateStatusForNewType(int col);

  const CompactSparseMatrix& matrix_;
  std::vector<Fractional> lower_bounds_, upper_bounds_;
  std::vector<Fractional> saved_lower_bounds_, saved_upper_bounds_;
  std::vector<VariableType> variable_type_;
  std::vector<VariableStatus> variable_status_;
  Bitset can_increase_, can_decrease_, relevance_, is_basic_, not_basic_,
      non_basic_boxed_variables_;
  int64_t num_entries_in_relevant_columns_ = 0;
  bool boxed_variables_are_relevant_ = true;
  bool in_dual_phase_one_ = false;
  std::vector<int>* change_log_ = nullptr;
};

}  // namespace milp

#endif  // MILP_SIMPLEX_H_
