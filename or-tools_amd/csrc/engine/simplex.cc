// MI355X revised-simplex engine: the host-side state machine of
// glop::RevisedSimplex (OR-Tools 9.7, ortools/glop/revised_simplex.cc and its
// helper classes), with every O(nnz(A)) pass executed by the HIP kernels of
// csrc/kernels through DeviceLp:
//   UpdateRow::ComputeUpdates*          (update_row.cc:196-306)  -> device
//   PrimalEdgeNorms::UpdateEdgeSquaredNorms dots (primal_edge_norms.cc:208-258)
//   ReducedCosts::ComputeReducedCosts   (reduced_costs.cc:352-423) -> device
//   ReducedCosts::ComputeMaximumDualResidual (reduced_costs.cc:96-110)
//   PrimalEdgeNorms::ComputeEdgeSquaredNorms, identity basis (:147-161)
//   VariableValues residual / basic-value SpMVs (variable_values.cc:101-131)
// The kernels reproduce the host loops' floating-point order, so the pivot
// sequence (basis, statuses, iteration count) is the one Glop's algorithm
// produces. Basis factorization and FTRAN/BTRAN stay on the host in round 1.
#include "simplex.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <queue>
#include <string>

#include "../../../include/mi_lp.h"
#include "device_lp.h"
#include "fibers.h"

// fibers.h's context switch (x86-64 SysV). The frame it pushes and pops:
// [control words][r15][r14][r13][r12][rbx][rbp][return address].
asm(R"(
  .text
  .globl milp_fiber_switch
  .type milp_fiber_switch, @function
milp_fiber_switch:
  pushq %rbp
  pushq %rbx
  pushq %r12
  pushq %r13
  pushq %r14
  pushq %r15
  subq $8, %rsp
  stmxcsr (%rsp)
  fnstcw 4(%rsp)
  movq %rsp, (%rdi)
  movq %rsi, %rsp
  ldmxcsr (%rsp)
  fldcw 4(%rsp)
  addq $8, %rsp
  popq %r15
  popq %r14
  popq %r13
  popq %r12
  popq %rbx
  popq %rbp
  ret
  .size milp_fiber_switch, .-milp_fiber_switch

  .globl milp_fiber_trampoline
  .type milp_fiber_trampoline, @function
milp_fiber_trampoline:
  movq %r12, %rdi
  callq *%r13
  ud2
  .size milp_fiber_trampoline, .-milp_fiber_trampoline
)");
#include "host_pool.h"

#include <chrono>
#include <mutex>

namespace milp {
namespace {
// Debug aid (env MILP_PHASE_TIMING=1): host wall time per phase of the primal
// or dual loop, printed to stderr when the loop ends.
struct PhaseClock {
  static constexpr int kPhases = 10;
  static constexpr const char* kPrimal[kPhases] = {
      "refactor+checks", "entering(pricing)", "direction", "ratio test", "values update",
      "edge norms",      "rc update",         "prices update", "pivot",  "other"};
  static constexpr const char* kDual[kPhases] = {
      "refactor+recompute", "leaving(pricing)", "btran rho",  "update row",
      "entering ratio test", "direction ftran", "rc update",  "dual norms (tau)",
      "values+pivot",        "other"};
  explicit PhaseClock(bool dual = false);
  const char* const* names;
  double ms[kPhases] = {};
  bool on = std::getenv("MILP_PHASE_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void Mark(int phase) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    ms[phase] += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  }
  void Dump(long long iterations);
  // MILP_PHASE_TIMING_EVERY=k: dump and restart every k iterations.
  const long long every = [] {
    const char* e = std::getenv("MILP_PHASE_TIMING_EVERY");
    return e ? std::atoll(e) : 0LL;
  }();
  long long window = 0;
  void Tick() {
    if (!on || every <= 0 || ++window < every) return;
    Dump(window);
    Reset();
  }
  void Reset();
};

// Finer split inside the phases (same switch): wall time of named sections.
enum SubPhase {
  kSubBtranY, kSubPricingCall, kSubCandidatesFull, kSubGetMaximum, kSubBtranW,
  kSubUpdateRowCall, kSubNormLoop, kSubQueue, kSubLuUpdate, kSubRefactorize,
  kSubBoxedScan, kSubFlipFtran, kSubRecomputeValues, kSubDualPrices, kSubFtranDirection,
  kSubTau, kSubFlipScatter, kSubFlipSolve, kSubFlipPrices, kSubRatioPrep, kSubRatioDevice,
  kSubRatioReplay, kSubSpecBegin, kNumSubPhases
};
const char* const kSubPhaseNames[kNumSubPhases] = {
    "btran y (c_B B^-1)", "pricing device call", "prices full rebuild", "GetMaximum",
    "btran w (B^-T d)",   "update-row device",   "norm update loop",    "price queue/replay",
    "basis update (MPF)", "refactorize (LU)", "boxed dual-feas scan", "flip update (FTRAN)",
    "recompute x_B",      "dual prices",       "ftran direction",   "tau ftran",
    "  flip: column scatter", "  flip: RightSolve", "  flip: x_B + prices",
    "  ratio: prepare (row, bits)", "  ratio: device call", "  ratio: host replay",
    "  ratio: speculative flips"};
double g_sub_ms[kNumSubPhases] = {};
double g_dual_candidates = 0.0;  // device ratio test: candidates returned
double g_dual_list = 0.0;        // update-row positions they were filtered from
const bool g_sub_on = std::getenv("MILP_PHASE_TIMING") != nullptr;
struct SubTimer {
  SubPhase p;
  std::chrono::steady_clock::time_point t0;
  bool stopped = false;
  explicit SubTimer(SubPhase q) : p(q) {
    if (g_sub_on) t0 = std::chrono::steady_clock::now();
  }
  void Stop() {
    if (g_sub_on && !stopped) {
      g_sub_ms[p] += std::chrono::duration<double, std::milli>(
                         std::chrono::steady_clock::now() - t0).count();
    }
    stopped = true;
  }
  ~SubTimer() { Stop(); }
};

PhaseClock::PhaseClock(bool dual) : names(dual ? kDual : kPrimal) {
  if (on) std::fill(g_sub_ms, g_sub_ms + kNumSubPhases, 0.0);
}

void PhaseClock::Reset() {
  std::fill(ms, ms + kPhases, 0.0);
  std::fill(g_ftran_ms, g_ftran_ms + kFtPieces, 0.0);
  std::fill(g_sub_ms, g_sub_ms + kNumSubPhases, 0.0);
  g_dual_candidates = g_dual_list = 0.0;
  window = 0;
}

void PhaseClock::Dump(long long iterations) {
  if (!on) return;
  std::fprintf(stderr, "[phase timing] %lld iterations\n", iterations);
  for (int i = 0; i < kPhases; ++i) {
    std::fprintf(stderr, "  %-18s %10.3f ms  (%.3f ms/it)\n", names[i], ms[i],
                 iterations > 0 ? ms[i] / iterations : 0.0);
  }
  if (g_dual_list > 0.0) {
    std::fprintf(stderr, "  device ratio test: %.0f candidates from %.0f update-row positions\n",
                 g_dual_candidates, g_dual_list);
  }
  {
    static const char* const kFt[kFtPieces] = {"ftran L", "ftran etas", "ftran U (call)",
                                                "  U copy-in", "  U launch+wait",
                                                "  U copy-out", "  U rows to consider",
                                                "  U host solve", "  U right-pool append"};
    for (int i = 0; i < kFtPieces; ++i) {
      std::fprintf(stderr, "  %-22s %10.3f ms  (%.3f ms/it)\n", kFt[i], g_ftran_ms[i],
                   iterations > 0 ? g_ftran_ms[i] / iterations : 0.0);
    }
  }
  std::fprintf(stderr, "  -- sections:\n");
  for (int i = 0; i < kNumSubPhases; ++i) {
    std::fprintf(stderr, "  %-22s %10.3f ms  (%.3f ms/it)\n", kSubPhaseNames[i], g_sub_ms[i],
                 iterations > 0 ? g_sub_ms[i] / iterations : 0.0);
  }
}
}  // namespace
}  // namespace milp

namespace milp {

// ---------------------------------------------------------------------------
// DynamicMaximum (pricing.h:152-345)
int DynamicMaximum::RandomizeIfManyChoices(int best) {
  if (equivalent_choices_.empty()) return best;
  equivalent_choices_.push_back(best);
  return equivalent_choices_[UniformInt(*random_,
                                        static_cast<int>(equivalent_choices_.size()) - 1)];
}

int DynamicMaximum::GetMaximum() {
  Fractional best_value = -kInfinity;
  int best_position = -1;
  equivalent_choices_.clear();
  if (!tops_.empty()) {
    int new_size = 0;
    for (size_t k = 0, n = tops_.size(); k < n; ++k) {
      const HeapElement e = tops_[k];
      if (!is_candidate_[e.index]) continue;
      if (values_[e.index] != e.value) continue;
      tops_[new_size++] = e;
      if (e.value >= best_value) {
        if (e.value == best_value) {
          equivalent_choices_.push_back(e.index);
          continue;
        }
        equivalent_choices_.clear();
        best_value = e.value;
        best_position = e.index;
      }
    }
    tops_.resize(new_size);
    if (new_size != 0) return RandomizeIfManyChoices(best_position);
  }
  threshold_ = -kInfinity;
  auto visit = [&](int position) {
    const Fractional value = values_[position];
    if (value < threshold_) return;
    UpdateTopK(position, value);
    if (value >= best_value) {
      if (value == best_value) {
        equivalent_choices_.push_back(position);
        return;
      }
      equivalent_choices_.clear();
      best_value = value;
      best_position = position;
    }
  };
  std::vector<int> processed;
  if (ScanCandidatesInParallel(&processed)) {
    for (const int position : processed) visit(position);
  } else {
    is_candidate_.ForEach(visit);
  }
  return RandomizeIfManyChoices(best_position);
}

void DynamicMaximum::BulkAddOrUpdate(const int* pos, const Fractional* value,
                                     const uint8_t* keep, size_t n) {
  constexpr int k = 31;
  constexpr int kMaxParts = 16;
  const bool parallel = n >= 8192 && HostPool::Get().threads() > 1 &&
                        static_cast<int>(tops_.size()) == k;
  if (!parallel) {
    for (size_t i = 0; i < n; ++i) {
      if (keep[i]) {
        AddOrUpdate(pos[i], value[i]);
      } else {
        Remove(pos[i]);
      }
    }
    return;
  }
  // The heap is full, so threshold_ is its minimum and an AddOrUpdate reaches
  // UpdateTopK iff its value is not below the minimum of the 31 largest
  // values so far (the heap's multiset). Pass 1: the writes (distinct
  // positions, whole candidate words per part are not needed: Set/Clear of
  // one bit is made atomic) and each part's 31 largest kept values; pass 2:
  // each part's acting entries from the multiset of the heap and the parts
  // before it.
  auto offer = [](std::vector<Fractional>* h, Fractional v) {
    if (static_cast<int>(h->size()) < k) {
      h->push_back(v);
      std::push_heap(h->begin(), h->end(), std::greater<Fractional>());
    } else if (v > h->front()) {
      std::pop_heap(h->begin(), h->end(), std::greater<Fractional>());
      h->back() = v;
      std::push_heap(h->begin(), h->end(), std::greater<Fractional>());
    }
  };
  std::vector<Fractional> tops[kMaxParts];
  bool has_nan[kMaxParts] = {};
  Fractional* values = values_.data();
  uint64_t* words = is_candidate_.mutable_data();
  // One plan for both passes (pass 2 indexes pass 1's per-part results).
  const RangePlan plan = PlanRanges(static_cast<int64_t>(n), 8192, 1);
  const int parts = RunRanges(plan, static_cast<int64_t>(n),
                              [&](int p, int64_t b, int64_t e) {
    std::vector<Fractional>& h = tops[p];
    h.clear();
    for (int64_t i = b; i < e; ++i) {
      const int q = pos[i];
      uint64_t* w = words + (q >> 6);
      const uint64_t bit = uint64_t{1} << (q & 63);
      if (keep[i]) {
        __atomic_fetch_or(w, bit, __ATOMIC_RELAXED);
        values[q] = value[i];
        if (value[i] != value[i]) has_nan[p] = true;
        offer(&h, value[i]);
      } else {
        __atomic_fetch_and(w, ~bit, __ATOMIC_RELAXED);
      }
    }
  });
  bool nan = parts > kMaxParts;
  for (int p = 0; p < parts && !nan; ++p) nan = has_nan[p];
  std::vector<int> acting;
  if (!nan) {
    std::vector<Fractional> incoming[kMaxParts];
    std::vector<Fractional> running;
    for (const HeapElement& e : tops_) offer(&running, e.value);
    for (int p = 0; p < parts; ++p) {
      incoming[p] = running;
      for (const Fractional v : tops[p]) offer(&running, v);
    }
    std::vector<int> found[kMaxParts];
    RunRanges(plan, static_cast<int64_t>(n), [&](int p, int64_t b, int64_t e) {
      std::vector<Fractional> h = incoming[p];
      std::vector<int>& out = found[p];
      out.clear();
      for (int64_t i = b; i < e; ++i) {
        if (!keep[i] || value[i] < h.front()) continue;
        out.push_back(static_cast<int>(i));
        offer(&h, value[i]);
      }
    });
    for (int p = 0; p < parts; ++p) acting.insert(acting.end(), found[p].begin(), found[p].end());
  } else {
    for (size_t i = 0; i < n; ++i) {
      if (keep[i]) acting.push_back(static_cast<int>(i));
    }
  }
  // The values and bits are final; the top-k sees the acting entries in order.
  for (const int i : acting) {
    if (value[i] >= threshold_) UpdateTopK(pos[i], value[i]);
  }
}

// The full scan above only acts on the candidates that are not below the
// threshold when the scan reaches them, and that threshold is the 31st
// largest value seen so far (UpdateTopK keeps the 31 largest values; an equal
// value only swaps an index). The host pool finds those candidates: pass 1
// gives each part its 31 largest values, pass 2 scans each part from the
// 31 largest of the parts before it, keeping the same multiset the heap
// would hold. The serial replay of the found candidates then makes the same
// UpdateTopK calls, RNG draws and tie lists as the plain scan.
bool DynamicMaximum::ScanCandidatesInParallel(std::vector<int>* processed) const {
  constexpr int k = 31;
  const int n = is_candidate_.size();
  if (n < (1 << 16) || HostPool::Get().threads() <= 1) return false;
  const uint64_t* words = is_candidate_.data();
  const int num_words = (n + 63) / 64;
  const Fractional* values = values_.data();
  constexpr int kMaxParts = 16;
  std::vector<Fractional> tops[kMaxParts];
  bool has_nan[kMaxParts] = {};
  auto offer = [](std::vector<Fractional>* h, Fractional v) {
    // Min-heap of the k largest values (multiset).
    if (static_cast<int>(h->size()) < k) {
      h->push_back(v);
      std::push_heap(h->begin(), h->end(), std::greater<Fractional>());
    } else if (v > h->front()) {
      std::pop_heap(h->begin(), h->end(), std::greater<Fractional>());
      h->back() = v;
      std::push_heap(h->begin(), h->end(), std::greater<Fractional>());
    }
  };
  const int parts = ParallelRanges(num_words, 1024, 1, [&](int p, int64_t w0, int64_t w1) {
    std::vector<Fractional>& h = tops[p];
    h.clear();
    for (int64_t w = w0; w < w1; ++w) {
      uint64_t bits = words[w];
      while (bits) {
        const int i = static_cast<int>(w * 64 + __builtin_ctzll(bits));
        bits &= bits - 1;
        if (i >= n) break;
        const Fractional v = values[i];
        if (v != v) has_nan[p] = true;
        offer(&h, v);
      }
    }
  });
  if (parts > kMaxParts) return false;
  for (int p = 0; p < parts; ++p) {
    if (has_nan[p]) return false;  // the plain scan's comparisons, not these
  }
  std::vector<Fractional> incoming[kMaxParts];
  {
    std::vector<Fractional> running;
    for (int p = 0; p < parts; ++p) {
      incoming[p] = running;
      for (const Fractional v : tops[p]) offer(&running, v);
    }
  }
  std::vector<int> found[kMaxParts];
  const int parts2 = ParallelRanges(num_words, 1024, 1, [&](int p, int64_t w0, int64_t w1) {
    std::vector<Fractional> h = incoming[p];
    std::vector<int>& out = found[p];
    out.clear();
    Fractional threshold = static_cast<int>(h.size()) < k ? -kInfinity : h.front();
    for (int64_t w = w0; w < w1; ++w) {
      uint64_t bits = words[w];
      while (bits) {
        const int i = static_cast<int>(w * 64 + __builtin_ctzll(bits));
        bits &= bits - 1;
        if (i >= n) break;
        const Fractional v = values[i];
        if (v < threshold) continue;
        out.push_back(i);
        offer(&h, v);
        threshold = static_cast<int>(h.size()) < k ? -kInfinity : h.front();
      }
    }
  });
  if (parts2 != parts) return false;
  processed->clear();
  for (int p = 0; p < parts; ++p) processed->insert(processed->end(), found[p].begin(), found[p].end());
  return true;
}

void DynamicMaximum::UpdateTopK(int position, Fractional value) {
  constexpr int k = 31;
  if (static_cast<int>(tops_.size()) < k) {
    tops_.push_back(HeapElement{position, value});
    if (static_cast<int>(tops_.size()) == k) {
      std::make_heap(tops_.begin(), tops_.end(), HeapLess());
      threshold_ = tops_[0].value;
    }
    return;
  }
  if (value == tops_[0].value) {
    if (AbslBernoulli(*random_, 0.5)) tops_[0].index = position;
    return;
  }
  int i = 0;
  constexpr int limit = k / 2;
  for (; i < limit;) {
    const int left_child = 2 * i + 1;
    const int right_child = left_child + 1;
    const Fractional l_value = tops_[left_child].value;
    const Fractional r_value = tops_[right_child].value;
    if (l_value > r_value) {
      if (value <= r_value) break;
      tops_[i] = tops_[right_child];
      i = right_child;
    } else {
      if (value <= l_value) break;
      tops_[i] = tops_[left_child];
      i = left_child;
    }
  }
  tops_[i] = HeapElement{position, value};
  threshold_ = tops_[0].value;
}

// ---------------------------------------------------------------------------
// VariablesInfo (variables_info.cc:14-476)
bool VariablesInfo::LoadBoundsAndReturnTrueIfUnchanged(
    const std::vector<double>& vlb, const std::vector<double>& vub,
    const std::vector<double>& clb, const std::vector<double>& cub) {
  const int num_cols = matrix_.num_cols();
  const int num_variables = static_cast<int>(vub.size());
  const int num_rows = static_cast<int>(clb.size());
  bool is_unchanged = (num_cols == static_cast<int>(lower_bounds_.size()));
  lower_bounds_.resize(num_cols, 0.0);
  upper_bounds_.resize(num_cols, 0.0);
  variable_type_.resize(num_cols, VariableType::FIXED_VARIABLE);
  for (int col = 0; col < num_variables; ++col) {
    if (lower_bounds_[col] != vlb[col] || upper_bounds_[col] != vub[col]) {
      lower_bounds_[col] = vlb[col];
      upper_bounds_[col] = vub[col];
      is_unchanged = false;
      variable_type_[col] = ComputeVariableType(col);
    }
  }
  for (int row = 0; row < num_rows; ++row) {
    const int col = num_variables + row;
    if (lower_bounds_[col] != -cub[row] || upper_bounds_[col] != -clb[row]) {
      lower_bounds_[col] = -cub[row];
      upper_bounds_[col] = -clb[row];
      is_unchanged = false;
      variable_type_[col] = ComputeVariableType(col);
    }
  }
  return is_unchanged;
}

void VariablesInfo::ResetStatusInfo() {
  const int num_cols = matrix_.num_cols();
  variable_status_.resize(num_cols, VariableStatus::FREE);
  can_increase_.ClearAndResize(num_cols);
  can_decrease_.ClearAndResize(num_cols);
  is_basic_.ClearAndResize(num_cols);
  not_basic_.ClearAndResize(num_cols);
  non_basic_boxed_variables_.ClearAndResize(num_cols);
  boxed_variables_are_relevant_ = true;
  num_entries_in_relevant_columns_ = 0;
  relevance_.ClearAndResize(num_cols);
}

void VariablesInfo::InitializeFromBasisState(int first_slack_col, int num_new_cols,
                                             const std::vector<VariableStatus>& state) {
  ResetStatusInfo();
  const int num_cols = static_cast<int>(lower_bounds_.size());
  const int first_new_col = first_slack_col - num_new_cols;
  const int ssize = static_cast<int>(state.size());
  for (int col = 0; col < num_cols; ++col) {
    VariableStatus status;
    if (col < first_new_col && col < ssize) {
      status = state[col];
    } else if (col >= first_slack_col && col - num_new_cols < ssize) {
      status = state[col - num_new_cols];
    } else {
      UpdateToNonBasicStatus(col, DefaultVariableStatus(col));
      continue;
    }
    switch (status) {
      case VariableStatus::BASIC:
        variable_status_[col] = VariableStatus::BASIC;
        is_basic_.Set(col, true);
        break;
      case VariableStatus::AT_LOWER_BOUND:
        if (lower_bounds_[col] == upper_bounds_[col]) {
          UpdateToNonBasicStatus(col, VariableStatus::FIXED_VALUE);
        } else {
          UpdateToNonBasicStatus(col, lower_bounds_[col] == -kInfinity
                                          ? DefaultVariableStatus(col)
                                          : status);
        }
        break;
      case VariableStatus::AT_UPPER_BOUND:
        if (lower_bounds_[col] == upper_bounds_[col]) {
          UpdateToNonBasicStatus(col, VariableStatus::FIXED_VALUE);
        } else {
          UpdateToNonBasicStatus(col, upper_bounds_[col] == kInfinity
                                          ? DefaultVariableStatus(col)
                                          : status);
        }
        break;
      default:
        UpdateToNonBasicStatus(col, DefaultVariableStatus(col));
    }
  }
}

int VariablesInfo::ChangeUnusedBasicVariablesToFree(const std::vector<int>& basis) {
  const int num_cols = static_cast<int>(lower_bounds_.size());
  is_basic_.ClearAndResize(num_cols);
  for (const int col : basis) UpdateToBasicStatus(col);
  int num_no_longer_in_basis = 0;
  for (int col = 0; col < num_cols; ++col) {
    if (!is_basic_[col] && variable_status_[col] == VariableStatus::BASIC) {
      ++num_no_longer_in_basis;
      if (variable_type_[col] == VariableType::FIXED_VARIABLE) {
        UpdateToNonBasicStatus(col, VariableStatus::FIXED_VALUE);
      } else {
        UpdateToNonBasicStatus(col, VariableStatus::FREE);
      }
    }
  }
  return num_no_longer_in_basis;
}

int VariablesInfo::SnapFreeVariablesToBound(Fractional distance,
                                            const std::vector<Fractional>& sv) {
  int num_changes = 0;
  const int num_cols = static_cast<int>(lower_bounds_.size());
  for (int col = 0; col < num_cols; ++col) {
    if (variable_status_[col] != VariableStatus::FREE) continue;
    if (variable_type_[col] == VariableType::UNCONSTRAINED) continue;
    const Fractional value = col < static_cast<int>(sv.size()) ? sv[col] : 0.0;
    const Fractional diff_ub = upper_bounds_[col] - value;
    const Fractional diff_lb = value - lower_bounds_[col];
    if (diff_lb <= diff_ub) {
      if (diff_lb <= distance) {
        ++num_changes;
        UpdateToNonBasicStatus(col, VariableStatus::AT_LOWER_BOUND);
      }
    } else {
      if (diff_ub <= distance) {
        ++num_changes;
        UpdateToNonBasicStatus(col, VariableStatus::AT_UPPER_BOUND);
      }
    }
  }
  return num_changes;
}

void VariablesInfo::InitializeToDefaultStatus() {
  ResetStatusInfo();
  const int num_cols = static_cast<int>(lower_bounds_.size());
  for (int col = 0; col < num_cols; ++col)
    UpdateToNonBasicStatus(col, DefaultVariableStatus(col));
}

VariableStatus VariablesInfo::DefaultVariableStatus(int col) const {
  if (lower_bounds_[col] == upper_bounds_[col]) return VariableStatus::FIXED_VALUE;
  if (lower_bounds_[col] == -kInfinity && upper_bounds_[col] == kInfinity)
    return VariableStatus::FREE;
  return std::fabs(lower_bounds_[col]) <= std::fabs(upper_bounds_[col])
             ? VariableStatus::AT_LOWER_BOUND
             : VariableStatus::AT_UPPER_BOUND;
}

void VariablesInfo::MakeBoxedVariableRelevant(bool value) {
  if (value == boxed_variables_are_relevant_) return;
  boxed_variables_are_relevant_ = value;
  const std::vector<int> boxed = non_basic_boxed_variables_.ToVector();
  if (value) {
    for (const int col : boxed)
      SetRelevance(col, variable_type_[col] != VariableType::FIXED_VARIABLE);
  } else {
    for (const int col : boxed) SetRelevance(col, false);
  }
}

void VariablesInfo::UpdateToBasicStatus(int col) {
  if (in_dual_phase_one_) {
    if (lower_bounds_[col] != 0.0) lower_bounds_[col] = -kInfinity;
    if (upper_bounds_[col] != 0.0) upper_bounds_[col] = +kInfinity;
    variable_type_[col] = ComputeVariableType(col);
  }
  if (change_log_ != nullptr) change_log_->push_back(col);
  variable_status_[col] = VariableStatus::BASIC;
  is_basic_.Set(col, true);
  not_basic_.Set(col, false);
  can_increase_.Set(col, false);
  can_decrease_.Set(col, false);
  non_basic_boxed_variables_.Set(col, false);
  SetRelevance(col, false);
}

void VariablesInfo::UpdateToNonBasicStatus(int col, VariableStatus status) {
  if (change_log_ != nullptr) change_log_->push_back(col);
  variable_status_[col] = status;
  is_basic_.Set(col, false);
  not_basic_.Set(col, true);
  can_increase_.Set(col, status == VariableStatus::AT_LOWER_BOUND ||
                             status == VariableStatus::FREE);
  can_decrease_.Set(col, status == VariableStatus::AT_UPPER_BOUND ||
                             status == VariableStatus::FREE);
  const bool boxed = variable_type_[col] == VariableType::UPPER_AND_LOWER_BOUNDED;
  non_basic_boxed_variables_.Set(col, boxed);
  const bool relevance = status != VariableStatus::FIXED_VALUE &&
                         (boxed_variables_are_relevant_ || !boxed);
  SetRelevance(col, relevance);
}

VariableType VariablesInfo::ComputeVariableType(int col) const {
  if (lower_bounds_[col] == -kInfinity) {
    if (upper_bounds_[col] == kInfinity) return VariableType::UNCONSTRAINED;
    return VariableType::UPPER_BOUNDED;
  } else if (upper_bounds_[col] == kInfinity) {
    return VariableType::LOWER_BOUNDED;
  } else if (lower_bounds_[col] == upper_bounds_[col]) {
    return VariableType::FIXED_VARIABLE;
  }
  return VariableType::UPPER_AND_LOWER_BOUNDED;
}

void VariablesInfo::SetRelevance(int col, bool relevance) {
  if (relevance_.IsSet(col) == relevance) return;
  if (relevance) {
    relevance_.Set(col);
    num_entries_in_relevant_columns_ += matrix_.ColumnNumEntries(col);
  } else {
    relevance_.Clear(col);
    num_entries_in_relevant_columns_ -= matrix_.ColumnNumEntries(col);
  }
}

void VariablesInfo::UpdateStatusForNewType(int col) {
  switch (variable_status_[col]) {
    case VariableStatus::BASIC:
      UpdateToBasicStatus(col);
      break;
    case VariableStatus::AT_LOWER_BOUND:
      if (lower_bounds_[col] == upper_bounds_[col]) {
        UpdateToNonBasicStatus(col, VariableStatus::FIXED_VALUE);
      } else if (lower_bounds_[col] == -kInfinity) {
        UpdateToNonBasicStatus(col, DefaultVariableStatus(col));
      } else {
        UpdateToNonBasicStatus(col, variable_status_[col]);
      }
      break;
    case VariableStatus::AT_UPPER_BOUND:
      if (lower_bounds_[col] == upper_bounds_[col]) {
        UpdateToNonBasicStatus(col, VariableStatus::FIXED_VALUE);
      } else if (upper_bounds_[col] == kInfinity) {
        UpdateToNonBasicStatus(col, DefaultVariableStatus(col));
      } else {
        UpdateToNonBasicStatus(col, variable_status_[col]);
      }
      break;
    default:
      UpdateToNonBasicStatus(col, DefaultVariableStatus(col));
  }
}

void VariablesInfo::TransformToDualPhaseIProblem(Fractional tol,
                                                 const std::vector<Fractional>& rc) {
  in_dual_phase_one_ = true;
  saved_lower_bounds_ = lower_bounds_;
  saved_upper_bounds_ = upper_bounds_;
  const int num_cols = matrix_.num_cols();
  for (int col = 0; col < num_cols; ++col) {
    switch (variable_type_[col]) {
      case VariableType::FIXED_VARIABLE:
      case VariableType::UPPER_AND_LOWER_BOUNDED:
        lower_bounds_[col] = 0.0;
        upper_bounds_[col] = 0.0;
        variable_type_[col] = VariableType::FIXED_VARIABLE;
        break;
      case VariableType::LOWER_BOUNDED:
        lower_bounds_[col] = 0.0;
        upper_bounds_[col] = 1.0;
        variable_type_[col] = VariableType::UPPER_AND_LOWER_BOUNDED;
        break;
      case VariableType::UPPER_BOUNDED:
        lower_bounds_[col] = -1.0;
        upper_bounds_[col] = 0.0;
        variable_type_[col] = VariableType::UPPER_AND_LOWER_BOUNDED;
        break;
      case VariableType::UNCONSTRAINED:
        lower_bounds_[col] = -1000.0;
        upper_bounds_[col] = 1000.0;
        variable_type_[col] = VariableType::UPPER_AND_LOWER_BOUNDED;
        break;
    }
    if (variable_type_[col] == VariableType::UPPER_AND_LOWER_BOUNDED) {
      if (rc[col] > tol) {
        variable_status_[col] = VariableStatus::AT_LOWER_BOUND;
      } else if (rc[col] < -tol) {
        variable_status_[col] = VariableStatus::AT_UPPER_BOUND;
      }
    }
    UpdateStatusForNewType(col);
  }
}

void VariablesInfo::EndDualPhaseI(Fractional tol, const std::vector<Fractional>& rc) {
  in_dual_phase_one_ = false;
  std::swap(saved_lower_bounds_, lower_bounds_);
  std::swap(saved_upper_bounds_, upper_bounds_);
  saved_lower_bounds_.clear();
  saved_upper_bounds_.clear();
  const int num_cols = matrix_.num_cols();
  for (int col = 0; col < num_cols; ++col) {
    variable_type_[col] = ComputeVariableType(col);
    if (variable_type_[col] == VariableType::UPPER_AND_LOWER_BOUNDED) {
      if (rc[col] > tol) {
        variable_status_[col] = VariableStatus::AT_LOWER_BOUND;
      } else if (rc[col] < -tol) {
        variable_status_[col] = VariableStatus::AT_UPPER_BOUND;
      }
    }
    UpdateStatusForNewType(col);
  }
}

// ---------------------------------------------------------------------------
// Dual edge norms shared by the handles of one batch call
// (mi_lp_batch_solve_bounds): the children of a search node start from the
// same basis of the same matrix, so the first child's norm recompute after
// the first factorization is every child's. Keyed by the factorization's
// content; a hit copies the values and replays the loop's deterministic-time
// bumps, so every result is the one a solve computing its own norms gets.
struct DualNormCache {
  struct Entry {
    uint64_t key;
    std::vector<int> basis, row_perm, col_perm;  // compared exactly on a hit
    std::shared_ptr<const std::vector<Fractional>> norms;
  };
  std::mutex mu;
  std::vector<Entry> entries;
  static constexpr size_t kMaxEntries = 8;
  std::shared_ptr<const std::vector<Fractional>> Find(uint64_t key, const std::vector<int>& basis,
                                                      const std::vector<int>& row_perm,
                                                      const std::vector<int>& col_perm) {
    std::lock_guard<std::mutex> l(mu);
    for (const auto& e : entries) {
      if (e.key == key && e.basis == basis && e.row_perm == row_perm && e.col_perm == col_perm) {
        return e.norms;
      }
    }
    return nullptr;
  }
  void Insert(uint64_t key, const std::vector<int>& basis, const std::vector<int>& row_perm,
              const std::vector<int>& col_perm, const std::vector<Fractional>& v) {
    std::lock_guard<std::mutex> l(mu);
    if (entries.size() >= kMaxEntries) return;
    for (const auto& e : entries) {
      if (e.key == key && e.basis == basis) return;
    }
    entries.push_back(
        Entry{key, basis, row_perm, col_perm, std::make_shared<const std::vector<Fractional>>(v)});
  }
};

// ---------------------------------------------------------------------------
// DualEdgeNorms (dual_edge_norms.cc)
class DualEdgeNorms {
  friend struct SdualBridge;
  friend struct SdualHooks;

 public:
  explicit DualEdgeNorms(const BasisFactorization& bf) : bf_(bf) {}
  void SetParameters(const GlopParameters& p) { params_ = p; }
  bool NeedsBasisRefactorization() const { return recompute_; }
  void Clear() { recompute_ = true; }
  void ResizeOnNewRows(int n) { norms_.resize(n, 1.0); }
  const std::vector<Fractional>& GetEdgeSquaredNorms() {
    if (recompute_) ComputeEdgeSquaredNorms();
    return norms_;
  }
  void UpdateDataOnBasisPermutation(const std::vector<int>& col_perm) {
    if (recompute_) return;
    std::vector<Fractional> tmp(norms_.size());
    for (size_t i = 0; i < col_perm.size(); ++i) tmp[col_perm[i]] = norms_[i];
    norms_.swap(tmp);
  }
  // dual_edge_norms.cc:49-80
  bool TestPrecision(int leaving_row, const ScatteredVector& rho) {
    if (recompute_) return true;
    const Fractional leaving_squared_norm = SquaredNorm(rho);
    const Fractional old_squared_norm = norms_[leaving_row];
    const Fractional acc = (std::sqrt(leaving_squared_norm) - std::sqrt(old_squared_norm)) /
                           std::sqrt(leaving_squared_norm);
    if (std::fabs(acc) > params_.recompute_edges_norm_threshold) recompute_ = true;
    norms_[leaving_row] = leaving_squared_norm;
    return old_squared_norm > 0.25 * leaving_squared_norm;
  }
  // UpdateBeforeBasisPivot will compute tau (if the iteration gets there).
  bool WillComputeTau() const { return !recompute_; }
  // dual_edge_norms.cc:82-118
  void UpdateBeforeBasisPivot(int /*entering_col*/, int leaving_row,
                              const ScatteredVector& direction,
                              const ScatteredVector& rho) {
    if (recompute_) return;
    SubTimer tau_timer(kSubTau);
    const std::vector<Fractional>& tau = bf_.RightSolveForTau(rho);
    const Fractional pivot = direction[leaving_row];
    const Fractional new_leaving_squared_norm = norms_[leaving_row] / Square(pivot);
    // Element-wise over the direction's distinct rows: split over the host pool.
    const std::vector<int>& rows = direction.non_zeros;
    ParallelRanges(static_cast<int64_t>(rows.size()), 16384, 1, [&](int, int64_t b, int64_t e) {
      for (int64_t k = b; k < e; ++k) {
        const int row = rows[k];
        const Fractional c = direction[row];
        norms_[row] += c * (c * new_leaving_squared_norm - 2.0 / pivot * tau[row]);
        const Fractional kLowerBound = 1e-4;
        if (norms_[row] < kLowerBound) {
          if (row == leaving_row) continue;
          norms_[row] = kLowerBound;
        }
      }
    });
    norms_[leaving_row] = new_leaving_squared_norm;
  }

 private:
  void ComputeEdgeSquaredNorms() {  // dual_edge_norms.cc:120-132
    const int num_rows = bf_.GetNumberOfRows();
    uint64_t key = 0;
    if (cache_ != nullptr && bf_.NumUpdates() == 0) {
      key = bf_.FactorizationContentKey();
      const auto hit = cache_->Find(key, bf_.basis(), bf_.lu().row_perm(),
                                    bf_.lu().GetColumnPermutation());
      if (hit != nullptr && static_cast<int>(hit->size()) == num_rows) {
        norms_ = *hit;
        for (int row = 0; row < num_rows; ++row) bf_.BumpDeterministicTimeForSolve(1);
        recompute_ = false;
        return;
      }
    }
    norms_.resize(num_rows, 0.0);
    for (int row = 0; row < num_rows; ++row) norms_[row] = bf_.DualEdgeSquaredNorm(row);
    recompute_ = false;
    if (key != 0) {
      cache_->Insert(key, bf_.basis(), bf_.lu().row_perm(), bf_.lu().GetColumnPermutation(),
                     norms_);
    }
  }
 public:
  void SetCache(DualNormCache* cache) { cache_ = cache; }

 private:
  DualNormCache* cache_ = nullptr;
  const BasisFactorization& bf_;
  GlopParameters params_;
  bool recompute_ = true;
  std::vector<Fractional> norms_;
};

// ---------------------------------------------------------------------------
// UpdateRow (update_row.cc)
class UpdateRow {
  friend struct SdualBridge;
  friend struct SdualHooks;

 public:
  UpdateRow(const CompactSparseMatrix& m, const CompactSparseMatrix& t,
            const VariablesInfo& vi, const std::vector<int>& basis,
            const BasisFactorization& bf, DeviceLp* dev)
      : matrix_(m), transposed_matrix_(t), variables_info_(vi), basis_(basis), bf_(bf),
        dev_(dev) {}
  void SetParameters(const GlopParameters& p) { params_ = p; }
  void Invalidate() {
    Materialize();
    left_inverse_computed_for_ = kInvalidRow;
    update_row_computed_for_ = kInvalidRow;
  }
  const ScatteredVector& GetUnitRowLeftInverse() const { return rho_; }
  const ScatteredVector& ComputeAndGetUnitRowLeftInverse(int leaving_row) {
    Invalidate();
    bf_.TemporaryLeftSolveForUnitRow(leaving_row, &rho_);
    return rho_;
  }
  void ComputeUnitRowLeftInverse(int leaving_row) {
    if (left_inverse_computed_for_ == leaving_row) return;
    Materialize();  // a deferred pass still needs the current rho
    left_inverse_computed_for_ = leaving_row;
    bf_.LeftSolveForUnitRow(leaving_row, &rho_);
  }
  void ComputeUpdateRow(int leaving_row);
  bool IsComputedFor(int leaving_row) const {
    return update_row_computed_for_ == leaving_row;
  }
  const std::vector<Fractional>& GetCoefficients() const {
    Materialize();
    EnsureHost();
    return coefficient_;
  }
  const std::vector<int>& GetNonZeroPositions() const {
    Materialize();
    EnsureHost();
    return non_zero_position_list_;
  }
  // Listed positions are mirrored on the host; any other position holds
  // whatever the device update-row kernels left there (same write rules as
  // the host loops), so it is read back from the device.
  Fractional GetCoefficient(int col) const {
    Materialize();
    if (host_stale_ && col == known_col_) return known_value_;
    EnsureHost();
    if (col < static_cast<int>(listed_.size()) && listed_[col]) return coefficient_[col];
    return dev_->ReadCoefficient(col);
  }
  // Dual device mode: the update row stays on the device; the host copy is
  // read back only if host code asks for it. A coefficient the device ratio
  // test already returned can be registered and served without a readback.
  void SetLazyFetch(bool on) { lazy_fetch_ = on; }
  void SetKnownCoefficient(int col, Fractional value) {
    known_col_ = col;
    known_value_ = value;
  }
  void MaterializeOnDevice() { Materialize(); }
  // The column-wise pass is deferred until its result is first read, so the
  // primal edge-norm update can fuse its a_j . w dots into the same pass over
  // A. Returns true when that fused pass ran now; the dots are then served by
  // DeviceLp::ListDotsOverUpdateRow(w).
  bool MaterializeWithDots(const std::vector<Fractional>& w) {
    if (!pending_column_wise_) return false;
    RunColumnWise(&w);
    return true;
  }
  void Materialize() const {
    if (pending_column_wise_) const_cast<UpdateRow*>(this)->RunColumnWise(nullptr);
  }
  void ComputeFullUpdateRow(int leaving_row, std::vector<Fractional>* output) const;
  double DeterministicTime() const {
    return DeterministicTimeForFpOperations(num_operations_);
  }
  // Which algorithm ComputeUpdateRow() used last (exposed for parity tests).
  int last_algorithm() const { return last_algorithm_; }
  // Changes whenever the listed positions / coefficients are recomputed.
  uint64_t epoch() const { return epoch_; }

 private:
  void ComputeUpdatesRowWise();
  void ComputeUpdatesRowWiseHypersparse();
  void ComputeUpdatesColumnWise();
  void ComputeUpdatesForSingleRow(int row_as_col);
  void FetchFromDevice();
  void FetchOrDefer() {
    known_col_ = -1;
    if (lazy_fetch_) {
      host_stale_ = true;
    } else {
      host_stale_ = false;
      FetchFromDevice();
    }
  }
  void EnsureHost() const {
    if (!host_stale_) return;
    UpdateRow* self = const_cast<UpdateRow*>(this);
    self->host_stale_ = false;
    self->FetchFromDevice();
  }
  void RunColumnWise(const std::vector<Fractional>* w);

  const CompactSparseMatrix& matrix_;
  const CompactSparseMatrix& transposed_matrix_;
  const VariablesInfo& variables_info_;
  const std::vector<int>& basis_;
  const BasisFactorization& bf_;
  DeviceLp* dev_;
  std::vector<char> listed_;
  std::vector<Fractional> fetched_values_;
  GlopParameters params_;
  ScatteredVector rho_;
  std::vector<int> rho_filtered_non_zeros_;
  std::vector<int> non_zero_position_list_;
  Bitset non_zero_position_set_;
  std::vector<Fractional> coefficient_;
  int left_inverse_computed_for_ = kInvalidRow;
  int update_row_computed_for_ = kInvalidRow;
  int64_t num_operations_ = 0;
  int last_algorithm_ = -1;
  uint64_t epoch_ = 0;
  bool lazy_fetch_ = false;
  bool host_stale_ = false;
  int known_col_ = -1;
  Fractional known_value_ = 0.0;
  // Deferred column-wise pass: the relevance mask and work count it uses are
  // captured when Glop would have run it (update_row.cc:282-306).
  bool pending_column_wise_ = false;
  std::vector<uint64_t> pending_mask_;
  int64_t pending_relevant_entries_ = 0;
};

// update_row.cc:77-166
void UpdateRow::ComputeUpdateRow(int leaving_row) {
  if (update_row_computed_for_ == leaving_row) return;
  Materialize();
  update_row_computed_for_ = leaving_row;
  ComputeUnitRowLeftInverse(leaving_row);
  if (params_.use_transposed_matrix) {
    int64_t num_row_wise_entries = 0;
    const Fractional drop_tolerance = params_.drop_tolerance;
    rho_filtered_non_zeros_.clear();
    if (rho_.non_zeros.empty()) {
      const int size = rho_.size();
      for (int col = 0; col < size; ++col) {
        if (std::fabs(rho_.values[col]) > drop_tolerance) {
          rho_filtered_non_zeros_.push_back(col);
          num_row_wise_entries += transposed_matrix_.ColumnNumEntries(col);
        }
      }
    } else {
      for (const int col : rho_.non_zeros) {
        if (std::fabs(rho_.values[col]) > drop_tolerance) {
          rho_filtered_non_zeros_.push_back(col);
          num_row_wise_entries += transposed_matrix_.ColumnNumEntries(col);
        }
      }
    }
    if (rho_filtered_non_zeros_.size() == 1) {
      ComputeUpdatesForSingleRow(rho_filtered_non_zeros_.front());
      num_operations_ += num_row_wise_entries;
      last_algorithm_ = 0;
      return;
    }
    const int64_t num_col_wise_entries = variables_info_.GetNumEntriesInRelevantColumns();
    const double row_wise = static_cast<double>(num_row_wise_entries);
    if (row_wise < 0.5 * static_cast<double>(num_col_wise_entries)) {
      if (row_wise < 1.1 * static_cast<double>(matrix_.num_cols())) {
        ComputeUpdatesRowWiseHypersparse();
        num_operations_ += 5 * num_row_wise_entries + matrix_.num_cols() / 64;
        last_algorithm_ = 1;
      } else {
        ComputeUpdatesRowWise();
        num_operations_ += num_row_wise_entries + matrix_.num_rows();
        last_algorithm_ = 2;
      }
    } else {
      ComputeUpdatesColumnWise();
      num_operations_ += num_col_wise_entries + matrix_.num_cols();
      last_algorithm_ = 3;
    }
  } else {
    ComputeUpdatesColumnWise();
    num_operations_ +=
        variables_info_.GetNumEntriesInRelevantColumns() + matrix_.num_cols();
    last_algorithm_ = 3;
  }
}

// The four update-row algorithms (update_row.cc:196-306) run on the GPU;
// the host keeps Glop's algorithm choice (ComputeUpdateRow above) and mirrors
// the listed positions.
void UpdateRow::FetchFromDevice() {
  ++epoch_;
  {
    const int* pos = non_zero_position_list_.data();
    char* listed = listed_.data();
    ParallelRanges(static_cast<int64_t>(non_zero_position_list_.size()), 16384, 1,
                   [&](int, int64_t b, int64_t e) {
      for (int64_t k = b; k < e; ++k) listed[pos[k]] = 0;
    });
  }
  dev_->FetchUpdateRow(&non_zero_position_list_, &fetched_values_);
  const int* pos = non_zero_position_list_.data();
  const Fractional* vals = fetched_values_.data();
  char* listed = listed_.data();
  Fractional* coeff = coefficient_.data();
  ParallelRanges(static_cast<int64_t>(non_zero_position_list_.size()), 16384, 1,
                 [&](int, int64_t b, int64_t e) {
    for (int64_t k = b; k < e; ++k) {
      listed[pos[k]] = 1;
      coeff[pos[k]] = vals[k];
    }
  });
  // MILP_TRACE: one line per fetched update row (algorithm, list, values).
  static const char* trace = std::getenv("MILP_TRACE");
  if (trace != nullptr) {
    uint64_t hp = 1469598103934665603ull, hv = hp;
    for (size_t k = 0; k < non_zero_position_list_.size(); ++k) {
      hp = (hp ^ static_cast<uint32_t>(pos[k])) * 1099511628211ull;
      uint64_t bits;
      std::memcpy(&bits, &vals[k], sizeof(bits));
      hv = (hv ^ bits) * 1099511628211ull;
    }
    if (FILE* f = std::fopen((std::string(trace) + ".device").c_str(), "a")) {
      std::fprintf(f, "  update_row alg=%d n=%zu pos=%016llx val=%016llx\n", last_algorithm_,
                   non_zero_position_list_.size(), static_cast<unsigned long long>(hp),
                   static_cast<unsigned long long>(hv));
      std::fclose(f);
    }
  }
}

// update_row.cc:196-216
void UpdateRow::ComputeUpdatesRowWise() {
  SubTimer timer(kSubUpdateRowCall);
  coefficient_.resize(matrix_.num_cols(), 0.0);
  listed_.resize(matrix_.num_cols(), 0);
  dev_->SetMask(DeviceLp::kRelevant, variables_info_.GetIsRelevantBitRow().data(),
                variables_info_.GetIsRelevantBitRow().NumWords());
  dev_->UpdateRowRowWise(rho_filtered_non_zeros_, rho_.values, 2, params_.drop_tolerance);
  FetchOrDefer();
}

// update_row.cc:220-259
void UpdateRow::ComputeUpdatesRowWiseHypersparse() {
  SubTimer timer(kSubUpdateRowCall);
  coefficient_.resize(matrix_.num_cols(), 0.0);
  listed_.resize(matrix_.num_cols(), 0);
  dev_->SetMask(DeviceLp::kRelevant, variables_info_.GetIsRelevantBitRow().data(),
                variables_info_.GetIsRelevantBitRow().NumWords());
  dev_->UpdateRowRowWise(rho_filtered_non_zeros_, rho_.values, 1, params_.drop_tolerance);
  FetchOrDefer();
}

// update_row.cc:261-280
void UpdateRow::ComputeUpdatesForSingleRow(int row_as_col) {
  SubTimer timer(kSubUpdateRowCall);
  coefficient_.resize(matrix_.num_cols(), 0.0);
  listed_.resize(matrix_.num_cols(), 0);
  dev_->SetMask(DeviceLp::kRelevant, variables_info_.GetIsRelevantBitRow().data(),
                variables_info_.GetIsRelevantBitRow().NumWords());
  const std::vector<int> one(1, row_as_col);
  dev_->UpdateRowRowWise(one, rho_.values, 0, params_.drop_tolerance);
  FetchOrDefer();
}

// update_row.cc:282-306
void UpdateRow::ComputeUpdatesColumnWise() {
  coefficient_.resize(matrix_.num_cols(), 0.0);
  listed_.resize(matrix_.num_cols(), 0);
  const Bitset& relevant = variables_info_.GetIsRelevantBitRow();
  pending_mask_.assign(relevant.data(), relevant.data() + relevant.NumWords());
  pending_relevant_entries_ = variables_info_.GetNumEntriesInRelevantColumns();
  pending_column_wise_ = true;
}

void UpdateRow::RunColumnWise(const std::vector<Fractional>* w) {
  SubTimer timer(kSubUpdateRowCall);
  pending_column_wise_ = false;
  dev_->SetMask(DeviceLp::kRelevant, pending_mask_.data(),
                static_cast<int>(pending_mask_.size()));
  dev_->UpdateRowColumnWise(rho_.values, params_.drop_tolerance, pending_relevant_entries_,
                            w);
  FetchOrDefer();
}

// update_row.cc:311-332
void UpdateRow::ComputeFullUpdateRow(int leaving_row,
                                     std::vector<Fractional>* output) const {
  const int num_cols = matrix_.num_cols();
  output->assign(num_cols, 0.0);
  (*output)[basis_[leaving_row]] = 1.0;
  const Fractional drop_tolerance = params_.drop_tolerance;
  variables_info_.GetNotBasicBitRow().ForEach([&](int col) {
    const Fractional coeff = matrix_.ColumnScalarProduct(col, rho_.values.data());
    if (std::fabs(coeff) > drop_tolerance) (*output)[col] = coeff;
  });
}

// ---------------------------------------------------------------------------
// PrimalEdgeNorms (primal_edge_norms.cc)
class PrimalEdgeNorms {
  friend struct SdualBridge;

 public:
  PrimalEdgeNorms(const CompactSparseMatrix& m, const VariablesInfo& vi,
                  const BasisFactorization& bf, DeviceLp* dev)
      : matrix_(m), variables_info_(vi), bf_(bf), dev_(dev) {}
  void SetParameters(const GlopParameters& p) {
    FlushPendingUpdate();
    params_ = p;
  }
  void SetPricingRule(int rule) {
    FlushPendingUpdate();
    pricing_rule_ = rule;
  }

  // Parked steepest-edge update (engine-side scheduling, no Glop
  // counterpart). When the update row was built row-wise, the a_j . w dots of
  // UpdateEdgeSquaredNorms (primal_edge_norms.cc:229-233) need a pass over A
  // of their own. The update is parked instead, and completed by the next
  // pricing pass, which reads A anyway (ReducedCosts::ComputeReducedCosts ->
  // DeviceLp::Pricing with w), or by a standalone dots pass before anything
  // else reads the norms. PrimalPrices queues the price updates that read
  // the norms meanwhile and replays them, in order, on completion. The
  // arithmetic and its order are unchanged, so results stay bit-identical.
  void SetDeferral(bool on) { defer_enabled_ = on; }
  bool HasPendingUpdate() const { return pending_; }
  const std::vector<Fractional>& PendingDirectionLeftInverse() const {
    return direction_left_inverse_.values;
  }
  uint64_t PendingListEpoch() const { return pending_list_epoch_; }
  void CompletePendingUpdate(const std::vector<Fractional>& dots);
  void FlushPendingUpdate();
  void SetCompletionListener(std::function<void()> f) { on_complete_ = std::move(f); }

  void Clear() {
    FlushPendingUpdate();
    matrix_column_norms_.clear();
    recompute_edge_squared_norms_ = true;
    reset_devex_weights_ = true;
    for (bool* w : watchers_) *w = true;
  }
  bool NeedsBasisRefactorization() const {
    if (pricing_rule_ != 1) return false;
    return recompute_edge_squared_norms_;
  }
  const std::vector<Fractional>& GetSquaredNorms() {
    FlushPendingUpdate();
    switch (pricing_rule_) {
      case 0:
        return GetMatrixColumnNorms();
      case 1:
        return GetEdgeSquaredNorms();
      default:
        return GetDevexWeights();
    }
  }
  const std::vector<Fractional>& GetEdgeSquaredNorms() {
    FlushPendingUpdate();
    if (recompute_edge_squared_norms_) ComputeEdgeSquaredNorms();
    return edge_squared_norms_;
  }
  const std::vector<Fractional>& RawEdgeNorms() const { return edge_squared_norms_; }
  bool TestEnteringEdgeNormPrecision(int entering_col, const ScatteredVector& d);
  void StartDirectionLeftInverse(const ScatteredVector& d);
  void DropDirectionLeftInverse();
  void UpdateBeforeBasisPivot(int entering_col, int leaving_col, int leaving_row,
                              const ScatteredVector& direction, UpdateRow* update_row);
  void AddRecomputationWatcher(bool* w) { watchers_.push_back(w); }
  double DeterministicTime() const {
    return DeterministicTimeForFpOperations(num_operations_);
  }

 private:
  const std::vector<Fractional>& GetDevexWeights() {
    if (reset_devex_weights_) ResetDevexWeights();
    return devex_weights_;
  }
  const std::vector<Fractional>& GetMatrixColumnNorms() {
    if (matrix_column_norms_.empty()) ComputeMatrixColumnNorms();
    return matrix_column_norms_;
  }
  void ComputeMatrixColumnNorms() {
    matrix_column_norms_.resize(matrix_.num_cols(), 0.0);
    for (int col = 0; col < matrix_.num_cols(); ++col) {
      matrix_column_norms_[col] = SquaredNorm(matrix_.column(col));
      num_operations_ += matrix_.column(col).n;
    }
  }
  void ComputeEdgeSquaredNorms() {  // primal_edge_norms.cc:147-161
    edge_squared_norms_.resize(matrix_.num_cols(), 0.0);
    if (bf_.lu().IsIdentityFactorization()) {
      // 1 + ||a_j||^2 (lu_factorization.cc:130) for every relevant column at
      // once on the GPU; the per-solve deterministic-time bump is replayed.
      dev_->SetMask(DeviceLp::kRelevant, variables_info_.GetIsRelevantBitRow().data(),
                    variables_info_.GetIsRelevantBitRow().NumWords());
      dev_->ColumnSquaredNorms(&device_norms_);
      variables_info_.GetIsRelevantBitRow().ForEach([&](int col) {
        bf_.BumpDeterministicTimeForSolve(matrix_.ColumnNumEntries(col));
        edge_squared_norms_[col] = device_norms_[col];
      });
    } else {
      variables_info_.GetIsRelevantBitRow().ForEach([&](int col) {
        edge_squared_norms_[col] = 1.0 + bf_.RightSolveSquaredNorm(matrix_.column(col));
      });
    }
    recompute_edge_squared_norms_ = false;
  }
  void ComputeDirectionLeftInverse(int entering_col, const ScatteredVector& d);
  void SolveDirectionLeftInverse(const ScatteredVector& d, ScatteredVector* out) const;
  void UpdateEdgeSquaredNorms(int entering_col, int leaving_col, int leaving_row,
                              const std::vector<Fractional>& direction,
                              const UpdateRow& update_row);
  void ApplyNormUpdate(const std::vector<int>& positions,
                       const std::vector<Fractional>& coefficients,
                       const std::vector<Fractional>& dots, Fractional pivot,
                       Fractional leaving_squared_norm);
  int64_t CountEntries(const std::vector<int>& positions) const;
  void DeferEdgeSquaredNormsUpdate(int entering_col, int leaving_col, int leaving_row,
                                   const std::vector<Fractional>& direction,
                                   const UpdateRow& update_row);
  void UpdateDevexWeights(int entering_col, int leaving_col, int leaving_row,
                          const std::vector<Fractional>& direction,
                          const UpdateRow& update_row);
  void ResetDevexWeights() {
    if (params_.initialize_devex_with_column_norms) {
      devex_weights_ = GetMatrixColumnNorms();
    } else {
      devex_weights_.assign(matrix_.num_cols(), 1.0);
    }
    num_devex_updates_since_reset_ = 0;
    reset_devex_weights_ = false;
  }

  const CompactSparseMatrix& matrix_;
  const VariablesInfo& variables_info_;
  const BasisFactorization& bf_;
  DeviceLp* dev_;
  std::vector<Fractional> device_norms_;
  std::vector<Fractional> dots_;
  GlopParameters params_;
  int pricing_rule_ = 1;
  bool recompute_edge_squared_norms_ = true;
  bool reset_devex_weights_ = true;
  std::vector<Fractional> edge_squared_norms_;
  std::vector<Fractional> matrix_column_norms_;
  std::vector<Fractional> devex_weights_;
  int num_devex_updates_since_reset_ = 0;
  ScatteredVector direction_left_inverse_;
  ScatteredVector async_w_;
  uint64_t w_ticket_ = 0;
  int64_t num_operations_ = 0;
  std::vector<bool*> watchers_;
  // Parked update (see SetDeferral).
  bool defer_enabled_ = true;
  bool pending_ = false;
  Fractional pending_pivot_ = 0.0;
  Fractional pending_leaving_squared_norm_ = 0.0;
  const UpdateRow* pending_update_row_ = nullptr;
  uint64_t pending_row_epoch_ = 0;
  uint64_t pending_list_epoch_ = 0;
  std::function<void()> on_complete_;
};

// primal_edge_norms.cc:79-108
bool PrimalEdgeNorms::TestEnteringEdgeNormPrecision(int entering_col,
                                                    const ScatteredVector& d) {
  FlushPendingUpdate();
  if (!recompute_edge_squared_norms_) {
    const Fractional old_squared_norm = edge_squared_norms_[entering_col];
    const Fractional precise_squared_norm = 1.0 + SquaredNorm(d);
    edge_squared_norms_[entering_col] = precise_squared_norm;
    const Fractional precise_norm = std::sqrt(precise_squared_norm);
    const Fractional acc = (precise_norm - std::sqrt(old_squared_norm)) / precise_norm;
    if (std::fabs(acc) > params_.recompute_edges_norm_threshold) {
      recompute_edge_squared_norms_ = true;
      for (bool* w : watchers_) *w = true;
    }
    if (old_squared_norm < 0.25 * precise_squared_norm) return false;
  }
  return true;
}

// primal_edge_norms.cc:110-136
void PrimalEdgeNorms::UpdateBeforeBasisPivot(int entering_col, int leaving_col,
                                             int leaving_row,
                                             const ScatteredVector& direction,
                                             UpdateRow* update_row) {
  FlushPendingUpdate();
  if (!recompute_edge_squared_norms_) {
    update_row->ComputeUpdateRow(leaving_row);
    ComputeDirectionLeftInverse(entering_col, direction);
    // Column-wise update row and the a_j . w dots share one pass over A;
    // after a row-wise update row the dots ride on the next pricing pass.
    if (update_row->MaterializeWithDots(direction_left_inverse_.values) ||
        !defer_enabled_ || pricing_rule_ != 1) {
      UpdateEdgeSquaredNorms(entering_col, leaving_col, leaving_row, direction.values,
                             *update_row);
    } else {
      DeferEdgeSquaredNormsUpdate(entering_col, leaving_col, leaving_row, direction.values,
                                  *update_row);
    }
  }
  if (!reset_devex_weights_) {
    ++num_devex_updates_since_reset_;
    if (num_devex_updates_since_reset_ > params_.devex_weights_reset_period) {
      reset_devex_weights_ = true;
    } else {
      update_row->ComputeUpdateRow(leaving_row);
      UpdateDevexWeights(entering_col, leaving_col, leaving_row, direction.values,
                         *update_row);
    }
  }
}

// B^-T d needs only the direction: the factorization's worker computes it
// while the entering tests, the ratio test and the update row run
// (BasisFactorization::StartAsyncLeftSolve), into a copy of
// direction_left_inverse_ that replaces it when taken.
void PrimalEdgeNorms::StartDirectionLeftInverse(const ScatteredVector& d) {
  w_ticket_ = 0;
  if (pricing_rule_ != 1 || recompute_edge_squared_norms_ || pending_) return;
  w_ticket_ = bf_.StartAsyncLeftSolve([this, &d]() {
    async_w_ = direction_left_inverse_;
    SolveDirectionLeftInverse(d, &async_w_);
  });
}

void PrimalEdgeNorms::DropDirectionLeftInverse() {
  if (w_ticket_ != 0) bf_.DropAsync(w_ticket_);
  w_ticket_ = 0;
}

// primal_edge_norms.cc:166-199
void PrimalEdgeNorms::ComputeDirectionLeftInverse(int /*entering_col*/,
                                                  const ScatteredVector& d) {
  SubTimer timer(kSubBtranW);
  const uint64_t ticket = w_ticket_;
  w_ticket_ = 0;
  if (ticket != 0 && bf_.TakeAsync(ticket)) {
    std::swap(direction_left_inverse_, async_w_);
    return;
  }
  SolveDirectionLeftInverse(d, &direction_left_inverse_);
}

void PrimalEdgeNorms::SolveDirectionLeftInverse(const ScatteredVector& d,
                                                ScatteredVector* out) const {
  ScatteredVector& direction_left_inverse_ = *out;
  const int size = d.size();
  const double kThreshold = 0.05 * size;
  if (!direction_left_inverse_.non_zeros.empty() &&
      (direction_left_inverse_.non_zeros.size() + d.non_zeros.size() <
       2 * kThreshold)) {
    ClearAndResizeVectorWithNonZeros(size, &direction_left_inverse_);
    for (const int row : d.non_zeros) direction_left_inverse_[row] = d.values[row];
  } else {
    direction_left_inverse_.values = d.values;
    direction_left_inverse_.non_zeros.clear();
  }
  if (d.non_zeros.size() < kThreshold) {
    direction_left_inverse_.non_zeros = d.non_zeros;
  }
  bf_.LeftSolve(&direction_left_inverse_);
}

// primal_edge_norms.cc:208-258
void PrimalEdgeNorms::UpdateEdgeSquaredNorms(int entering_col, int leaving_col,
                                             int leaving_row,
                                             const std::vector<Fractional>& direction,
                                             const UpdateRow& update_row) {
  const Fractional pivot = -direction[leaving_row];
  const Fractional entering_squared_norm = edge_squared_norms_[entering_col];
  const Fractional leaving_squared_norm =
      std::max(1.0, entering_squared_norm / Square(pivot));
  SubTimer timer(kSubNormLoop);
  // a_j . (B^-T d) for every listed column in one GPU pass.
  dev_->ListDotsOverUpdateRow(direction_left_inverse_.values, &dots_);
  const std::vector<int>& positions = update_row.GetNonZeroPositions();
  num_operations_ += CountEntries(positions);
  ApplyNormUpdate(positions, update_row.GetCoefficients(), dots_, pivot, leaving_squared_norm);
  edge_squared_norms_[leaving_col] = leaving_squared_norm;
}

// The per-column loop of UpdateEdgeSquaredNorms (primal_edge_norms.cc:229-
// 244), positions in parallel (each writes its own norm).
void PrimalEdgeNorms::ApplyNormUpdate(const std::vector<int>& positions,
                                      const std::vector<Fractional>& coefficients,
                                      const std::vector<Fractional>& dots, Fractional pivot,
                                      Fractional leaving_squared_norm) {
  const Fractional factor = 2.0 / pivot;
  Fractional* norms = edge_squared_norms_.data();
  const Fractional* coeffs = coefficients.data();
  ParallelRanges(static_cast<int64_t>(positions.size()), 16384, 1,
                 [&](int, int64_t b, int64_t e) {
    for (int64_t k = b; k < e; ++k) {
      const int col = positions[k];
      const Fractional coeff = coeffs[col];
      norms[col] += coeff * (coeff * leaving_squared_norm + factor * dots[k]);
      const Fractional lower_bound = 1.0 + Square(coeff / pivot);
      if (norms[col] < lower_bound) norms[col] = lower_bound;
    }
  });
}

int64_t PrimalEdgeNorms::CountEntries(const std::vector<int>& positions) const {
  std::vector<int64_t> part(HostPool::Get().threads(), 0);
  const int parts = ParallelRanges(static_cast<int64_t>(positions.size()), 16384, 1,
                                   [&](int p, int64_t b, int64_t e) {
    int64_t n = 0;
    for (int64_t k = b; k < e; ++k) n += matrix_.ColumnNumEntries(positions[k]);
    part[p] = n;
  });
  int64_t total = 0;
  for (int p = 0; p < parts; ++p) total += part[p];
  return total;
}

// UpdateEdgeSquaredNorms split in two: the scalars now, the loop over the
// update row once its dots are known (CompletePendingUpdate).
void PrimalEdgeNorms::DeferEdgeSquaredNormsUpdate(int entering_col, int leaving_col,
                                                  int leaving_row,
                                                  const std::vector<Fractional>& direction,
                                                  const UpdateRow& update_row) {
  pending_pivot_ = -direction[leaving_row];
  const Fractional entering_squared_norm = edge_squared_norms_[entering_col];
  pending_leaving_squared_norm_ =
      std::max(1.0, entering_squared_norm / Square(pending_pivot_));
  num_operations_ += CountEntries(update_row.GetNonZeroPositions());
  // The leaving column is basic, hence not relevant and never one of the
  // listed positions: its final value can be written now.
  edge_squared_norms_[leaving_col] = pending_leaving_squared_norm_;
  pending_update_row_ = &update_row;
  pending_row_epoch_ = update_row.epoch();
  pending_list_epoch_ = dev_->list_epoch();
  pending_ = true;
}

void PrimalEdgeNorms::CompletePendingUpdate(const std::vector<Fractional>& dots) {
  if (!pending_) return;
  pending_ = false;
  if (pending_update_row_->epoch() != pending_row_epoch_) {
    throw DeviceError("update row recomputed under a parked edge-norm update");
  }
  const std::vector<int>& positions = pending_update_row_->GetNonZeroPositions();
  if (dots.size() != positions.size()) throw DeviceError("edge-norm dots size mismatch");
  {
    SubTimer timer(kSubNormLoop);
    ApplyNormUpdate(positions, pending_update_row_->GetCoefficients(), dots, pending_pivot_,
                    pending_leaving_squared_norm_);
  }
  if (on_complete_) on_complete_();
}

void PrimalEdgeNorms::FlushPendingUpdate() {
  if (!pending_) return;
  if (dev_->list_epoch() == pending_list_epoch_) {
    dev_->ListDotsOverUpdateRow(direction_left_inverse_.values, &dots_);
  } else {
    dev_->ListDots(pending_update_row_->GetNonZeroPositions(), direction_left_inverse_.values,
                   &dots_);
  }
  CompletePendingUpdate(dots_);
}

// primal_edge_norms.cc:260-281
void PrimalEdgeNorms::UpdateDevexWeights(int /*entering_col*/, int leaving_col,
                                         int leaving_row,
                                         const std::vector<Fractional>& direction,
                                         const UpdateRow& update_row) {
  KahanSum s;
  for (const Fractional v : direction) s.Add(Square(v));
  const Fractional entering_norm = std::sqrt(s.Value());
  const Fractional pivot_magnitude = std::fabs(direction[leaving_row]);
  const Fractional leaving_norm = std::max(1.0, entering_norm / pivot_magnitude);
  for (const int col : update_row.GetNonZeroPositions()) {
    const Fractional coeff = update_row.GetCoefficient(col);
    const Fractional update_vector_norm = std::fabs(coeff) * leaving_norm;
    devex_weights_[col] = std::max(devex_weights_[col], Square(update_vector_norm));
  }
  devex_weights_[leaving_col] = Square(leaving_norm);
}

// ---------------------------------------------------------------------------
// ReducedCosts (reduced_costs.cc:24-510)
class ReducedCosts {
  friend struct SdualBridge;
  friend struct SdualHooks;

 public:
  ReducedCosts(const CompactSparseMatrix& m, const std::vector<Fractional>& obj,
               const std::vector<int>& basis, const VariablesInfo& vi,
               const BasisFactorization& bf, Rng* random, DeviceLp* dev)
      : matrix_(m), objective_(obj), basis_(basis), variables_info_(vi), bf_(bf),
        random_(random), dev_(dev) {}
  void SetParameters(const GlopParameters& p) { params_ = p; }
  // The primal edge norms whose parked update the pricing pass completes.
  void SetDeferredNorms(PrimalEdgeNorms* norms) { deferred_norms_ = norms; }
  bool WillRecompute() const { return recompute_reduced_costs_; }
  bool NeedsBasisRefactorization() const { return must_refactorize_basis_; }
  Fractional TestEnteringReducedCostPrecision(int entering_col, const ScatteredVector& d);
  Fractional ComputeMaximumDualResidual();
  Fractional ComputeMaximumDualInfeasibility();
  Fractional ComputeMaximumDualInfeasibilityOnNonBoxedVariables();
  void UpdateBeforeBasisPivot(int entering_col, int leaving_row,
                              const ScatteredVector& direction, UpdateRow* update_row) {
    const int leaving_col = basis_[leaving_row];
    if (!recompute_reduced_costs_) {
      UpdateReducedCosts(entering_col, leaving_col, leaving_row, direction[leaving_row],
                         update_row);
    }
    UpdateBasicObjective(entering_col, leaving_row);
  }
  void SetNonBasicVariableCostToZero(int col, Fractional* current_cost) {
    SyncHost();  // primal only; never in dual device mode
    reduced_costs_[col] -= objective_[col];
    *current_cost = 0.0;
  }
  // Dual device mode (RevisedSimplex::DualDeviceMode): the device copy of the
  // reduced costs is the reference; the host vector is refreshed from it
  // only when host code reads it. The entering column's value is handed over
  // by the device ratio test.
  void EnterDeviceMode() {
    device_mode_ = true;
    host_stale_ = false;
  }
  void LeaveDeviceMode() {
    SyncHost();
    device_mode_ = false;
    known_col_ = -1;
  }
  bool InDeviceMode() const { return device_mode_; }
  void SetKnownReducedCost(int col, Fractional value) {
    known_col_ = col;
    known_value_ = value;
  }
  // The side effects of GetReducedCosts() (recompute, refactorization flag)
  // without refreshing the host copy.
  void PrepareForDeviceUse() {
    if (bf_.IsRefactorized()) must_refactorize_basis_ = false;
    if (recompute_reduced_costs_) ComputeReducedCosts();
  }
  bool AreReducedCostsPrecise() const { return are_reduced_costs_precise_; }
  bool AreReducedCostsRecomputed() const {
    return recompute_reduced_costs_ || are_reduced_costs_recomputed_;
  }
  void MakeReducedCostsPrecise() {
    if (are_reduced_costs_precise_) return;
    must_refactorize_basis_ = true;
    recompute_basic_objective_left_inverse_ = true;
    SetRecomputeReducedCostsAndNotifyWatchers();
  }
  void PerturbCosts();
  void ShiftCostIfNeeded(bool increasing_rc_is_needed, int col);
  bool HasCostShift() const { return has_cost_shift_; }
  void ClearAndRemoveCostShifts() {
    has_cost_shift_ = false;
    cost_perturbations_.assign(matrix_.num_cols(), 0.0);
    recompute_basic_objective_ = true;
    recompute_basic_objective_left_inverse_ = true;
    are_reduced_costs_precise_ = false;
    SetRecomputeReducedCostsAndNotifyWatchers();
  }
  void ResetForNewObjective() {
    recompute_basic_objective_ = true;
    recompute_basic_objective_left_inverse_ = true;
    are_reduced_costs_precise_ = false;
    SetRecomputeReducedCostsAndNotifyWatchers();
  }
  void UpdateDataOnBasisPermutation() {
    recompute_basic_objective_ = true;
    recompute_basic_objective_left_inverse_ = true;
  }
  const std::vector<Fractional>& GetReducedCosts() {
    SyncHost();
    if (bf_.IsRefactorized()) must_refactorize_basis_ = false;
    if (recompute_reduced_costs_) ComputeReducedCosts();
    return reduced_costs_;
  }
  const std::vector<Fractional>& RawReducedCosts() const {
    const_cast<ReducedCosts*>(this)->SyncHost();
    return reduced_costs_;
  }
  const std::vector<Fractional>& GetFullReducedCosts() {
    if (!are_reduced_costs_recomputed_) SetRecomputeReducedCostsAndNotifyWatchers();
    return GetReducedCosts();
  }
  const std::vector<Fractional>& GetDualValues() {
    ComputeBasicObjectiveLeftInverse();
    return basic_objective_left_inverse_.values;
  }
  Fractional GetDualFeasibilityTolerance() const { return dual_feasibility_tolerance_; }
  bool IsValidPrimalEnteringCandidate(int col) const {
    const Fractional rc = reduced_costs_[col];
    const Fractional tol = dual_feasibility_tolerance_;
    return (variables_info_.GetCanIncreaseBitRow().IsSet(col) && (rc < -tol)) ||
           (variables_info_.GetCanDecreaseBitRow().IsSet(col) && (rc > tol));
  }
  double DeterministicTime() const { return deterministic_time_; }
  void AddRecomputationWatcher(bool* w) { watchers_.push_back(w); }

 private:
  void ComputeBasicObjective() {  // reduced_costs.cc:338-350
    const int n = matrix_.num_rows();
    cost_perturbations_.resize(matrix_.num_cols(), 0.0);
    basic_objective_.resize(n, 0.0);
    for (int col = 0; col < n; ++col) {
      const int basis_col = basis_[col];
      basic_objective_[col] = objective_[basis_col] + cost_perturbations_[basis_col];
    }
    recompute_basic_objective_ = false;
    recompute_basic_objective_left_inverse_ = true;
  }
  void ComputeReducedCosts();
  void ComputeBasicObjectiveLeftInverse() {  // reduced_costs.cc:425-439
    SubTimer timer(kSubBtranY);
    if (recompute_basic_objective_) ComputeBasicObjective();
    basic_objective_left_inverse_.values = basic_objective_;
    basic_objective_left_inverse_.non_zeros.clear();
    bf_.LeftSolve(&basic_objective_left_inverse_);
    recompute_basic_objective_left_inverse_ = false;
  }
  void UpdateReducedCosts(int entering_col, int leaving_col, int leaving_row,
                          Fractional pivot, UpdateRow* update_row);
  void UpdateBasicObjective(int entering_col, int leaving_row) {
    basic_objective_[leaving_row] =
        objective_[entering_col] + cost_perturbations_[entering_col];
    recompute_basic_objective_left_inverse_ = true;
  }
  void SetRecomputeReducedCostsAndNotifyWatchers() {
    recompute_reduced_costs_ = true;
    for (bool* w : watchers_) *w = true;
  }
  void SyncHost() {
    if (!device_mode_ || !host_stale_) return;
    dev_->DualDownloadReducedCosts(&reduced_costs_);
    host_stale_ = false;
  }

  const CompactSparseMatrix& matrix_;
  const std::vector<Fractional>& objective_;
  const std::vector<int>& basis_;
  const VariablesInfo& variables_info_;
  const BasisFactorization& bf_;
  Rng* random_;
  DeviceLp* dev_;
  PrimalEdgeNorms* deferred_norms_ = nullptr;
  bool device_mode_ = false;
  bool host_stale_ = false;
  int known_col_ = -1;
  Fractional known_value_ = 0.0;
  std::vector<Fractional> fused_rc_;
  std::vector<Fractional> fused_dots_;
  std::vector<Fractional> shifted_objective_;
  std::vector<Fractional> dots_;
  GlopParameters params_;
  bool must_refactorize_basis_ = false;
  bool recompute_basic_objective_left_inverse_ = true;
  bool recompute_basic_objective_ = true;
  bool recompute_reduced_costs_ = true;
  bool are_reduced_costs_precise_ = false;
  bool are_reduced_costs_recomputed_ = false;
  bool has_cost_shift_ = false;
  std::vector<Fractional> basic_objective_;
  std::vector<Fractional> cost_perturbations_;
  std::vector<Fractional> reduced_costs_;
  ScatteredVector basic_objective_left_inverse_;
  Fractional dual_feasibility_tolerance_ = 0.0;
  std::vector<bool*> watchers_;
  double deterministic_time_ = 0.0;
};

// reduced_costs.cc:53-94
Fractional ReducedCosts::TestEnteringReducedCostPrecision(int entering_col,
                                                          const ScatteredVector& d) {
  if (recompute_basic_objective_) ComputeBasicObjective();
  const Fractional old_reduced_cost = reduced_costs_[entering_col];
  const Fractional precise_reduced_cost =
      objective_[entering_col] + cost_perturbations_[entering_col] -
      ScalarProduct(basic_objective_, d);
  reduced_costs_[entering_col] = precise_reduced_cost;
  if (!recompute_reduced_costs_) {
    const Fractional acc = old_reduced_cost - precise_reduced_cost;
    const Fractional scale =
        (std::fabs(precise_reduced_cost) <= 1.0) ? 1.0 : precise_reduced_cost;
    if (std::fabs(acc) / scale > params_.recompute_reduced_costs_threshold) {
      MakeReducedCostsPrecise();
    }
  }
  return precise_reduced_cost;
}

// reduced_costs.cc:96-110
Fractional ReducedCosts::ComputeMaximumDualResidual() {
  Fractional err = 0.0;
  const int num_rows = matrix_.num_rows();
  const std::vector<Fractional>& y = GetDualValues();
  if (dev_->host_small_ops()) {
    dots_.resize(num_rows);
    for (int row = 0; row < num_rows; ++row) dots_[row] = matrix_.ColumnScalarProduct(basis_[row], y);
  } else {
    dev_->ListDots(basis_, y, &dots_);  // a_{B(r)} . y on the GPU
  }
  for (int row = 0; row < num_rows; ++row) {
    const int basic_col = basis_[row];
    const Fractional residual =
        objective_[basic_col] + cost_perturbations_[basic_col] - dots_[row];
    err = std::max(err, std::fabs(residual));
  }
  return err;
}

// reduced_costs.cc:112-128
Fractional ReducedCosts::ComputeMaximumDualInfeasibility() {
  GetReducedCosts();
  Fractional m = 0.0;
  const Bitset& dec = variables_info_.GetCanDecreaseBitRow();
  const Bitset& inc = variables_info_.GetCanIncreaseBitRow();
  variables_info_.GetIsRelevantBitRow().ForEach([&](int col) {
    const Fractional rc = reduced_costs_[col];
    if ((inc.IsSet(col) && rc < 0.0) || (dec.IsSet(col) && rc > 0.0))
      m = std::max(m, std::fabs(rc));
  });
  return m;
}

// reduced_costs.cc:130-148
Fractional ReducedCosts::ComputeMaximumDualInfeasibilityOnNonBoxedVariables() {
  GetReducedCosts();
  Fractional m = 0.0;
  const Bitset& dec = variables_info_.GetCanDecreaseBitRow();
  const Bitset& inc = variables_info_.GetCanIncreaseBitRow();
  const Bitset& boxed = variables_info_.GetNonBasicBoxedVariables();
  variables_info_.GetNotBasicBitRow().ForEach([&](int col) {
    if (boxed[col]) return;
    const Fractional rc = reduced_costs_[col];
    if ((inc.IsSet(col) && rc < 0.0) || (dec.IsSet(col) && rc > 0.0))
      m = std::max(m, std::fabs(rc));
  });
  return m;
}

// reduced_costs.cc:226-275
void ReducedCosts::PerturbCosts() {
  Fractional max_cost_magnitude = 0.0;
  const int structural_size = matrix_.num_cols() - matrix_.num_rows();
  for (int col = 0; col < structural_size; ++col)
    max_cost_magnitude = std::max(max_cost_magnitude, std::fabs(objective_[col]));
  cost_perturbations_.assign(matrix_.num_cols(), 0.0);
  for (int col = 0; col < structural_size; ++col) {
    const Fractional objective = objective_[col];
    const Fractional magnitude =
        (1.0 + std::uniform_real_distribution<double>()(*random_)) *
        (params_.relative_cost_perturbation * std::fabs(objective) +
         params_.relative_max_cost_perturbation * max_cost_magnitude);
    switch (variables_info_.GetTypeRow()[col]) {
      case VariableType::UNCONSTRAINED:
      case VariableType::FIXED_VARIABLE:
        break;
      case VariableType::LOWER_BOUNDED:
        cost_perturbations_[col] = magnitude;
        break;
      case VariableType::UPPER_BOUNDED:
        cost_perturbations_[col] = -magnitude;
        break;
      case VariableType::UPPER_AND_LOWER_BOUNDED:
        if (objective > 0.0) {
          cost_perturbations_[col] = magnitude;
        } else if (objective < 0.0) {
          cost_perturbations_[col] = -magnitude;
        }
        break;
    }
  }
}

// reduced_costs.cc:277-294
void ReducedCosts::ShiftCostIfNeeded(bool increasing_rc_is_needed, int col) {
  const Fractional minimum_delta =
      params_.degenerate_ministep_factor * dual_feasibility_tolerance_;
  if (device_mode_) {
    if (known_col_ != col) throw DeviceError("dual device mode: entering reduced cost unknown");
    if (increasing_rc_is_needed && known_value_ <= -minimum_delta) return;
    if (!increasing_rc_is_needed && known_value_ >= minimum_delta) return;
    const Fractional delta = increasing_rc_is_needed ? minimum_delta : -minimum_delta;
    cost_perturbations_[col] -= known_value_ + delta;
    known_value_ = -delta;
    dev_->DualSetReducedCost(col, known_value_);
    host_stale_ = true;
    has_cost_shift_ = true;
    return;
  }
  if (increasing_rc_is_needed && reduced_costs_[col] <= -minimum_delta) return;
  if (!increasing_rc_is_needed && reduced_costs_[col] >= minimum_delta) return;
  const Fractional delta = increasing_rc_is_needed ? minimum_delta : -minimum_delta;
  cost_perturbations_[col] -= reduced_costs_[col] + delta;
  reduced_costs_[col] = -delta;
  has_cost_shift_ = true;
}

// reduced_costs.cc:352-423 (single-threaded path; the OMP branch does not
// compile upstream).
void ReducedCosts::ComputeReducedCosts() {
  if (recompute_basic_objective_left_inverse_) ComputeBasicObjectiveLeftInverse();
  Fractional dual_residual_error = 0.0;
  const int num_cols = matrix_.num_cols();
  reduced_costs_.resize(num_cols, 0.0);
  const Bitset& is_basic = variables_info_.GetIsBasicBitRow();
  cost_perturbations_.resize(num_cols, 0.0);
  shifted_objective_.resize(num_cols);
  for (int col = 0; col < num_cols; ++col)
    shifted_objective_[col] = objective_[col] + cost_perturbations_[col];
  // rc_j = (c_j + delta_j) - a_j . y for all N columns: the pricing SpMV.
  const std::vector<Fractional>& y = basic_objective_left_inverse_.values;
  SubTimer pricing_timer(kSubPricingCall);
  if (deferred_norms_ != nullptr && deferred_norms_->HasPendingUpdate()) {
    if (dev_->list_epoch() == deferred_norms_->PendingListEpoch()) {
      // One pass over A: rc for every column plus the parked edge-norm dots.
      // The parked update (and the price updates queued behind it) completes
      // while reduced_costs_ still holds the values they were issued with.
      dev_->Pricing(shifted_objective_, y, &fused_rc_,
                    &deferred_norms_->PendingDirectionLeftInverse(), &fused_dots_);
      deferred_norms_->CompletePendingUpdate(fused_dots_);
      reduced_costs_.swap(fused_rc_);
    } else {
      deferred_norms_->FlushPendingUpdate();
      dev_->Pricing(shifted_objective_, y, &reduced_costs_);
    }
  } else if (dev_->host_small_ops() && !device_mode_) {
    reduced_costs_.resize(num_cols);
    for (int col = 0; col < num_cols; ++col)
      reduced_costs_[col] = shifted_objective_[col] - matrix_.ColumnScalarProduct(col, y);
  } else {
    dev_->Pricing(shifted_objective_, y, &reduced_costs_);
  }
  if (device_mode_) {
    dev_->DualTakePricedReducedCosts();
    host_stale_ = false;
  }
  is_basic.ForEach([&](int col) {
    dual_residual_error = std::max(dual_residual_error, std::fabs(reduced_costs_[col]));
  });
  deterministic_time_ += DeterministicTimeForFpOperations(matrix_.num_entries());
  recompute_reduced_costs_ = false;
  are_reduced_costs_recomputed_ = true;
  are_reduced_costs_precise_ = bf_.IsRefactorized();
  dual_feasibility_tolerance_ = params_.dual_feasibility_tolerance;
  if (dual_residual_error > dual_feasibility_tolerance_) {
    dual_feasibility_tolerance_ = dual_residual_error;
  }
}

// reduced_costs.cc:444-488
void ReducedCosts::UpdateReducedCosts(int entering_col, int leaving_col, int leaving_row,
                                      Fractional pivot, UpdateRow* update_row) {
  if (recompute_reduced_costs_) return;
  if (device_mode_) {
    if (known_col_ != entering_col) {
      throw DeviceError("dual device mode: entering reduced cost unknown");
    }
    const Fractional entering_reduced_cost = known_value_;
    if (entering_reduced_cost == 0.0) {
      are_reduced_costs_precise_ = false;
      return;
    }
    are_reduced_costs_recomputed_ = false;
    are_reduced_costs_precise_ = false;
    update_row->ComputeUpdateRow(leaving_row);
    const Fractional new_leaving_reduced_cost = entering_reduced_cost / -pivot;
    dev_->DualUpdateReducedCosts(new_leaving_reduced_cost, leaving_col,
                                 new_leaving_reduced_cost, entering_col);
    host_stale_ = true;
    known_col_ = -1;
    return;
  }
  const Fractional entering_reduced_cost = reduced_costs_[entering_col];
  if (entering_reduced_cost == 0.0) {
    are_reduced_costs_precise_ = false;
    return;
  }
  are_reduced_costs_recomputed_ = false;
  are_reduced_costs_precise_ = false;
  update_row->ComputeUpdateRow(leaving_row);
  const Fractional new_leaving_reduced_cost = entering_reduced_cost / -pivot;
  const std::vector<int>& positions = update_row->GetNonZeroPositions();
  const Fractional* coeffs = update_row->GetCoefficients().data();
  Fractional* rc = reduced_costs_.data();
  ParallelRanges(static_cast<int64_t>(positions.size()), 16384, 1,
                 [&](int, int64_t b, int64_t e) {
    for (int64_t k = b; k < e; ++k) {
      const int col = positions[k];
      rc[col] += new_leaving_reduced_cost * coeffs[col];
    }
  });
  reduced_costs_[leaving_col] = new_leaving_reduced_cost;
  reduced_costs_[entering_col] = 0.0;
}

// ---------------------------------------------------------------------------
// PrimalPrices (reduced_costs.cc:512-600)
class PrimalPrices {
  friend struct SdualBridge;

 public:
  PrimalPrices(Rng* random, const VariablesInfo& vi, PrimalEdgeNorms* pen,
               ReducedCosts* rc)
      : prices_(random), variables_info_(vi), primal_edge_norms_(pen),
        reduced_costs_(rc) {
    reduced_costs_->AddRecomputationWatcher(&recompute_);
    primal_edge_norms_->AddRecomputationWatcher(&recompute_);
    primal_edge_norms_->SetCompletionListener([this]() { ReplayQueue(); });
  }
  int GetBestEnteringColumn() {
    // A parked edge-norm update completes inside the pricing pass when the
    // reduced costs are about to be recomputed, otherwise right here.
    if (!recompute_ || !reduced_costs_->WillRecompute()) {
      primal_edge_norms_->FlushPendingUpdate();
    }
    if (recompute_) {
      const std::vector<Fractional>& rc = reduced_costs_->GetReducedCosts();
      primal_edge_norms_->FlushPendingUpdate();  // no-op after the fused pass
      SubTimer timer(kSubCandidatesFull);
      prices_.ClearAndResize(static_cast<int>(rc.size()));
      RebuildEnteringCandidates();
      recompute_ = false;
    }
    SubTimer timer(kSubGetMaximum);
    return prices_.GetMaximum();
  }
  void UpdateBeforeBasisPivot(int entering_col, UpdateRow* update_row) {
    if (recompute_) return;
    if (primal_edge_norms_->HasPendingUpdate()) {
      QueueEnteringCandidates(entering_col, *update_row);
      return;
    }
    UpdateEnteringCandidates<false>(update_row->GetNonZeroPositions());
  }
  void RecomputePriceAt(int col) {
    if (recompute_) return;
    if (primal_edge_norms_->HasPendingUpdate()) {
      const bool valid = reduced_costs_->IsValidPrimalEnteringCandidate(col);
      if (valid) reduced_costs_->GetReducedCosts();  // its side effects happen now
      queue_.push_back(QueuedOp{col, valid ? kAdd : kRemove});
      return;
    }
    if (reduced_costs_->IsValidPrimalEnteringCandidate(col)) {
      const std::vector<Fractional>& sn = primal_edge_norms_->GetSquaredNorms();
      const std::vector<Fractional>& rc = reduced_costs_->GetReducedCosts();
      prices_.AddOrUpdate(col, Square(rc[col]) / sn[col]);
    } else {
      prices_.Remove(col);
    }
  }
  void SetAndDebugCheckThatColumnIsDualFeasible(int col) {
    if (recompute_) return;
    if (primal_edge_norms_->HasPendingUpdate()) {
      queue_.push_back(QueuedOp{col, kRemove});
      return;
    }
    prices_.Remove(col);
  }
  void ForceRecomputation() { recompute_ = true; }

 private:
  // Price updates issued while the edge-norm update is parked, replayed in
  // order once the norms are complete and before any reduced cost changes.
  // A single-column op has its candidate test done at issue time. The
  // update-row block (UpdateEnteringCandidates<false> over the listed
  // positions) is re-evaluated at replay from the live state: until then the
  // reduced costs of those positions, the tolerance and the can-increase /
  // can-decrease bits do not change, except the bits of the entering column
  // (UpdateBasis), whose decision is taken at issue time.
  enum OpKind : int8_t { kRemove = 0, kAdd = 1, kUpdateRowBlock = 2 };
  struct QueuedOp {
    int col;
    OpKind kind;
  };
  bool IsDualInfeasible(int col, Fractional reduced_cost, Fractional tolerance) const {
    return ((reduced_cost > tolerance) && variables_info_.GetCanDecreaseBitRow().IsSet(col)) !=
           ((reduced_cost < -tolerance) && variables_info_.GetCanIncreaseBitRow().IsSet(col));
  }
  void QueueEnteringCandidates(int entering_col, const UpdateRow& update_row) {
    SubTimer timer(kSubQueue);
    block_tolerance_ = reduced_costs_->GetDualFeasibilityTolerance();
    const std::vector<Fractional>& rc = reduced_costs_->GetReducedCosts();
    block_row_ = &update_row;
    block_epoch_ = update_row.epoch();
    block_entering_col_ = entering_col;
    block_entering_infeasible_ = IsDualInfeasible(entering_col, rc[entering_col],
                                                  block_tolerance_);
    queue_.push_back(QueuedOp{entering_col, kUpdateRowBlock});
  }
  void ReplayQueue() {
    SubTimer timer(kSubQueue);
    const std::vector<Fractional>& sn = primal_edge_norms_->RawEdgeNorms();
    const std::vector<Fractional>& rc = reduced_costs_->RawReducedCosts();
    // When the prices are about to be rebuilt from scratch (every reader
    // checks recompute_ first, GetBestEnteringColumn clears them), only the
    // top-k bookkeeping matters: it may draw from the RNG.
    const bool before_clear = recompute_;
    for (const QueuedOp& op : queue_) {
      if (op.kind == kUpdateRowBlock) {
        if (block_row_->epoch() != block_epoch_) {
          throw DeviceError("update row recomputed under queued price updates");
        }
        const int entering = block_entering_col_;
        const bool entering_infeasible = block_entering_infeasible_;
        const Fractional tolerance = block_tolerance_;
        UpdatePricesOver(block_row_->GetNonZeroPositions(), !before_clear, [&](int col) {
          return col == entering ? entering_infeasible : IsDualInfeasible(col, rc[col], tolerance);
        }, rc.data(), sn.data());
      } else if (op.kind == kAdd) {
        const Fractional price = Square(rc[op.col]) / sn[op.col];
        if (before_clear) {
          prices_.AddOrUpdateBeforeClear(op.col, price);
        } else {
          prices_.AddOrUpdate(op.col, price);
        }
      } else if (!before_clear) {
        prices_.Remove(op.col);
      }
    }
    queue_.clear();
  }
  const UpdateRow* block_row_ = nullptr;
  uint64_t block_epoch_ = 0;
  int block_entering_col_ = -1;
  bool block_entering_infeasible_ = false;
  Fractional block_tolerance_ = 0.0;
  std::vector<QueuedOp> queue_;
  // UpdateEnteringCandidates<from_clean_state=true> over the relevant
  // columns (reduced_costs.cc:557-600), walking the bitset words directly.
  void RebuildEnteringCandidates() {
    const Fractional tolerance = reduced_costs_->GetDualFeasibilityTolerance();
    const uint64_t* dec = variables_info_.GetCanDecreaseBitRow().data();
    const uint64_t* inc = variables_info_.GetCanIncreaseBitRow().data();
    const Bitset& relevant = variables_info_.GetIsRelevantBitRow();
    const uint64_t* rel = relevant.data();
    const Fractional* sn = primal_edge_norms_->GetSquaredNorms().data();
    const Fractional* rc = reduced_costs_->GetReducedCosts().data();
    Fractional* values = prices_.mutable_values();
    uint64_t* candidate = prices_.mutable_candidate_words();
    const int num_words = relevant.NumWords();
    part_adds_.resize(HostPool::Get().threads());
    // Words are split whole, so each candidate word has one writer.
    const int parts = ParallelRanges(num_words, kMinParallelWords, 1,
                                     [&](int p, int64_t w0, int64_t w1) {
      // A local vector (header on this thread's stack), handed back at the end.
      std::vector<PriceUpdate> adds;
      adds.swap(part_adds_[p].v);
      adds.clear();
      for (int64_t w = w0; w < w1; ++w) {
        uint64_t bits = rel[w];
        const uint64_t dec_w = dec[w];
        const uint64_t inc_w = inc[w];
        uint64_t set = 0;
        while (bits != 0) {
          const int b = __builtin_ctzll(bits);
          bits &= bits - 1;
          const int col = static_cast<int>(w << 6) + b;
          const Fractional reduced_cost = rc[col];
          const bool is_dual_infeasible = ((reduced_cost > tolerance) && ((dec_w >> b) & 1)) !=
                                          ((reduced_cost < -tolerance) && ((inc_w >> b) & 1));
          if (is_dual_infeasible) {
            const Fractional price = Square(reduced_cost) / sn[col];
            values[col] = price;
            set |= uint64_t{1} << b;
            adds.push_back(PriceUpdate{col, price});
          }
        }
        candidate[w] |= set;
      }
      part_adds_[p].v.swap(adds);
    });
    for (int p = 0; p < parts; ++p) {
      for (const PriceUpdate& u : part_adds_[p].v) prices_.ReplayTopK(u.col, u.price);
    }
  }
  // The per-position loop of UpdateEnteringCandidates / the queued
  // update-row block: add(col) decides dual infeasibility; with
  // write_state, AddOrUpdate or Remove, else only the top-k bookkeeping of
  // the adds (AddOrUpdateBeforeClear). Prices and candidate bits are written
  // in parallel (positions are distinct; bits with atomic word updates), the
  // top-k replay runs serially in position order.
  template <typename AddFn>
  void UpdatePricesOver(const std::vector<int>& cols, bool write_state, AddFn&& add,
                        const Fractional* rc, const Fractional* sn) {
    Fractional* values = prices_.mutable_values();
    uint64_t* candidate = prices_.mutable_candidate_words();
    part_adds_.resize(HostPool::Get().threads());
    const int parts = ParallelRanges(static_cast<int64_t>(cols.size()), kMinParallelPositions, 1,
                                     [&](int p, int64_t b, int64_t e) {
      std::vector<PriceUpdate> adds;
      adds.swap(part_adds_[p].v);
      adds.clear();
      for (int64_t k = b; k < e; ++k) {
        const int col = cols[k];
        const uint64_t mask = uint64_t{1} << (col & 63);
        if (add(col)) {
          const Fractional price = Square(rc[col]) / sn[col];
          if (write_state) {
            values[col] = price;
            __atomic_fetch_or(&candidate[col >> 6], mask, __ATOMIC_RELAXED);
          }
          adds.push_back(PriceUpdate{col, price});
        } else if (write_state) {
          __atomic_fetch_and(&candidate[col >> 6], ~mask, __ATOMIC_RELAXED);
        }
      }
      part_adds_[p].v.swap(adds);
    });
    for (int p = 0; p < parts; ++p) {
      for (const PriceUpdate& u : part_adds_[p].v) prices_.ReplayTopK(u.col, u.price);
    }
  }
  struct PriceUpdate {
    int col;
    Fractional price;
  };
  static constexpr int64_t kMinParallelWords = 256;        // 16384 columns
  static constexpr int64_t kMinParallelPositions = 16384;
  struct alignas(64) PartAdds {
    std::vector<PriceUpdate> v;
  };
  std::vector<PartAdds> part_adds_;
  template <bool from_clean_state>
  void UpdateEnteringCandidates(const std::vector<int>& cols) {
    const Fractional tolerance = reduced_costs_->GetDualFeasibilityTolerance();
    const Bitset& dec = variables_info_.GetCanDecreaseBitRow();
    const Bitset& inc = variables_info_.GetCanIncreaseBitRow();
    const std::vector<Fractional>& sn = primal_edge_norms_->GetSquaredNorms();
    const std::vector<Fractional>& rc = reduced_costs_->GetReducedCosts();
    UpdatePricesOver(cols, true, [&](int col) {
      const Fractional reduced_cost = rc[col];
      return ((reduced_cost > tolerance) && dec.IsSet(col)) !=
             ((reduced_cost < -tolerance) && inc.IsSet(col));
    }, rc.data(), sn.data());
    (void)from_clean_state;  // a clean state has no candidate to remove
  }
  bool recompute_ = true;
  DynamicMaximum prices_;
  const VariablesInfo& variables_info_;
  PrimalEdgeNorms* primal_edge_norms_;
  ReducedCosts* reduced_costs_;
};

// ---------------------------------------------------------------------------
// EnteringVariable (entering_variable.cc)
class EnteringVariable {
  friend struct SdualBridge;
  friend struct SdualHooks;

 public:
  EnteringVariable(const VariablesInfo& vi, Rng* random, ReducedCosts* rc)
      : variables_info_(vi), random_(random), reduced_costs_(rc) {}
  void SetParameters(const GlopParameters& p) { params_ = p; }
  Status DualChooseEnteringColumn(bool nothing_to_recompute, const UpdateRow& update_row,
                                  Fractional cost_variation,
                                  std::vector<int>* bound_flip_candidates,
                                  int* entering_col);
  Status DualPhaseIChooseEnteringColumn(bool nothing_to_recompute,
                                        const UpdateRow& update_row,
                                        Fractional cost_variation, int* entering_col);
  // DualChooseEnteringColumn in dual device mode: the device filters the
  // update row down to the breakpoints that can matter, the two Glop loops
  // run on them. Also returns the entering column's update-row coefficient
  // and reduced cost.
  Status DualChooseEnteringColumnDevice(bool nothing_to_recompute, DeviceLp* dev,
                                        Fractional cost_variation,
                                        std::vector<int>* bound_flip_candidates,
                                        int* entering_col, Fractional* entering_coeff,
                                        Fractional* entering_rc);
  double DeterministicTime() const {
    return DeterministicTimeForFpOperations(num_operations_);
  }
  // The last device ratio test's candidates (their update-row coefficients
  // and reduced costs): the speculative flip FTRAN's prediction reads them.
  const DeviceLp::DualCandidates& LastDeviceCandidates() const { return candidates_; }

 private:
  struct ColWithRatio {  // entering_variable.h:118-139
    int col;
    Fractional ratio;
    Fractional coeff_magnitude;
    ColWithRatio() = default;
    ColWithRatio(int c, Fractional reduced_cost, Fractional coeff_m)
        : col(c), ratio(reduced_cost / coeff_m), coeff_magnitude(coeff_m) {}
    bool operator<(const ColWithRatio& o) const {
      if (ratio == o.ratio) {
        if (coeff_magnitude == o.coeff_magnitude) return col > o.col;
        return coeff_magnitude < o.coeff_magnitude;
      }
      return ratio > o.ratio;
    }
  };
  const VariablesInfo& variables_info_;
  Rng* random_;
  ReducedCosts* reduced_costs_;
  GlopParameters params_;
  std::vector<int> equivalent_entering_choices_;
  std::vector<ColWithRatio> breakpoints_;
  std::vector<Fractional> bound_flip_magnitudes_;
  DeviceLp::DualCandidates candidates_;
  int64_t num_operations_ = 0;
};

// entering_variable.cc:37-239 over the device-filtered breakpoints. Only the
// slots with ratio <= B (1 + 1e-9) come back, B being the smallest Harris
// ratio over the breakpoints that can never be bound flipped: in the second
// loop such a breakpoint (or an earlier accepted one, with a larger
// coefficient and a smaller ratio) caps harris_ratio at <= B, so nothing
// with a larger ratio is popped, and a breakpoint beyond B can only prune
// breakpoints beyond B in the first loop. When many breakpoints remain, the
// device sorts them by ratio and walks them in pop order up to the first
// accepted one, a, and B becomes min(B, Harris ratio of a): no breakpoint
// before a is pruned by the first loop (a pruning breakpoint would have been
// accepted first), so the walk sees what the heap would pop. Both loops
// below are Glop's, in list order, over the returned subset.
Status EnteringVariable::DualChooseEnteringColumnDevice(bool nothing_to_recompute,
                                                        DeviceLp* dev,
                                                        Fractional cost_variation,
                                                        std::vector<int>* bound_flip_candidates,
                                                        int* entering_col,
                                                        Fractional* entering_coeff,
                                                        Fractional* entering_rc) {
  const Bitset& can_decrease = variables_info_.GetCanDecreaseBitRow();
  const Bitset& can_increase = variables_info_.GetCanIncreaseBitRow();
  const Bitset& is_boxed = variables_info_.GetNonBasicBoxedVariables();
  const Fractional threshold = nothing_to_recompute ? params_.minimum_acceptable_pivot
                                                    : params_.ratio_test_zero_threshold;
  Fractional variation_magnitude = std::fabs(cost_variation) - threshold;
  const Fractional harris_tolerance =
      params_.harris_tolerance_ratio * reduced_costs_->GetDualFeasibilityTolerance();
  const Fractional minimum_delta =
      params_.degenerate_ministep_factor * reduced_costs_->GetDualFeasibilityTolerance();
  SubTimer device_timer(kSubRatioDevice);
  dev->DualRatioCandidates(cost_variation > 0.0 ? 1.0 : -1.0, threshold, harris_tolerance,
                           minimum_delta, variation_magnitude, &candidates_);
  device_timer.Stop();
  SubTimer replay_timer(kSubRatioReplay);
  const DeviceLp::DualCandidates& cand = candidates_;
  num_operations_ += 10 * static_cast<int64_t>(cand.list_count);
  if (g_sub_on) {
    g_dual_candidates += static_cast<double>(cand.col.size());
    g_dual_list += cand.list_count;
  }
  breakpoints_.clear();
  Fractional harris_ratio = std::numeric_limits<Fractional>::max();
  const int num_candidates = static_cast<int>(cand.col.size());
  for (int k = 0; k < num_candidates; ++k) {
    const int col = cand.col[k];
    const Fractional coeff = (cost_variation > 0.0) ? cand.coeff[k] : -cand.coeff[k];
    const Fractional reduced_cost = cand.rc[k];
    ColWithRatio entry;
    if (can_decrease.IsSet(col) && coeff > threshold) {
      if (-reduced_cost > harris_ratio * coeff) continue;
      entry = ColWithRatio(col, -reduced_cost, coeff);
    } else if (can_increase.IsSet(col) && coeff < -threshold) {
      if (reduced_cost > harris_ratio * -coeff) continue;
      entry = ColWithRatio(col, reduced_cost, -coeff);
    } else {
      continue;
    }
    const Fractional hr = std::max(minimum_delta / entry.coeff_magnitude,
                                   entry.ratio + harris_tolerance / entry.coeff_magnitude);
    if (hr < harris_ratio) {
      if (is_boxed[col]) {
        const Fractional delta =
            variables_info_.GetBoundDifference(col) * entry.coeff_magnitude;
        if (delta >= variation_magnitude) harris_ratio = hr;
      } else {
        harris_ratio = hr;
      }
    }
    breakpoints_.push_back(entry);
  }
  std::make_heap(breakpoints_.begin(), breakpoints_.end());
  harris_ratio = std::numeric_limits<Fractional>::max();
  *entering_col = kInvalidCol;
  bound_flip_candidates->clear();
  bound_flip_magnitudes_.clear();
  Fractional step = 0.0;
  Fractional best_coeff = -1.0;
  equivalent_entering_choices_.clear();
  while (!breakpoints_.empty()) {
    const ColWithRatio top = breakpoints_.front();
    if (top.ratio > harris_ratio) break;
    if (variation_magnitude > 0.0) {
      if (is_boxed[top.col]) {
        variation_magnitude -=
            variables_info_.GetBoundDifference(top.col) * top.coeff_magnitude;
        if (variation_magnitude > 0.0) {
          bound_flip_candidates->push_back(top.col);
          bound_flip_magnitudes_.push_back(top.coeff_magnitude);
          std::pop_heap(breakpoints_.begin(), breakpoints_.end());
          breakpoints_.pop_back();
          continue;
        }
      }
    }
    if (top.coeff_magnitude >= best_coeff) {
      harris_ratio = std::min(
          harris_ratio, std::max(minimum_delta / top.coeff_magnitude,
                                 top.ratio + harris_tolerance / top.coeff_magnitude));
      if (top.coeff_magnitude == best_coeff && top.ratio == step) {
        equivalent_entering_choices_.push_back(top.col);
      } else {
        equivalent_entering_choices_.clear();
        best_coeff = top.coeff_magnitude;
        *entering_col = top.col;
        step = top.ratio;
      }
    }
    std::pop_heap(breakpoints_.begin(), breakpoints_.end());
    breakpoints_.pop_back();
  }
  if (!equivalent_entering_choices_.empty()) {
    equivalent_entering_choices_.push_back(*entering_col);
    *entering_col = equivalent_entering_choices_[UniformInt(
        *random_, static_cast<int>(equivalent_entering_choices_.size()) - 1)];
  }
  if (*entering_col == kInvalidCol) return Status::OK();
  const Fractional pivot_limit = params_.minimum_acceptable_pivot;
  if (best_coeff < pivot_limit && !bound_flip_candidates->empty()) {
    // |update_coefficients[col]| is the breakpoint's coefficient magnitude.
    for (int i = static_cast<int>(bound_flip_candidates->size()) - 1; i >= 0; --i) {
      const int col = (*bound_flip_candidates)[i];
      if (bound_flip_magnitudes_[i] < pivot_limit) continue;
      *entering_col = col;
      break;
    }
  }
  for (int k = 0; k < num_candidates; ++k) {
    if (cand.col[k] == *entering_col) {
      *entering_coeff = cand.coeff[k];
      *entering_rc = cand.rc[k];
      return Status::OK();
    }
  }
  throw DeviceError("dual device mode: entering column not among the candidates");
}

// entering_variable.cc:37-239
Status EnteringVariable::DualChooseEnteringColumn(bool nothing_to_recompute,
                                                  const UpdateRow& update_row,
                                                  Fractional cost_variation,
                                                  std::vector<int>* bound_flip_candidates,
                                                  int* entering_col) {
  const std::vector<Fractional>& update_coefficients = update_row.GetCoefficients();
  const std::vector<Fractional>& reduced_costs = reduced_costs_->GetReducedCosts();
  breakpoints_.clear();
  breakpoints_.reserve(update_row.GetNonZeroPositions().size());
  const Bitset& can_decrease = variables_info_.GetCanDecreaseBitRow();
  const Bitset& can_increase = variables_info_.GetCanIncreaseBitRow();
  const Bitset& is_boxed = variables_info_.GetNonBasicBoxedVariables();
  const Fractional threshold = nothing_to_recompute ? params_.minimum_acceptable_pivot
                                                    : params_.ratio_test_zero_threshold;
  Fractional variation_magnitude = std::fabs(cost_variation) - threshold;
  const Fractional harris_tolerance =
      params_.harris_tolerance_ratio * reduced_costs_->GetDualFeasibilityTolerance();
  Fractional harris_ratio = std::numeric_limits<Fractional>::max();
  const Fractional minimum_delta =
      params_.degenerate_ministep_factor * reduced_costs_->GetDualFeasibilityTolerance();
  num_operations_ += 10 * update_row.GetNonZeroPositions().size();
  for (const int col : update_row.GetNonZeroPositions()) {
    const Fractional coeff =
        (cost_variation > 0.0) ? update_coefficients[col] : -update_coefficients[col];
    ColWithRatio entry;
    if (can_decrease.IsSet(col) && coeff > threshold) {
      if (-reduced_costs[col] > harris_ratio * coeff) continue;
      entry = ColWithRatio(col, -reduced_costs[col], coeff);
    } else if (can_increase.IsSet(col) && coeff < -threshold) {
      if (reduced_costs[col] > harris_ratio * -coeff) continue;
      entry = ColWithRatio(col, reduced_costs[col], -coeff);
    } else {
      continue;
    }
    const Fractional hr = std::max(minimum_delta / entry.coeff_magnitude,
                                   entry.ratio + harris_tolerance / entry.coeff_magnitude);
    if (hr < harris_ratio) {
      if (is_boxed[col]) {
        const Fractional delta =
            variables_info_.GetBoundDifference(col) * entry.coeff_magnitude;
        if (delta >= variation_magnitude) harris_ratio = hr;
      } else {
        harris_ratio = hr;
      }
    }
    breakpoints_.push_back(entry);
  }
  std::make_heap(breakpoints_.begin(), breakpoints_.end());
  harris_ratio = std::numeric_limits<Fractional>::max();
  *entering_col = kInvalidCol;
  bound_flip_candidates->clear();
  Fractional step = 0.0;
  Fractional best_coeff = -1.0;
  equivalent_entering_choices_.clear();
  while (!breakpoints_.empty()) {
    const ColWithRatio top = breakpoints_.front();
    if (top.ratio > harris_ratio) break;
    if (variation_magnitude > 0.0) {
      if (is_boxed[top.col]) {
        variation_magnitude -=
            variables_info_.GetBoundDifference(top.col) * top.coeff_magnitude;
        if (variation_magnitude > 0.0) {
          bound_flip_candidates->push_back(top.col);
          std::pop_heap(breakpoints_.begin(), breakpoints_.end());
          breakpoints_.pop_back();
          continue;
        }
      }
    }
    if (top.coeff_magnitude >= best_coeff) {
      harris_ratio = std::min(
          harris_ratio, std::max(minimum_delta / top.coeff_magnitude,
                                 top.ratio + harris_tolerance / top.coeff_magnitude));
      if (top.coeff_magnitude == best_coeff && top.ratio == step) {
        equivalent_entering_choices_.push_back(top.col);
      } else {
        equivalent_entering_choices_.clear();
        best_coeff = top.coeff_magnitude;
        *entering_col = top.col;
        step = top.ratio;
      }
    }
    std::pop_heap(breakpoints_.begin(), breakpoints_.end());
    breakpoints_.pop_back();
  }
  if (!equivalent_entering_choices_.empty()) {
    equivalent_entering_choices_.push_back(*entering_col);
    *entering_col = equivalent_entering_choices_[UniformInt(
        *random_, static_cast<int>(equivalent_entering_choices_.size()) - 1)];
  }
  if (*entering_col == kInvalidCol) return Status::OK();
  const Fractional pivot_limit = params_.minimum_acceptable_pivot;
  if (best_coeff < pivot_limit && !bound_flip_candidates->empty()) {
    for (int i = static_cast<int>(bound_flip_candidates->size()) - 1; i >= 0; --i) {
      const int col = (*bound_flip_candidates)[i];
      if (std::fabs(update_coefficients[col]) < pivot_limit) continue;
      *entering_col = col;
      break;
    }
  }
  return Status::OK();
}

// entering_variable.cc:241-355
Status EnteringVariable::DualPhaseIChooseEnteringColumn(bool nothing_to_recompute,
                                                        const UpdateRow& update_row,
                                                        Fractional cost_variation,
                                                        int* entering_col) {
  const std::vector<Fractional>& update_coefficients = update_row.GetCoefficients();
  const std::vector<Fractional>& reduced_costs = reduced_costs_->GetReducedCosts();
  breakpoints_.clear();
  breakpoints_.reserve(update_row.GetNonZeroPositions().size());
  const Fractional threshold = nothing_to_recompute ? params_.minimum_acceptable_pivot
                                                    : params_.ratio_test_zero_threshold;
  const Fractional dual_feasibility_tolerance =
      reduced_costs_->GetDualFeasibilityTolerance();
  const Fractional harris_tolerance =
      params_.harris_tolerance_ratio * dual_feasibility_tolerance;
  const Fractional minimum_delta =
      params_.degenerate_ministep_factor * dual_feasibility_tolerance;
  const Bitset& can_decrease = variables_info_.GetCanDecreaseBitRow();
  const Bitset& can_increase = variables_info_.GetCanIncreaseBitRow();
  num_operations_ += 10 * update_row.GetNonZeroPositions().size();
  for (const int col : update_row.GetNonZeroPositions()) {
    if (std::fabs(update_coefficients[col]) < threshold) continue;
    const Fractional coeff =
        (cost_variation > 0.0) ? update_coefficients[col] : -update_coefficients[col];
    if (std::fabs(reduced_costs[col]) <= dual_feasibility_tolerance) {
      if (coeff > 0 && !can_decrease.IsSet(col)) continue;
      if (coeff < 0 && !can_increase.IsSet(col)) continue;
      if (coeff * reduced_costs[col] > 0.0) {
        breakpoints_.push_back(ColWithRatio(
            col, std::max(minimum_delta, harris_tolerance - std::fabs(reduced_costs[col])),
            std::fabs(coeff)));
        continue;
      }
    } else {
      if (coeff * reduced_costs[col] > 0.0) continue;
    }
    breakpoints_.push_back(ColWithRatio(
        col, std::fabs(reduced_costs[col]) + harris_tolerance, std::fabs(coeff)));
  }
  std::make_heap(breakpoints_.begin(), breakpoints_.end());
  Fractional pivot_magnitude = 0.0;
  *entering_col = kInvalidCol;
  Fractional step = -1.0;
  Fractional improvement = std::fabs(cost_variation);
  while (!breakpoints_.empty()) {
    const ColWithRatio top = breakpoints_.front();
    if (top.ratio > step && top.coeff_magnitude >= pivot_magnitude) {
      *entering_col = top.col;
      step = top.ratio;
      pivot_magnitude = top.coeff_magnitude;
    }
    improvement -= top.coeff_magnitude;
    if (can_decrease.IsSet(top.col) && can_increase.IsSet(top.col) &&
        std::fabs(reduced_costs[top.col]) > threshold) {
      improvement -= top.coeff_magnitude;
    }
    if (improvement <= 0.0) break;
    std::pop_heap(breakpoints_.begin(), breakpoints_.end());
    breakpoints_.pop_back();
  }
  return Status::OK();
}

// ---------------------------------------------------------------------------
// VariableValues (variable_values.cc)
class VariableValues {
  friend struct SdualBridge;
  friend struct SdualHooks;

 public:
  VariableValues(const GlopParameters& p, const CompactSparseMatrix& m,
                 const std::vector<int>& basis, const VariablesInfo& vi,
                 const BasisFactorization& bf, DualEdgeNorms* den, DynamicMaximum* dp,
                 DeviceLp* dev)
      : params_(p), matrix_(m), basis_(basis), variables_info_(vi), bf_(bf),
        dual_edge_norms_(den), dual_prices_(dp), dev_(dev) {}
  Fractional Get(int col) const { return variable_values_[col]; }
  void Set(int col, Fractional v) { variable_values_[col] = v; }
  const std::vector<Fractional>& GetDenseRow() const { return variable_values_; }
  void SetNonBasicVariableValueFromStatus(int col);
  void ResetAllNonBasicVariableValues(const std::vector<Fractional>& free_initial);
  void RecomputeBasicVariableValues();
  Fractional ComputeMaximumPrimalResidual() const;
  Fractional ComputeMaximumPrimalInfeasibility() const;
  void UpdateOnPivoting(const ScatteredVector& direction, int entering_col,
                        Fractional step) {
    const std::vector<int>& rows = direction.non_zeros;
    // Distinct rows hold distinct basic columns: split over the host pool.
    ParallelRanges(static_cast<int64_t>(rows.size()), 16384, 1, [&](int, int64_t b, int64_t e) {
      for (int64_t k = b; k < e; ++k) {
        if (k + 16 < e) __builtin_prefetch(variable_values_.data() + basis_[rows[k + 16]], 1);
        const int row = rows[k];
        const int col = basis_[row];
        variable_values_[col] -= direction.values[row] * step;
      }
    });
    variable_values_[entering_col] += step;
  }
  void UpdateGivenNonBasicVariables(const std::vector<int>& cols, bool update_basic);
  // Speculative flip FTRAN (engine; BasisFactorization::SpecFlipBegin): the
  // flips `cols` with value changes `deltas` the next iteration's
  // MakeBoxedVariableDualFeasible is expected to make, scattered as
  // UpdateGivenNonBasicVariables scatters them and solved ahead. That call
  // uses the result when it flips exactly these columns by exactly these
  // changes; SpecFlipDone drops a speculation nothing used.
  void SpecFlipBegin(const std::vector<int>& cols, const std::vector<Fractional>& deltas,
                     int entering_col, int leaving_row);
  void SpecFlipDone();
  void RecomputeDualPrices(bool put_more_importance_on_norm = false);
  void RecomputeDualPricesImpl(bool put_more_importance_on_norm, Fractional* delta);
  void UpdateDualPrices(const std::vector<int>& rows);
  template <typename Rows>
  bool UpdatePrimalPhaseICosts(const Rows& rows, std::vector<Fractional>* objective) {
    bool changed = false;
    const Fractional tolerance = params_.primal_feasibility_tolerance;
    for (const int row : rows) {
      const int col = basis_[row];
      Fractional new_cost = 0.0;
      if (GetUpperBoundInfeasibility(col) > tolerance) {
        new_cost = 1.0;
      } else if (GetLowerBoundInfeasibility(col) > tolerance) {
        new_cost = -1.0;
      }
      if (new_cost != (*objective)[col]) {
        changed = true;
        (*objective)[col] = new_cost;
      }
    }
    return changed;
  }

 private:
  std::vector<Fractional> price_scratch_;  // UpdateDualPrices' parallel pass
  std::vector<uint8_t> price_keep_;
  Fractional GetUpperBoundInfeasibility(int col) const {
    return variable_values_[col] - variables_info_.GetVariableUpperBounds()[col];
  }
  Fractional GetLowerBoundInfeasibility(int col) const {
    return variables_info_.GetVariableLowerBounds()[col] - variable_values_[col];
  }
  const GlopParameters& params_;
  const CompactSparseMatrix& matrix_;
  const std::vector<int>& basis_;
  const VariablesInfo& variables_info_;
  const BasisFactorization& bf_;
  bool put_more_importance_on_norm_ = false;
  DualEdgeNorms* dual_edge_norms_;
  DynamicMaximum* dual_prices_;
  DeviceLp* dev_;
  // UpdateGivenNonBasicVariables' scatter of the flips' value changes.
  void ScatterFlipChanges(const std::vector<int>& cols, const Fractional* deltas,
                          ScatteredVector* v) const;
  std::vector<Fractional> variable_values_;
  mutable ScatteredVector scratchpad_;
  ScatteredVector initially_all_zero_scratchpad_;
  std::vector<Fractional> flip_deltas_;
  bool spec_armed_ = false;
  std::vector<int> spec_cols_;
  std::vector<Fractional> spec_deltas_;
  ScatteredVector spec_scratch_;  // all zero between uses
 public:
  // MILP_SPEC_FLIP_STATS=1: speculations used / dropped, printed at exit.
  static std::atomic<int64_t> spec_used, spec_missed, spec_started;
};

void VariableValues::SetNonBasicVariableValueFromStatus(int col) {
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  variable_values_.resize(matrix_.num_cols(), 0.0);
  switch (variables_info_.GetStatusRow()[col]) {
    case VariableStatus::FIXED_VALUE:
    case VariableStatus::AT_LOWER_BOUND:
      variable_values_[col] = lb[col];
      break;
    case VariableStatus::AT_UPPER_BOUND:
      variable_values_[col] = ub[col];
      break;
    default:
      break;
  }
}

void VariableValues::ResetAllNonBasicVariableValues(const std::vector<Fractional>& fiv) {
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  const std::vector<VariableStatus>& st = variables_info_.GetStatusRow();
  const int num_cols = matrix_.num_cols();
  variable_values_.resize(num_cols, 0.0);
  for (int col = 0; col < num_cols; ++col) {
    switch (st[col]) {
      case VariableStatus::FIXED_VALUE:
      case VariableStatus::AT_LOWER_BOUND:
        variable_values_[col] = lb[col];
        break;
      case VariableStatus::AT_UPPER_BOUND:
        variable_values_[col] = ub[col];
        break;
      case VariableStatus::FREE:
        variable_values_[col] = col < static_cast<int>(fiv.size()) ? fiv[col] : 0.0;
        break;
      case VariableStatus::BASIC:
        break;
    }
  }
}

// Host forms of DeviceLp::RowSums / ListDots / Pricing for the sdual batch
// mode (DeviceLp::SetHostSmallOps): sparse.h's ColumnAddMultipleToDenseColumn
// and ColumnScalarProduct in column order, as the kernels sum.
namespace {
void HostRowSums(const CompactSparseMatrix& a, const std::vector<Fractional>& x,
                 const Bitset* skip, Fractional sign, std::vector<Fractional>* out) {
  out->assign(a.num_rows(), 0.0);
  for (int col = 0; col < a.num_cols(); ++col) {
    if (skip != nullptr && skip->IsSet(col)) continue;
    a.ColumnAddMultipleToDenseColumn(col, sign * x[col], out->data());
  }
}
}  // namespace

// variable_values.cc:101-118
void VariableValues::RecomputeBasicVariableValues() {
  SubTimer timer(kSubRecomputeValues);
  const int num_rows = matrix_.num_rows();
  scratchpad_.non_zeros.clear();
  // -sum over non-basic columns of x_j a_j, per row in column order (GPU).
  if (dev_->host_small_ops()) {
    HostRowSums(matrix_, variable_values_, &variables_info_.GetIsBasicBitRow(), -1.0,
                &scratchpad_.values);
  } else {
    dev_->SetMask(DeviceLp::kBasic, variables_info_.GetIsBasicBitRow().data(),
                  variables_info_.GetIsBasicBitRow().NumWords());
    dev_->RowSums(variable_values_, /*skip_basic=*/true, -1.0, &scratchpad_.values);
  }
  bf_.RightSolve(&scratchpad_);
  for (int row = 0; row < num_rows; ++row) variable_values_[basis_[row]] = scratchpad_[row];
  dual_prices_->Clear();
}

// variable_values.cc:120-131
Fractional VariableValues::ComputeMaximumPrimalResidual() const {
  scratchpad_.non_zeros.clear();
  if (dev_->host_small_ops()) {
    HostRowSums(matrix_, variable_values_, nullptr, 1.0, &scratchpad_.values);
  } else {
    dev_->RowSums(variable_values_, /*skip_basic=*/false, 1.0, &scratchpad_.values);
  }
  return InfinityNorm(scratchpad_.values);
}

// variable_values.cc:133-143
Fractional VariableValues::ComputeMaximumPrimalInfeasibility() const {
  Fractional pi = 0.0;
  for (int col = 0; col < matrix_.num_cols(); ++col) {
    const Fractional ci =
        std::max(GetUpperBoundInfeasibility(col), GetLowerBoundInfeasibility(col));
    pi = std::max(pi, ci);
  }
  return pi;
}

// variable_values.cc:179-227
std::atomic<int64_t> VariableValues::spec_used{0}, VariableValues::spec_missed{0},
    VariableValues::spec_started{0};
namespace {
struct SpecFlipStatsAtExit {
  ~SpecFlipStatsAtExit() {
    if (std::getenv("MILP_SPEC_FLIP_STATS") == nullptr) return;
    std::fprintf(stderr, "[spec flip] started %lld used %lld dropped %lld\n",
                 static_cast<long long>(VariableValues::spec_started.load()),
                 static_cast<long long>(VariableValues::spec_used.load()),
                 static_cast<long long>(VariableValues::spec_missed.load()));
  }
} g_spec_flip_stats_at_exit;
}  // namespace

void VariableValues::ScatterFlipChanges(const std::vector<int>& cols, const Fractional* deltas,
                                        ScatteredVector* v) const {
  v->values.resize(matrix_.num_rows(), 0.0);
  v->ClearSparseMask();
  bool use_dense = false;
  for (size_t i = 0; i < cols.size(); ++i) {
    if (use_dense) {
      matrix_.ColumnAddMultipleToDenseColumn(cols[i], deltas[i], v->values.data());
    } else {
      matrix_.ColumnAddMultipleToSparseScatteredColumn(cols[i], deltas[i], v);
      use_dense = v->ShouldUseDenseIteration();
    }
  }
  v->ClearSparseMask();
  v->ClearNonZerosIfTooDense();
}

void VariableValues::SpecFlipBegin(const std::vector<int>& cols,
                                   const std::vector<Fractional>& deltas, int entering_col,
                                   int leaving_row) {
  SpecFlipDone();
  ScatterFlipChanges(cols, deltas.data(), &spec_scratch_);
  if (!bf_.SpecFlipBegin(&spec_scratch_, entering_col, leaving_row)) {
    std::fill(spec_scratch_.values.begin(), spec_scratch_.values.end(), 0.0);
    spec_scratch_.non_zeros.clear();
    spec_scratch_.ClearSparseMask();
    return;
  }
  spec_cols_ = cols;
  spec_deltas_ = deltas;
  spec_armed_ = true;
  ++spec_started;
}

void VariableValues::SpecFlipDone() {
  if (!spec_armed_) return;
  spec_armed_ = false;
  bf_.SpecFlipDrop();
  ++spec_missed;
}

void VariableValues::UpdateGivenNonBasicVariables(const std::vector<int>& cols,
                                                  bool update_basic) {
  if (!update_basic) {
    for (const int col : cols) SetNonBasicVariableValueFromStatus(col);
    return;
  }
  SubTimer scatter_timer(kSubFlipScatter);
  flip_deltas_.resize(cols.size());
  for (size_t i = 0; i < cols.size(); ++i) {
    const Fractional old_value = variable_values_[cols[i]];
    SetNonBasicVariableValueFromStatus(cols[i]);
    flip_deltas_[i] = variable_values_[cols[i]] - old_value;
  }
  // The speculative solve is RightSolve's result for the same flips and
  // changes (same columns in the same order, the same bits).
  bool solved = false;
  if (spec_armed_) {
    scatter_timer.Stop();
    spec_armed_ = false;
    if (cols == spec_cols_ &&
        std::memcmp(flip_deltas_.data(), spec_deltas_.data(),
                    cols.size() * sizeof(Fractional)) == 0) {
      SubTimer solve_timer(kSubFlipSolve);
      solved = bf_.SpecFlipTake(&initially_all_zero_scratchpad_);
    } else {
      bf_.SpecFlipDrop();
    }
    ++(solved ? spec_used : spec_missed);
  }
  if (!solved) {
    ScatterFlipChanges(cols, flip_deltas_.data(), &initially_all_zero_scratchpad_);
    scatter_timer.Stop();
    SubTimer solve_timer(kSubFlipSolve);
    bf_.RightSolve(&initially_all_zero_scratchpad_);
  }
  SubTimer prices_timer(kSubFlipPrices);
  if (initially_all_zero_scratchpad_.non_zeros.empty()) {
    // x_B update, scratch reset and RecomputeDualPrices() in one pass: a
    // row's price reads only its own basic variable, so the three loops of
    // variable_values.cc:211-217 and :229-262 fuse row by row.
    RecomputeDualPricesImpl(false, initially_all_zero_scratchpad_.values.data());
    return;
  }
  for (const int row : initially_all_zero_scratchpad_.non_zeros) {
    variable_values_[basis_[row]] -= initially_all_zero_scratchpad_[row];
    initially_all_zero_scratchpad_[row] = 0.0;
  }
  UpdateDualPrices(initially_all_zero_scratchpad_.non_zeros);
  initially_all_zero_scratchpad_.non_zeros.clear();
}

// variable_values.cc:229-262
void VariableValues::RecomputeDualPrices(bool put_more_importance_on_norm) {
  RecomputeDualPricesImpl(put_more_importance_on_norm, nullptr);
}

// With delta != nullptr, first x[basis[row]] -= delta[row] and delta[row] =
// 0 (UpdateGivenNonBasicVariables' dense update). Rows are split over the
// host pool in 64-row ranges, so every candidate-bit word has one writer;
// DenseAddOrUpdate touches no shared state besides its own value and bit.
void VariableValues::RecomputeDualPricesImpl(bool put_more_importance_on_norm,
                                             Fractional* delta) {
  SubTimer timer(kSubDualPrices);
  const int num_rows = matrix_.num_rows();
  dual_prices_->ClearAndResize(num_rows);
  dual_prices_->StartDenseUpdates();
  put_more_importance_on_norm_ = put_more_importance_on_norm;
  const Fractional tolerance = params_.primal_feasibility_tolerance;
  const std::vector<Fractional>& sn = dual_edge_norms_->GetEdgeSquaredNorms();
  // The basic columns are scattered over arrays of N entries: their values
  // and bounds are prefetched a few rows ahead.
  Fractional* x = variable_values_.data();
  const Fractional* lb = variables_info_.GetVariableLowerBounds().data();
  const Fractional* ub = variables_info_.GetVariableUpperBounds().data();
  const int* basis = basis_.data();
  Fractional* values = dual_prices_->mutable_values();
  uint64_t* words = dual_prices_->mutable_candidate_words();
  ParallelRanges(num_rows, 16384, 64, [&](int, int64_t begin, int64_t end) {
    constexpr int kAhead = 16;
    for (int64_t row = begin; row < end; ++row) {
      if (row + kAhead < end) {
        const int ahead = basis[row + kAhead];
        __builtin_prefetch(x + ahead, 1);
        __builtin_prefetch(lb + ahead);
        __builtin_prefetch(ub + ahead);
      }
      const int col = basis[row];
      if (delta != nullptr) {
        x[col] -= delta[row];
        delta[row] = 0.0;
      }
      // GetUpperBoundInfeasibility / GetLowerBoundInfeasibility
      const Fractional inf = std::max(x[col] - ub[col], lb[col] - x[col]);
      if (inf > tolerance) {
        words[row >> 6] |= uint64_t{1} << (row & 63);
        values[row] =
            put_more_importance_on_norm ? std::fabs(inf) / sn[row] : Square(inf) / sn[row];
      }
    }
  });
}

// variable_values.cc:264-297
void VariableValues::UpdateDualPrices(const std::vector<int>& rows) {
  if (dual_prices_->Size() != matrix_.num_rows()) {
    RecomputeDualPrices(put_more_importance_on_norm_);
    return;
  }
  const Fractional tolerance = params_.primal_feasibility_tolerance;
  const std::vector<Fractional>& sn = dual_edge_norms_->GetEdgeSquaredNorms();
  const Fractional* x = variable_values_.data();
  const Fractional* lb = variables_info_.GetVariableLowerBounds().data();
  const Fractional* ub = variables_info_.GetVariableUpperBounds().data();
  const size_t n = rows.size();
  if (n >= 8192 && HostPool::Get().threads() > 1) {
    // Long lists (a dense direction): the prices, element by element with the
    // serial loop's expression, in parallel into scratch (-1: not a
    // candidate); then AddOrUpdate / Remove in list order, so the top-k
    // bookkeeping and its RNG draws are the serial loop's.
    price_scratch_.resize(n);
    price_keep_.resize(n);
    Fractional* price = price_scratch_.data();
    uint8_t* keep = price_keep_.data();
    const int* basis = basis_.data();
    const bool by_norm = put_more_importance_on_norm_;
    ParallelRanges(static_cast<int64_t>(n), 8192, 64, [&](int, int64_t b, int64_t e) {
      for (int64_t k = b; k < e; ++k) {
        if (k + 16 < e) {
          const int ahead = basis[rows[k + 16]];
          __builtin_prefetch(x + ahead);
          __builtin_prefetch(lb + ahead);
          __builtin_prefetch(ub + ahead);
        }
        const int row = rows[k];
        const int col = basis[row];
        const Fractional inf = std::max(x[col] - ub[col], lb[col] - x[col]);
        keep[k] = inf > tolerance ? 1 : 0;
        if (keep[k]) price[k] = by_norm ? std::fabs(inf) / sn[row] : Square(inf) / sn[row];
      }
    });
    dual_prices_->BulkAddOrUpdate(rows.data(), price, keep, n);
    return;
  }
  for (size_t k = 0; k < n; ++k) {
    if (k + 16 < n) {
      const int ahead = basis_[rows[k + 16]];
      __builtin_prefetch(x + ahead);
      __builtin_prefetch(lb + ahead);
      __builtin_prefetch(ub + ahead);
    }
    const int row = rows[k];
    const int col = basis_[row];
    const Fractional inf =
        std::max(GetUpperBoundInfeasibility(col), GetLowerBoundInfeasibility(col));
    if (inf > tolerance) {
      dual_prices_->AddOrUpdate(row, put_more_importance_on_norm_
                                         ? std::fabs(inf) / sn[row]
                                         : Square(inf) / sn[row]);
    } else {
      dual_prices_->Remove(row);
    }
  }
}

// ---------------------------------------------------------------------------
// InitialBasis::CompleteTriangularBasis (initial_basis.cc:126-206)
namespace {
int GetColumnCategory(VariableType t) {
  switch (t) {
    case VariableType::UNCONSTRAINED:
      return 2;
    case VariableType::LOWER_BOUNDED:
    case VariableType::UPPER_BOUNDED:
      return 3;
    case VariableType::UPPER_AND_LOWER_BOUNDED:
      return 4;
    case VariableType::FIXED_VARIABLE:
      return 5;
  }
  return 5;
}

template <bool only_allow_zero_cost_column>
void CompleteTriangularBasis(const CompactSparseMatrix& matrix,
                             const std::vector<Fractional>& objective,
                             const std::vector<Fractional>& lb,
                             const std::vector<Fractional>& ub,
                             const std::vector<VariableType>& type, int num_cols,
                             std::vector<int>* basis) {
  const int num_rows = matrix.num_rows();
  std::vector<char> can_be_replaced(num_rows, false);
  for (int row = 0; row < num_rows; ++row)
    if ((*basis)[row] == kInvalidCol) can_be_replaced[row] = true;
  MatrixNonZeroPattern residual_pattern;
  residual_pattern.Reset(num_rows, num_cols);
  for (int col = 0; col < num_cols; ++col) {
    if (only_allow_zero_cost_column && objective[col] != 0.0) continue;
    const ColumnView c = matrix.column(col);
    for (int64_t i = 0; i < c.n; ++i)
      if (can_be_replaced[c.rows[i]]) residual_pattern.AddEntry(c.rows[i], col);
  }
  std::vector<int> residual_singleton_column;
  Fractional max_scaled_abs_cost = 0.0;
  for (int col = 0; col < num_cols; ++col) {
    max_scaled_abs_cost = std::max(max_scaled_abs_cost, std::fabs(objective[col]));
    if (residual_pattern.ColDegree(col) == 1) residual_singleton_column.push_back(col);
  }
  const Fractional kBixbyWeight = 1000.0;
  max_scaled_abs_cost =
      (max_scaled_abs_cost == 0.0) ? 1.0 : kBixbyWeight * max_scaled_abs_cost;
  auto penalty = [&](int col) {  // initial_basis.cc:GetColumnPenalty
    const VariableType t = type[col];
    Fractional p = 0.0;
    if (t == VariableType::LOWER_BOUNDED) p = lb[col];
    if (t == VariableType::UPPER_BOUNDED) p = -ub[col];
    if (t == VariableType::UPPER_AND_LOWER_BOUNDED) p = lb[col] - ub[col];
    return p + std::fabs(objective[col]) / max_scaled_abs_cost;
  };
  // initial_basis.cc TriangularColumnComparator.
  auto cmp = [&](int a, int b) {
    if (a == b) return false;
    const int ca = GetColumnCategory(type[a]);
    const int cb = GetColumnCategory(type[b]);
    if (ca != cb) return ca > cb;
    if (matrix.ColumnNumEntries(a) != matrix.ColumnNumEntries(b))
      return matrix.ColumnNumEntries(a) > matrix.ColumnNumEntries(b);
    return penalty(a) > penalty(b);
  };
  std::priority_queue<int, std::vector<int>, std::function<bool(int, int)>> queue(
      cmp, std::vector<int>(residual_singleton_column.begin(),
                            residual_singleton_column.end()));
  while (!queue.empty()) {
    const int candidate = queue.top();
    queue.pop();
    if (residual_pattern.ColDegree(candidate) != 1) continue;
    int row = kInvalidRow;
    Fractional coeff = 0.0;
    Fractional max_magnitude = 0.0;
    const ColumnView c = matrix.column(candidate);
    for (int64_t i = 0; i < c.n; ++i) {
      max_magnitude = std::max(max_magnitude, std::fabs(c.coefs[i]));
      if (can_be_replaced[c.rows[i]]) {
        row = c.rows[i];
        coeff = c.coefs[i];
        break;
      }
    }
    const Fractional kStabilityThreshold = 0.01;
    if (std::fabs(coeff) < kStabilityThreshold * max_magnitude) continue;
    (*basis)[row] = candidate;
    can_be_replaced[row] = false;
    residual_pattern.DeleteRowAndColumn(row, candidate);
    for (const int col : residual_pattern.RowNonZero(row)) {
      if (col == candidate) continue;
      residual_pattern.DecreaseColDegree(col);
      if (residual_pattern.ColDegree(col) == 1) queue.push(col);
    }
  }
}
// initial_basis.cc:208-356 (GetMarosPriority, GetMarosBasis), restated as is:
// the first availability test of the residual pattern indexes `available`
// with the row number (upstream's expression).
int GetMarosPriority(VariableType t) {
  switch (t) {
    case VariableType::UNCONSTRAINED:
      return 3;
    case VariableType::LOWER_BOUNDED:
    case VariableType::UPPER_BOUNDED:
      return 2;
    case VariableType::UPPER_AND_LOWER_BOUNDED:
      return 1;
    case VariableType::FIXED_VARIABLE:
      return 0;
  }
  return 0;
}

template <bool only_allow_zero_cost_column>
void GetMarosBasis(const CompactSparseMatrix& matrix, const std::vector<Fractional>& objective,
                   const std::vector<VariableType>& type, int num_cols,
                   std::vector<int>* basis) {
  const int num_rows = matrix.num_rows();
  const int first_slack = num_cols - num_rows;
  basis->resize(num_rows);
  for (int row = 0; row < num_rows; ++row) (*basis)[row] = first_slack + row;
  std::vector<char> available(num_cols, true);
  for (int col = 0; col < first_slack; ++col) {
    if (type[col] == VariableType::FIXED_VARIABLE ||
        (only_allow_zero_cost_column && objective[col] != 0.0)) {
      available[col] = false;
    }
  }
  for (int col = first_slack; col < num_cols; ++col) {
    if (type[col] == VariableType::UNCONSTRAINED) available[col] = false;
  }
  MatrixNonZeroPattern residual_pattern;
  residual_pattern.Reset(num_rows, num_cols);
  for (int col = 0; col < first_slack; ++col) {
    const ColumnView c = matrix.column(col);
    for (int64_t i = 0; i < c.n; ++i) {
      if (available[c.rows[i]] && available[col]) residual_pattern.AddEntry(c.rows[i], col);
    }
  }
  for (int row = 0; row < num_rows; ++row) {
    if (residual_pattern.RowDegree(row) == 0) available[row + first_slack] = false;
  }
  auto row_priority = [&](int row) { return GetMarosPriority(type[row + first_slack]); };
  for (;;) {
    int max_row_priority_function = std::numeric_limits<int>::min();
    int max_rpf_row = kInvalidRow;
    for (int row = 0; row < num_rows; ++row) {
      if (available[row + first_slack]) {
        const int rpf = 10 * (3 - row_priority(row)) - residual_pattern.RowDegree(row);
        if (rpf > max_row_priority_function) {
          max_row_priority_function = rpf;
          max_rpf_row = row;
        }
      }
    }
    if (max_rpf_row == kInvalidRow) break;
    const Fractional kStabilityThreshold = 1e-3;
    int max_cpf_col = kInvalidCol;
    int max_col_priority_function = std::numeric_limits<int>::min();
    Fractional pivot_absolute_value = 0.0;
    for (const int col : residual_pattern.RowNonZero(max_rpf_row)) {
      if (!available[col]) continue;
      const int cpf = 10 * GetMarosPriority(type[col]) - residual_pattern.ColDegree(col);
      if (cpf > max_col_priority_function) {
        Fractional max_magnitude = 0;
        pivot_absolute_value = 0.0;
        const ColumnView c = matrix.column(col);
        for (int64_t i = 0; i < c.n; ++i) {
          const Fractional absolute_value = std::fabs(c.coefs[i]);
          if (c.rows[i] == max_rpf_row) pivot_absolute_value = absolute_value;
          max_magnitude = std::max(max_magnitude, absolute_value);
        }
        if (pivot_absolute_value >= kStabilityThreshold * max_magnitude) {
          max_col_priority_function = cpf;
          max_cpf_col = col;
        }
      }
    }
    if (max_cpf_col == kInvalidCol) {
      available[max_rpf_row + first_slack] = false;
      continue;
    }
    if (row_priority(max_rpf_row) >= GetMarosPriority(type[max_cpf_col])) {
      available[max_rpf_row + first_slack] = false;
      continue;
    }
    (*basis)[max_rpf_row] = max_cpf_col;
    available[max_cpf_col] = false;
    available[first_slack + max_rpf_row] = false;
    residual_pattern.DeleteRowAndColumn(max_rpf_row, max_cpf_col);
    for (const int col : residual_pattern.RowNonZero(max_rpf_row)) available[col] = false;
  }
}

// initial_basis.cc:43-103 (CompleteBixbyBasis) with ComputeCandidates and
// BixbyColumnComparator (:358-419) and lp_utils.cc:115-172 helpers.
void CompleteBixbyBasis(const CompactSparseMatrix& matrix, const std::vector<Fractional>& objective,
                        const std::vector<Fractional>& lb, const std::vector<Fractional>& ub,
                        const std::vector<VariableType>& type, int num_cols,
                        std::vector<int>* basis) {
  const int num_rows = matrix.num_rows();
  std::vector<char> can_be_replaced(num_rows, false);
  std::vector<char> has_zero_coefficient(num_rows, false);
  basis->resize(num_rows, kInvalidCol);
  for (int row = 0; row < num_rows; ++row) {
    if ((*basis)[row] == kInvalidCol) {
      can_be_replaced[row] = true;
      has_zero_coefficient[row] = true;
    }
  }
  std::vector<Fractional> scaled_diagonal_abs(num_rows, kInfinity);
  std::vector<int> candidates;
  Fractional max_scaled_abs_cost = 0.0;
  for (int col = 0; col < num_cols; ++col) {
    if (type[col] != VariableType::FIXED_VARIABLE && matrix.ColumnNumEntries(col) > 0) {
      candidates.push_back(col);
      max_scaled_abs_cost = std::max(max_scaled_abs_cost, std::fabs(objective[col]));
    }
  }
  const Fractional kBixbyWeight = 1000.0;
  max_scaled_abs_cost = (max_scaled_abs_cost == 0.0) ? 1.0 : kBixbyWeight * max_scaled_abs_cost;
  auto penalty = [&](int col) {
    const VariableType t = type[col];
    Fractional p = 0.0;
    if (t == VariableType::LOWER_BOUNDED) p = lb[col];
    if (t == VariableType::UPPER_BOUNDED) p = -ub[col];
    if (t == VariableType::UPPER_AND_LOWER_BOUNDED) p = lb[col] - ub[col];
    return p + std::fabs(objective[col]) / max_scaled_abs_cost;
  };
  std::sort(candidates.begin(), candidates.end(), [&](int a, int b) {
    if (a == b) return false;
    const int ca = GetColumnCategory(type[a]);
    const int cb = GetColumnCategory(type[b]);
    if (ca != cb) return ca < cb;
    return penalty(a) < penalty(b);
  });
  auto restricted_inf_norm = [](const ColumnView& c, const std::vector<char>& rows,
                                int* row_index) {
    Fractional norm = 0.0;
    for (int64_t i = 0; i < c.n; ++i) {
      if (rows[c.rows[i]] && std::fabs(c.coefs[i]) > norm) {
        norm = std::fabs(c.coefs[i]);
        *row_index = c.rows[i];
      }
    }
    return norm;
  };
  for (const int candidate_col_index : candidates) {
    bool enter_basis = false;
    const ColumnView candidate_col = matrix.column(candidate_col_index);
    Fractional inf_norm = 0.0;
    for (int64_t i = 0; i < candidate_col.n; ++i) {
      inf_norm = std::max(inf_norm, std::fabs(candidate_col.coefs[i]));
    }
    if (inf_norm != 1.0) continue;
    int candidate_row = kInvalidRow;
    Fractional candidate_coeff =
        restricted_inf_norm(candidate_col, has_zero_coefficient, &candidate_row);
    const Fractional kBixbyHighThreshold = 0.99;
    if (candidate_coeff > kBixbyHighThreshold) {
      enter_basis = true;
    } else {
      bool dominated = true;
      for (int64_t i = 0; i < candidate_col.n; ++i) {
        if (std::fabs(candidate_col.coefs[i]) > scaled_diagonal_abs[candidate_col.rows[i]]) {
          dominated = false;
          break;
        }
      }
      if (dominated) {
        candidate_coeff = restricted_inf_norm(candidate_col, can_be_replaced, &candidate_row);
        if (candidate_coeff != 0.0) enter_basis = true;
      }
    }
    if (enter_basis) {
      can_be_replaced[candidate_row] = false;
      for (int64_t i = 0; i < candidate_col.n; ++i) {
        if (candidate_col.coefs[i] != 0.0) has_zero_coefficient[candidate_col.rows[i]] = false;
      }
      const Fractional kBixbyLowThreshold = 0.01;
      scaled_diagonal_abs[candidate_row] = kBixbyLowThreshold * std::fabs(candidate_coeff);
      (*basis)[candidate_row] = candidate_col_index;
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// RevisedSimplex (revised_simplex.cc)
class RevisedSimplex {
  friend struct SdualBridge;
  friend struct SdualHooks;

 public:
  RevisedSimplex();
  void SetParameters(const GlopParameters& p) {  // revised_simplex.cc:3586-3593
    random_.seed(p.random_seed);
    initial_parameters_ = p;
    parameters_ = p;
    PropagateParameters();
  }
  Status Solve(const LinearProgram& lp, TimeLimit* time_limit);
  void ClearStateForNextSolve() {
    solution_state_.clear();
    variable_starting_values_.clear();
  }
  void LoadStateForNextSolve(const std::vector<VariableStatus>& s) {
    solution_state_ = s;
    solution_state_has_been_set_externally_ = true;
  }
  void NotifyThatMatrixIsUnchangedForNextSolve() { notify_that_matrix_is_unchanged_ = true; }
  // revised_simplex.cc:135-137
  void NotifyThatMatrixIsChangedForNextSolve() { notify_that_matrix_is_unchanged_ = false; }
  // revised_simplex.cc:126-129
  void SetStartingVariableValuesForNextSolve(const std::vector<Fractional>& values) {
    variable_starting_values_ = values;
  }
  void SetIntegralityScale(int col, Fractional scale);
  // revised_simplex.h:236 (called by sat/linear_programming_constraint.cc:424
  // before the scales are set again).
  void ClearIntegralityScales() { integrality_scale_.clear(); }
  bool objective_limit_reached() const { return objective_limit_reached_; }
  // revised_simplex.h:209-211 (UpdateRow::ComputeAndGetUnitRowLeftInverse).
  const ScatteredVector& GetUnitRowLeftInverse(int row) {
    return update_row_.ComputeAndGetUnitRowLeftInverse(row);
  }
  // revised_simplex.cc:3785-3806: row r of B^-1 A, one direction per column.
  // Returns triplets (row, col, value) in the order the reference fills its
  // per-row sparse rows.
  void ComputeDictionary(const std::vector<Fractional>* column_scales,
                         std::vector<std::vector<std::pair<int, Fractional>>>* rows);

  ProblemStatus GetProblemStatus() const { return problem_status_; }
  Fractional GetObjectiveValue() const { return solution_objective_value_; }
  int64_t GetNumberOfIterations() const { return num_iterations_; }
  Fractional GetVariableValue(int col) const { return variable_values_.Get(col); }
  Fractional GetReducedCost(int col) const { return solution_reduced_costs_[col]; }
  Fractional GetDualValue(int row) const { return solution_dual_values_[row]; }
  Fractional GetConstraintActivity(int row) const {
    return -variable_values_.Get(first_slack_col_ + row);
  }
  VariableStatus GetVariableStatus(int col) const {
    return variables_info_.GetStatusRow()[col];
  }
  VariableStatus GetConstraintStatus(int row) const {  // revised_simplex.cc:681-692
    const VariableStatus s = variables_info_.GetStatusRow()[first_slack_col_ + row];
    if (s == VariableStatus::AT_LOWER_BOUND) return VariableStatus::AT_UPPER_BOUND;
    if (s == VariableStatus::AT_UPPER_BOUND) return VariableStatus::AT_LOWER_BOUND;
    return s;
  }
  const std::vector<VariableStatus>& GetState() const { return solution_state_; }
  int GetBasis(int row) const { return basis_[row]; }
  const std::vector<Fractional>& GetPrimalRay() const { return solution_primal_ray_; }
  const std::vector<Fractional>& GetDualRay() const { return solution_dual_ray_; }
  const std::vector<Fractional>& GetDualRayRowCombination() const {
    return solution_dual_ray_row_combination_;
  }
  double DeterministicTime() const {  // revised_simplex.cc:731-739
    return DeterministicTimeForFpOperations(num_update_price_operations_) +
           basis_factorization_.DeterministicTime() + update_row_.DeterministicTime() +
           entering_variable_.DeterministicTime() + reduced_costs_.DeterministicTime() +
           primal_edge_norms_.DeterministicTime();
  }
  int num_rows() const { return num_rows_; }
  int num_cols() const { return num_cols_; }
  // Per-iteration timestamps (seconds since Solve start) for the CPU baseline.
  std::vector<double> iteration_times;
  bool record_iteration_times = false;
  // Called after every completed iteration (benchmark slicing, mi_lp_begin).
  std::function<void(int64_t)> iteration_hook;
  DeviceLp& device() { return device_; }
  int64_t NumFactorizations() const { return basis_factorization_.NumFactorizations(); }
  double FactorizationSeconds() const { return basis_factorization_.FactorizationSeconds(); }

 private:
  enum class Phase { FEASIBILITY, OPTIMIZATION, PUSH };
  void PropagateParameters() {
    basis_factorization_.SetParameters(parameters_.basis_refactorization_period,
                                       parameters_.dynamically_adjust_refactorization_period,
                                       parameters_.lu(),
                                       parameters_.use_middle_product_form_update);
    entering_variable_.SetParameters(parameters_);
    reduced_costs_.SetParameters(parameters_);
    dual_edge_norms_.SetParameters(parameters_);
    primal_edge_norms_.SetParameters(parameters_);
    update_row_.SetParameters(parameters_);
  }
  Status Initialize(const LinearProgram& lp);
  bool InitializeMatrixAndTestIfUnchanged(const LinearProgram& lp,
                                          bool* only_change_is_new_rows,
                                          bool* only_change_is_new_cols,
                                          int* num_new_cols);
  bool OldBoundsAreUnchangedAndNewVariablesHaveOneBoundAtZero(const LinearProgram& lp,
                                                              int num_new_cols);
  bool InitializeObjectiveAndTestIfUnchanged(const LinearProgram& lp);
  void InitializeObjectiveLimit();
  Status CreateInitialBasis();
  Status InitializeFirstBasis(const std::vector<int>& basis);
  void SaveState() {
    solution_state_ = variables_info_.GetStatusRow();
    solution_state_has_been_set_externally_ = false;
  }
  void SetNonBasicVariableStatusAndDeriveValue(int col, VariableStatus status) {
    variables_info_.UpdateToNonBasicStatus(col, status);
    variable_values_.SetNonBasicVariableValueFromStatus(col);
  }
  void UpdateBasis(int entering_col, int basis_row, VariableStatus leaving_status) {
    const int leaving_col = basis_[basis_row];
    variables_info_.UpdateToNonBasicStatus(leaving_col, leaving_status);
    basis_[basis_row] = entering_col;
    variables_info_.UpdateToBasicStatus(entering_col);
    update_row_.Invalidate();
  }
  void UseSingletonColumnInInitialBasis(std::vector<int>* basis);
  void CorrectErrorsOnVariableValues();
  void ComputeVariableValuesError();
  void ComputeDirection(int col);
  template <bool positive>
  Fractional GetRatio(const std::vector<Fractional>& lb, const std::vector<Fractional>& ub,
                      int row) const;
  template <bool positive>
  Fractional ComputeHarrisRatioAndLeavingCandidates(Fractional bound_flip_ratio,
                                                    SparseColumn* leaving_candidates) const;
  Status ChooseLeavingVariableRow(int entering_col, Fractional reduced_cost,
                                  bool* refactorize, int* leaving_row,
                                  Fractional* step_length, Fractional* target_bound);
  void PrimalPhaseIChooseLeavingVariableRow(int entering_col, Fractional reduced_cost,
                                            bool* refactorize, int* leaving_row,
                                            Fractional* step_length,
                                            Fractional* target_bound) const;
  Status DualChooseLeavingVariableRow(int* leaving_row, Fractional* cost_variation,
                                      Fractional* target_bound);
  void DualPhaseIUpdatePrice(int leaving_row, int entering_col);
  template <bool use_dense_update = false>
  void OnDualPriceChange(const std::vector<Fractional>& squared_norms, int row,
                         VariableType type, Fractional threshold);
  void DualPhaseIUpdatePriceOnReducedCostChange(const std::vector<int>& cols);
  Status DualPhaseIChooseLeavingVariableRow(int* leaving_row, Fractional* cost_variation,
                                            Fractional* target_bound);
  void MakeBoxedVariableDualFeasible(const std::vector<int>& cols, bool update_basic_values);
  // Dual device mode: phase II of the dual simplex keeps the reduced costs
  // and the update row on the device (MILP_DEVICE_DUAL=auto|force|off; auto:
  // N >= 65536). The host copy of the column status bits is mirrored on the
  // device through the VariablesInfo change log.
  bool DualDeviceEnabled() const;
  void BeginDualDeviceMode();
  void EndDualDeviceMode();
  void FlushColumnBits();
  // MakeBoxedVariableDualFeasible with the decisions taken on the device;
  // cols == nullptr: every non-basic boxed column.
  void SpeculateFlips(int entering_col, int leaving_row, Fractional entering_coeff,
                      Fractional entering_rc);
  void MakeBoxedVariableDualFeasibleOnDevice(const std::vector<int>* cols,
                                             bool update_basic_values);
  Fractional ComputeStepToMoveBasicVariableToBound(int leaving_row, Fractional target_bound) {
    const int leaving_col = basis_[leaving_row];
    const Fractional unscaled_step = variable_values_.Get(leaving_col) - target_bound;
    return unscaled_step / direction_[leaving_row];
  }
  void PermuteBasis();
  Status UpdateAndPivot(int entering_col, int leaving_row, Fractional target_bound);
  Status RefactorizeBasisIfNeeded(bool* refactorize) {
    if (*refactorize && !basis_factorization_.IsRefactorized()) {
      SubTimer timer(kSubRefactorize);
      MILP_RETURN_IF_ERROR(basis_factorization_.Refactorize());
      update_row_.Invalidate();
      PermuteBasis();
    }
    *refactorize = false;
    return Status::OK();
  }
  Status PrimalMinimize(TimeLimit* time_limit);
  Status DualMinimize(bool feasibility_phase, TimeLimit* time_limit);
  Status PrimalPush(TimeLimit* time_limit);
  Status Polish(TimeLimit* time_limit);
  Fractional ComputeObjectiveValue() const {
    return PreciseScalarProduct(objective_, variable_values_.GetDenseRow());
  }
  Fractional ComputeInitialProblemObjectiveValue() const {
    const Fractional sum = PreciseScalarProduct(objective_, variable_values_.GetDenseRow());
    return objective_scaling_factor_ * (sum + objective_offset_);
  }
  int ComputeNumberOfSuperBasicVariables() const {
    int n = 0;
    for (int col = 0; col < num_cols_; ++col)
      if (variables_info_.GetStatusRow()[col] == VariableStatus::FREE &&
          variable_values_.Get(col) != 0.0)
        ++n;
    return n;
  }
  void AdvanceDeterministicTime(TimeLimit* tl) {
    const double cur = DeterministicTime();
    tl->AdvanceDeterministicTime(cur - last_deterministic_time_update_);
    last_deterministic_time_update_ = cur;
  }
  // Debug aid (env MILP_TRACE=<path prefix>): one line per iteration with
  // bit-hashes of the iterate, to locate the first divergence between the
  // oracle and the device engine.
  static uint64_t HashBits(const std::vector<Fractional>& v) {
    uint64_t h = 1469598103934665603ull;
    for (const Fractional x : v) {
      uint64_t b;
      std::memcpy(&b, &x, sizeof(b));
      h = (h ^ b) * 1099511628211ull;
    }
    return h;
  }
  static uint64_t HashInts(const std::vector<int>& v) {
    uint64_t h = 1469598103934665603ull;
    for (const int x : v) h = (h ^ static_cast<uint32_t>(x)) * 1099511628211ull;
    return h;
  }
  void TraceIteration() {
    static const char* prefix = std::getenv("MILP_TRACE");
    if (prefix == nullptr) return;
    primal_edge_norms_.FlushPendingUpdate();  // hash the norms Glop has here
    const std::string path = std::string(prefix) + ".device";
    FILE* f = std::fopen(path.c_str(), "a");
    if (f == nullptr) return;
    std::fprintf(f, "it=%lld phase=%d basis=%016llx x=%016llx rc=%016llx se=%016llx obj=%a"
                 " ent=%d lr=%d step=%a rcq=%a d=%016llx/%016llx/%016llx\n",
                 static_cast<long long>(num_iterations_), static_cast<int>(phase_),
                 static_cast<unsigned long long>(HashInts(basis_)),
                 static_cast<unsigned long long>(HashBits(variable_values_.GetDenseRow())),
                 static_cast<unsigned long long>(HashBits(reduced_costs_.RawReducedCosts())),
                 static_cast<unsigned long long>(HashBits(primal_edge_norms_.RawEdgeNorms())),
                 ComputeObjectiveValue(), trace_entering_, trace_leaving_row_, trace_step_,
                 trace_reduced_cost_, static_cast<unsigned long long>(g_ftran_hash[0]),
                 static_cast<unsigned long long>(g_ftran_hash[1]),
                 static_cast<unsigned long long>(g_ftran_hash[2]));
    trace_entering_ = trace_leaving_row_ = -1;
    trace_step_ = trace_reduced_cost_ = 0.0;
    g_ftran_hash[0] = g_ftran_hash[1] = g_ftran_hash[2] = 0;
    // MILP_TRACE_DUMP=k: raw x, rc and basis at iterations k-1 and k.
    static const char* dump = std::getenv("MILP_TRACE_DUMP");
    if (dump != nullptr && num_iterations_ + 1 >= std::atoll(dump) &&
        num_iterations_ <= std::atoll(dump)) {
      const std::string base = std::string(prefix) + ".it" + std::to_string(num_iterations_) +
                               ".%s";
      auto put = [&](const char* what, const void* p, size_t bytes) {
        char name[512];
        std::snprintf(name, sizeof(name), base.c_str(), what);
        if (FILE* d = std::fopen((std::string(name) + ".device").c_str(), "wb")) {
          std::fwrite(p, 1, bytes, d);
          std::fclose(d);
        }
      };
      put("x", variable_values_.GetDenseRow().data(), sizeof(Fractional) * num_cols_);
      put("rc", reduced_costs_.RawReducedCosts().data(), sizeof(Fractional) * num_cols_);
      put("basis", basis_.data(), sizeof(int) * num_rows_);
      put("d", direction_.values.data(), sizeof(Fractional) * direction_.values.size());
    }
    if (num_cols_ <= 64) {
      const std::vector<Fractional>* vs[3] = {&variable_values_.GetDenseRow(),
                                              &reduced_costs_.RawReducedCosts(),
                                              &primal_edge_norms_.RawEdgeNorms()};
      const char* names[3] = {"x", "rc", "se"};
      for (int k = 0; k < 3; ++k) {
        std::fprintf(f, "  %s:", names[k]);
        for (const Fractional v : *vs[k]) std::fprintf(f, " %a", v);
        std::fprintf(f, "\n");
      }
    }
    std::fclose(f);
  }
  int trace_entering_ = -1;
  int trace_leaving_row_ = -1;
  Fractional trace_step_ = 0.0;
  Fractional trace_reduced_cost_ = 0.0;
  void OnIterationDone(TimeLimit* tl) {
    TraceIteration();
    ++num_iterations_;
    if (record_iteration_times) iteration_times.push_back(tl->GetElapsedTime());
    if (iteration_hook) iteration_hook(num_iterations_);
  }

  DeviceLp device_;  // must outlive (be declared before) its users below
  bool device_matrix_uploaded_ = false;
  ProblemStatus problem_status_ = ProblemStatus::INIT;
  int num_rows_ = 0;
  int num_cols_ = 0;
  int first_slack_col_ = 0;
  CompactSparseMatrix compact_matrix_;
  CompactSparseMatrix transposed_matrix_;
  Fractional primal_objective_limit_ = kInfinity;
  Fractional dual_objective_limit_ = kInfinity;
  std::vector<Fractional> objective_;
  Fractional objective_offset_ = 0.0;
  Fractional objective_scaling_factor_ = 1.0;
  std::vector<Fractional> dual_infeasibility_improvement_direction_;
  int num_dual_infeasible_positions_ = 0;
  ScatteredVector initially_all_zero_scratchpad_;
  std::vector<int> basis_;
  Fractional solution_objective_value_ = 0.0;
  std::vector<Fractional> solution_dual_values_;
  std::vector<Fractional> solution_reduced_costs_;
  std::vector<Fractional> solution_primal_ray_;
  std::vector<Fractional> solution_dual_ray_;
  std::vector<Fractional> solution_dual_ray_row_combination_;
  std::vector<VariableStatus> solution_state_;
  bool solution_state_has_been_set_externally_ = true;
  std::vector<Fractional> variable_starting_values_;
  std::vector<Fractional> integrality_scale_;  // SetIntegralityScale
  bool notify_that_matrix_is_unchanged_ = false;
  ScatteredVector direction_;
  Fractional direction_infinity_norm_ = 0.0;
  std::vector<Fractional> error_;
  Rng random_;
  GlopParameters parameters_;
  GlopParameters initial_parameters_;
  BasisFactorization basis_factorization_;
  VariablesInfo variables_info_;
  PrimalEdgeNorms primal_edge_norms_;
  DualEdgeNorms dual_edge_norms_;
  DynamicMaximum dual_prices_;
  VariableValues variable_values_;
  UpdateRow update_row_;
  ReducedCosts reduced_costs_;
  EnteringVariable entering_variable_;
  PrimalPrices primal_prices_;
  std::vector<Fractional> dual_pricing_vector_;
  std::vector<int> bound_flip_candidates_;
  int64_t num_iterations_ = 0;
  int64_t num_update_price_operations_ = 0;
  double last_deterministic_time_update_ = 0.0;
  Phase phase_ = Phase::FEASIBILITY;
  bool objective_limit_reached_ = false;
  SparseColumn leaving_candidates_;
  std::vector<int> equivalent_leaving_choices_;
  bool dual_device_mode_ = false;
  std::vector<int> status_log_;
  std::vector<int> flush_cols_;
  std::vector<uint8_t> flush_bits_;
  std::vector<uint8_t> flip_flags_;
  std::vector<int> spec_pos_;  // SpeculateFlips: candidate index by column (-1)
  std::vector<int> spec_cols_;
  std::vector<Fractional> spec_deltas_;
  // Device dual segment (csrc/sdual): 0 off, 1 on the host (the same
  // restatement compiled for the CPU, a debugging aid), 2 on the device.
  int sdual_mode_ = 0;
  int saved_sdual_mode_ = 0;
  int batch_depth_ = 0;
  std::vector<char> sdual_buffer_;
  int64_t sdual_segments_ = 0;
  int64_t sdual_iterations_ = 0;
  // -1: no segment (the host runs the iteration), else SdualBridge::Continue's
  // answer: kReturn (DualMinimize returns *status), kLoopTop, kBody.
  int RunSdualSegment(TimeLimit* tl, bool* refactorize, Status* status);
  // The same for the primal loop (csrc/sdual/sprimal_core.h): batch solves
  // with MILP_SPRIMAL=on (device) or host; MILP_SDUAL=host runs it on the host.
  int sprimal_mode_ = 0;
  int RunSprimalSegment(TimeLimit* tl, bool* refactorize, Status* status);

 public:
  // The batch APIs run the phase-II dual loop of their LPs as device
  // segments (one workgroup per LP, csrc/sdual) when many LPs
  // are in flight, and the batched-launch path (host loop, batched small
  // kernels) when few are: a segment iteration is a chain of dependent
  // memory round trips on one wave (~0.4-0.5 ms at m = 2 250), so segments
  // only win by numbers (measured: 128 children 760 LPs/s on segments
  // against 2 009 batched-launch; 1 024 children 4 650 against 3 359).
  // MILP_SDUAL=off / host / device forces a mode; MILP_SDUAL_MIN_LPS sets
  // the in-flight count from which segments are the default (512).
  void SetBatchMode(bool on, int lps_in_flight = 1 << 30) {
    const int batch_mode = [lps_in_flight] {  // read per batch call (tests switch it)
      const char* e = std::getenv("MILP_SDUAL");
      if (e == nullptr) {
        int min_lps = 512;
        if (const char* v = std::getenv("MILP_SDUAL_MIN_LPS")) min_lps = std::atoi(v);
        return lps_in_flight >= min_lps ? 2 : 0;
      }
      if (std::strcmp(e, "host") == 0) return 1;
      if (std::strcmp(e, "device") == 0 || std::strcmp(e, "on") == 0) return 2;
      return 0;
    }();
    static const bool host_ops = [] {
      const char* e = std::getenv("MILP_SDUAL_HOSTOPS");
      return e == nullptr || std::atoi(e) != 0;
    }();
    // A handle may be passed more than once to one batch call: only the
    // outermost on/off pair saves and restores the mode.
    if (on) {
      if (batch_depth_++ == 0) {
        saved_sdual_mode_ = sdual_mode_;
        sdual_mode_ = batch_mode;
        sprimal_mode_ = SprimalMode();
      }
    } else if (batch_depth_ > 0 && --batch_depth_ == 0) {
      sdual_mode_ = saved_sdual_mode_;
      sprimal_mode_ = SprimalMode();
    }
    device_.SetHostSmallOps(batch_depth_ > 0 && sdual_mode_ == 2 && host_ops);
  }
  // Primal segments run where the dual ones do, when MILP_SPRIMAL is "on"
  // (read per call; tests switch it).
  int SprimalMode() const {
    const char* e = std::getenv("MILP_SPRIMAL");
    if (e == nullptr || std::strcmp(e, "on") != 0) return 0;
    return sdual_mode_;
  }
  // Whether this handle's batch solves use the device's segment pool.
  bool UsesSdualPool() const { return batch_depth_ > 0 && sdual_mode_ == 2; }
  // The batch's shared dual edge norms (DualNormCache), or none.
  void SetDualNormCache(DualNormCache* cache) { dual_edge_norms_.SetCache(cache); }
  // The batch's shared factorizations (LuShareCache), or none.
  void SetLuShareCache(LuShareCache* cache) { basis_factorization_.SetLuShareCache(cache); }
  void SdualCounters(int64_t* segments, int64_t* iterations) const {
    *segments = sdual_segments_;
    *iterations = sdual_iterations_;
  }
};

// ---------------------------------------------------------------------------
// Device dual simplex segment: the engine's side of csrc/sdual.
}  // namespace milp
#include "../sdual/sdual_core.h"
namespace milp {
struct SdualHooks {
  static bool Supported(const RevisedSimplex& rs) {
    return rs.sdual_mode_ != 0 && !rs.dual_device_mode_ && !rs.iteration_hook &&
           rs.device_.num_shards() == 1 && !rs.basis_factorization_.tau_u_pending_;
  }
  // Engine-only deferred work must be settled before the state is read: a
  // pending tau on the worker (dropped, as any other use of the factorization
  // would), a deferred column-wise update row, the host mirror of the row.
  static void PrepareForPack(RevisedSimplex& rs) {
    // A parked edge-norm update completes first (it reads the update row the
    // next lines may rebuild); its queued price updates replay with it.
    rs.primal_edge_norms_.FlushPendingUpdate();
    rs.primal_edge_norms_.DropDirectionLeftInverse();
    rs.basis_factorization_.DropAsync();
    rs.update_row_.Materialize();
    rs.update_row_.EnsureHost();
  }
  static void AfterUnpack(RevisedSimplex& rs, const sdual::Lp& s) {
    UpdateRow& ur = rs.update_row_;
    ur.listed_.assign(rs.num_cols_, 0);
    for (const int pos : ur.non_zero_position_list_) ur.listed_[pos] = 1;
    ur.host_stale_ = false;
    ur.known_col_ = -1;
    ur.pending_column_wise_ = false;
    ++ur.epoch_;
    ++rs.sdual_segments_;
    rs.sdual_iterations_ += s.iterations_done;
  }
};
#define SDUAL_DEVICE_RUNNER 1
#include "../sdual/sdual_bridge.inc"

// One segment (MILP_SDUAL=host: the host build of the same code).
int RevisedSimplex::RunSdualSegment(TimeLimit* tl, bool* refactorize, Status* status) {
  if (!SdualBridge::Supported(*this, tl)) return -1;
  if (sdual_mode_ == 1) {
    return SdualBridge::RunOnHost(*this, tl, refactorize, status, &sdual_buffer_);
  }
  return SdualBridge::RunOnDevice(*this, tl, refactorize, status);
}

int RevisedSimplex::RunSprimalSegment(TimeLimit* tl, bool* refactorize, Status* status) {
  if (sprimal_mode_ == 0 || !SdualBridge::SupportedPrimal(*this, tl)) return -1;
  if (sprimal_mode_ == 1) {
    return SdualBridge::RunOnHostPrimal(*this, tl, refactorize, status, &sdual_buffer_);
  }
  return SdualBridge::RunOnDevice(*this, tl, refactorize, status, /*primal=*/true);
}

RevisedSimplex::RevisedSimplex()
    : random_(42),
      basis_factorization_(&compact_matrix_, &basis_),
      variables_info_(compact_matrix_),
      primal_edge_norms_(compact_matrix_, variables_info_, basis_factorization_, &device_),
      dual_edge_norms_(basis_factorization_),
      dual_prices_(&random_),
      variable_values_(parameters_, compact_matrix_, basis_, variables_info_,
                       basis_factorization_, &dual_edge_norms_, &dual_prices_, &device_),
      update_row_(compact_matrix_, transposed_matrix_, variables_info_, basis_,
                  basis_factorization_, &device_),
      reduced_costs_(compact_matrix_, objective_, basis_, variables_info_,
                     basis_factorization_, &random_, &device_),
      entering_variable_(variables_info_, &random_, &reduced_costs_),
      primal_prices_(&random_, variables_info_, &primal_edge_norms_, &reduced_costs_) {
  reduced_costs_.SetDeferredNorms(&primal_edge_norms_);
  basis_factorization_.SetDeviceSolver(&device_);
  SetParameters(parameters_);
  if (const char* e = std::getenv("MILP_SDUAL")) {
    if (std::strcmp(e, "host") == 0) sdual_mode_ = 1;
    if (std::strcmp(e, "device") == 0 || std::strcmp(e, "on") == 0) sdual_mode_ = 2;
  }
  sprimal_mode_ = SprimalMode();
}

void SamplerAttachThread();       // engine/sampler.cc (MILP_SAMPLE_WALL)
void SamplerAttachBatchThread();  // (MILP_SAMPLE_WALL=batch)
void SamplerBatchCallBegin();

// revised_simplex.cc:139-635
Status RevisedSimplex::Solve(const LinearProgram& lp, TimeLimit* time_limit) {
  SamplerAttachThread();
  struct Cleanup {
    std::function<void()> f;
    ~Cleanup() { f(); }
  } cleanup{[this, time_limit]() { AdvanceDeterministicTime(time_limit); }};
  iteration_times.clear();
  MILP_RETURN_IF_ERROR(Initialize(lp));
  dual_infeasibility_improvement_direction_.clear();
  update_row_.Invalidate();
  problem_status_ = ProblemStatus::INIT;
  phase_ = Phase::FEASIBILITY;
  num_iterations_ = 0;
  solution_state_has_been_set_externally_ = true;

  const bool use_dual = parameters_.use_dual_simplex;
  primal_edge_norms_.SetPricingRule(parameters_.feasibility_rule);
  if (use_dual) {
    if (parameters_.perturb_costs_in_dual_simplex) reduced_costs_.PerturbCosts();
    if (parameters_.use_dedicated_dual_feasibility_algorithm) {
      variables_info_.MakeBoxedVariableRelevant(false);
      MILP_RETURN_IF_ERROR(DualMinimize(phase_ == Phase::FEASIBILITY, time_limit));
      if (problem_status_ != ProblemStatus::DUAL_INFEASIBLE) {
        MILP_RETURN_IF_ERROR(basis_factorization_.Refactorize());
        PermuteBasis();
        variables_info_.MakeBoxedVariableRelevant(true);
        reduced_costs_.MakeReducedCostsPrecise();
        MakeBoxedVariableDualFeasible(
            variables_info_.GetNonBasicBoxedVariables().ToVector(), false);
        variable_values_.RecomputeBasicVariableValues();
      }
    } else {
      reduced_costs_.MakeReducedCostsPrecise();
      bool refactorize = reduced_costs_.NeedsBasisRefactorization();
      MILP_RETURN_IF_ERROR(RefactorizeBasisIfNeeded(&refactorize));
      const Fractional initial_infeasibility =
          reduced_costs_.ComputeMaximumDualInfeasibilityOnNonBoxedVariables();
      if (initial_infeasibility < reduced_costs_.GetDualFeasibilityTolerance()) {
        problem_status_ = ProblemStatus::DUAL_FEASIBLE;
        MakeBoxedVariableDualFeasible(
            variables_info_.GetNonBasicBoxedVariables().ToVector(), false);
        variable_values_.RecomputeBasicVariableValues();
      } else {
        variables_info_.TransformToDualPhaseIProblem(
            reduced_costs_.GetDualFeasibilityTolerance(), reduced_costs_.GetReducedCosts());
        std::vector<Fractional> zero;
        variable_values_.ResetAllNonBasicVariableValues(zero);
        variable_values_.RecomputeBasicVariableValues();
        MILP_RETURN_IF_ERROR(DualMinimize(false, time_limit));
        variables_info_.EndDualPhaseI(reduced_costs_.GetDualFeasibilityTolerance(),
                                      reduced_costs_.GetFullReducedCosts());
        variable_values_.ResetAllNonBasicVariableValues(variable_starting_values_);
        variable_values_.RecomputeBasicVariableValues();
        if (problem_status_ == ProblemStatus::OPTIMAL) {
          if (reduced_costs_.ComputeMaximumDualInfeasibility() <
              reduced_costs_.GetDualFeasibilityTolerance() + 1e-6) {
            problem_status_ = ProblemStatus::DUAL_FEASIBLE;
          } else {
            problem_status_ = ProblemStatus::DUAL_INFEASIBLE;
          }
        }
      }
    }
  } else {
    MILP_RETURN_IF_ERROR(PrimalMinimize(time_limit));
    if (problem_status_ != ProblemStatus::PRIMAL_INFEASIBLE) {
      InitializeObjectiveAndTestIfUnchanged(lp);
      reduced_costs_.ResetForNewObjective();
    }
  }

  phase_ = Phase::OPTIMIZATION;
  primal_edge_norms_.SetPricingRule(parameters_.optimization_rule);

  for (int num_optims = 0;
       num_optims <= parameters_.max_number_of_reoptimizations &&
       !objective_limit_reached_ &&
       (num_iterations_ == 0 ||
        num_iterations_ < parameters_.max_number_of_iterations ||
        parameters_.max_number_of_iterations < 0) &&
       !time_limit->LimitReached() &&
       (problem_status_ == ProblemStatus::PRIMAL_FEASIBLE ||
        problem_status_ == ProblemStatus::DUAL_FEASIBLE);
       ++num_optims) {
    if (problem_status_ == ProblemStatus::PRIMAL_FEASIBLE) {
      MILP_RETURN_IF_ERROR(PrimalMinimize(time_limit));
    } else {
      MILP_RETURN_IF_ERROR(DualMinimize(phase_ == Phase::FEASIBILITY, time_limit));
    }
    // revised_simplex.cc:341-344
    if (!integrality_scale_.empty() && problem_status_ == ProblemStatus::OPTIMAL) {
      MILP_RETURN_IF_ERROR(Polish(time_limit));
    }
    variable_values_.ResetAllNonBasicVariableValues(variable_starting_values_);
    MILP_RETURN_IF_ERROR(basis_factorization_.Refactorize());
    PermuteBasis();
    variable_values_.RecomputeBasicVariableValues();
    reduced_costs_.ClearAndRemoveCostShifts();

    if (problem_status_ == ProblemStatus::PRIMAL_UNBOUNDED) {
      const Fractional tolerance = parameters_.solution_feasibility_tolerance;
      if (reduced_costs_.ComputeMaximumDualResidual() > tolerance ||
          variable_values_.ComputeMaximumPrimalResidual() > tolerance ||
          variable_values_.ComputeMaximumPrimalInfeasibility() > tolerance) {
        if (parameters_.change_status_to_imprecise) {
          problem_status_ = ProblemStatus::IMPRECISE;
        }
        break;
      }
      double max_magnitude = 0.0;
      double min_distance = kInfinity;
      const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
      const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
      double cost_delta = 0.0;
      for (int col = 0; col < num_cols_; ++col) {
        cost_delta += solution_primal_ray_[col] * objective_[col];
        if (solution_primal_ray_[col] > 0 && ub[col] != kInfinity) {
          const Fractional value = variable_values_.Get(col);
          const Fractional distance =
              (ub[col] - value + tolerance) / solution_primal_ray_[col];
          min_distance = std::min(distance, min_distance);
          max_magnitude = std::max(solution_primal_ray_[col], max_magnitude);
        }
        if (solution_primal_ray_[col] < 0 && lb[col] != -kInfinity) {
          const Fractional value = variable_values_.Get(col);
          const Fractional distance =
              (value - lb[col] + tolerance) / -solution_primal_ray_[col];
          min_distance = std::min(distance, min_distance);
          max_magnitude = std::max(-solution_primal_ray_[col], max_magnitude);
        }
      }
      if (min_distance * std::fabs(cost_delta) < 1 &&
          reduced_costs_.ComputeMaximumDualInfeasibility() <= tolerance) {
        problem_status_ = ProblemStatus::OPTIMAL;
      }
      break;
    }
    if (problem_status_ == ProblemStatus::DUAL_UNBOUNDED) {
      const Fractional tolerance = parameters_.solution_feasibility_tolerance;
      if (reduced_costs_.ComputeMaximumDualResidual() > tolerance ||
          variable_values_.ComputeMaximumPrimalResidual() > tolerance ||
          reduced_costs_.ComputeMaximumDualInfeasibility() > tolerance) {
        if (parameters_.change_status_to_imprecise) {
          problem_status_ = ProblemStatus::IMPRECISE;
        }
      }
      const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
      const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
      Fractional implied_lb = 0.0;
      Fractional error = 0.0;
      for (int col = 0; col < num_cols_; ++col) {
        const Fractional coeff = solution_dual_ray_row_combination_[col];
        if (coeff > 0) {
          if (lb[col] == -kInfinity) {
            error = std::max(error, coeff);
          } else {
            implied_lb += coeff * lb[col];
          }
        } else if (coeff < 0) {
          if (ub[col] == kInfinity) {
            error = std::max(error, -coeff);
          } else {
            implied_lb += coeff * ub[col];
          }
        }
      }
      if (implied_lb < tolerance || error > tolerance) {
        if (parameters_.change_status_to_imprecise) {
          problem_status_ = ProblemStatus::IMPRECISE;
        }
      }
      break;
    }
    if (problem_status_ == ProblemStatus::OPTIMAL) {
      const Fractional solution_tolerance = parameters_.solution_feasibility_tolerance;
      const Fractional primal_residual = variable_values_.ComputeMaximumPrimalResidual();
      const Fractional dual_residual = reduced_costs_.ComputeMaximumDualResidual();
      if (primal_residual > solution_tolerance || dual_residual > solution_tolerance) {
        if (parameters_.change_status_to_imprecise) {
          problem_status_ = ProblemStatus::IMPRECISE;
        }
      } else {
        const Fractional primal_tolerance =
            std::max(primal_residual, parameters_.primal_feasibility_tolerance);
        const Fractional dual_tolerance =
            std::max(dual_residual, parameters_.dual_feasibility_tolerance);
        const Fractional primal_infeasibility =
            variable_values_.ComputeMaximumPrimalInfeasibility();
        const Fractional dual_infeasibility =
            reduced_costs_.ComputeMaximumDualInfeasibility();
        if (primal_infeasibility > primal_tolerance &&
            dual_infeasibility > dual_tolerance) {
          if (parameters_.change_status_to_imprecise) {
            problem_status_ = ProblemStatus::IMPRECISE;
          }
        } else if (primal_infeasibility > primal_tolerance) {
          if (num_optims == parameters_.max_number_of_reoptimizations) break;
          problem_status_ = ProblemStatus::DUAL_FEASIBLE;
        } else if (dual_infeasibility > dual_tolerance) {
          if (num_optims == parameters_.max_number_of_reoptimizations) break;
          problem_status_ = ProblemStatus::PRIMAL_FEASIBLE;
        }
      }
    }
  }

  if (parameters_.change_status_to_imprecise &&
      problem_status_ != ProblemStatus::DUAL_INFEASIBLE) {
    const Fractional tolerance = parameters_.solution_feasibility_tolerance;
    if (variable_values_.ComputeMaximumPrimalResidual() > tolerance ||
        reduced_costs_.ComputeMaximumDualResidual() > tolerance) {
      problem_status_ = ProblemStatus::IMPRECISE;
    } else if (problem_status_ == ProblemStatus::DUAL_FEASIBLE ||
               problem_status_ == ProblemStatus::DUAL_UNBOUNDED ||
               problem_status_ == ProblemStatus::PRIMAL_INFEASIBLE) {
      if (reduced_costs_.ComputeMaximumDualInfeasibility() > tolerance) {
        problem_status_ = ProblemStatus::IMPRECISE;
      }
    } else if (problem_status_ == ProblemStatus::PRIMAL_FEASIBLE ||
               problem_status_ == ProblemStatus::PRIMAL_UNBOUNDED ||
               problem_status_ == ProblemStatus::DUAL_INFEASIBLE) {
      if (variable_values_.ComputeMaximumPrimalInfeasibility() > tolerance) {
        problem_status_ = ProblemStatus::IMPRECISE;
      }
    }
  }

  if (!variable_starting_values_.empty()) {
    const int num_super_basic = ComputeNumberOfSuperBasicVariables();
    if (num_super_basic > 0 && parameters_.push_to_vertex &&
        problem_status_ == ProblemStatus::OPTIMAL) {
      phase_ = Phase::PUSH;
      MILP_RETURN_IF_ERROR(PrimalPush(time_limit));
    }
  }

  solution_objective_value_ = ComputeInitialProblemObjectiveValue();
  solution_dual_values_ = reduced_costs_.GetDualValues();
  solution_reduced_costs_ = reduced_costs_.GetReducedCosts();
  SaveState();
  if (lp.maximize) {
    for (auto& v : solution_dual_values_) v = -v;
    for (auto& v : solution_reduced_costs_) v = -v;
  }
  if (problem_status_ == ProblemStatus::DUAL_UNBOUNDED ||
      problem_status_ == ProblemStatus::PRIMAL_UNBOUNDED) {
    solution_objective_value_ =
        (problem_status_ == ProblemStatus::DUAL_UNBOUNDED) ? kInfinity : -kInfinity;
    if (lp.maximize) solution_objective_value_ = -solution_objective_value_;
  }
  variable_starting_values_.clear();
  return Status::OK();
}

// revised_simplex.cc:836-926
void RevisedSimplex::UseSingletonColumnInInitialBasis(std::vector<int>* basis) {
  std::vector<int> singleton_column;
  std::vector<Fractional> cost_variation(num_cols_, 0.0);
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  for (int col = 0; col < num_cols_; ++col) {
    if (compact_matrix_.ColumnNumEntries(col) != 1) continue;
    if (lb[col] == ub[col]) continue;
    const Fractional slope = compact_matrix_.column(col).GetFirstCoefficient();
    if (variable_values_.Get(col) == lb[col]) {
      cost_variation[col] = objective_[col] / std::fabs(slope);
    } else {
      cost_variation[col] = -objective_[col] / std::fabs(slope);
    }
    singleton_column.push_back(col);
  }
  if (singleton_column.empty()) return;
  std::sort(singleton_column.begin(), singleton_column.end(),
            [&](int a, int b) { return cost_variation[a] < cost_variation[b]; });
  const std::vector<Fractional>& values = variable_values_.GetDenseRow();
  for (const int col : singleton_column) {
    const int row = compact_matrix_.column(col).GetFirstRow();
    if ((*basis)[row] == kInvalidCol) (*basis)[row] = col;
    if (error_[row] == 0.0) continue;
    const Fractional coeff = compact_matrix_.column(col).GetFirstCoefficient();
    const Fractional new_value = values[col] + error_[row] / coeff;
    if (new_value >= lb[col] && new_value <= ub[col]) {
      error_[row] = 0.0;
      (*basis)[row] = col;
      continue;
    }
    const Fractional box_width = variables_info_.GetBoundDifference(col);
    const Fractional error_sign = error_[row] / coeff;
    if (values[col] == lb[col] && error_sign > 0.0) {
      error_[row] -= coeff * box_width;
      SetNonBasicVariableStatusAndDeriveValue(col, VariableStatus::AT_UPPER_BOUND);
      continue;
    }
    if (values[col] == ub[col] && error_sign < 0.0) {
      error_[row] += coeff * box_width;
      SetNonBasicVariableStatusAndDeriveValue(col, VariableStatus::AT_LOWER_BOUND);
      continue;
    }
  }
}

// revised_simplex.cc:928-1002 + lp_data/matrix_utils.cc
// AreFirstColumnsAndRowsExactlyEquals.
bool RevisedSimplex::InitializeMatrixAndTestIfUnchanged(const LinearProgram& lp,
                                                        bool* only_change_is_new_rows,
                                                        bool* only_change_is_new_cols,
                                                        int* num_new_cols) {
  bool old_part_of_matrix_is_unchanged = true;
  {
    const int nr = num_rows_;
    const int nc = first_slack_col_;
    if (nr > lp.m || nr > compact_matrix_.num_rows() || nc > lp.n ||
        nc > compact_matrix_.num_cols()) {
      old_part_of_matrix_is_unchanged = false;
    } else {
      for (int col = 0; col < nc && old_part_of_matrix_is_unchanged; ++col) {
        const int64_t a0 = lp.col_starts[col];
        const int64_t na = lp.col_starts[col + 1] - a0;
        const ColumnView b = compact_matrix_.column(col);
        const int64_t end = std::min(na, b.n);
        if (end < na && lp.row_idx[a0 + end] < nr) old_part_of_matrix_is_unchanged = false;
        if (end < b.n && b.rows[end] < nr) old_part_of_matrix_is_unchanged = false;
        for (int64_t i = 0; i < end && old_part_of_matrix_is_unchanged; ++i) {
          if (lp.row_idx[a0 + i] != b.rows[i] || lp.vals[a0 + i] != b.coefs[i])
            old_part_of_matrix_is_unchanged = false;
        }
      }
    }
  }
  const int lp_first_slack = lp.n;
  if (old_part_of_matrix_is_unchanged && lp.m == num_rows_ &&
      lp_first_slack == first_slack_col_) {
    if (transposed_matrix_.IsEmpty()) {
      transposed_matrix_.PopulateFromTranspose(compact_matrix_);
      device_matrix_uploaded_ = false;
    }
    if (!device_matrix_uploaded_) {
      device_.UploadMatrix(compact_matrix_, transposed_matrix_);
      device_matrix_uploaded_ = true;
    }
    return true;
  }
  *only_change_is_new_rows = old_part_of_matrix_is_unchanged && lp.m > num_rows_ &&
                             lp_first_slack == first_slack_col_;
  *only_change_is_new_cols = old_part_of_matrix_is_unchanged && lp.m == num_rows_ &&
                             lp_first_slack > first_slack_col_;
  *num_new_cols = *only_change_is_new_cols ? lp_first_slack - first_slack_col_ : 0;
  first_slack_col_ = lp_first_slack;
  num_rows_ = lp.m;
  num_cols_ = lp_first_slack + lp.m;
  compact_matrix_.PopulateFromSparseMatrixAndAddSlacks(lp.m, lp.n, lp.col_starts.data(),
                                                       lp.row_idx.data(), lp.vals.data());
  transposed_matrix_.PopulateFromTranspose(compact_matrix_);
  device_.UploadMatrix(compact_matrix_, transposed_matrix_);
  device_matrix_uploaded_ = true;
  return false;
}

// revised_simplex.cc:1006-1052
bool RevisedSimplex::OldBoundsAreUnchangedAndNewVariablesHaveOneBoundAtZero(
    const LinearProgram& lp, int num_new_cols) {
  const int first_new_col = first_slack_col_ - num_new_cols;
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  for (int col = 0; col < first_new_col; ++col) {
    if (lb[col] != lp.col_lb[col] || ub[col] != lp.col_ub[col]) return false;
  }
  for (int col = first_new_col; col < first_slack_col_; ++col) {
    if (lp.col_lb[col] != 0.0 && lp.col_ub[col] != 0.0) return false;
  }
  for (int row = 0; row < num_rows_; ++row) {
    const int col = first_slack_col_ + row;
    if (lb[col - num_new_cols] != -lp.row_ub[row] ||
        ub[col - num_new_cols] != -lp.row_lb[row])
      return false;
  }
  return true;
}

// revised_simplex.cc:1054-1095
bool RevisedSimplex::InitializeObjectiveAndTestIfUnchanged(const LinearProgram& lp) {
  bool unchanged = true;
  objective_.resize(num_cols_, 0.0);
  for (int col = lp.n; col < num_cols_; ++col) {
    if (objective_[col] != 0.0) {
      unchanged = false;
      objective_[col] = 0.0;
    }
  }
  if (lp.maximize) {
    for (int col = 0; col < lp.n; ++col) {
      const Fractional coeff = -lp.obj[col];
      if (objective_[col] != coeff) {
        unchanged = false;
        objective_[col] = coeff;
      }
    }
    objective_offset_ = -lp.obj_offset;
    objective_scaling_factor_ = -lp.obj_scale;
  } else {
    for (int col = 0; col < lp.n; ++col) {
      const Fractional coeff = lp.obj[col];
      if (objective_[col] != coeff) {
        unchanged = false;
        objective_[col] = coeff;
      }
    }
    objective_offset_ = lp.obj_offset;
    objective_scaling_factor_ = lp.obj_scale;
  }
  return unchanged;
}

// revised_simplex.cc:1097-1127
void RevisedSimplex::InitializeObjectiveLimit() {
  objective_limit_reached_ = false;
  for (const bool set_dual : {true, false}) {
    const Fractional limit = (objective_scaling_factor_ >= 0.0) != set_dual
                                 ? parameters_.objective_lower_limit
                                 : parameters_.objective_upper_limit;
    const Fractional shifted_limit = limit / objective_scaling_factor_ - objective_offset_;
    if (set_dual) {
      dual_objective_limit_ = shifted_limit;
    } else {
      primal_objective_limit_ = shifted_limit;
    }
  }
}

// revised_simplex.cc:1134-1278
Status RevisedSimplex::CreateInitialBasis() {
  variables_info_.InitializeToDefaultStatus();
  variable_values_.ResetAllNonBasicVariableValues(variable_starting_values_);
  std::vector<int> basis(num_rows_, kInvalidCol);
  for (int row = 0; row < num_rows_; ++row) basis[row] = first_slack_col_ + row;
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  if (!parameters_.use_dual_simplex && parameters_.initial_basis != 3 &&
      parameters_.exploit_singleton_column_in_initial_basis) {
    for (int col = 0; col < num_cols_; ++col) {
      if (compact_matrix_.ColumnNumEntries(col) != 1) continue;
      const VariableStatus status = variables_info_.GetStatusRow()[col];
      const Fractional objective = objective_[col];
      if (objective > 0 && IsFinite(lb[col]) && status == VariableStatus::AT_UPPER_BOUND) {
        SetNonBasicVariableStatusAndDeriveValue(col, VariableStatus::AT_LOWER_BOUND);
      } else if (objective < 0 && IsFinite(ub[col]) &&
                 status == VariableStatus::AT_LOWER_BOUND) {
        SetNonBasicVariableStatusAndDeriveValue(col, VariableStatus::AT_UPPER_BOUND);
      }
    }
    ComputeVariableValuesError();
    basis.assign(num_rows_, kInvalidCol);
    UseSingletonColumnInInitialBasis(&basis);
    for (int row = 0; row < num_rows_; ++row)
      if (basis[row] == kInvalidCol) basis[row] = first_slack_col_ + row;
  }
  if (parameters_.initial_basis == 0) return InitializeFirstBasis(basis);
  if (parameters_.initial_basis == 3) {  // MAROS (revised_simplex.cc:1200-1216)
    if (parameters_.use_dual_simplex) {
      GetMarosBasis<true>(compact_matrix_, objective_, variables_info_.GetTypeRow(), num_cols_,
                          &basis);
    } else {
      GetMarosBasis<false>(compact_matrix_, objective_, variables_info_.GetTypeRow(), num_cols_,
                           &basis);
    }
    return InitializeFirstBasis(basis);
  }
  if (parameters_.initial_basis == 1 && parameters_.use_scaling) {  // BIXBY
    int num_fixed_variables = 0;
    for (int row = 0; row < static_cast<int>(basis.size()); ++row) {
      const int col = basis[row];
      if (lb[col] == ub[col]) {
        basis[row] = kInvalidCol;
        ++num_fixed_variables;
      }
    }
    if (num_fixed_variables != 0) {
      CompleteBixbyBasis(compact_matrix_, objective_, lb, ub, variables_info_.GetTypeRow(),
                         first_slack_col_, &basis);
    }
    return InitializeFirstBasis(basis);
  }
  if (parameters_.initial_basis == 2) {  // TRIANGULAR
    int num_fixed_variables = 0;
    for (int row = 0; row < static_cast<int>(basis.size()); ++row) {
      const int col = basis[row];
      if (lb[col] == ub[col]) {
        basis[row] = kInvalidCol;
        ++num_fixed_variables;
      }
    }
    if (num_fixed_variables != 0) {
      if (parameters_.use_dual_simplex) {
        CompleteTriangularBasis<true>(compact_matrix_, objective_, lb, ub,
                                      variables_info_.GetTypeRow(), num_cols_, &basis);
      } else {
        CompleteTriangularBasis<false>(compact_matrix_, objective_, lb, ub,
                                       variables_info_.GetTypeRow(), num_cols_, &basis);
      }
      const Status status = InitializeFirstBasis(basis);
      if (status.ok()) return status;
      for (int row = 0; row < num_rows_; ++row) basis[row] = first_slack_col_ + row;
    }
  }
  return InitializeFirstBasis(basis);
}

// revised_simplex.cc:1280-1332
Status RevisedSimplex::InitializeFirstBasis(const std::vector<int>& basis) {
  basis_ = basis;
  basis_.resize(num_rows_, kInvalidCol);
  for (int row = 0; row < num_rows_; ++row)
    if (basis_[row] == kInvalidCol) basis_[row] = first_slack_col_ + row;
  MILP_RETURN_IF_ERROR(basis_factorization_.Initialize());
  PermuteBasis();
  const Fractional cond = basis_factorization_.ComputeInfinityNormConditionNumberUpperBound();
  if (cond > parameters_.initial_condition_number_threshold) {
    return Status(Status::ERROR_LU, "The matrix condition number upper bound is too high");
  }
  for (int row = 0; row < num_rows_; ++row) variables_info_.UpdateToBasicStatus(basis_[row]);
  variable_values_.ResetAllNonBasicVariableValues(variable_starting_values_);
  variable_values_.RecomputeBasicVariableValues();
  return Status::OK();
}

// revised_simplex.cc:1334-1565
Status RevisedSimplex::Initialize(const LinearProgram& lp) {
  parameters_ = initial_parameters_;
  PropagateParameters();
  int num_new_cols = 0;
  bool only_change_is_new_rows = false;
  bool only_change_is_new_cols = false;
  bool matrix_is_unchanged = true;
  bool only_new_bounds = false;
  if (solution_state_.empty() || !notify_that_matrix_is_unchanged_) {
    matrix_is_unchanged = InitializeMatrixAndTestIfUnchanged(
        lp, &only_change_is_new_rows, &only_change_is_new_cols, &num_new_cols);
    only_new_bounds = only_change_is_new_cols && num_new_cols > 0 &&
                      OldBoundsAreUnchangedAndNewVariablesHaveOneBoundAtZero(lp, num_new_cols);
  }
  notify_that_matrix_is_unchanged_ = false;
  const bool objective_is_unchanged = InitializeObjectiveAndTestIfUnchanged(lp);
  const bool bounds_are_unchanged = variables_info_.LoadBoundsAndReturnTrueIfUnchanged(
      lp.col_lb, lp.col_ub, lp.row_lb, lp.row_ub);
  if (matrix_is_unchanged && parameters_.allow_simplex_algorithm_change) {
    if (objective_is_unchanged && !bounds_are_unchanged) {
      parameters_.use_dual_simplex = true;
      PropagateParameters();
    }
    if (bounds_are_unchanged && !objective_is_unchanged) {
      parameters_.use_dual_simplex = false;
      PropagateParameters();
    }
  }
  InitializeObjectiveLimit();

  bool solve_from_scratch = true;
  if (!solution_state_.empty() && !solution_state_has_been_set_externally_) {
    if (!parameters_.use_dual_simplex) {
      dual_edge_norms_.Clear();
      dual_pricing_vector_.clear();
      if (matrix_is_unchanged && bounds_are_unchanged) {
        reduced_costs_.ClearAndRemoveCostShifts();
        solve_from_scratch = false;
      } else if (only_change_is_new_cols && only_new_bounds) {
        variables_info_.InitializeFromBasisState(first_slack_col_, num_new_cols,
                                                 solution_state_);
        variable_values_.ResetAllNonBasicVariableValues(variable_starting_values_);
        const int first_new_col = first_slack_col_ - num_new_cols;
        for (int& c : basis_)
          if (c >= first_new_col) c += num_new_cols;
        primal_edge_norms_.Clear();
        reduced_costs_.ClearAndRemoveCostShifts();
        solve_from_scratch = false;
      }
    } else {
      primal_edge_norms_.Clear();
      if (objective_is_unchanged) {
        if (matrix_is_unchanged) {
          if (!bounds_are_unchanged) {
            variables_info_.InitializeFromBasisState(first_slack_col_, 0, solution_state_);
            variable_values_.ResetAllNonBasicVariableValues(variable_starting_values_);
            variable_values_.RecomputeBasicVariableValues();
          }
          solve_from_scratch = false;
        } else if (only_change_is_new_rows) {
          variables_info_.InitializeFromBasisState(first_slack_col_, 0, solution_state_);
          dual_edge_norms_.ResizeOnNewRows(num_rows_);
          reduced_costs_.ClearAndRemoveCostShifts();
          dual_pricing_vector_.clear();
          if (InitializeFirstBasis(basis_).ok()) solve_from_scratch = false;
        }
      }
    }
  }

  if (solve_from_scratch && !solution_state_.empty()) {
    basis_factorization_.Clear();
    reduced_costs_.ClearAndRemoveCostShifts();
    primal_edge_norms_.Clear();
    dual_edge_norms_.Clear();
    dual_pricing_vector_.clear();
    variables_info_.InitializeFromBasisState(first_slack_col_, 0, solution_state_);
    std::vector<int> candidates = variables_info_.GetIsBasicBitRow().ToVector();
    if (static_cast<int>(candidates.size()) == num_rows_) {
      basis_ = candidates;
      if (InitializeFirstBasis(basis_).ok()) solve_from_scratch = false;
    }
    if (solve_from_scratch) {
      basis_ = basis_factorization_.ComputeInitialBasis(candidates);
      variables_info_.ChangeUnusedBasicVariablesToFree(basis_);
      variables_info_.SnapFreeVariablesToBound(parameters_.crossover_bound_snapping_distance,
                                               variable_starting_values_);
      if (InitializeFirstBasis(basis_).ok()) solve_from_scratch = false;
    }
  }

  if (solve_from_scratch) {
    basis_factorization_.Clear();
    reduced_costs_.ClearAndRemoveCostShifts();
    primal_edge_norms_.Clear();
    dual_edge_norms_.Clear();
    dual_pricing_vector_.clear();
    MILP_RETURN_IF_ERROR(CreateInitialBasis());
  }
  return Status::OK();
}

// revised_simplex.cc:1663-1693
void RevisedSimplex::CorrectErrorsOnVariableValues() {
  const Fractional primal_residual = variable_values_.ComputeMaximumPrimalResidual();
  const bool recompute = primal_residual >= parameters_.harris_tolerance_ratio *
                                                parameters_.primal_feasibility_tolerance;
  if (const char* e = std::getenv("MILP_TRACE_RESIDUAL")) {  // debugging aid
    if (FILE* f = std::fopen(e, "a")) {
      std::fprintf(f, "it=%lld residual=%a recompute=%d\n", static_cast<long long>(num_iterations_),
                   primal_residual, recompute ? 1 : 0);
      std::fclose(f);
    }
  }
  if (recompute) variable_values_.RecomputeBasicVariableValues();
}

void RevisedSimplex::ComputeVariableValuesError() {
  if (device_.host_small_ops()) {
    HostRowSums(compact_matrix_, variable_values_.GetDenseRow(), nullptr, -1.0, &error_);
  } else {
    device_.RowSums(variable_values_.GetDenseRow(), /*skip_basic=*/false, -1.0, &error_);
  }
}

// revised_simplex.cc:1695-1720
void RevisedSimplex::ComputeDirection(int col) {
  SubTimer timer(kSubFtranDirection);
  primal_edge_norms_.DropDirectionLeftInverse();  // its job reads direction_
  basis_factorization_.RightSolveForProblemColumn(col, &direction_);
  direction_infinity_norm_ = 0.0;
  if (direction_.non_zeros.empty()) {
    ParallelAppendNonZeros(direction_.values.data(), 0, num_rows_, &direction_.non_zeros,
                           static_cast<std::vector<Fractional>*>(nullptr),
                           &direction_infinity_norm_);
  } else {
    for (const int row : direction_.non_zeros) {
      direction_infinity_norm_ =
          std::max(direction_infinity_norm_, std::fabs(direction_[row]));
    }
  }
}

// revised_simplex.cc:1732-1754
template <bool positive>
Fractional RevisedSimplex::GetRatio(const std::vector<Fractional>& lb,
                                    const std::vector<Fractional>& ub, int row) const {
  const int col = basis_[row];
  const Fractional direction = direction_[row];
  const Fractional value = variable_values_.Get(col);
  if (positive) {
    if (direction > 0.0) return (ub[col] - value) / direction;
    return (lb[col] - value) / direction;
  } else {
    if (direction > 0.0) return (value - lb[col]) / direction;
    return (value - ub[col]) / direction;
  }
}

// revised_simplex.cc:1756-1806
template <bool positive>
Fractional RevisedSimplex::ComputeHarrisRatioAndLeavingCandidates(
    Fractional bound_flip_ratio, SparseColumn* leaving_candidates) const {
  const Fractional harris_tolerance =
      parameters_.harris_tolerance_ratio * parameters_.primal_feasibility_tolerance;
  const Fractional minimum_delta =
      parameters_.degenerate_ministep_factor * parameters_.primal_feasibility_tolerance;
  Fractional harris_ratio = bound_flip_ratio;
  leaving_candidates->Clear();
  const Fractional threshold = basis_factorization_.IsRefactorized()
                                   ? parameters_.minimum_acceptable_pivot
                                   : parameters_.ratio_test_zero_threshold;
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  for (const int row : direction_.non_zeros) {
    const Fractional magnitude = std::fabs(direction_[row]);
    if (magnitude <= threshold) continue;
    const Fractional ratio = GetRatio<positive>(lb, ub, row);
    if (ratio <= harris_ratio) {
      leaving_candidates->SetCoefficient(row, ratio);
      harris_ratio = std::min(harris_ratio, std::max(minimum_delta / magnitude,
                                                     ratio + harris_tolerance / magnitude));
    }
  }
  return harris_ratio;
}

namespace {
bool IsRatioMoreOrEquallyStable(Fractional candidate, Fractional current) {
  if (current >= 0.0) return candidate >= 0.0 && candidate <= current;
  return candidate >= current;
}
}  // namespace

// revised_simplex.cc:1829-2003
Status RevisedSimplex::ChooseLeavingVariableRow(int entering_col, Fractional reduced_cost,
                                                bool* refactorize, int* leaving_row,
                                                Fractional* step_length,
                                                Fractional* target_bound) {
  equivalent_leaving_choices_.clear();
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  while (true) {
    const Fractional entering_value = variable_values_.Get(entering_col);
    Fractional current_ratio = (reduced_cost > 0.0) ? entering_value - lb[entering_col]
                                                    : ub[entering_col] - entering_value;
    const Fractional harris_ratio =
        (reduced_cost > 0.0)
            ? ComputeHarrisRatioAndLeavingCandidates<true>(current_ratio, &leaving_candidates_)
            : ComputeHarrisRatioAndLeavingCandidates<false>(current_ratio,
                                                            &leaving_candidates_);
    if (current_ratio <= harris_ratio) {
      *leaving_row = kInvalidRow;
      *step_length = current_ratio;
      break;
    }
    Fractional pivot_magnitude = 0.0;
    *leaving_row = kInvalidRow;
    equivalent_leaving_choices_.clear();
    for (int64_t k = 0; k < leaving_candidates_.num_entries(); ++k) {
      const Fractional ratio = leaving_candidates_.coefs[k];
      if (ratio > harris_ratio) continue;
      const int row = leaving_candidates_.rows[k];
      const Fractional candidate_magnitude = std::fabs(direction_[row]);
      if (candidate_magnitude < pivot_magnitude) continue;
      if (candidate_magnitude == pivot_magnitude) {
        if (!IsRatioMoreOrEquallyStable(ratio, current_ratio)) continue;
        if (ratio == current_ratio) {
          equivalent_leaving_choices_.push_back(row);
          continue;
        }
      }
      equivalent_leaving_choices_.clear();
      current_ratio = ratio;
      pivot_magnitude = candidate_magnitude;
      *leaving_row = row;
    }
    if (!equivalent_leaving_choices_.empty()) {
      equivalent_leaving_choices_.push_back(*leaving_row);
      *leaving_row = equivalent_leaving_choices_[UniformInt(
          random_, static_cast<int>(equivalent_leaving_choices_.size()) - 1)];
    }
    if (current_ratio <= 0.0) {
      const Fractional minimum_delta =
          parameters_.degenerate_ministep_factor * parameters_.primal_feasibility_tolerance;
      *step_length = minimum_delta / pivot_magnitude;
    } else {
      *step_length = current_ratio;
    }
    if (pivot_magnitude < parameters_.small_pivot_threshold * direction_infinity_norm_) {
      if (!basis_factorization_.IsRefactorized()) {
        *refactorize = true;
        return Status::OK();
      }
    }
    break;
  }
  if (*leaving_row != kInvalidRow) {
    const bool is_reduced_cost_positive = (reduced_cost > 0.0);
    const bool is_leaving_coeff_positive = (direction_[*leaving_row] > 0.0);
    *target_bound = (is_reduced_cost_positive == is_leaving_coeff_positive)
                        ? ub[basis_[*leaving_row]]
                        : lb[basis_[*leaving_row]];
  }
  return Status::OK();
}

namespace {
// revised_simplex.cc:2010-2035
struct BreakPoint {
  int row;
  Fractional ratio;
  Fractional coeff_magnitude;
  Fractional target_bound;
  bool operator<(const BreakPoint& o) const {
    if (ratio == o.ratio) {
      if (coeff_magnitude == o.coeff_magnitude) return row > o.row;
      return coeff_magnitude < o.coeff_magnitude;
    }
    return ratio > o.ratio;
  }
};
}  // namespace

// revised_simplex.cc:2039-2145
void RevisedSimplex::PrimalPhaseIChooseLeavingVariableRow(
    int entering_col, Fractional reduced_cost, bool* refactorize, int* leaving_row,
    Fractional* step_length, Fractional* target_bound) const {
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  const Fractional entering_value = variable_values_.Get(entering_col);
  Fractional current_ratio = (reduced_cost > 0.0) ? entering_value - lb[entering_col]
                                                  : ub[entering_col] - entering_value;
  std::vector<BreakPoint> breakpoints;
  const Fractional tolerance = parameters_.primal_feasibility_tolerance;
  for (const int row : direction_.non_zeros) {
    const Fractional direction = reduced_cost > 0.0 ? direction_[row] : -direction_[row];
    const Fractional magnitude = std::fabs(direction);
    if (magnitude < tolerance) continue;
    const int col = basis_[row];
    const Fractional value = variable_values_.Get(col);
    const Fractional lower_bound = lb[col];
    const Fractional upper_bound = ub[col];
    const Fractional to_lower = (lower_bound - tolerance - value) / direction;
    const Fractional to_upper = (upper_bound + tolerance - value) / direction;
    if (to_lower >= 0.0 && to_lower < current_ratio)
      breakpoints.push_back(BreakPoint{row, to_lower, magnitude, lower_bound});
    if (to_upper >= 0.0 && to_upper < current_ratio)
      breakpoints.push_back(BreakPoint{row, to_upper, magnitude, upper_bound});
  }
  std::make_heap(breakpoints.begin(), breakpoints.end());
  Fractional improvement = std::fabs(reduced_cost);
  Fractional best_magnitude = 0.0;
  *leaving_row = kInvalidRow;
  while (!breakpoints.empty()) {
    const BreakPoint top = breakpoints.front();
    if (top.coeff_magnitude > best_magnitude) {
      *leaving_row = top.row;
      current_ratio = top.ratio;
      best_magnitude = top.coeff_magnitude;
      *target_bound = top.target_bound;
    }
    improvement -= top.coeff_magnitude;
    if (improvement <= 0.0) break;
    std::pop_heap(breakpoints.begin(), breakpoints.end());
    breakpoints.pop_back();
  }
  if (*leaving_row != kInvalidRow) {
    const Fractional threshold = parameters_.small_pivot_threshold * direction_infinity_norm_;
    if (best_magnitude < threshold && !basis_factorization_.IsRefactorized()) {
      *refactorize = true;
      return;
    }
  }
  *step_length = current_ratio;
}

// revised_simplex.cc:2148-2181
Status RevisedSimplex::DualChooseLeavingVariableRow(int* leaving_row,
                                                    Fractional* cost_variation,
                                                    Fractional* target_bound) {
  if (dual_prices_.Size() == 0) {
    variable_values_.RecomputeDualPrices(parameters_.dual_price_prioritize_norm);
  }
  *leaving_row = dual_prices_.GetMaximum();
  if (*leaving_row == kInvalidRow) return Status::OK();
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  const int leaving_col = basis_[*leaving_row];
  const Fractional value = variable_values_.Get(leaving_col);
  if (value < lb[leaving_col]) {
    *cost_variation = lb[leaving_col] - value;
    *target_bound = lb[leaving_col];
  } else {
    *cost_variation = ub[leaving_col] - value;
    *target_bound = ub[leaving_col];
  }
  return Status::OK();
}

namespace {
bool IsDualPhaseILeavingCandidate(Fractional cost, VariableType type, Fractional threshold) {
  if (cost == 0.0) return false;
  return type == VariableType::UPPER_AND_LOWER_BOUNDED ||
         type == VariableType::FIXED_VARIABLE ||
         (type == VariableType::UPPER_BOUNDED && cost < -threshold) ||
         (type == VariableType::LOWER_BOUNDED && cost > threshold);
}
}  // namespace

// revised_simplex.cc:2198-2215
template <bool use_dense_update>
void RevisedSimplex::OnDualPriceChange(const std::vector<Fractional>& squared_norm, int row,
                                       VariableType type, Fractional threshold) {
  const Fractional price = dual_pricing_vector_[row];
  const bool is_candidate = IsDualPhaseILeavingCandidate(price, type, threshold);
  if (is_candidate) {
    if (use_dense_update) {
      dual_prices_.DenseAddOrUpdate(row, Square(price) / squared_norm[row]);
    } else {
      dual_prices_.AddOrUpdate(row, Square(price) / squared_norm[row]);
    }
  } else {
    dual_prices_.Remove(row);
  }
}

// revised_simplex.cc:2217-2267
void RevisedSimplex::DualPhaseIUpdatePrice(int leaving_row, int entering_col) {
  if (reduced_costs_.AreReducedCostsRecomputed() ||
      dual_edge_norms_.NeedsBasisRefactorization() || dual_pricing_vector_.empty()) {
    return;
  }
  const std::vector<VariableType>& variable_type = variables_info_.GetTypeRow();
  const Fractional threshold = parameters_.ratio_test_zero_threshold;
  const std::vector<Fractional>& squared_norms = dual_edge_norms_.GetEdgeSquaredNorms();
  const Fractional step = dual_pricing_vector_[leaving_row] / direction_[leaving_row];
  for (const int row : direction_.non_zeros) {
    dual_pricing_vector_[row] -= direction_[row] * step;
    OnDualPriceChange(squared_norms, row, variable_type[basis_[row]], threshold);
  }
  dual_pricing_vector_[leaving_row] = step;
  dual_pricing_vector_[leaving_row] -=
      dual_infeasibility_improvement_direction_[entering_col];
  if (dual_infeasibility_improvement_direction_[entering_col] != 0.0) {
    --num_dual_infeasible_positions_;
  }
  dual_infeasibility_improvement_direction_[entering_col] = 0.0;
  dual_infeasibility_improvement_direction_[basis_[leaving_row]] = 0.0;
  OnDualPriceChange(squared_norms, leaving_row, variable_type[entering_col], threshold);
}

// revised_simplex.cc:2269-2333
void RevisedSimplex::DualPhaseIUpdatePriceOnReducedCostChange(const std::vector<int>& cols) {
  bool something_to_do = false;
  const Bitset& can_decrease = variables_info_.GetCanDecreaseBitRow();
  const Bitset& can_increase = variables_info_.GetCanIncreaseBitRow();
  const std::vector<Fractional>& reduced_costs = reduced_costs_.GetReducedCosts();
  const Fractional tolerance = reduced_costs_.GetDualFeasibilityTolerance();
  for (const int col : cols) {
    const Fractional reduced_cost = reduced_costs[col];
    const Fractional sign = (can_increase.IsSet(col) && reduced_cost < -tolerance) ? 1.0
                            : (can_decrease.IsSet(col) && reduced_cost > tolerance) ? -1.0
                                                                                    : 0.0;
    if (sign != dual_infeasibility_improvement_direction_[col]) {
      if (sign == 0.0) {
        --num_dual_infeasible_positions_;
      } else if (dual_infeasibility_improvement_direction_[col] == 0.0) {
        ++num_dual_infeasible_positions_;
      }
      if (!something_to_do) {
        initially_all_zero_scratchpad_.values.resize(num_rows_, 0.0);
        initially_all_zero_scratchpad_.ClearSparseMask();
        initially_all_zero_scratchpad_.non_zeros.clear();
        something_to_do = true;
      }
      num_update_price_operations_ += 10 * compact_matrix_.ColumnNumEntries(col);
      compact_matrix_.ColumnAddMultipleToSparseScatteredColumn(
          col, sign - dual_infeasibility_improvement_direction_[col],
          &initially_all_zero_scratchpad_);
      dual_infeasibility_improvement_direction_[col] = sign;
    }
  }
  if (something_to_do) {
    initially_all_zero_scratchpad_.ClearNonZerosIfTooDense();
    initially_all_zero_scratchpad_.ClearSparseMask();
    const std::vector<Fractional>& squared_norms = dual_edge_norms_.GetEdgeSquaredNorms();
    const std::vector<VariableType>& variable_type = variables_info_.GetTypeRow();
    const Fractional threshold = parameters_.ratio_test_zero_threshold;
    basis_factorization_.RightSolve(&initially_all_zero_scratchpad_);
    if (initially_all_zero_scratchpad_.non_zeros.empty()) {
      dual_prices_.StartDenseUpdates();
      for (int row = 0; row < num_rows_; ++row) {
        if (initially_all_zero_scratchpad_[row] == 0.0) continue;
        dual_pricing_vector_[row] += initially_all_zero_scratchpad_[row];
        OnDualPriceChange<true>(squared_norms, row, variable_type[basis_[row]], threshold);
      }
      initially_all_zero_scratchpad_.values.assign(num_rows_, 0.0);
    } else {
      for (const int row : initially_all_zero_scratchpad_.non_zeros) {
        dual_pricing_vector_[row] += initially_all_zero_scratchpad_[row];
        OnDualPriceChange(squared_norms, row, variable_type[basis_[row]], threshold);
        initially_all_zero_scratchpad_[row] = 0.0;
      }
    }
    initially_all_zero_scratchpad_.non_zeros.clear();
  }
}

// revised_simplex.cc:2335-2388
Status RevisedSimplex::DualPhaseIChooseLeavingVariableRow(int* leaving_row,
                                                          Fractional* cost_variation,
                                                          Fractional* target_bound) {
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  if (reduced_costs_.AreReducedCostsRecomputed() ||
      dual_edge_norms_.NeedsBasisRefactorization() || dual_pricing_vector_.empty()) {
    num_dual_infeasible_positions_ = 0;
    dual_pricing_vector_.assign(num_rows_, 0.0);
    dual_prices_.ClearAndResize(num_rows_);
    dual_infeasibility_improvement_direction_.assign(num_cols_, 0.0);
    DualPhaseIUpdatePriceOnReducedCostChange(
        variables_info_.GetIsRelevantBitRow().ToVector());
  } else {
    DualPhaseIUpdatePriceOnReducedCostChange(update_row_.GetNonZeroPositions());
  }
  *leaving_row = kInvalidRow;
  if (num_dual_infeasible_positions_ == 0) return Status::OK();
  *leaving_row = dual_prices_.GetMaximum();
  if (*leaving_row == kInvalidRow) return Status::OK();
  *cost_variation = dual_pricing_vector_[*leaving_row];
  const int leaving_col = basis_[*leaving_row];
  if (*cost_variation < 0.0) {
    *target_bound = ub[leaving_col];
  } else {
    *target_bound = lb[leaving_col];
  }
  return Status::OK();
}

// revised_simplex.cc:2390-2437
void RevisedSimplex::MakeBoxedVariableDualFeasible(const std::vector<int>& cols,
                                                   bool update_basic_values) {
  SubTimer timer(kSubBoxedScan);
  std::vector<int> changed_cols;
  const Fractional threshold = reduced_costs_.GetDualFeasibilityTolerance();
  const std::vector<Fractional>& reduced_costs = reduced_costs_.GetReducedCosts();
  const std::vector<VariableStatus>& variable_status = variables_info_.GetStatusRow();
  for (const int col : cols) {
    const Fractional reduced_cost = reduced_costs[col];
    const VariableStatus status = variable_status[col];
    if (reduced_cost > threshold && status == VariableStatus::AT_UPPER_BOUND) {
      variables_info_.UpdateToNonBasicStatus(col, VariableStatus::AT_LOWER_BOUND);
      changed_cols.push_back(col);
    } else if (reduced_cost < -threshold && status == VariableStatus::AT_LOWER_BOUND) {
      variables_info_.UpdateToNonBasicStatus(col, VariableStatus::AT_UPPER_BOUND);
      changed_cols.push_back(col);
    }
  }
  if (!changed_cols.empty()) {
    SubTimer flip_timer(kSubFlipFtran);
    variable_values_.UpdateGivenNonBasicVariables(changed_cols, update_basic_values);
  }
}

// revised_simplex.cc:2475-2502
void RevisedSimplex::PermuteBasis() {
  const std::vector<int> col_perm = basis_factorization_.GetColumnPermutation();
  if (col_perm.empty()) return;
  {
    std::vector<int> tmp(basis_.size());
    for (size_t i = 0; i < col_perm.size(); ++i) tmp[col_perm[i]] = basis_[i];
    basis_.swap(tmp);
  }
  if (!dual_pricing_vector_.empty()) {
    std::vector<Fractional> tmp(dual_pricing_vector_.size());
    for (size_t i = 0; i < col_perm.size(); ++i) tmp[col_perm[i]] = dual_pricing_vector_[i];
    dual_pricing_vector_.swap(tmp);
  }
  reduced_costs_.UpdateDataOnBasisPermutation();
  dual_edge_norms_.UpdateDataOnBasisPermutation(col_perm);
  basis_factorization_.SetColumnPermutationToIdentity();
}

// revised_simplex.cc:2504-2575
Status RevisedSimplex::UpdateAndPivot(int entering_col, int leaving_row,
                                      Fractional target_bound) {
  Fractional pivot_from_update_row;
  if (update_row_.IsComputedFor(leaving_row)) {
    pivot_from_update_row = update_row_.GetCoefficient(entering_col);
  } else {
    update_row_.ComputeUnitRowLeftInverse(leaving_row);
    pivot_from_update_row = compact_matrix_.ColumnScalarProduct(
        entering_col, update_row_.GetUnitRowLeftInverse().values.data());
  }
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  const int leaving_col = basis_[leaving_row];
  const VariableStatus leaving_variable_status =
      lb[leaving_col] == ub[leaving_col] ? VariableStatus::FIXED_VALUE
      : target_bound == lb[leaving_col]  ? VariableStatus::AT_LOWER_BOUND
                                         : VariableStatus::AT_UPPER_BOUND;
  UpdateBasis(entering_col, leaving_row, leaving_variable_status);
  const Fractional pivot_from_direction = direction_[leaving_row];
  const Fractional diff = std::fabs(pivot_from_update_row - pivot_from_direction);
  if (diff > parameters_.refactorization_threshold *
                 (1.0 + std::min(std::fabs(pivot_from_update_row),
                                 std::fabs(pivot_from_direction)))) {
    if (basis_factorization_.NumUpdates() < 10) {
      Fractional threshold = parameters_.lu_factorization_pivot_threshold;
      threshold = std::min(threshold * 1.5, 0.9);
      parameters_.lu_factorization_pivot_threshold = threshold;
      basis_factorization_.SetLuParameters(parameters_.lu());
    }
    SubTimer timer(kSubRefactorize);
    MILP_RETURN_IF_ERROR(basis_factorization_.ForceRefactorization());
  } else {
    SubTimer timer(kSubLuUpdate);
    MILP_RETURN_IF_ERROR(basis_factorization_.Update(entering_col, leaving_row, direction_));
  }
  if (basis_factorization_.IsRefactorized()) PermuteBasis();
  return Status::OK();
}

// revised_simplex.cc:2751-3045
Status RevisedSimplex::PrimalMinimize(TimeLimit* time_limit) {
  struct Cleanup {
    std::function<void()> f;
    ~Cleanup() { f(); }
  } cleanup{[this, time_limit]() {
    try {
      primal_edge_norms_.FlushPendingUpdate();  // nothing parked leaves the loop
    } catch (const DeviceError&) {
      // The device failed; the next device call reports it.
    }
    AdvanceDeterministicTime(time_limit);
  }};
  {
    const char* defer = std::getenv("MILP_DEFER_NORMS");
    primal_edge_norms_.SetDeferral(defer == nullptr || std::strcmp(defer, "0") != 0);
  }
  PhaseClock clock;
  const int64_t first_iteration = num_iterations_;
  struct DumpAtExit {
    PhaseClock* c;
    const int64_t* it;
    int64_t first;
    ~DumpAtExit() { c->Dump(static_cast<long long>(*it - first)); }
  } dump{&clock, &num_iterations_, first_iteration};
  g_trace_ftran = std::getenv("MILP_TRACE") != nullptr;
  bool refactorize = false;
  primal_prices_.ForceRecomputation();
  if (phase_ == Phase::FEASIBILITY) {
    objective_.assign(num_cols_, 0.0);
    std::vector<int> all_rows(num_rows_);
    for (int r = 0; r < num_rows_; ++r) all_rows[r] = r;
    variable_values_.UpdatePrimalPhaseICosts(all_rows, &objective_);
    reduced_costs_.ResetForNewObjective();
  }
  while (true) {
    if (!refactorize && reduced_costs_.NeedsBasisRefactorization()) refactorize = true;
    if (!refactorize && primal_edge_norms_.NeedsBasisRefactorization()) refactorize = true;
    MILP_RETURN_IF_ERROR(RefactorizeBasisIfNeeded(&refactorize));
    if (basis_factorization_.IsRefactorized()) {
      CorrectErrorsOnVariableValues();
      if (phase_ == Phase::FEASIBILITY) {
        std::vector<int> all_rows(num_rows_);
        for (int r = 0; r < num_rows_; ++r) all_rows[r] = r;
        if (variable_values_.UpdatePrimalPhaseICosts(all_rows, &objective_)) {
          reduced_costs_.ResetForNewObjective();
        }
      }
      if (phase_ == Phase::OPTIMIZATION &&
          ComputeObjectiveValue() < primal_objective_limit_) {
        problem_status_ = ProblemStatus::PRIMAL_FEASIBLE;
        objective_limit_reached_ = true;
        return Status::OK();
      }
    } else if (phase_ == Phase::FEASIBILITY) {
      if (variable_values_.UpdatePrimalPhaseICosts(direction_.non_zeros, &objective_)) {
        reduced_costs_.ResetForNewObjective();
      }
    }

    if (sprimal_mode_ != 0) {
      Status sp_status;
      int sp;
      do {
        sp = RunSprimalSegment(time_limit, &refactorize, &sp_status);
      } while (sp == SdualBridge::kBody);
      if (sp == SdualBridge::kLoopTop) continue;
      if (sp == SdualBridge::kReturn) return sp_status;
    }
    clock.Mark(0);
    const int entering_col = primal_prices_.GetBestEnteringColumn();
    clock.Mark(1);
    if (entering_col == kInvalidCol) {
      if (reduced_costs_.AreReducedCostsPrecise() && basis_factorization_.IsRefactorized()) {
        if (phase_ == Phase::FEASIBILITY) {
          const Fractional primal_infeasibility =
              variable_values_.ComputeMaximumPrimalInfeasibility();
          if (primal_infeasibility < parameters_.primal_feasibility_tolerance) {
            problem_status_ = ProblemStatus::PRIMAL_FEASIBLE;
          } else {
            problem_status_ = ProblemStatus::PRIMAL_INFEASIBLE;
          }
        } else {
          problem_status_ = ProblemStatus::OPTIMAL;
        }
        break;
      }
      reduced_costs_.MakeReducedCostsPrecise();
      refactorize = true;
      continue;
    }

    ComputeDirection(entering_col);
    primal_edge_norms_.StartDirectionLeftInverse(direction_);
    if (!primal_edge_norms_.TestEnteringEdgeNormPrecision(entering_col, direction_)) {
      primal_prices_.RecomputePriceAt(entering_col);
      continue;
    }
    const Fractional reduced_cost =
        reduced_costs_.TestEnteringReducedCostPrecision(entering_col, direction_);
    primal_prices_.RecomputePriceAt(entering_col);
    if (!reduced_costs_.IsValidPrimalEnteringCandidate(entering_col)) {
      reduced_costs_.MakeReducedCostsPrecise();
      continue;
    }
    AdvanceDeterministicTime(time_limit);
    if (num_iterations_ == parameters_.max_number_of_iterations ||
        time_limit->LimitReached()) {
      break;
    }

    clock.Mark(2);
    Fractional step_length;
    int leaving_row;
    Fractional target_bound;
    if (phase_ == Phase::FEASIBILITY) {
      PrimalPhaseIChooseLeavingVariableRow(entering_col, reduced_cost, &refactorize,
                                           &leaving_row, &step_length, &target_bound);
    } else {
      MILP_RETURN_IF_ERROR(ChooseLeavingVariableRow(entering_col, reduced_cost,
                                                      &refactorize, &leaving_row,
                                                      &step_length, &target_bound));
    }
    clock.Mark(3);
    if (refactorize) continue;

    if (step_length == kInfinity || step_length == -kInfinity) {
      if (!basis_factorization_.IsRefactorized() ||
          !reduced_costs_.AreReducedCostsPrecise()) {
        reduced_costs_.MakeReducedCostsPrecise();
        refactorize = true;
        continue;
      }
      if (phase_ == Phase::FEASIBILITY) {
        problem_status_ = ProblemStatus::ABNORMAL;
      } else {
        problem_status_ = ProblemStatus::PRIMAL_UNBOUNDED;
        solution_primal_ray_.assign(num_cols_, 0.0);
        for (int row = 0; row < num_rows_; ++row) {
          solution_primal_ray_[basis_[row]] = -direction_[row];
        }
        solution_primal_ray_[entering_col] = 1.0;
        if (reduced_cost > 0.0) {
          for (auto& v : solution_primal_ray_) v = -v;
        }
      }
      break;
    }

    Fractional step = (reduced_cost > 0.0) ? -step_length : step_length;
    if (phase_ == Phase::FEASIBILITY && leaving_row != kInvalidRow) {
      step = ComputeStepToMoveBasicVariableToBound(leaving_row, target_bound);
    }
    trace_entering_ = entering_col;
    trace_leaving_row_ = leaving_row;
    trace_step_ = step;
    trace_reduced_cost_ = reduced_cost;
    const int leaving_col = (leaving_row == kInvalidRow) ? kInvalidCol : basis_[leaving_row];
    bool is_degenerate = false;
    if (leaving_row != kInvalidRow) {
      const Fractional dir = -direction_[leaving_row] * step;
      is_degenerate = (dir == 0.0) ||
                      (dir > 0.0 && variable_values_.Get(leaving_col) >= target_bound) ||
                      (dir < 0.0 && variable_values_.Get(leaving_col) <= target_bound);
    }
    variable_values_.UpdateOnPivoting(direction_, entering_col, step);
    clock.Mark(4);
    if (leaving_row != kInvalidRow) {
      primal_edge_norms_.UpdateBeforeBasisPivot(entering_col, basis_[leaving_row],
                                                leaving_row, direction_, &update_row_);
      clock.Mark(5);
      reduced_costs_.UpdateBeforeBasisPivot(entering_col, leaving_row, direction_,
                                            &update_row_);
      clock.Mark(6);
      primal_prices_.UpdateBeforeBasisPivot(entering_col, &update_row_);
      clock.Mark(7);
      if (!is_degenerate) variable_values_.Set(leaving_col, target_bound);
      MILP_RETURN_IF_ERROR(UpdateAndPivot(entering_col, leaving_row, target_bound));
      clock.Mark(8);
    } else {
      if (step > 0.0) {
        SetNonBasicVariableStatusAndDeriveValue(entering_col, VariableStatus::AT_UPPER_BOUND);
      } else if (step < 0.0) {
        SetNonBasicVariableStatusAndDeriveValue(entering_col, VariableStatus::AT_LOWER_BOUND);
      }
      primal_prices_.SetAndDebugCheckThatColumnIsDualFeasible(entering_col);
    }
    if (phase_ == Phase::FEASIBILITY && leaving_row != kInvalidRow) {
      variable_values_.SetNonBasicVariableValueFromStatus(leaving_col);
      reduced_costs_.SetNonBasicVariableCostToZero(leaving_col, &objective_[leaving_col]);
      primal_prices_.RecomputePriceAt(leaving_col);
    }
    OnIterationDone(time_limit);
    clock.Mark(9);
  }
  return Status::OK();
}

bool RevisedSimplex::DualDeviceEnabled() const {
  const char* e = std::getenv("MILP_DEVICE_DUAL");
  if (e != nullptr && std::strcmp(e, "off") == 0) return false;
  if (e != nullptr && std::strcmp(e, "force") == 0) return true;
  return num_cols_ >= 65536;
}

void RevisedSimplex::BeginDualDeviceMode() {
  std::vector<uint8_t> bits(num_cols_);
  std::vector<Fractional> bound_diff(num_cols_);
  for (int col = 0; col < num_cols_; ++col) {
    bits[col] = variables_info_.ColumnBits(col);
    bound_diff[col] = variables_info_.GetBoundDifference(col);
  }
  // The raw host values: if a recompute is pending it replaces them (on the
  // device) at the first read, exactly when Glop would recompute.
  device_.DualBegin(reduced_costs_.RawReducedCosts(), bits, bound_diff);
  reduced_costs_.EnterDeviceMode();
  update_row_.SetLazyFetch(true);
  device_.SetListMirror(false);
  status_log_.clear();
  variables_info_.SetChangeLog(&status_log_);
  dual_device_mode_ = true;
}

void RevisedSimplex::EndDualDeviceMode() {
  dual_device_mode_ = false;
  variables_info_.SetChangeLog(nullptr);
  status_log_.clear();
  update_row_.SetLazyFetch(false);
  device_.SetListMirror(true);
  // Bring the last update row to the host while the device list is intact
  // (later ListDots calls reuse the list-value buffer).
  update_row_.GetNonZeroPositions();
  reduced_costs_.LeaveDeviceMode();
}

void RevisedSimplex::FlushColumnBits() {
  if (status_log_.empty()) return;
  std::sort(status_log_.begin(), status_log_.end());
  status_log_.erase(std::unique(status_log_.begin(), status_log_.end()), status_log_.end());
  flush_cols_.assign(status_log_.begin(), status_log_.end());
  flush_bits_.resize(flush_cols_.size());
  for (size_t i = 0; i < flush_cols_.size(); ++i) {
    flush_bits_[i] = variables_info_.ColumnBits(flush_cols_[i]);
  }
  status_log_.clear();
  device_.DualSetColBits(flush_cols_, flush_bits_);
}

// revised_simplex.cc:2391-2437. The per-column decisions do not depend on
// each other, so they are taken in one device pass and applied in order.
// Speculative flip FTRAN (VariableValues::SpecFlipBegin): the flips the
// next iteration's MakeBoxedVariableDualFeasible(bound_flip_candidates_)
// (revised_simplex.cc:2391-2437) is expected to make, predicted from the
// candidates' reduced costs after this pivot's update (reduced_costs.cc:
// 444-488, with the update row's entering coefficient for the pivot). A
// wrong prediction costs the speculative solve only: the next iteration
// uses it only for exactly the flips and value changes it makes.
void RevisedSimplex::SpeculateFlips(int entering_col, int leaving_row, Fractional entering_coeff,
                                    Fractional entering_rc) {
  const DeviceLp::DualCandidates& cand = entering_variable_.LastDeviceCandidates();
  const int n = static_cast<int>(cand.col.size());
  spec_pos_.resize(variables_info_.GetStatusRow().size(), -1);
  for (int k = 0; k < n; ++k) spec_pos_[cand.col[k]] = k;
  const Fractional threshold = reduced_costs_.GetDualFeasibilityTolerance();
  const Fractional step = entering_rc == 0.0 ? 0.0 : entering_rc / -entering_coeff;
  const std::vector<VariableStatus>& status = variables_info_.GetStatusRow();
  const std::vector<Fractional>& lb = variables_info_.GetVariableLowerBounds();
  const std::vector<Fractional>& ub = variables_info_.GetVariableUpperBounds();
  spec_cols_.clear();
  spec_deltas_.clear();
  for (const int col : bound_flip_candidates_) {
    const int k = spec_pos_[col];
    if (col == entering_col || k < 0) continue;
    const Fractional rc = cand.rc[k] + step * cand.coeff[k];
    if (rc > threshold && status[col] == VariableStatus::AT_UPPER_BOUND) {
      spec_cols_.push_back(col);
      spec_deltas_.push_back(lb[col] - variable_values_.Get(col));
    } else if (rc < -threshold && status[col] == VariableStatus::AT_LOWER_BOUND) {
      spec_cols_.push_back(col);
      spec_deltas_.push_back(ub[col] - variable_values_.Get(col));
    }
  }
  for (int k = 0; k < n; ++k) spec_pos_[cand.col[k]] = -1;
  if (spec_cols_.empty()) return;
  variable_values_.SpecFlipBegin(spec_cols_, spec_deltas_, entering_col, leaving_row);
}

void RevisedSimplex::MakeBoxedVariableDualFeasibleOnDevice(const std::vector<int>* cols,
                                                           bool update_basic_values) {
  std::vector<int> changed_cols;
  const Fractional threshold = reduced_costs_.GetDualFeasibilityTolerance();
  reduced_costs_.PrepareForDeviceUse();  // GetReducedCosts() side effects
  {
    SubTimer timer(kSubBoxedScan);
    FlushColumnBits();
    device_.DualBoxedFlips(cols, threshold, &flip_flags_);
    const std::vector<VariableStatus>& variable_status = variables_info_.GetStatusRow();
    const int n = static_cast<int>(flip_flags_.size());
    for (int i = 0; i < n; ++i) {
      if (!flip_flags_[i]) continue;
      const int col = cols != nullptr ? (*cols)[i] : i;
      if (variable_status[col] == VariableStatus::AT_UPPER_BOUND) {
        variables_info_.UpdateToNonBasicStatus(col, VariableStatus::AT_LOWER_BOUND);
      } else {
        variables_info_.UpdateToNonBasicStatus(col, VariableStatus::AT_UPPER_BOUND);
      }
      changed_cols.push_back(col);
    }
  }
  if (!changed_cols.empty()) {
    SubTimer flip_timer(kSubFlipFtran);
    variable_values_.UpdateGivenNonBasicVariables(changed_cols, update_basic_values);
  }
}

// revised_simplex.cc:3058-3367
Status RevisedSimplex::DualMinimize(bool feasibility_phase, TimeLimit* time_limit) {
  struct Cleanup {
    std::function<void()> f;
    ~Cleanup() { f(); }
  } cleanup{[this, time_limit]() { AdvanceDeterministicTime(time_limit); }};
  PhaseClock clock(/*dual=*/true);
  const int64_t first_iteration = num_iterations_;
  struct DumpAtExit {
    PhaseClock* c;
    const int64_t* it;
    int64_t first;
    ~DumpAtExit() { c->Dump(static_cast<long long>(*it - first)); }
  } dump{&clock, &num_iterations_, first_iteration};
  const bool device_mode = !feasibility_phase && DualDeviceEnabled();
  if (device_mode) BeginDualDeviceMode();
  struct EndDeviceMode {
    RevisedSimplex* s;
    bool on;
    ~EndDeviceMode() {
      if (!on) return;
      try {
        s->EndDualDeviceMode();
      } catch (const DeviceError&) {
        // The device failed; the next device call reports it.
      }
    }
  } end_device_mode{this, device_mode};
  // A speculative flip FTRAN still pending when the loop leaves is dropped
  // (its device solve waited for).
  struct DropSpec {
    VariableValues* v;
    ~DropSpec() {
      try {
        v->SpecFlipDone();
      } catch (const DeviceError&) {
      }
    }
  } drop_spec{&variable_values_};
  const bool spec_flip = device_mode && device_.SpecFlipEnabled() &&
                         parameters_.use_middle_product_form_update;
  bool refactorize = false;
  bound_flip_candidates_.clear();
  int leaving_row;
  Fractional cost_variation;
  Fractional target_bound;
  int entering_col;
  while (true) {
    const bool old_refactorize_value = refactorize;
    if (!refactorize && reduced_costs_.NeedsBasisRefactorization()) refactorize = true;
    if (!refactorize && dual_edge_norms_.NeedsBasisRefactorization()) refactorize = true;
    MILP_RETURN_IF_ERROR(RefactorizeBasisIfNeeded(&refactorize));
    if (basis_factorization_.IsRefactorized()) {
      if (feasibility_phase || old_refactorize_value) {
        reduced_costs_.MakeReducedCostsPrecise();
      }
      if (!feasibility_phase) {
        if (dual_device_mode_) {
          MakeBoxedVariableDualFeasibleOnDevice(nullptr, false);
        } else {
          MakeBoxedVariableDualFeasible(
              variables_info_.GetNonBasicBoxedVariables().ToVector(), false);
        }
        variable_values_.RecomputeBasicVariableValues();
        variable_values_.RecomputeDualPrices(parameters_.dual_price_prioritize_norm);
        if (phase_ == Phase::OPTIMIZATION && dual_objective_limit_ != kInfinity &&
            ComputeObjectiveValue() > dual_objective_limit_) {
          problem_status_ = ProblemStatus::DUAL_FEASIBLE;
          objective_limit_reached_ = true;
          return Status::OK();
        }
      }
    } else {
      if (!feasibility_phase) {
        if (dual_device_mode_) {
          MakeBoxedVariableDualFeasibleOnDevice(&bound_flip_candidates_, true);
        } else {
          MakeBoxedVariableDualFeasible(bound_flip_candidates_, true);
        }
        bound_flip_candidates_.clear();
        variable_values_.UpdateDualPrices(direction_.non_zeros);
      }
    }
    variable_values_.SpecFlipDone();  // a speculation the flips did not use
    clock.Mark(0);

    // Phase II, or dual phase I (sd_run's dual_phase1). A warm start's phase
    // I begins with the reduced costs to recompute, which keeps its first
    // leaving choice on the host (SdualBridge::Supported).
    if (sdual_mode_ != 0) {
      Status sd_status;
      int sd;
      do {
        sd = RunSdualSegment(time_limit, &refactorize, &sd_status);
      } while (sd == SdualBridge::kBody);
      if (sd == SdualBridge::kLoopTop) continue;
      if (sd == SdualBridge::kReturn) return sd_status;
    }
    if (feasibility_phase) {
      MILP_RETURN_IF_ERROR(
          DualPhaseIChooseLeavingVariableRow(&leaving_row, &cost_variation, &target_bound));
    } else {
      MILP_RETURN_IF_ERROR(
          DualChooseLeavingVariableRow(&leaving_row, &cost_variation, &target_bound));
    }
    clock.Mark(1);
    if (leaving_row == kInvalidRow) {
      if (!basis_factorization_.IsRefactorized() || reduced_costs_.HasCostShift()) {
        reduced_costs_.ClearAndRemoveCostShifts();
        refactorize = true;
        continue;
      }
      if (feasibility_phase) {
        problem_status_ = num_dual_infeasible_positions_ == 0
                              ? ProblemStatus::DUAL_FEASIBLE
                              : ProblemStatus::DUAL_INFEASIBLE;
      } else {
        problem_status_ = ProblemStatus::OPTIMAL;
      }
      return Status::OK();
    }

    update_row_.ComputeUnitRowLeftInverse(leaving_row);
    clock.Mark(2);
    if (!dual_edge_norms_.TestPrecision(leaving_row, update_row_.GetUnitRowLeftInverse())) {
      if (feasibility_phase) {
        const Fractional price = dual_pricing_vector_[leaving_row];
        const std::vector<Fractional>& sn = dual_edge_norms_.GetEdgeSquaredNorms();
        dual_prices_.AddOrUpdate(leaving_row, Square(price) / sn[leaving_row]);
      } else {
        variable_values_.UpdateDualPrices({leaving_row});
      }
      continue;
    }
    // tau = B^-1 rho needs only rho: it is computed on the factorization's
    // worker thread while the update row, ratio test and direction run.
    // Small bases compute it on this thread while the GPU computes the update
    // row (launched first, fetched after).
    const bool tau_inline = dual_edge_norms_.WillComputeTau() && !dual_device_mode_ &&
                            basis_factorization_.InlineTauEnabled();
    if (dual_edge_norms_.WillComputeTau() && !tau_inline) {
      basis_factorization_.StartAsyncTau(update_row_.GetUnitRowLeftInverse());
    }
    if (tau_inline) update_row_.SetLazyFetch(true);
    update_row_.ComputeUpdateRow(leaving_row);
    if (tau_inline) {
      basis_factorization_.ComputeTauNow(update_row_.GetUnitRowLeftInverse());
      update_row_.SetLazyFetch(false);
    }
    if (!dual_device_mode_) update_row_.GetNonZeroPositions();  // timed as the update row
    clock.Mark(3);

    if (feasibility_phase) {
      MILP_RETURN_IF_ERROR(entering_variable_.DualPhaseIChooseEnteringColumn(
          reduced_costs_.AreReducedCostsPrecise(), update_row_, cost_variation,
          &entering_col));
    } else if (dual_device_mode_) {
      const bool nothing_to_recompute = reduced_costs_.AreReducedCostsPrecise();
      SubTimer prep_timer(kSubRatioPrep);
      update_row_.MaterializeOnDevice();
      reduced_costs_.PrepareForDeviceUse();  // GetReducedCosts() side effects
      FlushColumnBits();
      prep_timer.Stop();
      Fractional coeff = 0.0;
      Fractional rc = 0.0;
      MILP_RETURN_IF_ERROR(entering_variable_.DualChooseEnteringColumnDevice(
          nothing_to_recompute, &device_, cost_variation, &bound_flip_candidates_,
          &entering_col, &coeff, &rc));
      if (entering_col != kInvalidCol) {
        update_row_.SetKnownCoefficient(entering_col, coeff);
        reduced_costs_.SetKnownReducedCost(entering_col, rc);
        if (spec_flip && !bound_flip_candidates_.empty()) {
          SubTimer spec_timer(kSubSpecBegin);
          SpeculateFlips(entering_col, leaving_row, coeff, rc);
        }
      }
    } else {
      MILP_RETURN_IF_ERROR(entering_variable_.DualChooseEnteringColumn(
          reduced_costs_.AreReducedCostsPrecise(), update_row_, cost_variation,
          &bound_flip_candidates_, &entering_col));
    }
    clock.Mark(4);

    if (entering_col == kInvalidCol) {
      if (!reduced_costs_.AreReducedCostsPrecise()) {
        refactorize = true;
        continue;
      }
      if (feasibility_phase) {
        problem_status_ = ProblemStatus::ABNORMAL;
      } else {
        problem_status_ = ProblemStatus::DUAL_UNBOUNDED;
        solution_dual_ray_ = update_row_.GetUnitRowLeftInverse().values;
        update_row_.ComputeFullUpdateRow(leaving_row, &solution_dual_ray_row_combination_);
        if (cost_variation < 0) {
          for (auto& v : solution_dual_ray_) v = -v;
          for (auto& v : solution_dual_ray_row_combination_) v = -v;
        }
      }
      return Status::OK();
    }

    const Fractional entering_coeff = update_row_.GetCoefficient(entering_col);
    if (std::fabs(entering_coeff) < parameters_.dual_small_pivot_threshold &&
        !reduced_costs_.AreReducedCostsPrecise()) {
      refactorize = true;
      continue;
    }
    ComputeDirection(entering_col);
    clock.Mark(5);
    if (std::fabs(direction_[leaving_row]) <
        parameters_.small_pivot_threshold * direction_infinity_norm_) {
      if (!reduced_costs_.AreReducedCostsPrecise()) {
        refactorize = true;
        continue;
      }
    }
    AdvanceDeterministicTime(time_limit);
    if (num_iterations_ == parameters_.max_number_of_iterations ||
        time_limit->LimitReached()) {
      return Status::OK();
    }
    const bool increasing_rc_is_needed = (cost_variation > 0.0) == (entering_coeff > 0.0);
    reduced_costs_.ShiftCostIfNeeded(increasing_rc_is_needed, entering_col);
    reduced_costs_.UpdateBeforeBasisPivot(entering_col, leaving_row, direction_,
                                          &update_row_);
    if (dual_device_mode_ && !bound_flip_candidates_.empty()) {
      // The next loop top's MakeBoxedVariableDualFeasible decisions, from the
      // reduced costs just updated (taken there if nothing changed them).
      device_.DualBoxedFlipsEarly(bound_flip_candidates_,
                                  reduced_costs_.GetDualFeasibilityTolerance());
    }
    clock.Mark(6);
    dual_edge_norms_.UpdateBeforeBasisPivot(entering_col, leaving_row, direction_,
                                            update_row_.GetUnitRowLeftInverse());
    clock.Mark(7);
    Fractional primal_step = 0.0;
    if (feasibility_phase) {
      DualPhaseIUpdatePrice(leaving_row, entering_col);
    } else {
      primal_step = ComputeStepToMoveBasicVariableToBound(leaving_row, target_bound);
      variable_values_.UpdateOnPivoting(direction_, entering_col, primal_step);
    }
    const int leaving_col = basis_[leaving_row];
    MILP_RETURN_IF_ERROR(UpdateAndPivot(entering_col, leaving_row, target_bound));
    variable_values_.SetNonBasicVariableValueFromStatus(leaving_col);
    clock.Mark(8);
    OnIterationDone(time_limit);
    clock.Mark(9);
    clock.Tick();
  }
  return Status::OK();
}

// revised_simplex.cc:2588-2593
void RevisedSimplex::SetIntegralityScale(int col, Fractional scale) {
  if (col >= static_cast<int>(integrality_scale_.size())) {
    integrality_scale_.resize(col + 1, 0.0);
  }
  integrality_scale_[col] = scale;
}

// revised_simplex.cc:2595-2734: after an optimal solve with integrality
// scales set, up to 5 degenerate pivots among zero-reduced-cost columns that
// make the basic solution less fractional.
Status RevisedSimplex::Polish(TimeLimit* time_limit) {
  struct Cleanup {
    std::function<void()> f;
    ~Cleanup() { f(); }
  } cleanup{[this, time_limit]() { AdvanceDeterministicTime(time_limit); }};
  const std::vector<Fractional>& rc = reduced_costs_.GetReducedCosts();
  std::vector<int> candidates;
  variables_info_.GetNotBasicBitRow().ForEach([&](int col) {
    if (!variables_info_.GetIsRelevantBitRow()[col]) return;
    if (std::fabs(rc[col]) < 1e-9) candidates.push_back(col);
  });
  bool refactorize = false;
  int num_pivots = 0;
  for (int i = 0; i < 10; ++i) {
    AdvanceDeterministicTime(time_limit);
    if (time_limit->LimitReached()) break;
    if (num_pivots >= 5) break;
    if (candidates.empty()) break;
    const int index = UniformInt(random_, static_cast<int>(candidates.size()) - 1);
    const int entering_col = candidates[index];
    std::swap(candidates[index], candidates.back());
    candidates.pop_back();
    // The entering variable must move in a feasible direction.
    Fractional fake_rc = 1.0;
    if (!variables_info_.GetCanDecreaseBitRow()[entering_col]) fake_rc = -1.0;
    if (reduced_costs_.NeedsBasisRefactorization()) refactorize = true;
    MILP_RETURN_IF_ERROR(RefactorizeBasisIfNeeded(&refactorize));
    ComputeDirection(entering_col);
    Fractional step_length;
    int leaving_row;
    Fractional target_bound;
    bool local_refactorize = false;
    MILP_RETURN_IF_ERROR(ChooseLeavingVariableRow(entering_col, fake_rc, &local_refactorize,
                                             &leaving_row, &step_length, &target_bound));
    if (local_refactorize) continue;
    if (step_length == kInfinity || step_length == -kInfinity) continue;
    if (std::fabs(step_length) <= 1e-6) continue;
    if (leaving_row != kInvalidRow && std::fabs(direction_[leaving_row]) < 0.1) continue;
    const Fractional step = (fake_rc > 0.0) ? -step_length : step_length;
    // Change of the total fractionality if the pivot is made.
    const auto get_diff = [this](int col, Fractional old_value, Fractional new_value) {
      if (col >= static_cast<int>(integrality_scale_.size()) ||
          integrality_scale_[col] == 0.0) {
        return 0.0;
      }
      const Fractional s = integrality_scale_[col];
      return (std::fabs(new_value * s - std::round(new_value * s)) -
              std::fabs(old_value * s - std::round(old_value * s)));
    };
    Fractional diff = get_diff(entering_col, variable_values_.Get(entering_col),
                               variable_values_.Get(entering_col) + step);
    for (const int row : direction_.non_zeros) {
      const int col = basis_[row];
      const Fractional old_value = variable_values_.Get(col);
      const Fractional new_value = old_value - direction_[row] * step;
      diff += get_diff(col, old_value, new_value);
    }
    if (diff > -1e-2) continue;
    num_pivots++;
    variable_values_.UpdateOnPivoting(direction_, entering_col, step);
    if (leaving_row == kInvalidRow) {  // a bound flip of the entering column
      if (step > 0.0) {
        SetNonBasicVariableStatusAndDeriveValue(entering_col, VariableStatus::AT_UPPER_BOUND);
      } else if (step < 0.0) {
        SetNonBasicVariableStatusAndDeriveValue(entering_col, VariableStatus::AT_LOWER_BOUND);
      }
      continue;
    }
    const int leaving_col = basis_[leaving_row];
    update_row_.ComputeUpdateRow(leaving_row);
    primal_edge_norms_.UpdateBeforeBasisPivot(entering_col, leaving_col, leaving_row,
                                              direction_, &update_row_);
    dual_edge_norms_.UpdateBeforeBasisPivot(entering_col, leaving_row, direction_,
                                            update_row_.GetUnitRowLeftInverse());
    reduced_costs_.UpdateBeforeBasisPivot(entering_col, leaving_row, direction_, &update_row_);
    const Fractional dir = -direction_[leaving_row] * step;
    const bool is_degenerate =
        (dir == 0.0) ||
        (dir > 0.0 && variable_values_.Get(leaving_col) >= target_bound) ||
        (dir < 0.0 && variable_values_.Get(leaving_col) <= target_bound);
    if (!is_degenerate) variable_values_.Set(leaving_col, target_bound);
    MILP_RETURN_IF_ERROR(UpdateAndPivot(entering_col, leaving_row, target_bound));
  }
  return Status::OK();
}

void RevisedSimplex::ComputeDictionary(const std::vector<Fractional>* column_scales,
                                       std::vector<std::vector<std::pair<int, Fractional>>>* rows) {
  rows->assign(num_rows_, {});
  for (int col = 0; col < num_cols_; ++col) {
    ComputeDirection(col);
    for (const int row : direction_.non_zeros) {
      if (column_scales == nullptr) {
        (*rows)[row].emplace_back(col, direction_[row]);
        continue;
      }
      const Fractional numerator =
          col < static_cast<int>(column_scales->size()) ? (*column_scales)[col] : 1.0;
      const Fractional denominator =
          basis_[row] < static_cast<int>(column_scales->size()) ? (*column_scales)[basis_[row]]
                                                                : 1.0;
      (*rows)[row].emplace_back(col, direction_[row] * (numerator / denominator));
    }
  }
}

// revised_simplex.cc:3369-3543
Status RevisedSimplex::PrimalPush(TimeLimit* time_limit) {
  bool refactorize = false;
  primal_edge_norms_.Clear();
  dual_edge_norms_.Clear();
  update_row_.Invalidate();
  reduced_costs_.ClearAndRemoveCostShifts();
  std::vector<int> super_basic_cols;
  variables_info_.GetNotBasicBitRow().ForEach([&](int col) {
    if (variables_info_.GetStatusRow()[col] == VariableStatus::FREE &&
        variable_values_.Get(col) != 0)
      super_basic_cols.push_back(col);
  });
  while (!super_basic_cols.empty()) {
    AdvanceDeterministicTime(time_limit);
    if (time_limit->LimitReached()) break;
    MILP_RETURN_IF_ERROR(RefactorizeBasisIfNeeded(&refactorize));
    if (basis_factorization_.IsRefactorized()) CorrectErrorsOnVariableValues();
    const int entering_col = super_basic_cols.back();
    Fractional fake_rc;
    const Fractional entering_value = variable_values_.Get(entering_col);
    if (variables_info_.GetTypeRow()[entering_col] == VariableType::UNCONSTRAINED) {
      fake_rc = entering_value > 0 ? 1.0 : -1.0;
    } else {
      const Fractional diff_ub =
          variables_info_.GetVariableUpperBounds()[entering_col] - entering_value;
      const Fractional diff_lb =
          entering_value - variables_info_.GetVariableLowerBounds()[entering_col];
      fake_rc = diff_lb <= diff_ub ? 1.0 : -1.0;
    }
    ComputeDirection(entering_col);
    Fractional step_length;
    int leaving_row;
    Fractional target_bound;
    MILP_RETURN_IF_ERROR(ChooseLeavingVariableRow(entering_col, fake_rc, &refactorize,
                                                    &leaving_row, &step_length,
                                                    &target_bound));
    if (refactorize) continue;
    super_basic_cols.pop_back();
    if (step_length == kInfinity || step_length == -kInfinity) {
      if (variables_info_.GetTypeRow()[entering_col] == VariableType::UNCONSTRAINED) {
        step_length = std::fabs(entering_value);
      } else {
        problem_status_ = ProblemStatus::ABNORMAL;
        break;
      }
    }
    const Fractional step = (fake_rc > 0.0) ? -step_length : step_length;
    const int leaving_col = (leaving_row == kInvalidRow) ? kInvalidCol : basis_[leaving_row];
    bool is_degenerate = false;
    if (leaving_row != kInvalidRow) {
      const Fractional dir = -direction_[leaving_row] * step;
      is_degenerate = (dir == 0.0) ||
                      (dir > 0.0 && variable_values_.Get(leaving_col) >= target_bound) ||
                      (dir < 0.0 && variable_values_.Get(leaving_col) <= target_bound);
    }
    variable_values_.UpdateOnPivoting(direction_, entering_col, step);
    if (leaving_row != kInvalidRow) {
      if (!is_degenerate) variable_values_.Set(leaving_col, target_bound);
      MILP_RETURN_IF_ERROR(UpdateAndPivot(entering_col, leaving_row, target_bound));
    } else {
      if (variables_info_.GetTypeRow()[entering_col] == VariableType::UNCONSTRAINED) {
        variable_values_.Set(entering_col, 0.0);
      } else if (step > 0.0) {
        SetNonBasicVariableStatusAndDeriveValue(entering_col, VariableStatus::AT_UPPER_BOUND);
      } else if (step < 0.0) {
        SetNonBasicVariableStatusAndDeriveValue(entering_col, VariableStatus::AT_LOWER_BOUND);
      }
    }
    OnIterationDone(time_limit);
  }
  return Status::OK();
}

}  // namespace milp


// ===========================================================================
// C ABI (include/mi_lp.h).
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <thread>

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>

#include <hip/hip_runtime_api.h>

struct mi_lp {
  milp::RevisedSimplex simplex;
  std::vector<std::vector<std::pair<int, double>>> dictionary;  // mi_lp_compute_dictionary
  milp::GlopParameters params;
  milp::LinearProgram lp;
  int device = 0;
  bool loaded = false;
  bool solved = false;
  std::string error;
  // benchmark slicing (mi_lp_begin / mi_lp_run_until / mi_lp_finish)
  std::thread worker;
  std::mutex mu;
  std::condition_variable cv;
  int64_t pause_at = -1;
  int64_t current_iteration = 0;
  bool paused = false;
  bool finished = false;
  bool running = false;
  volatile int32_t stop = 0;  // mi_lp_stop: interrupts like a time limit
  mi_lp_result pending{};
};

namespace {

milp::GlopParameters FromAbi(const mi_glop_params& p) {
  milp::GlopParameters g;
  g.use_dual_simplex = p.use_dual_simplex;
  g.feasibility_rule = p.feasibility_rule;
  g.optimization_rule = p.optimization_rule;
  g.initial_basis = p.initial_basis;
  g.use_transposed_matrix = p.use_transposed_matrix;
  g.basis_refactorization_period = p.basis_refactorization_period;
  g.dynamically_adjust_refactorization_period = p.dynamically_adjust_refactorization_period;
  g.change_status_to_imprecise = p.change_status_to_imprecise;
  g.markowitz_zlatev_parameter = p.markowitz_zlatev_parameter;
  g.allow_simplex_algorithm_change = p.allow_simplex_algorithm_change;
  g.devex_weights_reset_period = p.devex_weights_reset_period;
  g.use_middle_product_form_update = p.use_middle_product_form_update;
  g.initialize_devex_with_column_norms = p.initialize_devex_with_column_norms;
  g.exploit_singleton_column_in_initial_basis = p.exploit_singleton_column_in_initial_basis;
  g.random_seed = p.random_seed;
  g.perturb_costs_in_dual_simplex = p.perturb_costs_in_dual_simplex;
  g.use_dedicated_dual_feasibility_algorithm = p.use_dedicated_dual_feasibility_algorithm;
  g.push_to_vertex = p.push_to_vertex;
  g.dual_price_prioritize_norm = p.dual_price_prioritize_norm;
  g.use_scaling = p.use_scaling;
  g.max_number_of_iterations = p.max_number_of_iterations;
  g.refactorization_threshold = p.refactorization_threshold;
  g.recompute_reduced_costs_threshold = p.recompute_reduced_costs_threshold;
  g.recompute_edges_norm_threshold = p.recompute_edges_norm_threshold;
  g.primal_feasibility_tolerance = p.primal_feasibility_tolerance;
  g.dual_feasibility_tolerance = p.dual_feasibility_tolerance;
  g.ratio_test_zero_threshold = p.ratio_test_zero_threshold;
  g.harris_tolerance_ratio = p.harris_tolerance_ratio;
  g.small_pivot_threshold = p.small_pivot_threshold;
  g.minimum_acceptable_pivot = p.minimum_acceptable_pivot;
  g.drop_tolerance = p.drop_tolerance;
  g.solution_feasibility_tolerance = p.solution_feasibility_tolerance;
  g.max_number_of_reoptimizations = p.max_number_of_reoptimizations;
  g.lu_factorization_pivot_threshold = p.lu_factorization_pivot_threshold;
  g.max_time_in_seconds = p.max_time_in_seconds;
  g.max_deterministic_time = p.max_deterministic_time;
  g.markowitz_singularity_threshold = p.markowitz_singularity_threshold;
  g.dual_small_pivot_threshold = p.dual_small_pivot_threshold;
  g.objective_lower_limit = p.objective_lower_limit;
  g.objective_upper_limit = p.objective_upper_limit;
  g.degenerate_ministep_factor = p.degenerate_ministep_factor;
  g.relative_cost_perturbation = p.relative_cost_perturbation;
  g.relative_max_cost_perturbation = p.relative_max_cost_perturbation;
  g.initial_condition_number_threshold = p.initial_condition_number_threshold;
  g.crossover_bound_snapping_distance = p.crossover_bound_snapping_distance;
  return g;
}

// LPSolver's validity checks (lp_solver.cc:185-202, LinearProgram::IsValid).
bool ValidLp(const milp::LinearProgram& lp) {
  if (lp.m < 0 || lp.n < 0 || lp.col_starts.size() != static_cast<size_t>(lp.n) + 1)
    return false;
  if (lp.col_starts[0] != 0) return false;
  for (int c = 0; c < lp.n; ++c) {
    if (lp.col_starts[c + 1] < lp.col_starts[c]) return false;
    for (int64_t k = lp.col_starts[c]; k < lp.col_starts[c + 1]; ++k) {
      const int r = lp.row_idx[k];
      if (r < 0 || r >= lp.m) return false;
      if (k > lp.col_starts[c] && r <= lp.row_idx[k - 1]) return false;
      if (!(lp.vals[k] != 0.0) || !milp::IsFinite(lp.vals[k])) return false;
    }
  }
  auto bad_bounds = [](const std::vector<double>& lo, const std::vector<double>& hi) {
    for (size_t i = 0; i < lo.size(); ++i) {
      if (!(lo[i] <= hi[i]) || lo[i] == milp::kInfinity || hi[i] == -milp::kInfinity)
        return true;
    }
    return false;
  };
  if (bad_bounds(lp.col_lb, lp.col_ub) || bad_bounds(lp.row_lb, lp.row_ub)) return false;
  for (const double c : lp.obj)
    if (!milp::IsFinite(c)) return false;
  return milp::IsFinite(lp.obj_offset) && milp::IsFinite(lp.obj_scale) && lp.obj_scale != 0.0;
}

void RunSolve(mi_lp* h, const volatile int32_t* interrupt, mi_lp_result* out) {
  std::memset(out, 0, sizeof(*out));
  h->error.clear();
  if (!h->loaded) {
    out->error_code = MI_LP_ERROR_STATE;
    out->problem_status = MI_LP_INIT;
    h->error = "mi_lp_solve before mi_lp_load";
    return;
  }
  if (!ValidLp(h->lp)) {  // lp_solver.cc:185-202 -> INVALID_PROBLEM
    out->problem_status = MI_LP_INVALID_PROBLEM;
    out->error_code = MI_LP_OK;
    h->solved = false;
    return;
  }
  try {
    (void)hipSetDevice(h->device);
    h->simplex.SetParameters(h->params);
    milp::TimeLimit tl;
    tl.max_seconds = h->params.max_time_in_seconds;
    tl.max_deterministic = h->params.max_deterministic_time;
    tl.interrupt = interrupt;
    const milp::Status s = h->simplex.Solve(h->lp, &tl);
    h->simplex.device().Synchronize();
    out->error_code = static_cast<int32_t>(s.code);
    out->problem_status = s.ok() ? static_cast<int32_t>(h->simplex.GetProblemStatus())
                                 : MI_LP_ABNORMAL;  // lp_solver.cc:654-657
    out->iterations = h->simplex.GetNumberOfIterations();
    out->objective = h->simplex.GetObjectiveValue();
    out->deterministic_time = h->simplex.DeterministicTime();
    out->solve_seconds = tl.GetElapsedTime();
    if (!s.ok()) h->error = s.msg;
    h->solved = true;
  } catch (const milp::DeviceError& e) {
    h->error = e.what();
    out->error_code = MI_LP_ERROR_DEVICE;
    out->problem_status = MI_LP_ABNORMAL;
    h->solved = false;
  } catch (const std::exception& e) {
    // Nothing may unwind through extern "C" or out of a batch worker thread.
    h->error = std::string("engine exception: ") + e.what();
    out->error_code = MI_LP_ERROR_INTERNAL;
    out->problem_status = MI_LP_ABNORMAL;
    h->solved = false;
  } catch (...) {
    h->error = "engine exception";
    out->error_code = MI_LP_ERROR_INTERNAL;
    out->problem_status = MI_LP_ABNORMAL;
    h->solved = false;
  }
}

// A batch entry whose setup failed: reported like a failed solve, the other
// entries of the batch are unaffected.
void FailEntry(mi_lp* h, int code, const char* what, mi_lp_result* out) {
  std::memset(out, 0, sizeof(*out));
  out->error_code = code;
  out->problem_status = MI_LP_ABNORMAL;
  h->error = what;
  h->solved = false;
}

int LoadLp(mi_lp* h, int32_t m, int32_t n, const int64_t* cs, const int32_t* ri,
           const double* vals, const double* clb, const double* cub, const double* rlb,
           const double* rub, const double* obj, double obj_offset, double obj_scale,
           int32_t maximize);

}  // namespace

extern "C" {

void mi_glop_params_default(mi_glop_params* p) {
  p->use_dual_simplex = 0;
  p->feasibility_rule = MI_LP_STEEPEST_EDGE;
  p->optimization_rule = MI_LP_STEEPEST_EDGE;
  p->initial_basis = MI_LP_BASIS_TRIANGULAR;
  p->use_transposed_matrix = 1;
  p->basis_refactorization_period = 64;
  p->dynamically_adjust_refactorization_period = 1;
  p->change_status_to_imprecise = 1;
  p->markowitz_zlatev_parameter = 3;
  p->allow_simplex_algorithm_change = 0;
  p->devex_weights_reset_period = 150;
  p->use_middle_product_form_update = 1;
  p->initialize_devex_with_column_norms = 1;
  p->exploit_singleton_column_in_initial_basis = 1;
  p->random_seed = 1;
  p->perturb_costs_in_dual_simplex = 0;
  p->use_dedicated_dual_feasibility_algorithm = 1;
  p->push_to_vertex = 1;
  p->dual_price_prioritize_norm = 0;
  p->use_scaling = 1;
  p->max_number_of_iterations = -1;
  p->refactorization_threshold = 1e-9;
  p->recompute_reduced_costs_threshold = 1e-8;
  p->recompute_edges_norm_threshold = 100.0;
  p->primal_feasibility_tolerance = 1e-8;
  p->dual_feasibility_tolerance = 1e-8;
  p->ratio_test_zero_threshold = 1e-9;
  p->harris_tolerance_ratio = 0.5;
  p->small_pivot_threshold = 1e-6;
  p->minimum_acceptable_pivot = 1e-6;
  p->drop_tolerance = 1e-14;
  p->solution_feasibility_tolerance = 1e-6;
  p->max_number_of_reoptimizations = 40;
  p->lu_factorization_pivot_threshold = 0.01;
  p->max_time_in_seconds = milp::kInfinity;
  p->max_deterministic_time = milp::kInfinity;
  p->markowitz_singularity_threshold = 1e-15;
  p->dual_small_pivot_threshold = 1e-4;
  p->objective_lower_limit = -milp::kInfinity;
  p->objective_upper_limit = milp::kInfinity;
  p->degenerate_ministep_factor = 0.01;
  p->relative_cost_perturbation = 1e-5;
  p->relative_max_cost_perturbation = 1e-7;
  p->initial_condition_number_threshold = 1e50;
  p->crossover_bound_snapping_distance = milp::kInfinity;
}

// MILP_CRASH_REPORT=1: a SIGSEGV/SIGBUS/SIGABRT handler that prints each
// frame as library+offset (dladdr), so a crash inside another library's
// teardown can be attributed, then re-raises with the default action.
namespace {
void CrashReport(int sig, siginfo_t* info, void*) {
  void* frames[48];
  const int n = backtrace(frames, 48);
  std::fprintf(stderr, "[mi_lp crash report] signal %d, fault address %p, %d frames\n", sig,
               info != nullptr ? info->si_addr : nullptr, n);
  for (int i = 0; i < n; ++i) {
    Dl_info d{};
    if (dladdr(frames[i], &d) != 0 && d.dli_fname != nullptr) {
      std::fprintf(stderr, "  #%02d %p %s+0x%lx (%s)\n", i, frames[i], d.dli_fname,
                   static_cast<unsigned long>(reinterpret_cast<uintptr_t>(frames[i]) -
                                              reinterpret_cast<uintptr_t>(d.dli_fbase)),
                   d.dli_sname != nullptr ? d.dli_sname : "?");
    } else {
      std::fprintf(stderr, "  #%02d %p (no mapping)\n", i, frames[i]);
    }
  }
  std::fflush(stderr);
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) void InstallCrashReport() {
  const char* e = std::getenv("MILP_CRASH_REPORT");
  if (e == nullptr || std::atoi(e) == 0) return;
  struct sigaction sa {};
  sa.sa_sigaction = CrashReport;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
  sigemptyset(&sa.sa_mask);
  for (int sig : {SIGSEGV, SIGBUS, SIGABRT}) sigaction(sig, &sa, nullptr);
}
}  // namespace

int mi_lp_shutdown(void) {
  milp::ShutdownDevices();
  // MILP_DEVICE_RESET_AT_EXIT=1 (profiling runs only): release every HIP
  // resource of every device through the runtime, so that a profiler's own
  // exit-time teardown finds nothing left to release. Under rocprofv3 --pmc
  // a run that executed the device dual segments otherwise ends in a SIGSEGV
  // inside rocprofiler-sdk's static destructors (calling into HSA) after the
  // counters are written (scripts/pmc_teardown_probe.py bisects it: a torch
  // kernel, a single engine solve, a batch with MILP_SDUAL=off and a
  // scratch-using kernel all exit 0).
  if (const char* e = std::getenv("MILP_DEVICE_RESET_AT_EXIT")) {
    if (std::atoi(e) != 0) {
      int n = 0;
      if (hipGetDeviceCount(&n) == hipSuccess) {
        for (int d = 0; d < n; ++d) {
          if (hipSetDevice(d) == hipSuccess) {
            (void)hipDeviceSynchronize();
            (void)hipDeviceReset();
          }
        }
      }
    }
  }
  return MI_LP_OK;
}

int mi_lp_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int mi_lp_create(int device, mi_lp** out) {
  if (out == nullptr) return MI_LP_ERROR_NULL;
  *out = nullptr;
  mi_lp* h = new (std::nothrow) mi_lp();
  if (h == nullptr) return MI_LP_ERROR_INTERNAL;
  try {
    h->simplex.device().Init(device);
  } catch (const milp::DeviceError& e) {
    std::fprintf(stderr, "mi_lp_create: %s\n", e.what());
    delete h;
    return MI_LP_ERROR_DEVICE;
  }
  h->device = device;
  mi_glop_params p;
  mi_glop_params_default(&p);
  h->params = FromAbi(p);
  *out = h;
  return MI_LP_OK;
}

int mi_lp_destroy(mi_lp* h) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  if (h->worker.joinable()) {
    {
      std::lock_guard<std::mutex> l(h->mu);
      h->pause_at = -1;
    }
    h->cv.notify_all();
    h->worker.join();
  }
  delete h;
  return MI_LP_OK;
}

const char* mi_lp_last_error(const mi_lp* h) {
  return h == nullptr ? "null handle" : h->error.c_str();
}

int mi_lp_set_params(mi_lp* h, const mi_glop_params* p) {
  if (h == nullptr || p == nullptr) return MI_LP_ERROR_NULL;
  h->params = FromAbi(*p);
  return MI_LP_OK;
}

int mi_lp_load(mi_lp* h, int32_t m, int32_t n, const int64_t* cs, const int32_t* ri,
               const double* vals, const double* clb, const double* cub, const double* rlb,
               const double* rub, const double* obj, double obj_offset, double obj_scale,
               int32_t maximize) {
  if (h == nullptr || cs == nullptr) return MI_LP_ERROR_NULL;
  if (m < 0 || n < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  if (h->running) return MI_LP_ERROR_STATE;
  if (cs[n] > 0 && (ri == nullptr || vals == nullptr)) return MI_LP_ERROR_NULL;
  if ((n > 0 && (clb == nullptr || cub == nullptr || obj == nullptr)) ||
      (m > 0 && (rlb == nullptr || rub == nullptr))) {
    return MI_LP_ERROR_NULL;
  }
  try {
    return LoadLp(h, m, n, cs, ri, vals, clb, cub, rlb, rub, obj, obj_offset, obj_scale,
                  maximize);
  } catch (const std::exception& e) {
    h->loaded = false;
    h->solved = false;
    h->error = std::string("mi_lp_load: ") + e.what();
    return MI_LP_ERROR_INTERNAL;
  }
}

}  // extern "C"

namespace {
int LoadLp(mi_lp* h, int32_t m, int32_t n, const int64_t* cs, const int32_t* ri,
           const double* vals, const double* clb, const double* cub, const double* rlb,
           const double* rub, const double* obj, double obj_offset, double obj_scale,
           int32_t maximize) {
  milp::LinearProgram& lp = h->lp;
  lp.m = m;
  lp.n = n;
  lp.col_starts.assign(cs, cs + n + 1);
  const int64_t nnz = cs[n];
  if (nnz < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  lp.row_idx.assign(ri, ri + nnz);
  lp.vals.assign(vals, vals + nnz);
  lp.col_lb.assign(clb, clb + n);
  lp.col_ub.assign(cub, cub + n);
  lp.row_lb.assign(rlb, rlb + m);
  lp.row_ub.assign(rub, rub + m);
  lp.obj.assign(obj, obj + n);
  lp.obj_offset = obj_offset;
  lp.obj_scale = obj_scale;
  lp.maximize = maximize != 0;
  {
    // 64-bit multiply-xor over the matrix words (a few GB/s; once per load).
    uint64_t f = 0x243f6a8885a308d3ull ^ (static_cast<uint64_t>(m) << 32 | static_cast<uint32_t>(n));
    auto mix = [&f](uint64_t v) {
      f ^= v + 0x9e3779b97f4a7c15ull + (f << 6) + (f >> 2);
      f *= 0xff51afd7ed558ccdull;
    };
    for (const int64_t v : lp.col_starts) mix(static_cast<uint64_t>(v));
    for (int64_t k = 0; k < nnz; ++k) {
      uint64_t bits;
      std::memcpy(&bits, &lp.vals[k], 8);
      mix(bits ^ (static_cast<uint64_t>(static_cast<uint32_t>(lp.row_idx[k])) << 1));
    }
    lp.matrix_fingerprint = f;
  }
  h->loaded = true;
  h->solved = false;
  return MI_LP_OK;
}
// No begun solve, or one that is parked (paused or finished): its state may
// be read.
bool SolveIsParked(const mi_lp* h) {
  mi_lp* m = const_cast<mi_lp*>(h);
  std::lock_guard<std::mutex> l(m->mu);
  return !m->running || m->paused || m->finished;
}
}  // namespace

extern "C" {

int mi_lp_load_basis_state(mi_lp* h, const int8_t* st, int32_t len) {
  if (h == nullptr || (st == nullptr && len > 0)) return MI_LP_ERROR_NULL;
  if (len < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  try {
    std::vector<milp::VariableStatus> s(len);
    for (int i = 0; i < len; ++i) {
      if (st[i] < 0 || st[i] > 4) return MI_LP_ERROR_INVALID_PROBLEM;
      s[i] = static_cast<milp::VariableStatus>(st[i]);
    }
    h->simplex.LoadStateForNextSolve(s);
  } catch (const std::exception& e) {
    h->error = std::string("mi_lp_load_basis_state: ") + e.what();
    return MI_LP_ERROR_INTERNAL;
  }
  return MI_LP_OK;
}

int mi_lp_set_variable_bounds(mi_lp* h, const double* col_lb, const double* col_ub) {
  if (h == nullptr || col_lb == nullptr || col_ub == nullptr) return MI_LP_ERROR_NULL;
  if (!h->loaded) return MI_LP_ERROR_STATE;
  try {
    h->lp.col_lb.assign(col_lb, col_lb + h->lp.n);
    h->lp.col_ub.assign(col_ub, col_ub + h->lp.n);
  } catch (const std::exception& e) {
    h->error = std::string("mi_lp_set_variable_bounds: ") + e.what();
    return MI_LP_ERROR_INTERNAL;
  }
  return MI_LP_OK;
}

int mi_lp_clear_basis_state(mi_lp* h) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  h->simplex.ClearStateForNextSolve();
  return MI_LP_OK;
}

int mi_lp_notify_matrix_unchanged(mi_lp* h) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  h->simplex.NotifyThatMatrixIsUnchangedForNextSolve();
  return MI_LP_OK;
}

int mi_lp_notify_matrix_changed(mi_lp* h) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  h->simplex.NotifyThatMatrixIsChangedForNextSolve();
  return MI_LP_OK;
}

int mi_lp_set_starting_variable_values(mi_lp* h, const double* values, int32_t len) {
  if (h == nullptr || (values == nullptr && len > 0)) return MI_LP_ERROR_NULL;
  if (len < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  try {
    h->simplex.SetStartingVariableValuesForNextSolve(std::vector<double>(values, values + len));
  } catch (const std::exception& e) {
    h->error = e.what();
    return MI_LP_ERROR_INTERNAL;
  }
  return MI_LP_OK;
}

int mi_lp_set_integrality_scale(mi_lp* h, int32_t col, double scale) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  if (col < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  try {
    h->simplex.SetIntegralityScale(col, scale);
  } catch (const std::exception& e) {
    h->error = e.what();
    return MI_LP_ERROR_INTERNAL;
  }
  return MI_LP_OK;
}

int mi_lp_clear_integrality_scales(mi_lp* h) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  h->simplex.ClearIntegralityScales();
  return MI_LP_OK;
}

int mi_lp_objective_limit_reached(const mi_lp* h, int32_t* reached) {
  if (h == nullptr || reached == nullptr) return MI_LP_ERROR_NULL;
  *reached = h->simplex.objective_limit_reached() ? 1 : 0;
  return MI_LP_OK;
}

int mi_lp_get_unit_row_left_inverse(mi_lp* h, int32_t row, double* values, int32_t* non_zeros,
                                    int32_t* num_non_zeros) {
  if (h == nullptr || values == nullptr) return MI_LP_ERROR_NULL;
  if (!h->solved) return MI_LP_ERROR_STATE;
  if (row < 0 || row >= h->lp.m) return MI_LP_ERROR_INVALID_PROBLEM;
  try {
    (void)hipSetDevice(h->device);
    const milp::ScatteredVector& v = h->simplex.GetUnitRowLeftInverse(row);
    for (int r = 0; r < h->lp.m; ++r) values[r] = v.values[r];
    if (num_non_zeros != nullptr) *num_non_zeros = static_cast<int32_t>(v.non_zeros.size());
    if (non_zeros != nullptr) {
      for (size_t k = 0; k < v.non_zeros.size(); ++k) non_zeros[k] = v.non_zeros[k];
    }
  } catch (const milp::DeviceError& e) {
    h->error = e.what();
    return MI_LP_ERROR_DEVICE;
  } catch (const std::exception& e) {
    h->error = e.what();
    return MI_LP_ERROR_INTERNAL;
  }
  return MI_LP_OK;
}

int mi_lp_compute_dictionary(mi_lp* h, const double* column_scales, int32_t scales_len,
                             int64_t* nnz) {
  if (h == nullptr || nnz == nullptr || (column_scales == nullptr && scales_len > 0)) {
    return MI_LP_ERROR_NULL;
  }
  if (!h->solved) return MI_LP_ERROR_STATE;
  try {
    (void)hipSetDevice(h->device);
    std::vector<double> scales;
    if (column_scales != nullptr) scales.assign(column_scales, column_scales + scales_len);
    h->simplex.ComputeDictionary(column_scales != nullptr ? &scales : nullptr, &h->dictionary);
    int64_t total = 0;
    for (const auto& r : h->dictionary) total += static_cast<int64_t>(r.size());
    *nnz = total;
  } catch (const milp::DeviceError& e) {
    h->error = e.what();
    return MI_LP_ERROR_DEVICE;
  } catch (const std::exception& e) {
    h->error = e.what();
    return MI_LP_ERROR_INTERNAL;
  }
  return MI_LP_OK;
}

int mi_lp_get_dictionary(const mi_lp* h, int64_t* row_starts, int32_t* cols, double* values) {
  if (h == nullptr || row_starts == nullptr || cols == nullptr || values == nullptr) {
    return MI_LP_ERROR_NULL;
  }
  if (static_cast<int>(h->dictionary.size()) != h->lp.m) return MI_LP_ERROR_STATE;
  int64_t k = 0;
  for (int r = 0; r < h->lp.m; ++r) {
    row_starts[r] = k;
    for (const auto& e : h->dictionary[r]) {
      cols[k] = e.first;
      values[k] = e.second;
      ++k;
    }
  }
  row_starts[h->lp.m] = k;
  return MI_LP_OK;
}

int mi_lp_solve(mi_lp* h, const volatile int32_t* interrupt, mi_lp_result* out) {
  if (h == nullptr || out == nullptr) return MI_LP_ERROR_NULL;
  if (h->running) return MI_LP_ERROR_STATE;
  RunSolve(h, interrupt, out);
  return out->error_code;
}

#define MI_LP_REQUIRE_SOLVED(h)                  \
  do {                                           \
    if ((h) == nullptr) return MI_LP_ERROR_NULL; \
    if (!(h)->solved) return MI_LP_ERROR_STATE;  \
  } while (0)

int mi_lp_get_primal(const mi_lp* h, double* x) {
  MI_LP_REQUIRE_SOLVED(h);
  for (int c = 0; c < h->lp.n; ++c) x[c] = h->simplex.GetVariableValue(c);
  return MI_LP_OK;
}
int mi_lp_get_reduced_costs(const mi_lp* h, double* rc) {
  MI_LP_REQUIRE_SOLVED(h);
  for (int c = 0; c < h->lp.n; ++c) rc[c] = h->simplex.GetReducedCost(c);
  return MI_LP_OK;
}
int mi_lp_get_duals(const mi_lp* h, double* y) {
  MI_LP_REQUIRE_SOLVED(h);
  for (int r = 0; r < h->lp.m; ++r) y[r] = h->simplex.GetDualValue(r);
  return MI_LP_OK;
}
int mi_lp_get_activities(const mi_lp* h, double* a) {
  MI_LP_REQUIRE_SOLVED(h);
  for (int r = 0; r < h->lp.m; ++r) a[r] = h->simplex.GetConstraintActivity(r);
  return MI_LP_OK;
}
int mi_lp_get_statuses(const mi_lp* h, int8_t* var, int8_t* cons) {
  MI_LP_REQUIRE_SOLVED(h);
  for (int c = 0; c < h->lp.n; ++c) var[c] = static_cast<int8_t>(h->simplex.GetVariableStatus(c));
  for (int r = 0; r < h->lp.m; ++r)
    cons[r] = static_cast<int8_t>(h->simplex.GetConstraintStatus(r));
  return MI_LP_OK;
}
int mi_lp_get_basis(const mi_lp* h, int32_t* b) {
  MI_LP_REQUIRE_SOLVED(h);
  for (int r = 0; r < h->lp.m; ++r) b[r] = h->simplex.GetBasis(r);
  return MI_LP_OK;
}
int mi_lp_get_state(const mi_lp* h, int8_t* st) {
  MI_LP_REQUIRE_SOLVED(h);
  const auto& s = h->simplex.GetState();
  for (size_t i = 0; i < s.size(); ++i) st[i] = static_cast<int8_t>(s[i]);
  return MI_LP_OK;
}
int mi_lp_get_primal_ray(const mi_lp* h, double* v) {
  MI_LP_REQUIRE_SOLVED(h);
  const auto& r = h->simplex.GetPrimalRay();
  for (size_t i = 0; i < r.size(); ++i) v[i] = r[i];
  return MI_LP_OK;
}
int mi_lp_get_dual_ray(const mi_lp* h, double* v) {
  MI_LP_REQUIRE_SOLVED(h);
  const auto& r = h->simplex.GetDualRay();
  for (size_t i = 0; i < r.size(); ++i) v[i] = r[i];
  return MI_LP_OK;
}
int mi_lp_get_dual_ray_row_combination(const mi_lp* h, double* v) {
  MI_LP_REQUIRE_SOLVED(h);
  const auto& r = h->simplex.GetDualRayRowCombination();
  for (size_t i = 0; i < r.size(); ++i) v[i] = r[i];
  return MI_LP_OK;
}

// --- benchmark slicing -----------------------------------------------------
int mi_lp_begin(mi_lp* h, int64_t pause_at) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  if (h->running) return MI_LP_ERROR_STATE;
  h->running = true;
  h->finished = false;
  h->paused = false;
  h->stop = 0;
  h->pause_at = pause_at;
  h->current_iteration = 0;
  h->simplex.iteration_hook = [h](int64_t it) {
    std::unique_lock<std::mutex> l(h->mu);
    h->current_iteration = it;
    while (h->pause_at >= 0 && it >= h->pause_at) {
      h->simplex.device().Synchronize();
      h->paused = true;
      h->cv.notify_all();
      h->cv.wait(l);
    }
    h->paused = false;
  };
  h->worker = std::thread([h]() {
    RunSolve(h, &h->stop, &h->pending);
    std::lock_guard<std::mutex> l(h->mu);
    h->finished = true;
    h->cv.notify_all();
  });
  std::unique_lock<std::mutex> l(h->mu);
  h->cv.wait(l, [h]() { return h->paused || h->finished; });
  return MI_LP_OK;
}

int mi_lp_run_until(mi_lp* h, int64_t pause_at, int32_t* finished, int64_t* iterations) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  if (!h->running) return MI_LP_ERROR_STATE;
  std::unique_lock<std::mutex> l(h->mu);
  if (!h->finished) {
    h->pause_at = pause_at;
    h->paused = false;
    h->cv.notify_all();
    h->cv.wait(l, [h]() { return h->paused || h->finished; });
  }
  if (finished) *finished = h->finished ? 1 : 0;
  if (iterations) *iterations = h->current_iteration;
  return MI_LP_OK;
}

int mi_lp_stop(mi_lp* h) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  if (!h->running) return MI_LP_ERROR_STATE;
  {
    std::lock_guard<std::mutex> l(h->mu);
    h->stop = 1;
    h->pause_at = -1;
  }
  h->cv.notify_all();
  return MI_LP_OK;
}

int mi_lp_finish(mi_lp* h, mi_lp_result* out) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  if (!h->running) return MI_LP_ERROR_STATE;
  {
    std::lock_guard<std::mutex> l(h->mu);
    h->pause_at = -1;
  }
  h->cv.notify_all();
  h->worker.join();
  h->simplex.iteration_hook = nullptr;
  h->running = false;
  if (out) *out = h->pending;
  return h->pending.error_code;
}

int mi_lp_get_kernel_stats(const mi_lp* h, mi_lp_kernel_stats* s) {
  if (h == nullptr || s == nullptr) return MI_LP_ERROR_NULL;
  *s = const_cast<mi_lp*>(h)->simplex.device().stats();
  return MI_LP_OK;
}
int mi_lp_reset_kernel_stats(mi_lp* h) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  h->simplex.device().ResetStats();
  return MI_LP_OK;
}
int mi_lp_set_kernel_timing_ids(mi_lp* h, uint32_t id_mask) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  h->simplex.device().SetTiming(id_mask != 0, id_mask);
  return MI_LP_OK;
}
int mi_lp_set_kernel_timing(mi_lp* h, int32_t enable) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  h->simplex.device().SetTiming(enable != 0);
  return MI_LP_OK;
}

int mi_lp_set_exchange(mi_lp* h, int32_t rank, int32_t world, void* ctx,
                       mi_lp_allgather_fn allgather) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  if (h->running) return MI_LP_ERROR_STATE;
  try {
    (void)hipSetDevice(h->device);
    h->simplex.device().SetExchange(rank, world, ctx, allgather);
  } catch (const milp::DeviceError& e) {
    h->error = e.what();
    return MI_LP_ERROR_DEVICE;
  } catch (const std::exception& e) {
    h->error = e.what();
    return MI_LP_ERROR_INTERNAL;
  }
  return MI_LP_OK;
}

int mi_lp_record_iteration_times(mi_lp* h, int32_t enable) {
  if (h == nullptr) return MI_LP_ERROR_NULL;
  if (!SolveIsParked(h)) return MI_LP_ERROR_STATE;
  h->simplex.record_iteration_times = enable != 0;
  return MI_LP_OK;
}

int64_t mi_lp_get_iteration_times(const mi_lp* h, double* out, int64_t cap) {
  if (h == nullptr) return -MI_LP_ERROR_NULL;
  if (!SolveIsParked(h)) return -MI_LP_ERROR_STATE;
  const std::vector<double>& t = h->simplex.iteration_times;
  const int64_t n = std::min<int64_t>(cap, static_cast<int64_t>(t.size()));
  for (int64_t i = 0; out != nullptr && i < n; ++i) out[i] = t[i];
  return static_cast<int64_t>(t.size());
}

int mi_lp_get_run_counters(const mi_lp* h, mi_lp_run_counters* c) {
  if (h == nullptr || c == nullptr) return MI_LP_ERROR_NULL;
  if (!SolveIsParked(h)) return MI_LP_ERROR_STATE;
  std::memset(c, 0, sizeof(*c));
  c->factorizations = h->simplex.NumFactorizations();
  c->factorization_seconds = h->simplex.FactorizationSeconds();
  c->iterations = h->simplex.GetNumberOfIterations();
  const_cast<mi_lp*>(h)->simplex.device().TriScheduleShape(&c->u_levels, &c->u_outputs,
                                                          &c->u_entries);
  h->simplex.SdualCounters(&c->sdual_segments, &c->sdual_iterations);
  return MI_LP_OK;
}

}  // extern "C"

namespace {

// Back to single launches after a batch call (a device error there is the
// handle's next call's to report).
void SetSmallBatchSafe(mi_lp* h, bool on) {
  h->simplex.SetBatchMode(on);
  try {
    h->simplex.device().SetSmallBatch(on);
  } catch (const std::exception& e) {
    h->error = e.what();
  }
}
// The devices whose segment pool a batch call uses: when the last batch
// call on a device ends, its resident pool grid is told to stop.
struct PoolScope {
  std::vector<int> devices;
  std::vector<int> lps;  // handles of this call on devices[i]
  PoolScope(mi_lp* const* hs, int count) {
    std::vector<int> all, n;
    for (int i = 0; i < count; ++i) {
      if (!hs[i]->simplex.UsesSdualPool()) continue;
      const int d = hs[i]->device;
      const auto it = std::find(all.begin(), all.end(), d);
      if (it != all.end()) {
        ++n[it - all.begin()];
        continue;
      }
      all.push_back(d);
      n.push_back(1);
    }
    for (size_t k = 0; k < all.size(); ++k) {
      try {
        milp::SdualPoolScope(all[k], true, n[k]);
        devices.push_back(all[k]);
        lps.push_back(n[k]);
      } catch (const std::exception&) {
        // the segment itself reports the device error
      }
    }
  }
  ~PoolScope() {
    for (size_t k = 0; k < devices.size(); ++k) {
      try {
        milp::SdualPoolScope(devices[k], false, lps[k]);
      } catch (const std::exception&) {
      }
    }
  }
};
}  // namespace

extern "C" {

int mi_lp_batch_solve(mi_lp* const* handles, int32_t count, int32_t num_threads,
                      mi_lp_result* results) {
  milp::SamplerBatchCallBegin();
  if (handles == nullptr || results == nullptr) return MI_LP_ERROR_NULL;
  if (count < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  for (int i = 0; i < count; ++i) {
    if (handles[i] == nullptr) return MI_LP_ERROR_NULL;
  }
  if (num_threads < 1) num_threads = 1;
  // Each thread drives several LPs at once on fibers (fibers.h), their
  // small update rows going out in batched launches (SmallBatcher): while one
  // LP waits for the device, the thread runs another one's host work.
  // MILP_BATCH_FIBERS=k (default 4), MILP_SMALL_BATCH=0 turns batching off.
  int fibers = 4;
  if (const char* e = std::getenv("MILP_BATCH_FIBERS")) fibers = std::max(1, std::atoi(e));
  // MILP_BATCH_TRACE: the batch call's phases on stderr (setup, last solve
  // done, threads joined, teardown).
  static const bool trace = std::getenv("MILP_BATCH_TRACE") != nullptr;
  const auto t_start = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!trace) return;
    std::fprintf(stderr, "[batch] %-22s %9.3f s\n", what,
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
  };
  std::atomic<int> solved(0);
  const int in_flight = static_cast<int>(std::min<int64_t>(count, int64_t(num_threads) * fibers));
  for (int i = 0; i < count; ++i) {
    handles[i]->simplex.SetBatchMode(true, in_flight);
    handles[i]->simplex.device().SetSmallBatch(true);
  }
  mark("batch mode on");
  auto pool_scope = std::make_unique<PoolScope>(handles, count);
  mark("pool scope");
  // Largest LPs first (LPT order, weight (nnz + m) * m as in the multi-GPU
  // partition of mi_glop.distributed): the long solves start early instead of
  // forming the tail of the batch.
  std::vector<int> order(count);
  for (int i = 0; i < count; ++i) order[i] = i;
  auto weight = [&](int i) {
    const milp::LinearProgram& lp = handles[i]->lp;
    const double nnz = lp.col_starts.empty() ? 0.0 : double(lp.col_starts.back());
    return (nnz + lp.m) * double(lp.m);
  };
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return weight(a) > weight(b); });
  // The heaviest LPs (MILP_BATCH_PRIORITY_LPS, default 8) on high-priority
  // streams: their chains set the batch's wall (config 3: 4 -> 8 took the
  // suite from 6.8-6.9 to 7.7-7.8 LPs/s over three runs, gpurun_out/r06_j,k).
  static const int priority_lps = [] {
    const char* e = std::getenv("MILP_BATCH_PRIORITY_LPS");
    return e != nullptr ? std::max(0, std::atoi(e)) : 8;
  }();
  const int prioritized = count > num_threads ? std::min(priority_lps, count) : 0;
  for (int k = 0; k < prioritized; ++k) {
    try {
      handles[order[k]]->simplex.device().SetBatchPriority(true);
    } catch (const std::exception& e) {
      handles[order[k]]->error = e.what();
    }
  }
  // MILP_BATCH_DEDICATED=k: the k heaviest LPs each on a thread of their
  // own (no fibers), the rest on num_threads - k pooled threads.
  const int dedicated = [&] {
    const char* e = std::getenv("MILP_BATCH_DEDICATED");
    const int k = e != nullptr ? std::max(0, std::atoi(e)) : 0;
    return count > num_threads ? std::min({k, count, num_threads - 1}) : 0;
  }();
  std::atomic<int> next(dedicated);
  std::vector<std::thread> pool;
  // MILP_BATCH_HOST_POOL=1: the batch's LPs may also use the host pool.
  static const bool batch_pool = [] {
    const char* e = std::getenv("MILP_BATCH_HOST_POOL");
    return e != nullptr && std::atoi(e) != 0;
  }();
  for (int k = 0; k < dedicated; ++k) {
    pool.emplace_back([&, k]() {
      milp::SamplerAttachBatchThread();
      milp::HostSerialScope serial(!batch_pool);
      const int i = order[k];
      (void)hipSetDevice(handles[i]->device);
      RunSolve(handles[i], nullptr, &results[i]);
      if (solved.fetch_add(1) + 1 == count) mark("last solve done");
    });
  }
  for (int t = 0; t < num_threads - dedicated; ++t) {
    pool.emplace_back([&]() {
      milp::SamplerAttachBatchThread();
      milp::HostSerialScope serial(!batch_pool && num_threads > 1);
      std::vector<std::function<void()>> tasks;
      for (int f = 0; f < fibers; ++f) {
        tasks.push_back([&]() {
          while (true) {
            const int at = next.fetch_add(1);
            if (at >= count) break;
            const int i = order[at];
            (void)hipSetDevice(handles[i]->device);
            milp::SetFiberWeight(weight(i));
            RunSolve(handles[i], nullptr, &results[i]);
            milp::SetFiberWeight(0.0);
            if (solved.fetch_add(1) + 1 == count) mark("last solve done");
          }
        });
      }
      milp::RunFibers(std::move(tasks));
    });
  }
  for (auto& th : pool) th.join();
  mark("threads joined");
  for (int k = 0; k < prioritized; ++k) {
    try {
      handles[order[k]]->simplex.device().SetBatchPriority(false);
    } catch (const std::exception& e) {
      handles[order[k]]->error = e.what();
    }
  }
  for (int i = 0; i < count; ++i) SetSmallBatchSafe(handles[i], false);
  mark("batch mode off");
  pool_scope.reset();
  mark("pool scope closed");
  return MI_LP_OK;  // per-entry outcomes are in results[i]
}

// One search node's children: LP i = the workers' common LP with variable
// bounds lbs/ubs[i * n ...], warm-started from warm_state when given.
// Workers (handles loaded with the same LP, any devices) pull LPs from a
// shared counter, one host thread per worker. n and warm_len are checked
// against the workers' LP; a child whose setup fails is reported in its own
// result (ABNORMAL + error code) and is not solved.
int mi_lp_batch_solve_bounds(mi_lp* const* workers, int32_t num_workers, int32_t count,
                             const double* lbs, const double* ubs, const int8_t* warm_state,
                             int32_t warm_len, mi_lp_result* results) {
  milp::SamplerBatchCallBegin();
  if (workers == nullptr || lbs == nullptr || ubs == nullptr || results == nullptr) {
    return MI_LP_ERROR_NULL;
  }
  if (num_workers < 1 || count < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  for (int w = 0; w < num_workers; ++w) {
    if (workers[w] == nullptr) return MI_LP_ERROR_NULL;
    if (!workers[w]->loaded || workers[w]->lp.n != workers[0]->lp.n ||
        workers[w]->lp.m != workers[0]->lp.m) {
      return MI_LP_ERROR_STATE;
    }
    if (workers[w]->running) return MI_LP_ERROR_STATE;
  }
  const int64_t n = workers[0]->lp.n;
  if (warm_state != nullptr && warm_len != n + workers[0]->lp.m) {
    return MI_LP_ERROR_INVALID_PROBLEM;
  }
  // At most kBatchThreads host threads (MILP_BATCH_THREADS): worker w runs on
  // thread w % threads, the workers of one thread interleaved as fibers at
  // their device waits (fibers.h), their small update rows sent in batched
  // launches (SmallBatcher; MILP_SMALL_BATCH=0 turns batching off).
  constexpr int kBatchThreads = 16;
  int threads = std::min(num_workers, kBatchThreads);
  if (const char* e = std::getenv("MILP_BATCH_THREADS")) {
    threads = std::max(1, std::min(num_workers, std::atoi(e)));
  }
  // The children share one basis: its dual edge norms and its factorization
  // are computed once for the call (DualNormCache, LuShareCache; a hit
  // replays the deterministic-time bumps, so every result and every
  // handle's deterministic time are those of a child computing its own).
  // MILP_BATCH_SHARED_NORMS=0 / MILP_BATCH_SHARED_LU=0 turn them off. Read
  // per call (tests switch them).
  auto env_on = [](const char* name) {
    const char* e = std::getenv(name);
    return e == nullptr || std::atoi(e) != 0;
  };
  // Only between handles that loaded the same matrix (fingerprint at load;
  // the cache entries also compare their basis exactly on a hit).
  bool same_matrix = true;
  for (int w = 1; w < num_workers; ++w) {
    same_matrix = same_matrix &&
                  workers[w]->lp.matrix_fingerprint == workers[0]->lp.matrix_fingerprint &&
                  workers[w]->lp.col_starts.back() == workers[0]->lp.col_starts.back();
  }
  const bool shared_norms = same_matrix && env_on("MILP_BATCH_SHARED_NORMS");
  const bool shared_lu = same_matrix && env_on("MILP_BATCH_SHARED_LU");
  milp::DualNormCache norm_cache;
  milp::LuShareCache lu_cache;
  const int in_flight = std::min(num_workers, count);
  for (int w = 0; w < num_workers; ++w) {
    workers[w]->simplex.SetBatchMode(true, in_flight);
    workers[w]->simplex.device().SetSmallBatch(true);
    if (shared_norms && warm_state != nullptr) workers[w]->simplex.SetDualNormCache(&norm_cache);
    if (shared_lu && warm_state != nullptr) workers[w]->simplex.SetLuShareCache(&lu_cache);
  }
  PoolScope pool_scope(workers, num_workers);
  std::atomic<int> next(0);
  auto worker_loop = [&](mi_lp* h) {
    (void)hipSetDevice(h->device);
    while (true) {
      const int i = next.fetch_add(1);
      if (i >= count) break;
      int rc = mi_lp_set_variable_bounds(h, lbs + i * n, ubs + i * n);
      if (rc != MI_LP_OK) {
        FailEntry(h, rc, "mi_lp_set_variable_bounds failed", &results[i]);
        continue;
      }
      if (warm_state != nullptr) {
        rc = mi_lp_load_basis_state(h, warm_state, warm_len);
        if (rc != MI_LP_OK) {
          FailEntry(h, rc, "mi_lp_load_basis_state failed", &results[i]);
          continue;
        }
      }
      RunSolve(h, nullptr, &results[i]);
    }
  };
  // Workers are dealt to threads device by device (a thread's fibers never
  // span two GPUs; each device's workers get a share of the threads in
  // proportion to their number), all pulling children from one counter.
  std::vector<int> order(num_workers);
  for (int w = 0; w < num_workers; ++w) order[w] = w;
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return workers[a]->device < workers[b]->device; });
  std::vector<std::vector<mi_lp*>> per_thread(threads);
  {
    int t = 0;
    for (int w0 = 0; w0 < num_workers;) {
      int w1 = w0;
      while (w1 < num_workers && workers[order[w1]]->device == workers[order[w0]]->device) ++w1;
      const int group = w1 - w0;
      const int share = std::max(1, static_cast<int>(int64_t(group) * threads / num_workers));
      for (int k = 0; k < group; ++k) per_thread[(t + k % share) % threads].push_back(workers[order[w0 + k]]);
      t = (t + share) % threads;
      w0 = w1;
    }
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    if (per_thread[t].empty()) continue;
    pool.emplace_back([&, t]() {
      milp::SamplerAttachBatchThread();
      std::vector<std::function<void()>> tasks;
      for (mi_lp* h : per_thread[t]) tasks.push_back([&worker_loop, h]() { worker_loop(h); });
      milp::RunFibers(std::move(tasks));
    });
  }
  for (auto& th : pool) th.join();
  for (int w = 0; w < num_workers; ++w) {
    workers[w]->simplex.SetDualNormCache(nullptr);
    workers[w]->simplex.SetLuShareCache(nullptr);
    SetSmallBatchSafe(workers[w], false);
  }
  return MI_LP_OK;  // per-entry outcomes are in results[i]
}

// SURVEY 8(b) mi_lp_batch_solve(hs, count, num_gpus, ...): the handles'
// devices must lie in [0, num_gpus); each device's handles are solved by a
// pool of threads_per_gpu threads of their own (fibers per thread, batched
// launches, largest LPs first), every device at once.
int mi_lp_batch_solve_gpus(mi_lp* const* handles, int32_t count, int32_t num_gpus,
                           int32_t threads_per_gpu, mi_lp_result* results) {
  if (handles == nullptr || results == nullptr) return MI_LP_ERROR_NULL;
  if (count < 0 || num_gpus < 1) return MI_LP_ERROR_INVALID_PROBLEM;
  std::vector<std::vector<int>> by_device(num_gpus);
  for (int i = 0; i < count; ++i) {
    if (handles[i] == nullptr) return MI_LP_ERROR_NULL;
    const int d = handles[i]->device;
    if (d < 0 || d >= num_gpus) return MI_LP_ERROR_INVALID_PROBLEM;
    by_device[d].push_back(i);
  }
  try {
    std::vector<std::vector<mi_lp*>> hs(num_gpus);
    std::vector<std::vector<mi_lp_result>> rs(num_gpus);
    for (int d = 0; d < num_gpus; ++d) {
      for (const int i : by_device[d]) hs[d].push_back(handles[i]);
      rs[d].resize(hs[d].size());
    }
    std::vector<std::thread> per_device;
    for (int d = 0; d < num_gpus; ++d) {
      if (hs[d].empty()) continue;
      per_device.emplace_back([&, d]() {
        (void)hipSetDevice(d);
        mi_lp_batch_solve(hs[d].data(), static_cast<int32_t>(hs[d].size()), threads_per_gpu,
                          rs[d].data());
      });
    }
    for (auto& th : per_device) th.join();
    for (int d = 0; d < num_gpus; ++d) {
      for (size_t k = 0; k < by_device[d].size(); ++k) results[by_device[d][k]] = rs[d][k];
    }
  } catch (const std::exception&) {
    return MI_LP_ERROR_INTERNAL;
  }
  return MI_LP_OK;
}

}  // extern "C"

// Development aid (scripts/probe_batch.py): zero the MILP_SDUAL_PROFILE
// counters after a warm-up batch.
extern "C" void milp_sdual_profile_reset() {
  milp::SdualBridge::ResetProfile();
  milp::SdualProfileReset();
}

// Speculative flip FTRAN counters (process-wide): out[0] started, out[1]
// used by the next iteration, out[2] dropped. Read by the GPU tests.
extern "C" void milp_spec_flip_stats(int64_t* out) {
  out[0] = milp::VariableValues::spec_started.load();
  out[1] = milp::VariableValues::spec_used.load();
  out[2] = milp::VariableValues::spec_missed.load();
}
