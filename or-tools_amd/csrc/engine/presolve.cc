// Glop's presolve passes (glop/preprocessor.cc) and their postsolve, as
// MainLpPreprocessor runs them (preprocessor.cc:76-147). See presolve.h.
//
// Each pass keeps the reference's data flow: marks columns/rows for deletion
// while it scans, edits bounds/costs/entries in place, deletes at the end,
// and stores what its RecoverSolution needs. Helpers restate lp_utils.h
// (SumWithOneMissing, ScalarProduct), base/accurate_sum.h (AccurateSum),
// util/fp_utils.h (IsSmallerWithinTolerance), lp_data.cc (DeleteColumns,
// DeleteRows, PopulateFromDual), sparse_vector.h:849-929
// (AddMultipleToSparseVectorInternal) and matrix_utils.cc:27-173
// (FindProportionalColumns; the row-pattern hash is our own mix, which only
// groups candidates and does not change the mapping).
#include "presolve.h"

#include <algorithm>
#include <cmath>
#include <deque>
#include <limits>
#include <set>
#include <utility>

namespace milp {
namespace presolve {

namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

bool IsFinite(double v) { return v > -kInf && v < kInf; }  // lp_types.h:95-97

// util/fp_utils.h:158-161.
bool IsSmallerWithinTolerance(double x, double y, double tolerance) {
  if (y == kInf || y == -kInf) return x <= y;
  return x <= y + tolerance * std::max(1.0, std::min(std::fabs(x), std::fabs(y)));
}

// base/accurate_sum.h AccurateSum.
struct KahanSum {
  double sum = 0.0, err = 0.0;
  void Add(double v) {
    err += v;
    const double t = sum + err;
    err += sum - t;
    sum = t;
  }
  double Value() const { return sum; }
};

// lp_utils.h:324-387 SumWithOneMissing<supported_infinity_is_positive>.
template <bool kPositive>
struct SumWithOneMissing {
  int num_infinities = 0;
  KahanSum sum;
  double Infinity() const { return kPositive ? kInf : -kInf; }
  void Add(double x) {
    if (!IsFinite(x)) {
      ++num_infinities;
      return;
    }
    if (!IsFinite(sum.Value())) return;
    sum.Add(x);
  }
  double Sum() const { return num_infinities > 0 ? Infinity() : sum.Value(); }
  double SumWithout(double x) const {
    if (IsFinite(x)) {
      if (num_infinities > 0) return Infinity();
      return sum.Value() - x;
    }
    if (num_infinities > 1) return Infinity();
    return sum.Value();
  }
  double SumWithoutLb(double c) const {
    if (!IsFinite(c)) return SumWithout(c);
    return SumWithout(c) - std::fabs(c) * 1e-12;
  }
  double SumWithoutUb(double c) const {
    if (!IsFinite(c)) return SumWithout(c);
    return SumWithout(c) + std::fabs(c) * 1e-12;
  }
};
using SumNegInf = SumWithOneMissing<false>;
using SumPosInf = SumWithOneMissing<true>;

// lp_utils.h:85-92: dense . sparse, entry order.
double ScalarProduct(const std::vector<double>& u, const SparseVec& v) {
  double sum = 0.0;
  for (const Entry& e : v) sum += u[e.index] * e.coeff;
  return sum;
}

// lp_utils.h:120-128.
double PreciseScalarProduct(const std::vector<double>& u, const SparseVec& v) {
  KahanSum sum;
  for (const Entry& e : v) sum.Add(u[e.index] * e.coeff);
  return sum.Value();
}

// preprocessor.cc:349-369.
int8_t ComputeVariableStatus(double value, double lb, double ub) {
  if (lb == ub) return kFixedValue;
  if (value == lb) return kAtLowerBound;
  if (value == ub) return kAtUpperBound;
  return kFree;
}

// preprocessor.cc:372-375.
double MinInMagnitudeOrZeroIfInfinite(double a, double b) {
  const double value = std::fabs(a) < std::fabs(b) ? a : b;
  return IsFinite(value) ? value : 0.0;
}

// preprocessor.cc:456-471.
void SubtractColumnMultipleFromConstraintBound(int32_t col, double multiple, Lp* lp) {
  for (const Entry& e : lp->cols[col]) {
    const double delta = multiple * e.coeff;
    lp->row_lb[e.index] -= delta;
    lp->row_ub[e.index] -= delta;
  }
  lp->offset = lp->offset + lp->obj[col] * multiple;
}

// sparse_vector.h:849-929: *acc = multiplier * a + *acc, merged in index
// order; entries at common_index are dropped (delete_common) or kept from acc.
void AddMultipleToSparseVector(const SparseVec& a, bool delete_common, double multiplier,
                               int32_t common_index, double drop_tolerance, SparseVec* acc) {
  const SparseVec& b = *acc;
  SparseVec c;
  c.reserve(a.size() + b.size());
  size_t ia = 0, ib = 0;
  while (ia < a.size() && ib < b.size()) {
    const int32_t index_a = a[ia].index;
    const int32_t index_b = b[ib].index;
    if (index_a == index_b) {
      if (index_a != common_index) {
        const double a_coeff_mul = multiplier * a[ia].coeff;
        const double sum = a_coeff_mul + b[ib].coeff;
        if (std::fabs(sum) > drop_tolerance) c.push_back({index_a, sum});
      } else if (!delete_common) {
        c.push_back(b[ib]);
      }
      ++ia;
      ++ib;
    } else if (index_a < index_b) {
      c.push_back({index_a, multiplier * a[ia].coeff});
      ++ia;
    } else {
      c.push_back(b[ib]);
      ++ib;
    }
  }
  for (; ia < a.size(); ++ia) c.push_back({a[ia].index, multiplier * a[ia].coeff});
  for (; ib < b.size(); ++ib) c.push_back(b[ib]);
  acc->swap(c);
}

// SparseMatrix::PopulateFromTranspose of an m-row "matrix" given as columns.
std::vector<SparseVec> TransposeOf(const std::vector<SparseVec>& cols, int32_t num_rows) {
  std::vector<SparseVec> t(num_rows);
  std::vector<int32_t> count(num_rows, 0);
  for (const SparseVec& col : cols) {
    for (const Entry& e : col) ++count[e.index];
  }
  for (int32_t r = 0; r < num_rows; ++r) t[r].reserve(count[r]);
  for (int32_t c = 0; c < static_cast<int32_t>(cols.size()); ++c) {
    for (const Entry& e : cols[c]) t[e.index].push_back({c, e.coeff});
  }
  return t;
}

// --- matrix_utils.cc:27-173 FindProportionalColumns -------------------------
bool AreColumnsProportional(const SparseVec& a, const SparseVec& b, double tolerance) {
  if (a.size() != b.size()) return false;
  double multiple = 0.0;
  bool a_is_larger = true;
  for (size_t i = 0; i < a.size(); ++i) {
    if (a[i].index != b[i].index) return false;
    const double coeff_a = a[i].coeff;
    const double coeff_b = b[i].coeff;
    if (multiple == 0.0) {
      a_is_larger = std::fabs(coeff_a) > std::fabs(coeff_b);
      multiple = a_is_larger ? coeff_a / coeff_b : coeff_b / coeff_a;
    } else {
      if (a_is_larger) {
        if (std::fabs(coeff_a / coeff_b - multiple) > tolerance) return false;
      } else {
        if (std::fabs(coeff_b / coeff_a - multiple) > tolerance) return false;
      }
    }
  }
  return true;
}

struct Fingerprint {
  int32_t col;
  int64_t hash;
  double value;
  bool operator<(const Fingerprint& o) const {
    if (hash == o.hash) return value < o.value;
    return hash < o.hash;
  }
};

Fingerprint ComputeFingerprint(int32_t col, const SparseVec& column) {
  uint64_t h = 0x9e3779b97f4a7c15ull;
  double min_abs = std::numeric_limits<double>::max();
  double max_abs = 0.0;
  double sum = 0.0;
  for (const Entry& e : column) {
    h ^= static_cast<uint64_t>(static_cast<uint32_t>(e.index)) + 0x9e3779b97f4a7c15ull +
         (h << 6) + (h >> 2);
    h *= 0xff51afd7ed558ccdull;
    sum += e.coeff;
    min_abs = std::min(min_abs, std::fabs(e.coeff));
    max_abs = std::max(max_abs, std::fabs(e.coeff));
  }
  const double inverse_dynamic_range = min_abs / max_abs;
  const double scaled_average =
      std::fabs(sum) / (static_cast<double>(column.size()) * max_abs);
  return {col, static_cast<int64_t>(h), inverse_dynamic_range + scaled_average};
}

std::vector<int32_t> FindProportionalColumns(const std::vector<SparseVec>& matrix,
                                             double tolerance) {
  const int32_t num_cols = static_cast<int32_t>(matrix.size());
  std::vector<int32_t> mapping(num_cols, -1);
  std::vector<Fingerprint> fingerprints;
  for (int32_t col = 0; col < num_cols; ++col) {
    if (!matrix[col].empty()) fingerprints.push_back(ComputeFingerprint(col, matrix[col]));
  }
  std::sort(fingerprints.begin(), fingerprints.end());
  for (size_t i = 0; i < fingerprints.size(); ++i) {
    const int32_t col_a = fingerprints[i].col;
    if (mapping[col_a] != -1) continue;
    for (size_t j = i + 1; j < fingerprints.size(); ++j) {
      const int32_t col_b = fingerprints[j].col;
      if (mapping[col_b] != -1) continue;
      if (fingerprints[i].hash != fingerprints[j].hash ||
          !(std::fabs(fingerprints[i].value - fingerprints[j].value) < tolerance)) {
        break;
      }
      if (AreColumnsProportional(matrix[col_a], matrix[col_b], tolerance)) {
        mapping[col_b] = col_a;
      }
    }
  }
  for (int32_t col = 0; col < num_cols; ++col) {
    if (mapping[col] == -1) continue;
    const int32_t new_representative = mapping[mapping[col]];
    if (new_representative != -1) {
      mapping[col] = new_representative;
    } else if (mapping[col] > col) {
      mapping[mapping[col]] = col;
      mapping[col] = -1;
    }
  }
  return mapping;
}

// --- preprocessor.cc:211-338 helpers ----------------------------------------
class ColumnsSaver {
 public:
  void Save(int32_t col, const SparseVec& column) { saved_.emplace(col, column); }
  void SaveIfNotAlreadyDone(int32_t col, const SparseVec& column) {
    saved_.emplace(col, column);
  }
  const SparseVec& SavedOrEmpty(int32_t col) const {
    const auto it = saved_.find(col);
    return it == saved_.end() ? empty_ : it->second;
  }
  const SparseVec& Saved(int32_t col) const { return saved_.at(col); }

 private:
  SparseVec empty_;
  std::map<int32_t, SparseVec> saved_;
};

class ColumnDeletion {
 public:
  void Mark(int32_t col, double value = 0.0, int8_t status = kFree) {
    if (col >= static_cast<int32_t>(deleted_.size())) {
      deleted_.resize(col + 1, false);
      value_.resize(col + 1, 0.0);
      status_.resize(col + 1, kFree);
    }
    deleted_[col] = true;
    value_[col] = value;
    status_[col] = status;
  }
  bool IsMarked(int32_t col) const {
    return col < static_cast<int32_t>(deleted_.size()) && deleted_[col];
  }
  bool Empty() const { return deleted_.empty(); }
  const std::vector<bool>& Marked() const { return deleted_; }
  double StoredValue(int32_t col) const { return value_[col]; }
  void Clear() {
    deleted_.clear();
    value_.clear();
    status_.clear();
  }
  // RestoreDeletedColumns (preprocessor.cc:262-287).
  void Restore(Solution* s) const {
    std::vector<double> primal;
    std::vector<int8_t> vstat;
    size_t old = 0;
    for (size_t col = 0; col < deleted_.size(); ++col) {
      if (deleted_[col]) {
        primal.push_back(value_[col]);
        vstat.push_back(status_[col]);
      } else {
        primal.push_back(s->primal[old]);
        vstat.push_back(s->vstat[old]);
        ++old;
      }
    }
    for (; old < s->primal.size(); ++old) {
      primal.push_back(s->primal[old]);
      vstat.push_back(s->vstat[old]);
    }
    s->primal.swap(primal);
    s->vstat.swap(vstat);
  }

 private:
  std::vector<bool> deleted_;
  std::vector<double> value_;
  std::vector<int8_t> status_;
};

class RowDeletion {
 public:
  void Mark(int32_t row) {
    if (row >= static_cast<int32_t>(deleted_.size())) deleted_.resize(row + 1, false);
    deleted_[row] = true;
  }
  void Unmark(int32_t row) {
    if (row >= static_cast<int32_t>(deleted_.size())) return;
    deleted_[row] = false;
  }
  bool IsMarked(int32_t row) const {
    return row < static_cast<int32_t>(deleted_.size()) && deleted_[row];
  }
  bool Empty() const { return deleted_.empty(); }
  const std::vector<bool>& Marked() const { return deleted_; }
  // RestoreDeletedRows (preprocessor.cc:312-338): dual 0.0, BASIC.
  void Restore(Solution* s) const {
    std::vector<double> dual;
    std::vector<int8_t> cstat;
    size_t old = 0;
    for (size_t row = 0; row < deleted_.size(); ++row) {
      if (deleted_[row]) {
        dual.push_back(0.0);
        cstat.push_back(kBasic);
      } else {
        dual.push_back(s->dual[old]);
        cstat.push_back(s->cstat[old]);
        ++old;
      }
    }
    for (; old < s->dual.size(); ++old) {
      dual.push_back(s->dual[old]);
      cstat.push_back(s->cstat[old]);
    }
    s->dual.swap(dual);
    s->cstat.swap(cstat);
  }

 private:
  std::vector<bool> deleted_;
};

}  // namespace

// --- LinearProgram ------------------------------------------------------------
int64_t Lp::num_entries() const {
  int64_t n = 0;
  for (const SparseVec& c : cols) n += static_cast<int64_t>(c.size());
  return n;
}

std::vector<SparseVec> Lp::Transpose() const { return TransposeOf(cols, num_rows); }

void Lp::DeleteColumns(const std::vector<bool>& del) {
  if (del.empty()) return;
  int32_t k = 0;
  for (int32_t c = 0; c < num_cols(); ++c) {
    if (c < static_cast<int32_t>(del.size()) && del[c]) continue;
    if (k != c) {
      cols[k].swap(cols[c]);
      col_lb[k] = col_lb[c];
      col_ub[k] = col_ub[c];
      obj[k] = obj[c];
    }
    ++k;
  }
  cols.resize(k);
  col_lb.resize(k);
  col_ub.resize(k);
  obj.resize(k);
}

void Lp::DeleteRows(const std::vector<bool>& del) {
  if (del.empty()) return;
  std::vector<int32_t> perm(num_rows, -1);
  int32_t k = 0;
  for (int32_t r = 0; r < num_rows; ++r) {
    if (r < static_cast<int32_t>(del.size()) && del[r]) continue;
    row_lb[k] = row_lb[r];
    row_ub[k] = row_ub[r];
    perm[r] = k++;
  }
  row_lb.resize(k);
  row_ub.resize(k);
  num_rows = k;
  for (SparseVec& col : cols) {
    size_t w = 0;
    for (const Entry& e : col) {
      const int32_t nr = perm[e.index];
      if (nr != -1) col[w++] = {nr, e.coeff};
    }
    col.resize(w);
  }
}

int32_t Lp::AddColumn(double lb, double ub, double cost) {
  cols.emplace_back();
  col_lb.push_back(lb);
  col_ub.push_back(ub);
  obj.push_back(cost);
  return num_cols() - 1;
}

// --- Preprocessor base (preprocessor.h:47-100) ----------------------------------
class Pass {
 public:
  explicit Pass(const Params& p) : params_(p) {}
  virtual ~Pass() = default;
  virtual bool Run(Lp* lp) = 0;
  virtual void Recover(Solution* s) const = 0;
  int32_t status() const { return status_; }

 protected:
  bool SmallerWithinFeasibility(double a, double b) const {
    return IsSmallerWithinTolerance(a, b, params_.solution_feasibility_tolerance);
  }
  bool SmallerWithinZero(double a, double b) const {
    return IsSmallerWithinTolerance(a, b, params_.preprocessor_zero_tolerance);
  }
  int32_t status_ = kInit;
  const Params& params_;
};

namespace {

// --- EmptyColumnPreprocessor (preprocessor.cc:397-445) ------------------------
class EmptyColumnPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    for (int32_t col = 0; col < lp->num_cols(); ++col) {
      if (!lp->cols[col].empty()) continue;
      const double lb = lp->col_lb[col];
      const double ub = lp->col_ub[col];
      const double cost = lp->MinCost(col);
      double value;
      if (cost == 0) {
        value = ub != kInf ? ub : (lb != -kInf ? lb : 0.0);
      } else {
        value = cost > 0 ? lb : ub;
        if (!IsFinite(value)) {
          status_ = kInfeasibleOrUnbounded;
          return false;
        }
        lp->offset = lp->offset + value * lp->obj[col];
      }
      del_.Mark(col, value, ComputeVariableStatus(value, lb, ub));
    }
    lp->DeleteColumns(del_.Marked());
    return !del_.Empty();
  }
  void Recover(Solution* s) const override { del_.Restore(s); }

 private:
  ColumnDeletion del_;
};

// --- ProportionalColumnPreprocessor (preprocessor.cc:497-835) -----------------
class ProportionalColumnPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    std::vector<int32_t> mapping =
        FindProportionalColumns(lp->cols, params_.preprocessor_zero_tolerance);
    std::vector<int32_t> prop;
    for (int32_t col = 0; col < static_cast<int32_t>(mapping.size()); ++col) {
      const int32_t rep = mapping[col];
      if (rep != -1) {
        if (mapping[rep] == -1) {
          prop.push_back(rep);
          mapping[rep] = rep;
        }
        prop.push_back(col);
      }
    }
    if (prop.empty()) return false;
    const int32_t num_cols = lp->num_cols();
    factors_.assign(num_cols, 0.0);
    for (const int32_t col : prop) factors_[col] = lp->cols[col][0].coeff;

    std::vector<double> slope_lb(num_cols, -kInf), slope_ub(num_cols, kInf);
    for (const int32_t col : prop) {
      const int32_t rep = mapping[col];
      bool upper_bounded = lp->col_ub[col] == kInf;  // rc >= 0
      bool lower_bounded = lp->col_lb[col] == -kInf;  // rc <= 0
      if (factors_[col] < 0.0) std::swap(lower_bounded, upper_bounded);
      const double slope = lp->MinCost(col) / factors_[col];
      if (lower_bounded) slope_lb[rep] = std::max(slope_lb[rep], slope);
      if (upper_bounded) slope_ub[rep] = std::min(slope_ub[rep], slope);
    }
    for (const int32_t col : prop) {
      const int32_t rep = mapping[col];
      if (rep == col && !SmallerWithinFeasibility(slope_lb[rep], slope_ub[rep])) {
        status_ = kInfeasibleOrUnbounded;
        return false;
      }
    }
    for (const int32_t col : prop) {
      const int32_t rep = mapping[col];
      const double slope = lp->MinCost(col) / factors_[col];
      bool can_fix = false;
      double target = 0.0;
      const double lb = lp->col_lb[col];
      const double ub = lp->col_ub[col];
      if (!SmallerWithinFeasibility(slope_lb[rep], slope)) {
        can_fix = true;
        target = factors_[col] >= 0.0 ? ub : lb;
      } else if (!SmallerWithinFeasibility(slope, slope_ub[rep])) {
        can_fix = true;
        target = factors_[col] >= 0.0 ? lb : ub;
      }
      if (can_fix) {
        mapping[col] = -1;
        if (!IsFinite(target)) {
          status_ = kInfeasibleOrUnbounded;
          return false;
        }
        SubtractColumnMultipleFromConstraintBound(col, target, lp);
        del_.Mark(col, target, ComputeVariableStatus(target, lb, ub));
      }
    }
    struct Sorted {
      int32_t col, rep;
      double scaled_cost;
      bool operator<(const Sorted& o) const {
        if (rep == o.rep) {
          if (scaled_cost == o.scaled_cost) return col < o.col;
          return scaled_cost < o.scaled_cost;
        }
        return rep < o.rep;
      }
    };
    std::vector<Sorted> sorted;
    for (const int32_t col : prop) {
      if (mapping[col] != -1) {
        sorted.push_back({col, mapping[col], lp->obj[col] / factors_[col]});
      }
    }
    std::sort(sorted.begin(), sorted.end());
    merged_.assign(num_cols, -1);
    lbs_.assign(num_cols, -kInf);
    ubs_.assign(num_cols, kInf);
    new_lbs_.assign(num_cols, -kInf);
    new_ubs_.assign(num_cols, kInf);
    for (size_t i = 0; i < sorted.size();) {
      const int32_t target_col = sorted[i].col;
      const int32_t target_rep = sorted[i].rep;
      const double target_cost = sorted[i].scaled_cost;
      lbs_[target_col] = lp->col_lb[target_col];
      ubs_[target_col] = lp->col_ub[target_col];
      int num_merged = 0;
      for (++i; i < sorted.size(); ++i) {
        if (sorted[i].rep != target_rep) break;
        if (std::fabs(sorted[i].scaled_cost - target_cost) >=
            params_.preprocessor_zero_tolerance) {
          break;
        }
        ++num_merged;
        const int32_t col = sorted[i].col;
        const double lb = lp->col_lb[col];
        const double ub = lp->col_ub[col];
        lbs_[col] = lb;
        ubs_[col] = ub;
        merged_[col] = target_col;
        const double bound_factor = factors_[col] / factors_[target_col];
        const double target_value = MinInMagnitudeOrZeroIfInfinite(lb, ub);
        double lower_diff = (lb - target_value) * bound_factor;
        double upper_diff = (ub - target_value) * bound_factor;
        if (bound_factor < 0.0) std::swap(lower_diff, upper_diff);
        lp->col_lb[target_col] = lp->col_lb[target_col] + lower_diff;
        lp->col_ub[target_col] = lp->col_ub[target_col] + upper_diff;
        SubtractColumnMultipleFromConstraintBound(col, target_value, lp);
        del_.Mark(col, target_value, ComputeVariableStatus(target_value, lb, ub));
      }
      if (num_merged > 0) {
        merged_[target_col] = target_col;
        const double target_value =
            MinInMagnitudeOrZeroIfInfinite(lbs_[target_col], ubs_[target_col]);
        lp->col_lb[target_col] = lp->col_lb[target_col] - target_value;
        lp->col_ub[target_col] = lp->col_ub[target_col] - target_value;
        SubtractColumnMultipleFromConstraintBound(target_col, target_value, lp);
        new_lbs_[target_col] = lp->col_lb[target_col];
        new_ubs_[target_col] = lp->col_ub[target_col];
      }
    }
    lp->DeleteColumns(del_.Marked());
    return !del_.Empty();
  }

  void Recover(Solution* s) const override {
    del_.Restore(s);
    const int32_t num_cols = static_cast<int32_t>(merged_.size());
    std::vector<bool> rep_basic(num_cols, false), dist_to_ub(num_cols, false);
    std::vector<double> distance(num_cols, 0.0), wanted(num_cols, 0.0);
    for (int32_t col = 0; col < num_cols; ++col) {
      if (merged_[col] != col) continue;
      const double value = s->primal[col];
      const double to_ub = new_ubs_[col] - value;
      const double to_lb = value - new_lbs_[col];
      if (to_ub < to_lb) {
        distance[col] = to_ub;
        dist_to_ub[col] = true;
      } else {
        distance[col] = to_lb;
        dist_to_ub[col] = false;
      }
      rep_basic[col] = s->vstat[col] == kBasic;
      wanted[col] = value;
      s->primal[col] = MinInMagnitudeOrZeroIfInfinite(lbs_[col], ubs_[col]);
      s->vstat[col] = ComputeVariableStatus(s->primal[col], lbs_[col], ubs_[col]);
    }
    for (int32_t col = 0; col < num_cols; ++col) {
      const int32_t rep = merged_[col];
      if (rep == -1) continue;
      if (IsFinite(distance[rep])) {
        const double bound_factor = factors_[col] / factors_[rep];
        const double scaled_distance = distance[rep] / std::fabs(bound_factor);
        const double width = ubs_[col] - lbs_[col];
        const bool to_upper = (bound_factor > 0.0) == dist_to_ub[rep];
        if (width <= scaled_distance) {
          s->primal[col] = to_upper ? lbs_[col] : ubs_[col];
          s->vstat[col] = ComputeVariableStatus(s->primal[col], lbs_[col], ubs_[col]);
          distance[rep] -= width * std::fabs(bound_factor);
        } else {
          s->primal[col] = to_upper ? ubs_[col] - scaled_distance : lbs_[col] + scaled_distance;
          s->vstat[col] = rep_basic[rep]
                              ? static_cast<int8_t>(kBasic)
                              : ComputeVariableStatus(s->primal[col], lbs_[col], ubs_[col]);
          distance[rep] = 0.0;
          rep_basic[rep] = false;
        }
      } else {
        const double error = wanted[rep];
        if (error == 0.0) {
          if (rep_basic[rep]) {
            s->vstat[col] = kBasic;
            rep_basic[rep] = false;
          }
        } else {
          const double bound_factor = factors_[col] / factors_[rep];
          const bool use_this = (error * bound_factor > 0.0) ? (ubs_[col] == kInf)
                                                             : (lbs_[col] == -kInf);
          if (use_this) {
            wanted[rep] = 0.0;
            s->primal[col] += error / bound_factor;
            if (rep_basic[rep]) {
              s->vstat[col] = kBasic;
              rep_basic[rep] = false;
            } else {
              s->vstat[col] = kFree;
            }
          }
        }
      }
    }
  }

 private:
  ColumnDeletion del_;
  std::vector<double> factors_;
  std::vector<int32_t> merged_;
  std::vector<double> lbs_, ubs_, new_lbs_, new_ubs_;
};

// --- ProportionalRowPreprocessor (preprocessor.cc:841-1084) -------------------
class ProportionalRowPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    const int32_t num_rows = lp->num_rows;
    const std::vector<SparseVec> t = lp->Transpose();
    factors_.assign(num_rows, 0.0);
    for (int32_t row = 0; row < num_rows; ++row) {
      if (!t[row].empty()) factors_[row] = t[row][0].coeff;
    }
    std::vector<double> lower(num_rows, -kInf), upper(num_rows, kInf);
    ub_sources_.assign(num_rows, -1);
    lb_sources_.assign(num_rows, -1);
    std::vector<int32_t> mapping = FindProportionalColumns(t, params_.preprocessor_zero_tolerance);
    std::vector<bool> is_rep(num_rows, false);
    for (int32_t row = 0; row < num_rows; ++row) {
      const int32_t rep = mapping[row];
      if (rep != -1) {
        mapping[rep] = rep;
        is_rep[rep] = true;
      }
    }
    for (int32_t row = 0; row < num_rows; ++row) {
      if (mapping[row] == -1) continue;
      del_.Mark(row);
      const int32_t rep = mapping[row];
      const double factor = factors_[rep] / factors_[row];
      double implied_lb = factor * lp->row_lb[row];
      double implied_ub = factor * lp->row_ub[row];
      if (factor < 0.0) std::swap(implied_lb, implied_ub);
      if (implied_lb >= lower[rep]) {
        lower[rep] = implied_lb;
        lb_sources_[rep] = row;
      }
      if (implied_ub <= upper[rep]) {
        upper[rep] = implied_ub;
        ub_sources_[rep] = row;
      }
    }
    for (int32_t row = 0; row < num_rows; ++row) {
      if (!is_rep[row]) continue;
      const int32_t lsrc = lb_sources_[row];
      const int32_t usrc = ub_sources_[row];
      lb_sources_[row] = -1;
      ub_sources_[row] = -1;
      if (lsrc == usrc) {
        del_.Unmark(lsrc);
        continue;
      }
      if (!SmallerWithinFeasibility(lower[row], upper[row])) {
        status_ = kPrimalInfeasible;
        return false;
      }
      if (lp->row_lb[lsrc] == lp->row_ub[lsrc]) {
        del_.Unmark(lsrc);
        continue;
      }
      if (lp->row_lb[usrc] == lp->row_ub[usrc]) {
        del_.Unmark(usrc);
        continue;
      }
      int32_t new_rep = lsrc;
      int32_t other = usrc;
      if (std::fabs(factors_[new_rep]) < std::fabs(factors_[other])) std::swap(new_rep, other);
      const double factor = factors_[new_rep] / factors_[other];
      double new_lb = factor * lp->row_lb[other];
      double new_ub = factor * lp->row_ub[other];
      if (factor < 0.0) std::swap(new_lb, new_ub);
      lb_sources_[new_rep] = new_rep;
      ub_sources_[new_rep] = new_rep;
      if (new_lb > lp->row_lb[new_rep]) {
        lb_sources_[new_rep] = other;
      } else {
        new_lb = lp->row_lb[new_rep];
      }
      if (new_ub < lp->row_ub[new_rep]) {
        ub_sources_[new_rep] = other;
      } else {
        new_ub = lp->row_ub[new_rep];
      }
      const int32_t new_lsrc = lb_sources_[new_rep];
      if (new_lsrc == ub_sources_[new_rep]) {
        del_.Unmark(new_lsrc);
        lb_sources_[new_rep] = -1;
        ub_sources_[new_rep] = -1;
        continue;
      }
      if (new_lb > new_ub) {
        if (lb_sources_[new_rep] == new_rep) {
          new_ub = lp->row_lb[new_rep];
        } else {
          new_lb = lp->row_ub[new_rep];
        }
      }
      del_.Unmark(new_rep);
      lp->row_lb[new_rep] = new_lb;
      lp->row_ub[new_rep] = new_ub;
    }
    maximize_ = lp->maximize;
    lp->DeleteRows(del_.Marked());
    return !del_.Empty();
  }

  void Recover(Solution* s) const override {
    del_.Restore(s);
    const int32_t num_rows = static_cast<int32_t>(s->dual.size());
    for (int32_t row = 0; row < num_rows; ++row) {
      const int32_t lsrc = lb_sources_[row];
      const int32_t usrc = ub_sources_[row];
      if (lsrc == -1 && usrc == -1) continue;
      int8_t status = s->cstat[row];
      if (status == kBasic) continue;
      if (status == kFixedValue) {
        const double corrected = maximize_ ? -s->dual[row] : s->dual[row];
        if (corrected != 0.0) status = corrected > 0.0 ? kAtLowerBound : kAtUpperBound;
      }
      if (lsrc != row && status == kAtLowerBound) {
        const double factor = factors_[row] / factors_[lsrc];
        s->dual[lsrc] = factor * s->dual[row];
        s->dual[row] = 0.0;
        s->cstat[row] = kBasic;
        s->cstat[lsrc] = factor > 0.0 ? kAtLowerBound : kAtUpperBound;
      }
      if (usrc != row && status == kAtUpperBound) {
        const double factor = factors_[row] / factors_[usrc];
        s->dual[usrc] = factor * s->dual[row];
        s->dual[row] = 0.0;
        s->cstat[row] = kBasic;
        s->cstat[usrc] = factor > 0.0 ? kAtUpperBound : kAtLowerBound;
      }
      if (s->cstat[row] == kFixedValue) {
        s->cstat[row] = lsrc != row ? kAtUpperBound : kAtLowerBound;
      }
    }
  }

 private:
  RowDeletion del_;
  std::vector<double> factors_;
  std::vector<int32_t> lb_sources_, ub_sources_;
  bool maximize_ = false;
};

// --- FixedVariablePreprocessor (preprocessor.cc:1090-1117) ---------------------
class FixedVariablePass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    for (int32_t col = 0; col < lp->num_cols(); ++col) {
      const double lb = lp->col_lb[col];
      if (lb == lp->col_ub[col]) {
        SubtractColumnMultipleFromConstraintBound(col, lb, lp);
        del_.Mark(col, lb, kFixedValue);
      }
    }
    lp->DeleteColumns(del_.Marked());
    return !del_.Empty();
  }
  void Recover(Solution* s) const override { del_.Restore(s); }

 private:
  ColumnDeletion del_;
};

// --- ForcingAndImpliedFreeConstraintPreprocessor (preprocessor.cc:1123-1373) --
class ForcingAndImpliedFreePass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    const int32_t num_rows = lp->num_rows;
    const int32_t num_cols = lp->num_cols();
    std::vector<double> implied_lb(num_rows, 0), implied_ub(num_rows, 0);
    std::vector<int> degree(num_rows, 0);
    for (int32_t col = 0; col < num_cols; ++col) {
      const double lower = lp->col_lb[col];
      const double upper = lp->col_ub[col];
      for (const Entry& e : lp->cols[col]) {
        if (e.coeff > 0.0) {
          implied_lb[e.index] += lower * e.coeff;
          implied_ub[e.index] += upper * e.coeff;
        } else {
          implied_lb[e.index] += upper * e.coeff;
          implied_ub[e.index] += lower * e.coeff;
        }
        ++degree[e.index];
      }
    }
    int num_forcing = 0;
    forcing_up_.assign(num_rows, false);
    std::vector<bool> forcing_down(num_rows, false);
    for (int32_t row = 0; row < num_rows; ++row) {
      if (degree[row] == 0) continue;
      const double lower = lp->row_lb[row];
      const double upper = lp->row_ub[row];
      if (!SmallerWithinFeasibility(lower, implied_ub[row]) ||
          !SmallerWithinFeasibility(implied_lb[row], upper)) {
        status_ = kPrimalInfeasible;
        return false;
      }
      if (SmallerWithinZero(implied_ub[row], lower)) {
        forcing_down[row] = true;
        ++num_forcing;
        continue;
      }
      if (SmallerWithinZero(upper, implied_lb[row])) {
        forcing_up_[row] = true;
        ++num_forcing;
        continue;
      }
      if (SmallerWithinZero(lower, implied_lb[row]) && SmallerWithinZero(implied_ub[row], upper)) {
        lp->row_lb[row] = -kInf;
        lp->row_ub[row] = kInf;
      }
    }
    if (num_forcing > 0) {
      maximize_ = lp->maximize;
      costs_.resize(num_cols, 0.0);
      for (int32_t col = 0; col < num_cols; ++col) {
        const SparseVec& column = lp->cols[col];
        const double lower = lp->col_lb[col];
        const double upper = lp->col_ub[col];
        bool forced = false;
        double target = 0.0;
        for (const Entry& e : column) {
          if (forcing_down[e.index]) {
            const double candidate = e.coeff < 0.0 ? lower : upper;
            if (forced && candidate != target) {
              if (SmallerWithinZero(upper, lower)) {
                target = std::fabs(lower) < std::fabs(upper) ? lower : upper;
                continue;
              }
              status_ = kPrimalInfeasible;
              return false;
            }
            target = candidate;
            forced = true;
          }
          if (forcing_up_[e.index]) {
            const double candidate = e.coeff < 0.0 ? upper : lower;
            if (forced && candidate != target) {
              if (SmallerWithinZero(upper, lower)) {
                target = std::fabs(lower) < std::fabs(upper) ? lower : upper;
                continue;
              }
              status_ = kPrimalInfeasible;
              return false;
            }
            target = candidate;
            forced = true;
          }
        }
        if (forced) {
          SubtractColumnMultipleFromConstraintBound(col, target, lp);
          cdel_.Mark(col, target, ComputeVariableStatus(target, lower, upper));
          saver_.Save(col, column);
          costs_[col] = lp->obj[col];
        }
      }
      for (int32_t row = 0; row < num_rows; ++row) {
        if (forcing_down[row] || forcing_up_[row]) rdel_.Mark(row);
      }
    }
    lp->DeleteColumns(cdel_.Marked());
    lp->DeleteRows(rdel_.Marked());
    return !cdel_.Empty();
  }

  void Recover(Solution* s) const override {
    cdel_.Restore(s);
    rdel_.Restore(s);
    struct Del {
      int32_t row, col;
      double coeff;
    };
    std::vector<Del> entries;
    const int32_t size = static_cast<int32_t>(cdel_.Marked().size());
    for (int32_t col = 0; col < size; ++col) {
      if (!cdel_.IsMarked(col)) continue;
      int32_t last_row = -1;
      double last_coeff = 0.0;
      for (const Entry& e : saver_.Saved(col)) {
        if (rdel_.IsMarked(e.index)) {
          last_row = e.index;
          last_coeff = e.coeff;
        }
      }
      if (last_row != -1) entries.push_back({last_row, col, last_coeff});
    }
    std::sort(entries.begin(), entries.end(), [](const Del& a, const Del& b) {
      if (a.row == b.row) return a.col < b.col;
      return a.row < b.row;
    });
    for (size_t i = 0; i < entries.size();) {
      const int32_t row = entries[i].row;
      double new_dual = 0.0;
      int32_t new_basic = -1;
      for (; i < entries.size(); ++i) {
        if (entries[i].row != row) break;
        const int32_t col = entries[i].col;
        const double sp = ScalarProduct(s->dual, saver_.Saved(col));
        const double rc = costs_[col] - sp;
        const double bound = rc / entries[i].coeff;
        if (forcing_up_[row] == !maximize_) {
          if (bound < new_dual) {
            new_dual = bound;
            new_basic = col;
          }
        } else {
          if (bound > new_dual) {
            new_dual = bound;
            new_basic = col;
          }
        }
      }
      if (new_basic != -1) {
        s->dual[row] = new_dual;
        s->vstat[new_basic] = kBasic;
        s->cstat[row] = forcing_up_[row] ? kAtUpperBound : kAtLowerBound;
      }
    }
  }

 private:
  ColumnDeletion cdel_;
  RowDeletion rdel_;
  ColumnsSaver saver_;
  std::vector<double> costs_;
  std::vector<bool> forcing_up_;
  bool maximize_ = false;
};

// --- ImpliedFreePreprocessor (preprocessor.cc:1393-1610) ------------------------
class ImpliedFreePass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    if (!params_.use_implied_free_preprocessor) return false;
    const int32_t num_rows = lp->num_rows;
    const int32_t num_cols = lp->num_cols();
    std::vector<SumNegInf> lb_sums(num_rows);
    std::vector<SumPosInf> ub_sums(num_rows);
    for (int32_t col = 0; col < num_cols; ++col) {
      const double lb = lp->col_lb[col];
      const double ub = lp->col_ub[col];
      for (const Entry& e : lp->cols[col]) {
        double entry_lb = e.coeff * lb;
        double entry_ub = e.coeff * ub;
        if (e.coeff < 0.0) std::swap(entry_lb, entry_ub);
        lb_sums[e.index].Add(entry_lb);
        ub_sums[e.index].Add(entry_ub);
      }
    }
    for (int32_t row = 0; row < num_rows; ++row) {
      lb_sums[row].Add(-lp->row_ub[row]);
      ub_sums[row].Add(-lp->row_lb[row]);
    }
    std::vector<bool> used_rows(num_rows, false);
    postsolve_status_.assign(num_cols, kFree);
    offsets_.assign(num_cols, 0.0);
    std::vector<std::pair<int64_t, int32_t>> by_degree;
    by_degree.reserve(num_cols);
    for (int32_t col = 0; col < num_cols; ++col) {
      by_degree.push_back({static_cast<int64_t>(lp->cols[col].size()), col});
    }
    std::sort(by_degree.begin(), by_degree.end());
    int num_implied_free = 0;
    for (const auto& cd : by_degree) {
      const int32_t col = cd.second;
      const double lb = lp->col_lb[col];
      const double ub = lp->col_ub[col];
      if (!IsFinite(lb) && !IsFinite(ub)) continue;
      if (lb == ub) continue;
      double overall_lb = -kInf;
      double overall_ub = kInf;
      for (const Entry& e : lp->cols[col]) {
        if (used_rows[e.index]) continue;
        const double coeff = e.coeff;
        double entry_lb = coeff * lb;
        double entry_ub = coeff * ub;
        if (coeff < 0.0) std::swap(entry_lb, entry_ub);
        const double implied_lb = coeff > 0.0 ? -ub_sums[e.index].SumWithoutUb(entry_ub) / coeff
                                              : -lb_sums[e.index].SumWithoutLb(entry_lb) / coeff;
        const double implied_ub = coeff > 0.0 ? -lb_sums[e.index].SumWithoutLb(entry_lb) / coeff
                                              : -ub_sums[e.index].SumWithoutUb(entry_ub) / coeff;
        overall_lb = std::max(overall_lb, implied_lb);
        overall_ub = std::min(overall_ub, implied_ub);
      }
      if (!SmallerWithinFeasibility(overall_lb, ub) ||
          !SmallerWithinFeasibility(lb, overall_ub) ||
          !SmallerWithinFeasibility(overall_lb, overall_ub)) {
        status_ = kPrimalInfeasible;
        return false;
      }
      if (SmallerWithinZero(ub, overall_lb) || SmallerWithinZero(overall_ub, lb)) continue;
      if (SmallerWithinZero(overall_ub, overall_lb)) continue;
      if (SmallerWithinZero(lb, overall_lb) && SmallerWithinZero(overall_ub, ub)) {
        ++num_implied_free;
        lp->col_lb[col] = -kInf;
        lp->col_ub[col] = kInf;
        for (const Entry& e : lp->cols[col]) used_rows[e.index] = true;
        const double offset = MinInMagnitudeOrZeroIfInfinite(lb, ub);
        if (offset != 0.0) {
          offsets_[col] = offset;
          SubtractColumnMultipleFromConstraintBound(col, offset, lp);
        }
        postsolve_status_[col] = ComputeVariableStatus(offset, lb, ub);
      }
    }
    return num_implied_free > 0;
  }

  void Recover(Solution* s) const override {
    const int32_t num_cols = static_cast<int32_t>(s->vstat.size());
    for (int32_t col = 0; col < num_cols; ++col) {
      if (postsolve_status_[col] == kFree) continue;
      if (s->vstat[col] == kFree) s->vstat[col] = postsolve_status_[col];
      s->primal[col] += offsets_[col];
    }
  }

 private:
  std::vector<int8_t> postsolve_status_;
  std::vector<double> offsets_;
};

// --- DoubletonFreeColumnPreprocessor (preprocessor.cc:1616-1781) --------------
class DoubletonFreeColumnPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    std::vector<SparseVec> t = lp->Transpose();
    const int32_t num_cols = lp->num_cols();
    for (int32_t dcol = 0; dcol < num_cols; ++dcol) {
      const SparseVec& column = lp->cols[dcol];
      if (column.size() != 2) continue;
      if (lp->col_lb[dcol] != -kInf) continue;
      if (lp->col_ub[dcol] != kInf) continue;
      Restore r;
      r.col = dcol;
      r.cost = lp->obj[dcol];
      int index = 0;
      for (const Entry& e : column) {
        if (del_.IsMarked(e.index)) break;
        r.row[index] = e.index;
        r.coeff[index] = e.coeff;
        ++index;
      }
      if (index != 2) continue;
      if (std::fabs(r.coeff[kDeleted]) < std::fabs(r.coeff[kModified])) {
        std::swap(r.coeff[kDeleted], r.coeff[kModified]);
        std::swap(r.row[kDeleted], r.row[kModified]);
      }
      r.deleted_row.swap(t[r.row[kDeleted]]);
      {
        double new_lb = lp->row_lb[r.row[kDeleted]];
        double new_ub = lp->row_ub[r.row[kDeleted]];
        new_lb /= r.coeff[kDeleted];
        new_ub /= r.coeff[kDeleted];
        if (r.coeff[kDeleted] < 0.0) std::swap(new_lb, new_ub);
        lp->col_lb[r.col] = new_lb;
        lp->col_ub[r.col] = new_ub;
      }
      AddMultipleToSparseVector(r.deleted_row, false, -r.coeff[kModified] / r.coeff[kDeleted],
                                r.col, params_.drop_tolerance, &t[r.row[kModified]]);
      if (r.cost != 0.0) {
        for (const Entry& e : r.deleted_row) {
          const int32_t col = e.index;
          if (col == r.col) continue;
          const double new_obj = lp->obj[col] - e.coeff * r.cost / r.coeff[kDeleted];
          lp->obj[col] = std::fabs(new_obj) > params_.drop_tolerance ? new_obj : 0.0;
        }
      }
      del_.Mark(r.row[kDeleted]);
      stack_.push_back(std::move(r));
    }
    if (!del_.Empty()) {
      lp->cols = TransposeOf(t, num_cols);  // UseTransposeMatrixAsReference
      lp->DeleteRows(del_.Marked());
      return true;
    }
    return false;
  }

  void Recover(Solution* s) const override {
    del_.Restore(s);
    for (auto it = stack_.rbegin(); it != stack_.rend(); ++it) {
      const Restore& r = *it;
      switch (s->vstat[r.col]) {
        case kFixedValue:
          s->cstat[r.row[kDeleted]] = kFixedValue;
          break;
        case kAtUpperBound:
          s->cstat[r.row[kDeleted]] = r.coeff[kDeleted] > 0.0 ? kAtUpperBound : kAtLowerBound;
          break;
        case kAtLowerBound:
          s->cstat[r.row[kDeleted]] = r.coeff[kDeleted] > 0.0 ? kAtLowerBound : kAtUpperBound;
          break;
        case kFree:
          s->cstat[r.row[kDeleted]] = kFree;
          break;
        default:
          break;
      }
      {
        double value = s->primal[r.col];
        for (const Entry& e : r.deleted_row) {
          if (e.index == r.col) continue;
          value -= (e.coeff / r.coeff[kDeleted]) * s->primal[e.index];
        }
        s->primal[r.col] = value;
      }
      if (s->vstat[r.col] != kBasic) {
        s->vstat[r.col] = kBasic;
        const double rc = r.cost - r.coeff[kModified] * s->dual[r.row[kModified]];
        s->dual[r.row[kDeleted]] = rc / r.coeff[kDeleted];
      }
    }
  }

 private:
  enum { kDeleted = 0, kModified = 1 };
  struct Restore {
    int32_t col = 0;
    double cost = 0.0;
    int32_t row[2] = {0, 0};
    double coeff[2] = {0.0, 0.0};
    SparseVec deleted_row;  // the deleted row as a column (entries by column)
  };
  std::vector<Restore> stack_;
  RowDeletion del_;
};

// --- UnconstrainedVariablePreprocessor (preprocessor.cc:1787-2172) ------------
class UnconstrainedVariablePass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    const double low_tolerance = params_.preprocessor_zero_tolerance;
    const double high_tolerance = 1e-4;
    const int32_t num_rows = lp->num_rows;
    const int32_t num_cols = lp->num_cols();
    transpose_ = lp->Transpose();
    dual_lb_.assign(num_rows, -kInf);
    dual_ub_.assign(num_rows, kInf);
    for (int32_t row = 0; row < num_rows; ++row) {
      if (lp->row_lb[row] == -kInf) dual_ub_[row] = 0.0;
      if (lp->row_ub[row] == kInf) dual_lb_[row] = 0.0;
    }
    std::vector<bool> part_lb(num_cols, false), part_ub(num_cols, false);
    std::deque<int32_t> queue;
    std::vector<bool> in_queue(num_cols, true);
    std::vector<int32_t> changed_rows;
    for (int32_t col = 0; col < num_cols; ++col) queue.push_back(col);
    const int64_t limit = 5 * static_cast<int64_t>(num_cols);
    for (int64_t count = 0; !queue.empty() && count < limit; ++count) {
      const int32_t col = queue.front();
      queue.pop_front();
      in_queue[col] = false;
      if (cdel_.IsMarked(col)) continue;
      const SparseVec& column = lp->cols[col];
      const double col_cost = lp->MinCost(col);
      const double col_lb = lp->col_lb[col];
      const double col_ub = lp->col_ub[col];
      SumNegInf rc_lb;
      SumPosInf rc_ub;
      rc_lb.Add(col_cost);
      rc_ub.Add(col_cost);
      for (const Entry& e : column) {
        if (rdel_.IsMarked(e.index)) continue;
        const double coeff = e.coeff;
        if (coeff > 0.0) {
          rc_lb.Add(-coeff * dual_ub_[e.index]);
          rc_ub.Add(-coeff * dual_lb_[e.index]);
        } else {
          rc_lb.Add(-coeff * dual_lb_[e.index]);
          rc_ub.Add(-coeff * dual_ub_[e.index]);
        }
      }
      bool can_be_removed = false;
      double target = 0.0;
      bool rc_away_from_zero = false;
      if (rc_ub.Sum() <= low_tolerance) {
        can_be_removed = true;
        target = col_ub;
        rc_away_from_zero = rc_ub.Sum() <= -high_tolerance;
        can_be_removed = !part_ub[col];
      }
      if (rc_lb.Sum() >= -low_tolerance) {
        if (!can_be_removed || !IsFinite(target)) {
          can_be_removed = true;
          target = col_lb;
          rc_away_from_zero = rc_lb.Sum() >= high_tolerance;
          can_be_removed = !part_lb[col];
        }
      }
      if (can_be_removed) {
        if (IsFinite(target)) {
          cdel_.Mark(col, target, ComputeVariableStatus(target, col_lb, col_ub));
          continue;
        }
        if (rc_away_from_zero) {
          status_ = kInfeasibleOrUnbounded;
          return false;
        }
        if (col_cost != 0.0) continue;
        const double sign_correction = target == kInf ? 1.0 : -1.0;
        bool skip = false;
        for (const Entry& e : column) {
          const double direction = sign_correction * e.coeff;
          const bool blocking = direction > 0.0 ? lp->row_ub[e.index] != kInf
                                                : lp->row_lb[e.index] != -kInf;
          if (blocking) {
            skip = true;
            break;
          }
        }
        if (skip) continue;
        RemoveZeroCostUnconstrainedVariable(col, target, lp);
        continue;
      }
      if (col_lb != -kInf && col_ub != kInf) continue;
      changed_rows.clear();
      for (const Entry& e : column) {
        if (rdel_.IsMarked(e.index)) continue;
        const double c = e.coeff;
        const int32_t row = e.index;
        if (col_ub == kInf) {
          if (c > 0.0) {
            const double candidate = rc_ub.SumWithoutUb(-c * dual_lb_[row]) / c;
            if (candidate < dual_ub_[row]) {
              dual_ub_[row] = candidate;
              part_lb[col] = true;
              changed_rows.push_back(row);
            }
          } else {
            const double candidate = rc_ub.SumWithoutUb(-c * dual_ub_[row]) / c;
            if (candidate > dual_lb_[row]) {
              dual_lb_[row] = candidate;
              part_lb[col] = true;
              changed_rows.push_back(row);
            }
          }
        }
        if (col_lb == -kInf) {
          if (c > 0.0) {
            const double candidate = rc_lb.SumWithoutLb(-c * dual_ub_[row]) / c;
            if (candidate > dual_lb_[row]) {
              dual_lb_[row] = candidate;
              part_ub[col] = true;
              changed_rows.push_back(row);
            }
          } else {
            const double candidate = rc_lb.SumWithoutLb(-c * dual_lb_[row]) / c;
            if (candidate < dual_ub_[row]) {
              dual_ub_[row] = candidate;
              part_ub[col] = true;
              changed_rows.push_back(row);
            }
          }
        }
      }
      for (const int32_t row : changed_rows) {
        for (const Entry& e : transpose_[row]) {
          if (!in_queue[e.index]) {
            queue.push_back(e.index);
            in_queue[e.index] = true;
          }
        }
      }
    }
    const int32_t end = static_cast<int32_t>(cdel_.Marked().size());
    for (int32_t col = 0; col < end; ++col) {
      if (cdel_.IsMarked(col)) {
        SubtractColumnMultipleFromConstraintBound(col, cdel_.StoredValue(col), lp);
      }
    }
    transpose_.clear();
    lp->DeleteColumns(cdel_.Marked());
    lp->DeleteRows(rdel_.Marked());
    return !cdel_.Empty() || !rdel_.Empty();
  }

  void Recover(Solution* s) const override {
    cdel_.Restore(s);
    rdel_.Restore(s);
    struct Del {
      int32_t row, col;
      double coeff;
    };
    std::vector<Del> entries;
    const int32_t num_rows = static_cast<int32_t>(s->dual.size());
    for (int32_t row = 0; row < num_rows; ++row) {
      if (!rdel_.IsMarked(row)) continue;
      int32_t last_col = -1;
      double last_coeff = 0.0;
      for (const Entry& e : rows_saver_.Saved(row)) {
        if (e.index < static_cast<int32_t>(unbounded_.size()) && unbounded_[e.index]) {
          last_col = e.index;
          last_coeff = e.coeff;
        }
      }
      if (last_col != -1) entries.push_back({row, last_col, last_coeff});
    }
    std::sort(entries.begin(), entries.end(), [](const Del& a, const Del& b) {
      if (a.col == b.col) return a.row < b.row;
      return a.col < b.col;
    });
    for (size_t i = 0; i < entries.size();) {
      const int32_t col = entries[i].col;
      double shift = 0.0;
      int32_t row_at_bound = -1;
      for (; i < entries.size(); ++i) {
        if (entries[i].col != col) break;
        const int32_t row = entries[i].row;
        if (!IsFinite(rhs_[row])) continue;
        const double activity = rhs_[row] - ScalarProduct(s->primal, rows_saver_.Saved(row));
        if (activity * sign_[row] < 0.0) {
          const double bound = activity / entries[i].coeff;
          if (std::fabs(bound) > std::fabs(shift)) {
            shift = bound;
            row_at_bound = row;
          }
        }
      }
      s->primal[col] += shift;
      if (row_at_bound != -1) {
        s->vstat[col] = kBasic;
        s->cstat[row_at_bound] = sign_[row_at_bound] == 1.0 ? kAtUpperBound : kAtLowerBound;
      }
    }
  }

 private:
  // preprocessor.cc:1800-1839.
  void RemoveZeroCostUnconstrainedVariable(int32_t col, double target, Lp* lp) {
    if (rhs_.empty()) {
      rhs_.resize(lp->num_rows, 0.0);
      sign_.resize(lp->num_rows, 1.0);
      unbounded_.resize(lp->num_cols(), false);
    }
    const bool unbounded_up = target == kInf;
    for (const Entry& e : lp->cols[col]) {
      const int32_t row = e.index;
      if (!rdel_.IsMarked(row)) {
        rdel_.Mark(row);
        rows_saver_.Save(row, transpose_[row]);
      }
      const bool ub_relevant = e.coeff > 0.0 ? !unbounded_up : unbounded_up;
      sign_[row] = ub_relevant ? 1.0 : -1.0;
      rhs_[row] = ub_relevant ? lp->row_ub[row] : lp->row_lb[row];
    }
    unbounded_[col] = true;
    const double initial = MinInMagnitudeOrZeroIfInfinite(lp->col_lb[col], lp->col_ub[col]);
    cdel_.Mark(col, initial, ComputeVariableStatus(initial, lp->col_lb[col], lp->col_ub[col]));
  }

  ColumnDeletion cdel_;
  RowDeletion rdel_;
  ColumnsSaver rows_saver_;
  std::vector<SparseVec> transpose_;
  std::vector<double> dual_lb_, dual_ub_, rhs_, sign_;
  std::vector<bool> unbounded_;
};

// --- FreeConstraintPreprocessor (preprocessor.cc:2178-2198) ---------------------
class FreeConstraintPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    for (int32_t row = 0; row < lp->num_rows; ++row) {
      if (lp->row_lb[row] == -kInf && lp->row_ub[row] == kInf) del_.Mark(row);
    }
    lp->DeleteRows(del_.Marked());
    return !del_.Empty();
  }
  void Recover(Solution* s) const override { del_.Restore(s); }

 private:
  RowDeletion del_;
};

// --- EmptyConstraintPreprocessor (preprocessor.cc:2204-2246) --------------------
class EmptyConstraintPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    std::vector<int> degree(lp->num_rows, 0);
    for (const SparseVec& col : lp->cols) {
      for (const Entry& e : col) ++degree[e.index];
    }
    for (int32_t row = 0; row < lp->num_rows; ++row) {
      if (degree[row] != 0) continue;
      if (!SmallerWithinFeasibility(lp->row_lb[row], 0) ||
          !SmallerWithinFeasibility(0, lp->row_ub[row])) {
        status_ = kPrimalInfeasible;
        return false;
      }
      del_.Mark(row);
    }
    lp->DeleteRows(del_.Marked());
    return !del_.Empty();
  }
  void Recover(Solution* s) const override { del_.Restore(s); }

 private:
  RowDeletion del_;
};

// --- SingletonPreprocessor (preprocessor.cc:2252-2978) -------------------------
class SingletonPass : public Pass {
 public:
  using Pass::Pass;

  bool Run(Lp* lp) override {
    const std::vector<SparseVec>& matrix = lp->cols;
    const std::vector<SparseVec> transpose = lp->Transpose();
    const int32_t num_cols = lp->num_cols();
    const int32_t num_rows = lp->num_rows;
    std::vector<int64_t> col_degree(num_cols, 0), row_degree(num_rows, 0);
    std::vector<int32_t> col_queue, row_queue;
    for (int32_t col = 0; col < num_cols; ++col) {
      col_degree[col] = static_cast<int64_t>(matrix[col].size());
      if (col_degree[col] == 1) col_queue.push_back(col);
    }
    for (int32_t row = 0; row < num_rows; ++row) {
      row_degree[row] = static_cast<int64_t>(transpose[row].size());
      if (row_degree[row] == 1) row_queue.push_back(row);
    }
    while (status_ == kInit && (!col_queue.empty() || !row_queue.empty())) {
      while (status_ == kInit && !col_queue.empty()) {
        const int32_t col = col_queue.back();
        col_queue.pop_back();
        if (col_degree[col] <= 0) continue;
        const MatrixEntry e = SingletonColumnEntry(col, matrix);
        if (lp->obj[col] == 0.0) {
          DeleteZeroCostSingletonColumn(transpose, e, lp);
        } else {
          if (std::fabs(e.coeff) < params_.preprocessor_zero_tolerance) continue;
          if (MakeConstraintAnEqualityIfPossible(transpose, e, lp)) {
            DeleteSingletonColumnInEquality(transpose, e, lp);
          } else {
            continue;
          }
        }
        --row_degree[e.row];
        if (row_degree[e.row] == 1) row_queue.push_back(e.row);
      }
      while (status_ == kInit && !row_queue.empty()) {
        const int32_t row = row_queue.back();
        row_queue.pop_back();
        if (row_degree[row] <= 0) continue;
        const MatrixEntry e = SingletonRowEntry(row, transpose);
        DeleteSingletonRow(e, lp);
        --col_degree[e.col];
        if (col_degree[e.col] == 1) col_queue.push_back(e.col);
      }
    }
    if (status_ != kInit) return false;
    lp->DeleteColumns(cdel_.Marked());
    lp->DeleteRows(rdel_.Marked());
    return !cdel_.Empty() || !rdel_.Empty();
  }

  void Recover(Solution* s) const override {
    cdel_.Restore(s);
    rdel_.Restore(s);
    for (int i = static_cast<int>(undo_.size()) - 1; i >= 0; --i) {
      const Undo& u = undo_[i];
      const SparseVec& saved_col = cols_saver_.SavedOrEmpty(u.col);
      const SparseVec& saved_row = rows_saver_.SavedOrEmpty(u.row);
      switch (u.type) {
        case kSingletonRow:
          SingletonRowUndo(u, saved_col, s);
          break;
        case kZeroCostSingletonColumn:
          ZeroCostSingletonColumnUndo(u, saved_row, s);
          break;
        case kSingletonColumnInEquality:
          SingletonColumnInEqualityUndo(u, saved_row, s);
          break;
        case kMakeConstraintAnEquality:
          if (s->cstat[u.row] == kFixedValue) s->cstat[u.row] = u.constraint_status;
          break;
      }
    }
  }

 private:
  enum UndoType {
    kSingletonRow,
    kZeroCostSingletonColumn,
    kSingletonColumnInEquality,
    kMakeConstraintAnEquality,
  };
  struct MatrixEntry {
    int32_t row, col;
    double coeff;
  };
  // SingletonUndo (preprocessor.cc:2252-2262): the LP values at push time.
  struct Undo {
    UndoType type;
    bool is_max;
    int32_t row, col;
    double coeff, cost, vlb, vub, clb, cub;
    int8_t constraint_status;
  };
  Undo MakeUndo(UndoType type, const Lp& lp, const MatrixEntry& e, int8_t status) const {
    return {type,          lp.maximize,      e.row,           e.col,
            e.coeff,       lp.obj[e.col],    lp.col_lb[e.col], lp.col_ub[e.col],
            lp.row_lb[e.row], lp.row_ub[e.row], status};
  }

  MatrixEntry SingletonColumnEntry(int32_t col, const std::vector<SparseVec>& matrix) {
    for (const Entry& e : matrix[col]) {
      if (!rdel_.IsMarked(e.index)) return {e.index, col, e.coeff};
    }
    status_ = kAbnormal;
    return {0, 0, 0.0};
  }
  MatrixEntry SingletonRowEntry(int32_t row, const std::vector<SparseVec>& transpose) {
    for (const Entry& e : transpose[row]) {
      if (!cdel_.IsMarked(e.index)) return {row, e.index, e.coeff};
    }
    status_ = kAbnormal;
    return {0, 0, 0.0};
  }

  // preprocessor.cc:2284-2351.
  void DeleteSingletonRow(const MatrixEntry& e, Lp* lp) {
    double implied_lb = lp->row_lb[e.row] / e.coeff;
    double implied_ub = lp->row_ub[e.row] / e.coeff;
    if (e.coeff < 0.0) std::swap(implied_lb, implied_ub);
    const double old_lb = lp->col_lb[e.col];
    const double old_ub = lp->col_ub[e.col];
    const double potential_error = std::fabs(params_.preprocessor_zero_tolerance / e.coeff);
    double new_lb = implied_lb - potential_error > old_lb ? implied_lb : old_lb;
    double new_ub = implied_ub + potential_error < old_ub ? implied_ub : old_ub;
    if (new_ub == -kInf || new_lb == kInf) {
      status_ = kPrimalInfeasible;
      return;
    }
    if (new_ub < new_lb) {
      if (!SmallerWithinFeasibility(new_lb, new_ub)) {
        status_ = kPrimalInfeasible;
        return;
      }
      if (new_lb == lp->col_lb[e.col]) new_ub = new_lb;
      if (new_ub == lp->col_ub[e.col]) new_lb = new_ub;
      new_ub = new_lb;
    }
    rdel_.Mark(e.row);
    undo_.push_back(MakeUndo(kSingletonRow, *lp, e, kFree));
    cols_saver_.SaveIfNotAlreadyDone(e.col, lp->cols[e.col]);
    lp->col_lb[e.col] = new_lb;
    lp->col_ub[e.col] = new_ub;
  }

  // preprocessor.cc:2354-2424.
  static void SingletonRowUndo(const Undo& u, const SparseVec& saved_col, Solution* s) {
    const int8_t status = s->vstat[u.col];
    if (status == kBasic || status == kFree) return;
    double implied_lb = u.clb / u.coeff;
    double implied_ub = u.cub / u.coeff;
    if (u.coeff < 0.0) std::swap(implied_lb, implied_ub);
    const bool lb_changed = implied_lb > u.vlb;
    const bool ub_changed = implied_ub < u.vub;
    if (!lb_changed && !ub_changed) return;
    if (status == kAtLowerBound && !lb_changed) return;
    if (status == kAtUpperBound && !ub_changed) return;
    const double rc = u.cost - ScalarProduct(s->dual, saved_col);
    const double rc_min = u.is_max ? -rc : rc;
    if (status == kFixedValue) {
      if (rc_min >= 0.0 && !lb_changed) {
        s->vstat[u.col] = kAtLowerBound;
        return;
      }
      if (rc_min <= 0.0 && !ub_changed) {
        s->vstat[u.col] = kAtUpperBound;
        return;
      }
    }
    s->dual[u.row] = rc / u.coeff;
    int8_t new_status = status;  // VariableToConstraintStatus
    if (status == kFixedValue && (!lb_changed || !ub_changed)) {
      new_status = lb_changed ? kAtLowerBound : kAtUpperBound;
    }
    if (u.coeff < 0.0) {
      if (new_status == kAtLowerBound) {
        new_status = kAtUpperBound;
      } else if (new_status == kAtUpperBound) {
        new_status = kAtLowerBound;
      }
    }
    s->vstat[u.col] = kBasic;
    s->cstat[u.row] = new_status;
  }

  // preprocessor.cc:2426-2436.
  static void UpdateConstraintBoundsWithVariableBounds(const MatrixEntry& e, Lp* lp) {
    double lower_delta = -e.coeff * lp->col_ub[e.col];
    double upper_delta = -e.coeff * lp->col_lb[e.col];
    if (e.coeff < 0.0) std::swap(lower_delta, upper_delta);
    lp->row_lb[e.row] = lp->row_lb[e.row] + lower_delta;
    lp->row_ub[e.row] = lp->row_ub[e.row] + upper_delta;
  }

  // preprocessor.cc:2479-2488.
  void DeleteZeroCostSingletonColumn(const std::vector<SparseVec>& transpose,
                                     const MatrixEntry& e, Lp* lp) {
    undo_.push_back(MakeUndo(kZeroCostSingletonColumn, *lp, e, kFree));
    rows_saver_.SaveIfNotAlreadyDone(e.row, transpose[e.row]);
    UpdateConstraintBoundsWithVariableBounds(e, lp);
    cdel_.Mark(e.col);
  }

  // preprocessor.cc:2491-2615.
  void ZeroCostSingletonColumnUndo(const Undo& u, const SparseVec& saved_row,
                                   Solution* s) const {
    if (u.vub == u.vlb) {
      s->primal[u.col] = u.vlb;
      s->vstat[u.col] = kFixedValue;
      return;
    }
    const int8_t ct_status = s->cstat[u.row];
    if (ct_status == kFixedValue) {
      const double corrected = u.is_max ? -s->dual[u.row] : s->dual[u.row];
      if (corrected > 0) {
        s->primal[u.col] = u.vlb;
        s->vstat[u.col] = kAtLowerBound;
      } else {
        s->primal[u.col] = u.vub;
        s->vstat[u.col] = kAtUpperBound;
      }
      return;
    } else if (ct_status == kAtLowerBound || ct_status == kAtUpperBound) {
      if ((ct_status == kAtUpperBound && u.coeff > 0.0) ||
          (ct_status == kAtLowerBound && u.coeff < 0.0)) {
        s->primal[u.col] = u.vlb;
        s->vstat[u.col] = kAtLowerBound;
      } else {
        s->primal[u.col] = u.vub;
        s->vstat[u.col] = kAtUpperBound;
      }
      if (u.cub == u.clb) s->cstat[u.row] = kFixedValue;
      return;
    }
    const double activity = ScalarProduct(s->primal, saved_row);
    const double tol = params_.preprocessor_zero_tolerance;
    if (u.vlb != -kInf) {
      const double at_lb = activity + u.coeff * u.vlb;
      if (IsSmallerWithinTolerance(u.clb, at_lb, tol) &&
          IsSmallerWithinTolerance(at_lb, u.cub, tol)) {
        s->primal[u.col] = u.vlb;
        s->vstat[u.col] = kAtLowerBound;
        return;
      }
    }
    if (u.vub != kInf) {
      const double at_ub = activity + u.coeff * u.vub;
      if (IsSmallerWithinTolerance(u.clb, at_ub, tol) &&
          IsSmallerWithinTolerance(at_ub, u.cub, tol)) {
        s->primal[u.col] = u.vub;
        s->vstat[u.col] = kAtUpperBound;
        return;
      }
    }
    if (u.clb == -kInf && u.cub == kInf) {
      s->primal[u.col] = 0.0;
      s->vstat[u.col] = kFree;
      return;
    }
    s->vstat[u.col] = kBasic;
    if (u.clb == u.cub) {
      s->primal[u.col] = (u.clb - activity) / u.coeff;
      s->cstat[u.row] = kFixedValue;
      return;
    }
    bool to_lower;
    if (u.clb == -kInf) {
      to_lower = false;
    } else if (u.cub == kInf) {
      to_lower = true;
    } else {
      const double to_lb = (u.clb - activity) / u.coeff;
      const double to_ub = (u.cub - activity) / u.coeff;
      to_lower = std::max(u.vlb - to_lb, to_lb - u.vub) < std::max(u.vlb - to_ub, to_ub - u.vub);
    }
    if (to_lower) {
      s->primal[u.col] = (u.clb - activity) / u.coeff;
      s->cstat[u.row] = kAtLowerBound;
    } else {
      s->primal[u.col] = (u.cub - activity) / u.coeff;
      s->cstat[u.row] = kAtUpperBound;
    }
  }

  // preprocessor.cc:2617-2657.
  void DeleteSingletonColumnInEquality(const std::vector<SparseVec>& transpose,
                                       const MatrixEntry& e, Lp* lp) {
    const SparseVec& row_as_column = transpose[e.row];
    undo_.push_back(MakeUndo(kSingletonColumnInEquality, *lp, e, kFree));
    rows_saver_.SaveIfNotAlreadyDone(e.row, row_as_column);
    const double rhs = lp->row_ub[e.row];
    const double cost = lp->obj[e.col];
    const double multiplier = cost / e.coeff;
    lp->offset = lp->offset + rhs * multiplier;
    for (const Entry& re : row_as_column) {
      const int32_t col = re.index;
      if (cdel_.IsMarked(col)) continue;
      double new_cost = lp->obj[col] - re.coeff * multiplier;
      if (std::fabs(new_cost) < params_.preprocessor_zero_tolerance) new_cost = 0.0;
      lp->obj[col] = new_cost;
    }
    UpdateConstraintBoundsWithVariableBounds(e, lp);
    cdel_.Mark(e.col);
  }

  // preprocessor.cc:2659-2672.
  void SingletonColumnInEqualityUndo(const Undo& u, const SparseVec& saved_row,
                                     Solution* s) const {
    ZeroCostSingletonColumnUndo(u, saved_row, s);
    s->dual[u.row] += u.cost / u.coeff;
    if (s->cstat[u.row] == kBasic) {
      s->vstat[u.col] = kBasic;
      s->cstat[u.row] = kFixedValue;
    }
  }

  // preprocessor.cc:2681-2833.
  bool MakeConstraintAnEqualityIfPossible(const std::vector<SparseVec>& transpose,
                                          const MatrixEntry& e, Lp* lp) {
    const double cst_lb = lp->row_lb[e.row];
    const double cst_ub = lp->row_ub[e.row];
    if (cst_lb == cst_ub) return true;
    if (cst_lb == -kInf && cst_ub == kInf) return false;
    if (e.row >= static_cast<int32_t>(cached_.size()) || !cached_[e.row]) {
      if (e.row >= static_cast<int32_t>(cached_.size())) {
        cached_.resize(e.row + 1, false);
        row_lb_sum_.resize(e.row + 1);
        row_ub_sum_.resize(e.row + 1);
      }
      cached_[e.row] = true;
      row_lb_sum_[e.row].Add(cst_lb);
      row_ub_sum_[e.row].Add(cst_ub);
      for (const Entry& re : transpose[e.row]) {
        const int32_t col = re.index;
        if (cdel_.IsMarked(col)) continue;
        if (re.coeff > 0.0) {
          row_lb_sum_[e.row].Add(-re.coeff * lp->col_ub[col]);
          row_ub_sum_[e.row].Add(-re.coeff * lp->col_lb[col]);
        } else {
          row_lb_sum_[e.row].Add(-re.coeff * lp->col_lb[col]);
          row_ub_sum_[e.row].Add(-re.coeff * lp->col_ub[col]);
        }
      }
    }
    const double c = e.coeff;
    const double lb = c > 0.0 ? row_lb_sum_[e.row].SumWithoutLb(-c * lp->col_ub[e.col]) / c
                              : row_ub_sum_[e.row].SumWithoutUb(-c * lp->col_ub[e.col]) / c;
    const double ub = c > 0.0 ? row_ub_sum_[e.row].SumWithoutUb(-c * lp->col_lb[e.col]) / c
                              : row_lb_sum_[e.row].SumWithoutLb(-c * lp->col_lb[e.col]) / c;
    const double cost = lp->MinCost(e.col);
    int8_t relaxed = kFixedValue;
    if (cost < 0.0 && SmallerWithinZero(ub, lp->col_ub[e.col])) {
      if (e.coeff > 0) {
        if (cst_ub == kInf) {
          status_ = kInfeasibleOrUnbounded;
        } else {
          relaxed = kAtUpperBound;
          lp->row_lb[e.row] = cst_ub;
          lp->row_ub[e.row] = cst_ub;
        }
      } else {
        if (cst_lb == -kInf) {
          status_ = kInfeasibleOrUnbounded;
        } else {
          relaxed = kAtLowerBound;
          lp->row_lb[e.row] = cst_lb;
          lp->row_ub[e.row] = cst_lb;
        }
      }
      if (status_ == kInfeasibleOrUnbounded) return false;
      lp->col_ub[e.col] = kInf;
    }
    if (cost > 0.0 && SmallerWithinZero(lp->col_lb[e.col], lb)) {
      if (e.coeff > 0) {
        if (cst_lb == -kInf) {
          status_ = kInfeasibleOrUnbounded;
        } else {
          relaxed = kAtLowerBound;
          lp->row_lb[e.row] = cst_lb;
          lp->row_ub[e.row] = cst_lb;
        }
      } else {
        if (cst_ub == kInf) {
          status_ = kInfeasibleOrUnbounded;
        } else {
          relaxed = kAtUpperBound;
          lp->row_lb[e.row] = cst_ub;
          lp->row_ub[e.row] = cst_ub;
        }
      }
      if (status_ == kInfeasibleOrUnbounded) return false;
      lp->col_lb[e.col] = -kInf;
    }
    if (lp->row_lb[e.row] == lp->row_ub[e.row]) {
      undo_.push_back(MakeUndo(kMakeConstraintAnEquality, *lp, e, relaxed));
      return true;
    }
    return false;
  }

  ColumnDeletion cdel_;
  RowDeletion rdel_;
  ColumnsSaver cols_saver_, rows_saver_;
  std::vector<Undo> undo_;
  std::vector<bool> cached_;
  std::vector<SumNegInf> row_lb_sum_;
  std::vector<SumPosInf> row_ub_sum_;
};

// --- SingletonColumnSignPreprocessor (preprocessor.cc:3058-3100) ---------------
class SingletonColumnSignPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    if (lp->num_cols() == 0) return false;
    changed_.clear();
    for (int32_t col = 0; col < lp->num_cols(); ++col) {
      SparseVec& column = lp->cols[col];
      const double cost = lp->obj[col];
      if (column.size() == 1 && column[0].coeff < 0) {
        column[0].coeff *= -1.0;
        const double lb = lp->col_lb[col];
        lp->col_lb[col] = -lp->col_ub[col];
        lp->col_ub[col] = -lb;
        lp->obj[col] = -cost;
        changed_.push_back(col);
      }
    }
    return !changed_.empty();
  }
  void Recover(Solution* s) const override {
    for (const int32_t col : changed_) {
      s->primal[col] = -s->primal[col];
      if (s->vstat[col] == kAtUpperBound) {
        s->vstat[col] = kAtLowerBound;
      } else if (s->vstat[col] == kAtLowerBound) {
        s->vstat[col] = kAtUpperBound;
      }
    }
  }

 private:
  std::vector<int32_t> changed_;
};

// --- DoubletonEqualityRowPreprocessor (preprocessor.cc:3106-3475) --------------
class DoubletonEqualityRowPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    saved_row_lb_ = lp->row_lb;
    saved_row_ub_ = lp->row_ub;
    saved_obj_ = lp->obj;
    const std::vector<SparseVec> original_t = lp->Transpose();
    std::vector<std::pair<int64_t, int32_t>> sorted_rows;
    for (int32_t row = 0; row < lp->num_rows; ++row) {
      const SparseVec& orow = original_t[row];
      if (orow.size() != 2 || lp->row_lb[row] != lp->row_ub[row]) continue;
      int64_t score = 0;
      for (const Entry& e : orow) score += static_cast<int64_t>(lp->cols[e.index].size());
      sorted_rows.push_back({score, row});
    }
    std::sort(sorted_rows.begin(), sorted_rows.end());
    for (const auto& p : sorted_rows) {
      const int32_t row = p.second;
      Restore r;
      int entry_index = 0;
      for (const Entry& e : original_t[row]) {
        if (cdel_.IsMarked(e.index)) continue;
        r.col[entry_index] = e.index;
        r.coeff[entry_index] = e.coeff;
        ++entry_index;
      }
      if (entry_index < 2) continue;
      r.row = row;
      r.rhs = lp->row_lb[row];
      for (int k = 0; k < 2; ++k) {
        r.lb[k] = lp->col_lb[r.col[k]];
        r.ub[k] = lp->col_ub[r.col[k]];
        r.cost[k] = lp->obj[r.col[k]];
      }
      if (r.lb[kDeleted] == r.ub[kDeleted] || r.lb[kModified] == r.ub[kModified]) continue;
      {
        const double carry_over_offset = r.rhs / r.coeff[kModified];
        const double carry_over_factor = -r.coeff[kDeleted] / r.coeff[kModified];
        if (!IsFinite(carry_over_offset) || !IsFinite(carry_over_factor) ||
            carry_over_factor == 0.0) {
          status_ = kAbnormal;
          break;
        }
        double lb = r.lb[kModified];
        double ub = r.ub[kModified];
        double carried_lb = r.lb[kDeleted] * carry_over_factor + carry_over_offset;
        double carried_ub = r.ub[kDeleted] * carry_over_factor + carry_over_offset;
        if (carry_over_factor < 0) std::swap(carried_lb, carried_ub);
        if (carried_lb <= lb) {
          r.at_lb = {kModified, kAtLowerBound, lb};
        } else {
          lb = carried_lb;
          r.at_lb = {kDeleted, carry_over_factor > 0 ? kAtLowerBound : kAtUpperBound,
                     carry_over_factor > 0 ? r.lb[kDeleted] : r.ub[kDeleted]};
        }
        if (carried_ub >= ub) {
          r.at_ub = {kModified, kAtUpperBound, ub};
        } else {
          ub = carried_ub;
          r.at_ub = {kDeleted, carry_over_factor > 0 ? kAtUpperBound : kAtLowerBound,
                     carry_over_factor > 0 ? r.ub[kDeleted] : r.lb[kDeleted]};
        }
        if (SmallerWithinZero(ub, lb)) continue;
        lp->col_lb[r.col[kModified]] = lb;
        lp->col_ub[r.col[kModified]] = ub;
      }
      restore_.push_back(r);
      const double substitution_factor = -r.coeff[kModified] / r.coeff[kDeleted];
      const double constant_offset_factor = r.rhs / r.coeff[kDeleted];
      if (!IsFinite(substitution_factor) || substitution_factor == 0.0 ||
          !IsFinite(constant_offset_factor)) {
        status_ = kAbnormal;
        break;
      }
      for (const int k : {kDeleted, kModified}) {
        saver_.SaveIfNotAlreadyDone(r.col[k], lp->cols[r.col[k]]);
      }
      AddMultipleToSparseVector(lp->cols[r.col[kDeleted]], true, substitution_factor, r.row,
                                params_.drop_tolerance, &lp->cols[r.col[kModified]]);
      {
        const double new_obj = r.cost[kModified] + substitution_factor * r.cost[kDeleted];
        lp->obj[r.col[kModified]] = std::fabs(new_obj) > params_.drop_tolerance ? new_obj : 0.0;
      }
      SubtractColumnMultipleFromConstraintBound(r.col[kDeleted], constant_offset_factor, lp);
      SparseVec().swap(lp->cols[r.col[kDeleted]]);
      cdel_.Mark(r.col[kDeleted]);
      rdel_.Mark(r.row);
    }
    if (status_ != kInit) return false;
    lp->DeleteColumns(cdel_.Marked());
    lp->DeleteRows(rdel_.Marked());
    return !cdel_.Empty();
  }

  void Recover(Solution* s) const override {
    cdel_.Restore(s);
    rdel_.Restore(s);
    const int32_t num_cols = static_cast<int32_t>(s->vstat.size());
    std::vector<bool> new_basic(num_cols, false);
    for (auto it = restore_.rbegin(); it != restore_.rend(); ++it) {
      const Restore& r = *it;
      switch (s->vstat[r.col[kModified]]) {
        case kFixedValue:
          break;
        case kFree:
        case kBasic:
          s->vstat[r.col[kDeleted]] = kBasic;
          new_basic[r.col[kDeleted]] = true;
          break;
        case kAtLowerBound:
        case kAtUpperBound: {
          const Backtrack& bt =
              s->vstat[r.col[kModified]] == kAtLowerBound ? r.at_lb : r.at_ub;
          const int32_t bounded = r.col[bt.choice];
          const int32_t basic = r.col[1 - bt.choice];
          s->vstat[bounded] = bt.status;
          s->primal[bounded] = bt.value;
          s->vstat[basic] = kBasic;
          new_basic[basic] = true;
          break;
        }
        default:
          break;
      }
      if (s->vstat[r.col[kDeleted]] == kBasic) {
        s->primal[r.col[kDeleted]] =
            (r.rhs - s->primal[r.col[kModified]] * r.coeff[kModified]) / r.coeff[kDeleted];
      }
      s->cstat[r.row] = kFixedValue;
    }
    std::vector<std::set<int>> col_to_index(num_cols);
    for (int i = 0; i < static_cast<int>(restore_.size()); ++i) {
      col_to_index[restore_[i].col[kModified]].insert(i);
      col_to_index[restore_[i].col[kDeleted]].insert(i);
    }
    std::vector<int32_t> singleton_col;
    for (int32_t col = 0; col < num_cols; ++col) {
      if (!new_basic[col]) continue;
      if (col_to_index[col].size() == 1) singleton_col.push_back(col);
    }
    while (!singleton_col.empty()) {
      const int32_t col = singleton_col.back();
      singleton_col.pop_back();
      if (!new_basic[col]) continue;
      if (col_to_index[col].empty()) continue;
      const int index = *col_to_index[col].begin();
      const Restore& r = restore_[index];
      const int choice = r.col[kModified] == col ? kModified : kDeleted;
      const SparseVec& saved_col = saver_.Saved(r.col[choice]);
      const double rc = saved_obj_[r.col[choice]] - PreciseScalarProduct(s->dual, saved_col);
      s->dual[r.row] = rc / r.coeff[choice];
      col_to_index[r.col[kDeleted]].erase(index);
      col_to_index[r.col[kModified]].erase(index);
      if (col_to_index[r.col[kDeleted]].size() == 1) singleton_col.push_back(r.col[kDeleted]);
      if (col_to_index[r.col[kModified]].size() == 1) singleton_col.push_back(r.col[kModified]);
    }
    // FixConstraintWithFixedStatuses (preprocessor.cc:3455-3475).
    const int32_t num_rows = static_cast<int32_t>(s->cstat.size());
    for (int32_t row = 0; row < num_rows; ++row) {
      if (s->cstat[row] != kFixedValue) continue;
      if (saved_row_lb_[row] == saved_row_ub_[row]) continue;
      s->cstat[row] = s->dual[row] > 0 ? kAtLowerBound : kAtUpperBound;
    }
  }

 private:
  enum { kDeleted = 0, kModified = 1 };
  struct Backtrack {
    int choice = kDeleted;
    int8_t status = kBasic;
    double value = 0.0;
  };
  struct Restore {
    int32_t row = 0;
    double rhs = 0.0;
    int32_t col[2] = {0, 0};
    double coeff[2] = {0.0, 0.0}, lb[2] = {0.0, 0.0}, ub[2] = {0.0, 0.0},
           cost[2] = {0.0, 0.0};
    Backtrack at_lb, at_ub;
  };
  ColumnDeletion cdel_;
  RowDeletion rdel_;
  std::vector<Restore> restore_;
  std::vector<double> saved_row_lb_, saved_row_ub_, saved_obj_;
  ColumnsSaver saver_;
};

// --- DualizerPreprocessor (preprocessor.cc:3491-3734) --------------------------
class DualizerPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    if (params_.solve_dual_problem == 1) return false;  // NEVER_DO
    primal_cols_ = lp->num_cols();
    primal_rows_ = lp->num_rows;
    primal_max_ = lp->maximize;
    if (params_.solve_dual_problem == 2) {  // LET_SOLVER_DECIDE
      if (1.0 * primal_rows_ < params_.dualizer_threshold * primal_cols_) return false;
    }
    const int32_t num_cols = lp->num_cols();
    lbs_.assign(num_cols, 0.0);
    ubs_.assign(num_cols, 0.0);
    for (int32_t col = 0; col < num_cols; ++col) {
      const double lower = lp->col_lb[col];
      const double upper = lp->col_ub[col];
      lbs_[col] = lower;
      ubs_[col] = upper;
      const double value = MinInMagnitudeOrZeroIfInfinite(lower, upper);
      if (value != 0.0) {
        lp->col_lb[col] = lower - value;
        lp->col_ub[col] = upper - value;
        SubtractColumnMultipleFromConstraintBound(col, value, lp);
      }
    }
    correspondence_.clear();
    for (int32_t row = 0; row < primal_rows_; ++row) {
      const double lb = lp->row_lb[row];
      const double ub = lp->row_ub[row];
      if (lb == ub) {
        correspondence_.push_back(kFixedValue);
      } else if (ub != kInf) {
        correspondence_.push_back(kAtUpperBound);
      } else if (lb != -kInf) {
        correspondence_.push_back(kAtLowerBound);
      } else {
        correspondence_.push_back(kFree);  // no free rows reach this pass
      }
    }
    slack_mapping_.clear();
    for (int32_t col = 0; col < primal_cols_; ++col) {
      if (lp->col_lb[col] != -kInf) {
        correspondence_.push_back(lp->col_ub[col] == lp->col_lb[col] ? kFixedValue
                                                                     : kAtLowerBound);
        slack_mapping_.push_back(col);
      }
    }
    for (int32_t col = 0; col < primal_cols_; ++col) {
      if (lp->col_ub[col] != kInf) {
        correspondence_.push_back(lp->col_ub[col] == lp->col_lb[col] ? kFixedValue
                                                                     : kAtUpperBound);
        slack_mapping_.push_back(col);
      }
    }
    Lp dual = PopulateFromDual(*lp);
    *lp = std::move(dual);
    return true;
  }

  void Recover(Solution* s) const override {
    std::vector<double> primal(primal_cols_, 0.0);
    std::vector<int8_t> vstat(primal_cols_, kFree);
    for (int32_t col = 0; col < primal_cols_; ++col) {
      const int32_t row = col;
      const double lower = lbs_[col];
      const double upper = ubs_[col];
      const double shift = MinInMagnitudeOrZeroIfInfinite(lower, upper);
      primal[col] = s->dual[row] + shift;
      if (s->cstat[row] != kBasic) {
        vstat[col] = kBasic;
      } else {
        vstat[col] = ComputeVariableStatus(shift, lower, upper);
      }
    }
    const int32_t begin = primal_rows_;
    const int32_t end = static_cast<int32_t>(correspondence_.size());
    for (int32_t index = begin; index < end; ++index) {
      if (s->vstat[index] == kBasic) {
        const int32_t col = slack_mapping_[index - begin];
        const int8_t status = correspondence_[index];
        vstat[col] = status;
        if (status == kAtUpperBound || status == kFixedValue) {
          primal[col] = ubs_[col];
        } else {
          primal[col] = lbs_[col];
        }
      }
    }
    std::vector<double> dual(primal_rows_, 0.0);
    std::vector<int8_t> cstat(primal_rows_, kFree);
    const double sign = primal_max_ ? -1 : 1;
    for (int32_t row = 0; row < primal_rows_; ++row) {
      const int32_t col = row;
      dual[row] = sign * s->primal[col];
      if (s->vstat[col] != kBasic) {
        cstat[row] = kBasic;
        if (duplicated_[row] != -1 && s->vstat[duplicated_[row]] == kBasic) {
          cstat[row] = kAtLowerBound;
        }
      } else {
        cstat[row] = correspondence_[col];
      }
      if (duplicated_[row] != -1) dual[row] += sign * s->primal[duplicated_[row]];
    }
    switch (s->status) {
      case kPrimalInfeasible: s->status = kDualInfeasible; break;
      case kDualInfeasible: s->status = kPrimalInfeasible; break;
      case kPrimalUnbounded: s->status = kDualUnbounded; break;
      case kDualUnbounded: s->status = kPrimalUnbounded; break;
      case kPrimalFeasible: s->status = kDualFeasible; break;
      case kDualFeasible: s->status = kPrimalFeasible; break;
      default: break;
    }
    s->primal.swap(primal);
    s->dual.swap(dual);
    s->vstat.swap(vstat);
    s->cstat.swap(cstat);
  }

 private:
  // LinearProgram::PopulateFromDual (lp_data.cc:766-862).
  Lp PopulateFromDual(const Lp& p) {
    Lp d;
    d.maximize = true;
    d.offset = p.offset;
    d.scale = p.scale;
    d.num_rows = p.num_cols();
    for (int32_t prow = 0; prow < p.num_rows; ++prow) {
      const double lb = p.row_lb[prow];
      const double ub = p.row_ub[prow];
      if (lb == ub) {
        d.AddColumn(-kInf, kInf, lb);
      } else if (ub != kInf) {
        d.AddColumn(-kInf, 0.0, ub);
      } else {
        d.AddColumn(0.0, kInf, lb);
      }
    }
    for (int32_t pcol = 0; pcol < p.num_cols(); ++pcol) {
      if (p.col_lb[pcol] != -kInf) {
        const int32_t col = d.AddColumn(0.0, kInf, p.col_lb[pcol]);
        d.cols[col].push_back({pcol, 1.0});
      }
    }
    for (int32_t pcol = 0; pcol < p.num_cols(); ++pcol) {
      if (p.col_ub[pcol] != kInf) {
        const int32_t col = d.AddColumn(-kInf, 0.0, p.col_ub[pcol]);
        d.cols[col].push_back({pcol, 1.0});
      }
    }
    d.row_lb.assign(d.num_rows, 0.0);
    d.row_ub.assign(d.num_rows, 0.0);
    for (int32_t pcol = 0; pcol < p.num_cols(); ++pcol) {
      const double bound = p.MinCost(pcol);
      d.row_lb[pcol] = bound;
      d.row_ub[pcol] = bound;
      for (const Entry& e : p.cols[pcol]) d.cols[e.index].push_back({pcol, e.coeff});
    }
    duplicated_.assign(p.num_rows, -1);
    for (int32_t prow = 0; prow < p.num_rows; ++prow) {
      const double lb = p.row_lb[prow];
      const double ub = p.row_ub[prow];
      const bool free_or_boxed =
          (lb == -kInf && ub == kInf) || (lb != -kInf && ub != kInf && lb != ub);
      if (free_or_boxed) {
        const int32_t col = d.AddColumn(0.0, kInf, lb);
        d.cols[col] = d.cols[prow];
        duplicated_[prow] = col;
      }
    }
    return d;
  }

  int32_t primal_cols_ = 0, primal_rows_ = 0;
  bool primal_max_ = false;
  std::vector<double> lbs_, ubs_;
  std::vector<int8_t> correspondence_;
  std::vector<int32_t> slack_mapping_, duplicated_;
};

// --- ShiftVariableBoundsPreprocessor (preprocessor.cc:3740-3849) --------------
class ShiftVariableBoundsPass : public Pass {
 public:
  using Pass::Pass;
  bool Run(Lp* lp) override {
    bool all_contain_zero = true;
    const int32_t num_cols = lp->num_cols();
    init_lbs_.assign(num_cols, 0.0);
    init_ubs_.assign(num_cols, 0.0);
    for (int32_t col = 0; col < num_cols; ++col) {
      init_lbs_[col] = lp->col_lb[col];
      init_ubs_[col] = lp->col_ub[col];
      if (0.0 < init_lbs_[col] || 0.0 > init_ubs_[col]) all_contain_zero = false;
    }
    if (all_contain_zero) return false;
    std::vector<KahanSum> row_offsets(lp->num_rows);
    KahanSum obj_offset;
    offsets_.assign(num_cols, 0.0);
    for (int32_t col = 0; col < num_cols; ++col) {
      if (0.0 < init_lbs_[col] || 0.0 > init_ubs_[col]) {
        const double offset = MinInMagnitudeOrZeroIfInfinite(init_lbs_[col], init_ubs_[col]);
        offsets_[col] = offset;
        lp->col_lb[col] = init_lbs_[col] - offset;
        lp->col_ub[col] = init_ubs_[col] - offset;
        for (const Entry& e : lp->cols[col]) row_offsets[e.index].Add(e.coeff * offset);
        obj_offset.Add(lp->obj[col] * offset);
      }
    }
    for (int32_t row = 0; row < lp->num_rows; ++row) {
      if (!std::isfinite(row_offsets[row].Value())) {
        status_ = kInvalidProblem;
        return false;
      }
      lp->row_lb[row] = lp->row_lb[row] - row_offsets[row].Value();
      lp->row_ub[row] = lp->row_ub[row] - row_offsets[row].Value();
    }
    if (!std::isfinite(obj_offset.Value())) {
      status_ = kInvalidProblem;
      return false;
    }
    lp->offset = lp->offset + obj_offset.Value();
    return true;
  }
  void Recover(Solution* s) const override {
    const int32_t num_cols = static_cast<int32_t>(s->vstat.size());
    for (int32_t col = 0; col < num_cols; ++col) {
      switch (s->vstat[col]) {
        case kFixedValue:
        case kAtLowerBound:
          s->primal[col] = init_lbs_[col];
          break;
        case kAtUpperBound:
          s->primal[col] = init_ubs_[col];
          break;
        case kBasic:
          s->primal[col] += offsets_[col];
          break;
        default:
          break;
      }
    }
  }

 private:
  std::vector<double> init_lbs_, init_ubs_, offsets_;
};

}  // namespace

// --- MainLpPreprocessor (preprocessor.cc:76-209) --------------------------------
MainPresolve::MainPresolve(const Params& p) : params_(p) {}
MainPresolve::~MainPresolve() = default;

void MainPresolve::RunPass(std::unique_ptr<Pass> pass, const char* name, Lp* lp) {
  if (status_ != kInit) return;
  if (lp->num_cols() == 0 && lp->num_rows == 0) {
    status_ = kOptimal;
    return;
  }
  if (pass->Run(lp)) {
    status_ = pass->status();
    stack_.push_back(std::move(pass));
    applied_.push_back(name);
  } else {
    status_ = pass->status();
  }
}

bool MainPresolve::Run(Lp* lp) {
  if (params_.use_preprocessing) {
    RunPass(std::make_unique<ShiftVariableBoundsPass>(params_), "ShiftVariableBounds", lp);
    const int kMaxNumPasses = 20;
    for (int i = 0; i < kMaxNumPasses; ++i) {
      const size_t old_size = stack_.size();
      RunPass(std::make_unique<FixedVariablePass>(params_), "FixedVariable", lp);
      RunPass(std::make_unique<SingletonPass>(params_), "Singleton", lp);
      RunPass(std::make_unique<ForcingAndImpliedFreePass>(params_),
              "ForcingAndImpliedFreeConstraint", lp);
      RunPass(std::make_unique<FreeConstraintPass>(params_), "FreeConstraint", lp);
      RunPass(std::make_unique<ImpliedFreePass>(params_), "ImpliedFree", lp);
      RunPass(std::make_unique<UnconstrainedVariablePass>(params_), "UnconstrainedVariable",
              lp);
      RunPass(std::make_unique<DoubletonFreeColumnPass>(params_), "DoubletonFreeColumn", lp);
      RunPass(std::make_unique<DoubletonEqualityRowPass>(params_), "DoubletonEqualityRow", lp);
      if (stack_.size() == old_size) break;
    }
    RunPass(std::make_unique<EmptyColumnPass>(params_), "EmptyColumn", lp);
    RunPass(std::make_unique<EmptyConstraintPass>(params_), "EmptyConstraint", lp);
    RunPass(std::make_unique<ProportionalColumnPass>(params_), "ProportionalColumn", lp);
    RunPass(std::make_unique<ProportionalRowPass>(params_), "ProportionalRow", lp);
    const size_t old_size = stack_.size();
    RunPass(std::make_unique<DualizerPass>(params_), "Dualizer", lp);
    if (old_size != stack_.size()) {
      RunPass(std::make_unique<SingletonPass>(params_), "Singleton", lp);
      RunPass(std::make_unique<FreeConstraintPass>(params_), "FreeConstraint", lp);
      RunPass(std::make_unique<UnconstrainedVariablePass>(params_), "UnconstrainedVariable",
              lp);
      RunPass(std::make_unique<EmptyColumnPass>(params_), "EmptyColumn", lp);
      RunPass(std::make_unique<EmptyConstraintPass>(params_), "EmptyConstraint", lp);
    }
    RunPass(std::make_unique<SingletonColumnSignPass>(params_), "SingletonColumnSign", lp);
  }
  return !stack_.empty();
}

void MainPresolve::Recover(Solution* s) {
  while (!stack_.empty()) {
    stack_.back()->Recover(s);
    stack_.pop_back();
  }
}

}  // namespace presolve
}  // namespace milp
