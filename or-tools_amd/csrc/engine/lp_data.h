// Host-side sparse data structures of the MI355X simplex engine.
//
// The engine keeps Glop's exact data model (OR-Tools 9.7 lp_data/): the
// constraint matrix [A | I] as CompactSparseMatrix, ScatteredVector for
// FTRAN/BTRAN results, bitsets for the variable classes. Keeping the same
// representation rules (dense/sparse switches, non-zero list order) is what
// lets the device kernels reproduce Glop's floating-point order exactly.
// Each piece cites the reference file:line it follows (paths relative to
// /root/reference/ortools).
#ifndef MILP_LP_DATA_H_
#define MILP_LP_DATA_H_

#include "host_pool.h"
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <utility>
#include <vector>

namespace milp {

// Host bridge of the device dual segment (csrc/sdual/sdual_bridge.inc).
struct SdualBridge;
struct SdualHooks;

using Fractional = double;
using RowIndex = int32_t;
using ColIndex = int32_t;
using EntryIndex = int64_t;

constexpr RowIndex kInvalidRow = -1;
constexpr ColIndex kInvalidCol = -1;
constexpr RowIndex kNonPivotal = -1;
constexpr double kInfinity = std::numeric_limits<double>::infinity();

// lp_utils.h:38
inline Fractional Square(Fractional f) { return f * f; }
// lp_types.h:421-424
inline double DeterministicTimeForFpOperations(int64_t n) {
  return 2e-9 * static_cast<double>(n);
}
// lp_types.h IsFinite(): value > -inf && value < inf.
inline bool IsFinite(Fractional v) { return v > -kInfinity && v < kInfinity; }

// lp_types.h:106-168
enum class ProblemStatus : int8_t {
  OPTIMAL,
  PRIMAL_INFEASIBLE,
  DUAL_INFEASIBLE,
  INFEASIBLE_OR_UNBOUNDED,
  PRIMAL_UNBOUNDED,
  DUAL_UNBOUNDED,
  INIT,
  PRIMAL_FEASIBLE,
  DUAL_FEASIBLE,
  ABNORMAL,
  INVALID_PROBLEM,
  IMPRECISE,
};
enum class VariableType : int8_t {
  UNCONSTRAINED,
  LOWER_BOUNDED,
  UPPER_BOUNDED,
  UPPER_AND_LOWER_BOUNDED,
  FIXED_VARIABLE
};
enum class VariableStatus : int8_t {
  BASIC,
  FIXED_VALUE,
  AT_LOWER_BOUND,
  AT_UPPER_BOUND,
  FREE,
};

// glop/status.h:29-44
struct Status {
  enum ErrorCode {
    GLOP_OK = 0,
    ERROR_LU = 1,
    ERROR_BOUND = 2,
    ERROR_NULL = 3,
    ERROR_INVALID_PROBLEM = 4
  };
  ErrorCode code = GLOP_OK;
  const char* msg = "";
  Status() = default;
  Status(ErrorCode c, const char* m) : code(c), msg(m) {}
  static Status OK() { return Status(); }
  bool ok() const { return code == GLOP_OK; }
};
#define MILP_RETURN_IF_ERROR(x)   \
  do {                              \
    const ::milp::Status _s = (x); \
    if (!_s.ok()) return _s;        \
  } while (0)

// util/bitset.h:413 Bitset64: iteration visits set positions in increasing
// order.
class Bitset {
 public:
  void ClearAndResize(int n) {
    size_ = n;
    w_.assign((n + 63) / 64, 0);
  }
  void Resize(int n) {
    w_.resize((n + 63) / 64, 0);
    if (n < size_ && (n & 63)) w_[n >> 6] &= (~0ull >> (64 - (n & 63)));
    size_ = n;
  }
  int size() const { return size_; }
  bool IsSet(int i) const { return (w_[i >> 6] >> (i & 63)) & 1; }
  bool operator[](int i) const { return IsSet(i); }
  void Set(int i) { w_[i >> 6] |= (1ull << (i & 63)); }
  void Clear(int i) { w_[i >> 6] &= ~(1ull << (i & 63)); }
  void Set(int i, bool v) {
    if (v) Set(i); else Clear(i);
  }
  void Intersection(const Bitset& o) {
    const size_t k = std::min(w_.size(), o.w_.size());
    for (size_t i = 0; i < k; ++i) w_[i] &= o.w_[i];
    for (size_t i = k; i < w_.size(); ++i) w_[i] = 0;
  }
  uint64_t Word(int b) const { return w_[b]; }
  const uint64_t* data() const { return w_.data(); }
  uint64_t* mutable_data() { return w_.data(); }
  int NumWords() const { return static_cast<int>(w_.size()); }
  template <typename F>
  void ForEach(F&& f) const {
    const int nb = static_cast<int>(w_.size());
    for (int b = 0; b < nb; ++b) {
      uint64_t word = w_[b];
      while (word) {
        const int t = __builtin_ctzll(word);
        const int i = b * 64 + t;
        if (i >= size_) return;
        f(i);
        word &= word - 1;
      }
    }
  }
  std::vector<int> ToVector() const {
    std::vector<int> v;
    ForEach([&](int i) { v.push_back(i); });
    return v;
  }
  // util/bitset.h:629-640
  bool ConditionalXorOfTwoBits(int i, bool use1, const Bitset& set1, bool use2,
                               const Bitset& set2) const {
    return ((use1 && set1.IsSet(i)) != (use2 && set2.IsSet(i)));
  }

 private:
  int size_ = 0;
  std::vector<uint64_t> w_;
};

// lp_data/scattered_vector.h:61-177
struct ScatteredVector {
  std::vector<Fractional> values;
  bool non_zeros_are_sorted = false;
  std::vector<int> non_zeros;
  std::vector<char> is_non_zero;
  static constexpr double kDefaultRatioForUsingDenseIteration = 0.8;

  Fractional operator[](int i) const { return values[i]; }
  Fractional& operator[](int i) { return values[i]; }
  int size() const { return static_cast<int>(values.size()); }

  void Add(int index, Fractional value) {
    values[index] += value;
    if (!is_non_zero[index] && value != 0.0) {
      is_non_zero[index] = true;
      non_zeros.push_back(index);
      non_zeros_are_sorted = false;
    }
  }
  void SortNonZerosIfNeeded() {
    if (!non_zeros_are_sorted) {
      std::sort(non_zeros.begin(), non_zeros.end());
      non_zeros_are_sorted = true;
    }
  }
  bool ShouldUseDenseIteration(double ratio) const {
    if (non_zeros.empty()) return true;
    return static_cast<double>(non_zeros.size()) >
           ratio * static_cast<double>(values.size());
  }
  bool ShouldUseDenseIteration() const {
    return ShouldUseDenseIteration(kDefaultRatioForUsingDenseIteration);
  }
  void ClearSparseMask() {
    if (ShouldUseDenseIteration()) {
      is_non_zero.assign(values.size(), false);
    } else {
      is_non_zero.resize(values.size(), false);
      for (const int i : non_zeros) is_non_zero[i] = false;
    }
  }
  void RepopulateSparseMask() {
    ClearSparseMask();
    for (const int i : non_zeros) is_non_zero[i] = true;
  }
  void ClearNonZerosIfTooDense(double ratio) {
    if (ShouldUseDenseIteration(ratio)) {
      ClearSparseMask();
      non_zeros.clear();
    }
  }
  void ClearNonZerosIfTooDense() {
    ClearNonZerosIfTooDense(kDefaultRatioForUsingDenseIteration);
  }
  size_t NumNonZerosEstimate() const {
    return non_zeros.empty() ? values.size() : non_zeros.size();
  }
};

// lp_utils.h:281-299
inline void ClearAndResizeVectorWithNonZeros(int size, ScatteredVector* v) {
  const double kSparseThreshold = 0.05;
  if (!v->non_zeros.empty() &&
      v->non_zeros.size() < kSparseThreshold * size) {
    for (const int index : v->non_zeros) v->values[index] = 0.0;
    v->values.resize(size, 0.0);
  } else if (size >= (1 << 16) && static_cast<int>(v->values.size()) == size) {
    // A long dense vector: zeroed by the host pool (the same bits).
    double* p = v->values.data();
    ParallelRanges(size, 1 << 16, 4096, [p](int, int64_t b, int64_t e) {
      std::fill(p + b, p + e, 0.0);
    });
  } else {
    v->values.assign(size, 0.0);
  }
  v->non_zeros.clear();
}

// lp_utils.h:54-76 (dense, blocked by 4)
inline Fractional ScalarProduct(const std::vector<Fractional>& u,
                                const std::vector<Fractional>& v) {
  Fractional sum = 0.0;
  size_t i = 0;
  const size_t num_blocks = u.size() / 4;
  for (size_t b = 0; b < num_blocks; ++b) {
    sum += (u[i] * v[i]) + (u[i + 1] * v[i + 1]) + (u[i + 2] * v[i + 2]) +
           (u[i + 3] * v[i + 3]);
    i += 4;
  }
  while (i < u.size()) {
    sum += u[i] * v[i];
    ++i;
  }
  return sum;
}
// lp_utils.h:92-103
inline Fractional ScalarProduct(const std::vector<Fractional>& u,
                                const ScatteredVector& v) {
  if (v.ShouldUseDenseIteration()) return ScalarProduct(u, v.values);
  Fractional sum = 0.0;
  for (const int i : v.non_zeros) sum += (u[i] * v.values[i]);
  return sum;
}
// lp_utils.cc:62-75
inline Fractional SquaredNorm(const std::vector<Fractional>& c) {
  Fractional sum = 0.0;
  size_t r = 0;
  const size_t num_blocks = c.size() / 4;
  for (size_t b = 0; b < num_blocks; ++b) {
    sum += Square(c[r]) + Square(c[r + 1]) + Square(c[r + 2]) +
           Square(c[r + 3]);
    r += 4;
  }
  while (r < c.size()) {
    sum += Square(c[r]);
    ++r;
  }
  return sum;
}
// lp_utils.cc:46-54
inline Fractional SquaredNorm(const ScatteredVector& v) {
  if (v.ShouldUseDenseIteration()) return SquaredNorm(v.values);
  Fractional sum = 0.0;
  for (const int i : v.non_zeros) sum += Square(v.values[i]);
  return sum;
}
// base/accurate_sum.h:23-40 (Kahan)
struct KahanSum {
  Fractional sum = 0.0, err = 0.0;
  void Add(Fractional value) {
    err += value;
    const Fractional new_sum = sum + err;
    err += sum - new_sum;
    sum = new_sum;
  }
  Fractional Value() const { return sum; }
};
// lp_utils.h:106-114
inline Fractional PreciseScalarProduct(const std::vector<Fractional>& u,
                                       const std::vector<Fractional>& v) {
  KahanSum s;
  for (size_t i = 0; i < u.size(); ++i) s.Add(u[i] * v[i]);
  return s.Value();
}
// lp_utils.cc:83-89
inline Fractional InfinityNorm(const std::vector<Fractional>& v) {
  Fractional n = 0.0;
  for (const Fractional x : v) n = std::max(n, std::fabs(x));
  return n;
}

// A read-only view of one column (lp_data/sparse_column.h ColumnView).
struct ColumnView {
  const int* rows = nullptr;
  const Fractional* coefs = nullptr;
  int64_t n = 0;
  int64_t num_entries() const { return n; }
  bool IsEmpty() const { return n == 0; }
  int GetFirstRow() const { return rows[0]; }
  Fractional GetFirstCoefficient() const { return coefs[0]; }
};
inline Fractional SquaredNorm(const ColumnView& c) {  // lp_utils.cc:22-29
  Fractional sum = 0.0;
  for (int64_t i = 0; i < c.n; ++i) sum += Square(c.coefs[i]);
  return sum;
}

// lp_data/sparse_vector.h SparseVector<RowIndex> (subset used by Markowitz).
struct SparseColumn {
  std::vector<int> rows;
  std::vector<Fractional> coefs;
  bool may_contain_duplicates = false;

  int64_t num_entries() const { return static_cast<int64_t>(rows.size()); }
  bool IsEmpty() const { return rows.empty(); }
  void Clear() {
    rows.clear();
    coefs.clear();
    may_contain_duplicates = false;
  }
  void Reserve(int64_t n) {
    rows.reserve(n);
    coefs.reserve(n);
  }
  void AddEntry(int r, Fractional v) {
    rows.push_back(r);
    coefs.push_back(v);
  }
  void SetCoefficient(int r, Fractional v) {  // sparse_vector.h:687-691
    AddEntry(r, v);
    may_contain_duplicates = true;
  }
  int GetFirstRow() const { return rows[0]; }
  Fractional GetFirstCoefficient() const { return coefs[0]; }
  ColumnView view() const {
    return ColumnView{rows.data(), coefs.data(), num_entries()};
  }
  // sparse_vector.h:546-580: entries sorted by row (stable), zeros
  // dropped, of equal rows only the last kept. Already strictly increasing
  // rows need no sort; long columns use a stable LSD radix sort on the row,
  // which orders exactly as the stable comparison sort does.
  void CleanUp() {
    const size_t n = rows.size();
    bool sorted = true;
    for (size_t i = 1; i < n; ++i) {
      if (rows[i] <= rows[i - 1]) {
        sorted = false;
        break;
      }
    }
    if (!sorted) {
      if (n >= 256) {
        RadixSortByRow();
      } else {
        std::vector<std::pair<int, Fractional>> e;
        e.reserve(n);
        for (size_t i = 0; i < n; ++i) e.emplace_back(rows[i], coefs[i]);
        std::stable_sort(e.begin(), e.end(),
                         [](const std::pair<int, Fractional>& a,
                            const std::pair<int, Fractional>& b) {
                           return a.first < b.first;
                         });
        for (size_t i = 0; i < n; ++i) {
          rows[i] = e[i].first;
          coefs[i] = e[i].second;
        }
      }
    }
    size_t new_size = 0;
    for (size_t i = 0; i < n; ++i) {
      if (coefs[i] == 0.0) continue;
      if (i + 1 == n || rows[i] != rows[i + 1]) {
        rows[new_size] = rows[i];
        coefs[new_size] = coefs[i];
        ++new_size;
      }
    }
    rows.resize(new_size);
    coefs.resize(new_size);
    may_contain_duplicates = false;
  }
  void RadixSortByRow() {
    constexpr int kBits = 11;
    constexpr int kBuckets = 1 << kBits;
    const size_t n = rows.size();
    int max_row = 0;
    for (size_t i = 0; i < n; ++i) max_row = std::max(max_row, rows[i]);
    static thread_local std::vector<int> tmp_rows;
    static thread_local std::vector<Fractional> tmp_coefs;
    tmp_rows.resize(n);
    tmp_coefs.resize(n);
    size_t count[kBuckets];
    for (int shift = 0; shift == 0 || (max_row >> shift) != 0; shift += kBits) {
      std::fill(count, count + kBuckets, size_t{0});
      for (size_t i = 0; i < n; ++i) ++count[(rows[i] >> shift) & (kBuckets - 1)];
      size_t sum = 0;
      for (int b = 0; b < kBuckets; ++b) {
        const size_t c = count[b];
        count[b] = sum;
        sum += c;
      }
      for (size_t i = 0; i < n; ++i) {
        const size_t dst = count[(rows[i] >> shift) & (kBuckets - 1)]++;
        tmp_rows[dst] = rows[i];
        tmp_coefs[dst] = coefs[i];
      }
      rows.swap(tmp_rows);
      coefs.swap(tmp_coefs);
    }
  }
  // sparse_vector.h:956-984
  void MoveTaggedEntriesTo(const std::vector<int>& index_perm,
                           SparseColumn* output) {
    const int64_t end = num_entries();
    int64_t i = 0;
    while (true) {
      if (i >= end) return;
      if (index_perm[rows[i]] >= 0) break;
      ++i;
    }
    output->AddEntry(rows[i], coefs[i]);
    for (int64_t j = i + 1; j < end; ++j) {
      if (index_perm[rows[j]] < 0) {
        rows[i] = rows[j];
        coefs[i] = coefs[j];
        ++i;
      } else {
        output->AddEntry(rows[j], coefs[j]);
      }
    }
    rows.resize(i);
    coefs.resize(i);
    output->may_contain_duplicates = true;
  }
  // sparse_vector.h:986-998
  Fractional LookUpCoefficient(int index) const {
    Fractional value = 0.0;
    for (size_t i = 0; i < rows.size(); ++i)
      if (rows[i] == index) value = coefs[i];
    return value;
  }
};

// lp_data/sparse.h:291-512 CompactSparseMatrix.
class CompactSparseMatrix {
 public:
  int num_rows() const { return num_rows_; }
  int num_cols() const { return num_cols_; }
  int64_t num_entries() const { return static_cast<int64_t>(coefficients_.size()); }
  bool IsEmpty() const { return coefficients_.empty(); }
  ColumnView column(int col) const {
    const int64_t s = starts_[col];
    return ColumnView{rows_.data() + s, coefficients_.data() + s,
                      starts_[col + 1] - s};
  }
  int64_t ColumnNumEntries(int col) const {
    return starts_[col + 1] - starts_[col];
  }
  bool ColumnIsEmpty(int col) const { return starts_[col + 1] == starts_[col]; }

  // sparse.cc:462-487
  void PopulateFromSparseMatrixAndAddSlacks(int m, int n, const int64_t* cs,
                                            const int32_t* ri,
                                            const double* vals) {
    num_cols_ = n + m;
    num_rows_ = m;
    const int64_t nnz = cs[n] - cs[0];
    starts_.assign(num_cols_ + 1, 0);
    coefficients_.assign(nnz + m, 0.0);
    rows_.assign(nnz + m, 0);
    int64_t index = 0;
    for (int col = 0; col < n; ++col) {
      starts_[col] = index;
      for (int64_t k = cs[col]; k < cs[col + 1]; ++k) {
        coefficients_[index] = vals[k];
        rows_[index] = ri[k];
        ++index;
      }
    }
    for (int row = 0; row < m; ++row) {
      starts_[n + row] = index;
      coefficients_[index] = 1.0;
      rows_[index] = row;
      ++index;
    }
    starts_[num_cols_] = index;
  }
  // sparse.cc:489-528
  void PopulateFromTranspose(const CompactSparseMatrix& input) {
    num_cols_ = input.num_rows();
    num_rows_ = input.num_cols();
    starts_.assign(num_cols_ + 2, 0);
    for (const int row : input.rows_) ++starts_[row + 2];
    for (size_t c = 2; c < starts_.size(); ++c) starts_[c] += starts_[c - 1];
    coefficients_.resize(starts_.back(), 0.0);
    rows_.resize(starts_.back(), kInvalidRow);
    starts_.pop_back();
    for (int col = 0; col < input.num_cols(); ++col) {
      for (int64_t i = input.starts_[col]; i < input.starts_[col + 1]; ++i) {
        const int tcol = input.rows_[i];
        const int64_t index = starts_[tcol + 1]++;
        coefficients_[index] = input.coefficients_[i];
        rows_[index] = col;
      }
    }
  }
  // Columns [c0, c1) of input as a matrix of their own (a column shard of
  // [A | I] for DeviceLp's split over several devices).
  void PopulateColumnSlice(const CompactSparseMatrix& input, int c0, int c1) {
    num_rows_ = input.num_rows_;
    num_cols_ = c1 - c0;
    const int64_t b = input.starts_[c0];
    const int64_t e = input.starts_[c1];
    starts_.resize(num_cols_ + 1);
    for (int c = 0; c <= num_cols_; ++c) starts_[c] = input.starts_[c0 + c] - b;
    rows_.assign(input.rows_.begin() + b, input.rows_.begin() + e);
    coefficients_.assign(input.coefficients_.begin() + b, input.coefficients_.begin() + e);
  }
  // sparse.cc:554-561
  void Reset(int num_rows) {
    num_rows_ = num_rows;
    num_cols_ = 0;
    rows_.clear();
    coefficients_.clear();
    starts_.clear();
    starts_.push_back(0);
  }
  // sparse.h:514-542: four strided accumulators, then the tail in order.
  Fractional ColumnScalarProduct(int col, const Fractional* vector) const {
    int64_t i = starts_[col];
    const int64_t end = starts_[col + 1];
    const int64_t shifted_end = end - 3;
    Fractional r1 = 0.0, r2 = 0.0, r3 = 0.0, r4 = 0.0;
    for (; i < shifted_end; i += 4) {
      r1 += coefficients_[i] * vector[rows_[i]];
      r2 += coefficients_[i + 1] * vector[rows_[i + 1]];
      r3 += coefficients_[i + 2] * vector[rows_[i + 2]];
      r4 += coefficients_[i + 3] * vector[rows_[i + 3]];
    }
    Fractional result = r1 + r2 + r3 + r4;
    if (i < end) {
      result += coefficients_[i] * vector[rows_[i]];
      if (i + 1 < end) {
        result += coefficients_[i + 1] * vector[rows_[i + 1]];
        if (i + 2 < end) result += coefficients_[i + 2] * vector[rows_[i + 2]];
      }
    }
    return result;
  }
  Fractional ColumnScalarProduct(int col, const std::vector<Fractional>& v) const {
    return ColumnScalarProduct(col, v.data());
  }
  // sparse.h:389-399
  void ColumnAddMultipleToDenseColumn(int col, Fractional multiplier,
                                      Fractional* dense) const {
    if (multiplier == 0.0) return;
    for (int64_t i = starts_[col]; i < starts_[col + 1]; ++i)
      dense[rows_[i]] += multiplier * coefficients_[i];
  }
  // sparse.h:403-413
  void ColumnAddMultipleToSparseScatteredColumn(int col, Fractional multiplier,
                                                ScatteredVector* c) const {
    if (multiplier == 0.0) return;
    for (int64_t i = starts_[col]; i < starts_[col + 1]; ++i)
      c->Add(rows_[i], multiplier * coefficients_[i]);
  }
  // sparse.h:440-455
  void ColumnCopyToClearedDenseColumnWithNonZeros(
      int col, std::vector<Fractional>* dense, std::vector<int>* nz) const {
    dense->resize(num_rows_, 0.0);
    nz->clear();
    for (int64_t i = starts_[col]; i < starts_[col + 1]; ++i) {
      (*dense)[rows_[i]] = coefficients_[i];
      nz->push_back(rows_[i]);
    }
  }
  // sparse.cc:576-623
  int AddDenseColumnPrefix(const std::vector<Fractional>& d, int start) {
    // The non-zeros of d[start..), increasing (host pool for long columns).
    ParallelAppendNonZeros(d.data(), start, static_cast<int64_t>(d.size()), &rows_,
                           &coefficients_);
    starts_.push_back(rows_.size());
    return num_cols_++;
  }
  int AddDenseColumn(const std::vector<Fractional>& d) {
    return AddDenseColumnPrefix(d, 0);
  }
  int AddDenseColumnWithNonZeros(const std::vector<Fractional>& d,
                                 const std::vector<int>& nz) {
    if (nz.empty()) return AddDenseColumn(d);
    for (const int r : nz) {
      if (d[r] != 0.0) {
        rows_.push_back(r);
        coefficients_.push_back(d[r]);
      }
    }
    starts_.push_back(rows_.size());
    return num_cols_++;
  }
  int AddAndClearColumnWithNonZeros(std::vector<Fractional>* col,
                                    std::vector<int>* nz) {
    for (const int r : *nz) {
      const Fractional v = (*col)[r];
      if (v != 0.0) {
        rows_.push_back(r);
        coefficients_.push_back(v);
        (*col)[r] = 0.0;
      }
    }
    nz->clear();
    starts_.push_back(rows_.size());
    return num_cols_++;
  }

  int num_rows_ = 0;
  int num_cols_ = 0;
  std::vector<Fractional> coefficients_;
  std::vector<int> rows_;
  std::vector<int64_t> starts_;
};

// The basis B as a view of some columns of the matrix (sparse.h:544-569).
struct CompactSparseMatrixView {
  const CompactSparseMatrix* m;
  const std::vector<int>* cols;
  int num_rows() const { return m->num_rows(); }
  int num_cols() const { return static_cast<int>(cols->size()); }
  bool IsEmpty() const { return m->IsEmpty(); }
  ColumnView column(int c) const { return m->column((*cols)[c]); }
  int64_t num_entries() const {
    int64_t n = 0;
    for (int c = 0; c < num_cols(); ++c) n += column(c).n;
    return n;
  }
  // sparse.cc:69-86
  Fractional ComputeInfinityNorm() const {
    std::vector<Fractional> row_sum(num_rows(), 0.0);
    for (int c = 0; c < num_cols(); ++c) {
      const ColumnView col = column(c);
      for (int64_t i = 0; i < col.n; ++i)
        row_sum[col.rows[i]] += std::fabs(col.coefs[i]);
    }
    Fractional norm = 0.0;
    for (const Fractional s : row_sum) norm = std::max(norm, s);
    return norm;
  }
};

}  // namespace milp

#endif  // MILP_LP_DATA_H_
