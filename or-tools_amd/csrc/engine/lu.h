// Host basis factorization of the MI355X simplex engine: Markowitz LU,
// triangular solves and middle-product-form rank-one updates, following
// Glop (OR-Tools 9.7): lp_data/sparse.{h,cc} TriangularMatrix,
// glop/markowitz.cc, glop/lu_factorization.cc, glop/rank_one_update.h,
// glop/basis_representation.cc. Factorization stays on the host in round 1
// (SURVEY.md 7 "Hard parts"); the O(nnz(A)) passes run on the GPU.
#ifndef MILP_LU_H_
#define MILP_LU_H_

#include <atomic>
#include <cstdint>
#include <functional>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>

#include "device_solver.h"
#include "lp_data.h"

namespace milp {

// Debug aid (MILP_TRACE): bit-hashes of the last problem-column FTRAN's
// stages (after L, after the rank-one etas, after U), printed with the
// per-iteration trace line so engine and oracle divergences can be located.
inline bool g_trace_ftran = false;
inline uint64_t g_ftran_hash[3] = {0, 0, 0};
inline uint64_t TraceHashVector(const std::vector<Fractional>& v, const std::vector<int>& nz) {
  uint64_t h = 1469598103934665603ull;
  for (const Fractional x : v) {
    uint64_t b;
    std::memcpy(&b, &x, sizeof(b));
    h = (h ^ b) * 1099511628211ull;
  }
  for (const int r : nz) h = (h ^ static_cast<uint32_t>(r)) * 1099511628211ull;
  return h;
}

// Which copy of the solve scratch a thread uses: 0 on the solver's thread,
// 1 on BasisFactorization's tau worker (the two run FTRANs concurrently).
inline thread_local int g_lu_slot = 0;
// Runs a scope with another solve slot (scratch and deferred bookkeeping).
struct LuSlotGuard {
  int saved;
  explicit LuSlotGuard(int slot) : saved(g_lu_slot) { g_lu_slot = slot; }
  ~LuSlotGuard() { g_lu_slot = saved; }
};

// Debug aid (MILP_PHASE_TIMING): host wall time of the pieces of the solver
// thread's FTRANs (L, etas, U) and of the device U/L solve calls (copy-in,
// launch + wait, copy-out). Printed with the phase timing.
enum FtranPiece {
  kFtL, kFtEtas, kFtU, kFtDevCopyIn, kFtDevRun, kFtDevCopyOut,
  kFtURows, kFtUHost, kFtUPool, kFtPieces
};
extern double g_ftran_ms[kFtPieces];
extern const bool g_ftran_timing;
struct FtranTimer {
  int p;
  std::chrono::steady_clock::time_point t0;
  explicit FtranTimer(int q) : p(q) {
    if (g_ftran_timing && g_lu_slot == 0) t0 = std::chrono::steady_clock::now();
  }
  void Lap(int next) {
    if (!g_ftran_timing || g_lu_slot != 0) return;
    const auto now = std::chrono::steady_clock::now();
    g_ftran_ms[p] += std::chrono::duration<double, std::milli>(now - t0).count();
    t0 = now;
    p = next;
  }
  ~FtranTimer() { Lap(p); }
};

// ---------------------------------------------------------------------------
// TriangularMatrix (sparse.h:583-921).
class TriangularMatrix : public CompactSparseMatrix {
 public:
  bool IsEmpty() const { return diagonal_coefficients_.empty(); }
  int64_t num_entries() const {
    return static_cast<int64_t>(num_cols_) +
           static_cast<int64_t>(coefficients_.size());
  }
  // sparse.cc:562-572
  void Reset(int num_rows, int col_capacity) {
    par_ready_[0] = par_ready_[1] = false;
    CompactSparseMatrix::Reset(num_rows);
    first_non_identity_column_ = 0;
    all_diagonal_coefficients_are_one_ = true;
    pruned_ends_.resize(col_capacity);
    diagonal_coefficients_.resize(col_capacity);
    starts_.resize(col_capacity + 1);
    starts_[0] = 0;
  }
  void Swap(TriangularMatrix* o) {
    par_ready_[0] = par_ready_[1] = false;
    o->par_ready_[0] = o->par_ready_[1] = false;
    std::swap(num_rows_, o->num_rows_);
    std::swap(num_cols_, o->num_cols_);
    coefficients_.swap(o->coefficients_);
    rows_.swap(o->rows_);
    starts_.swap(o->starts_);
    diagonal_coefficients_.swap(o->diagonal_coefficients_);
    std::swap(first_non_identity_column_, o->first_non_identity_column_);
    std::swap(all_diagonal_coefficients_are_one_,
              o->all_diagonal_coefficients_are_one_);
  }
  // sparse.cc:530-552
  void PopulateFromTranspose(const TriangularMatrix& input) {
    par_ready_[0] = par_ready_[1] = false;
    CompactSparseMatrix::PopulateFromTranspose(input);
    diagonal_coefficients_ = input.diagonal_coefficients_;
    all_diagonal_coefficients_are_one_ = input.all_diagonal_coefficients_are_one_;
    pruned_ends_.resize(num_cols_);
    for (int c = 0; c < num_cols_; ++c) pruned_ends_[c] = starts_[c + 1];
    first_non_identity_column_ = 0;
    const int end = static_cast<int>(diagonal_coefficients_.size());
    while (first_non_identity_column_ < end &&
           ColumnNumEntries(first_non_identity_column_) == 0 &&
           diagonal_coefficients_[first_non_identity_column_] == 1.0) {
      ++first_non_identity_column_;
    }
  }
  // sparse.cc:651-672
  void CloseCurrentColumn(Fractional diagonal_value) {
    par_ready_[0] = par_ready_[1] = false;
    diagonal_coefficients_[num_cols_] = diagonal_value;
    pruned_ends_[num_cols_] = coefficients_.size();
    ++num_cols_;
    starts_[num_cols_] = coefficients_.size();
    if (first_non_identity_column_ == num_cols_ - 1 && coefficients_.empty() &&
        diagonal_value == 1.0) {
      first_non_identity_column_ = num_cols_;
    }
    all_diagonal_coefficients_are_one_ =
        all_diagonal_coefficients_are_one_ && (diagonal_value == 1.0);
  }
  void AddDiagonalOnlyColumn(Fractional d) { CloseCurrentColumn(d); }
  // sparse.cc:678-691
  void AddTriangularColumn(const ColumnView& column, int diagonal_row) {
    Fractional diagonal_value = 0.0;
    for (int64_t i = 0; i < column.n; ++i) {
      if (column.rows[i] == diagonal_row) {
        diagonal_value = column.coefs[i];
      } else {
        rows_.push_back(column.rows[i]);
        coefficients_.push_back(column.coefs[i]);
      }
    }
    CloseCurrentColumn(diagonal_value);
  }
  // sparse.cc:693-708
  void AddAndNormalizeTriangularColumn(const SparseColumn& column,
                                       int diagonal_row, Fractional diag) {
    for (int64_t i = 0; i < column.num_entries(); ++i) {
      if (column.rows[i] != diagonal_row) {
        if (column.coefs[i] != 0.0) {
          rows_.push_back(column.rows[i]);
          coefficients_.push_back(column.coefs[i] / diag);
        }
      }
    }
    CloseCurrentColumn(1.0);
  }
  // sparse.cc:710-719
  void AddTriangularColumnWithGivenDiagonalEntry(const SparseColumn& column,
                                                 int /*diagonal_row*/,
                                                 Fractional diagonal_value) {
    for (int64_t i = 0; i < column.num_entries(); ++i) {
      rows_.push_back(column.rows[i]);
      coefficients_.push_back(column.coefs[i]);
    }
    CloseCurrentColumn(diagonal_value);
  }
  // sparse.cc:749-755
  void ApplyRowPermutationToNonDiagonalEntries(const std::vector<int>& perm) {
    par_ready_[0] = par_ready_[1] = false;
    for (auto& r : rows_) r = perm[r];
  }
  bool IsUpperTriangular() const {  // sparse.cc:739-747
    for (int c = 0; c < num_cols_; ++c) {
      if (diagonal_coefficients_[c] == 0.0) return false;
      for (int64_t i = starts_[c]; i < starts_[c + 1]; ++i)
        if (rows_[i] >= c) return false;
    }
    return true;
  }
  // sparse.cc:757-767 (+ SparseVector::CleanUp)
  void CopyColumnToSparseColumn(int col, SparseColumn* out) const {
    out->Clear();
    for (int64_t i = starts_[col]; i < starts_[col + 1]; ++i)
      out->SetCoefficient(rows_[i], coefficients_[i]);
    out->SetCoefficient(col, diagonal_coefficients_[col]);
    out->CleanUp();
  }
  int GetFirstNonIdentityColumn() const { return first_non_identity_column_; }
  Fractional GetDiagonalCoefficient(int c) const { return diagonal_coefficients_[c]; }
  bool ColumnIsDiagonalOnly(int c) const { return ColumnIsEmpty(c); }

  // sparse.cc:776-812
  void LowerSolve(std::vector<Fractional>* rhs) const { LowerSolveStartingAt(0, rhs); }
  void LowerSolveStartingAt(int start, std::vector<Fractional>* rhs) const {
    Fractional* x = rhs->data();
    const int begin = std::max(start, first_non_identity_column_);
    const int end = static_cast<int>(diagonal_coefficients_.size());
    const bool ones = all_diagonal_coefficients_are_one_;
    for (int col = begin; col < end; ++col) {
      const Fractional value = x[col];
      if (value == 0.0) continue;
      const Fractional coeff = ones ? value : value / diagonal_coefficients_[col];
      if (!ones) x[col] = coeff;
      for (int64_t i = starts_[col]; i < starts_[col + 1]; ++i)
        x[rows_[i]] -= coeff * coefficients_[i];
    }
  }
  // sparse.cc:814-846
  void UpperSolve(std::vector<Fractional>* rhs) const {
    Fractional* x = rhs->data();
    const int end = first_non_identity_column_;
    const bool ones = all_diagonal_coefficients_are_one_;
    for (int col = static_cast<int>(diagonal_coefficients_.size()) - 1;
         col >= end; --col) {
      const Fractional value = x[col];
      if (value == 0.0) continue;
      const Fractional coeff = ones ? value : value / diagonal_coefficients_[col];
      if (!ones) x[col] = coeff;
      for (int64_t i = starts_[col + 1] - 1; i >= starts_[col]; --i)
        x[rows_[i]] -= coeff * coefficients_[i];
    }
  }
  // One output of TransposeUpperSolve / TransposeLowerSolve, the loops' own
  // operations in their order (entries from the start / from the end).
  Fractional TransposeUpperOutput(const Fractional* x, int col) const {
    Fractional sum = x[col];
    int64_t i = starts_[col];
    const int64_t i_end = starts_[col + 1];
    const int64_t shifted_end = i_end - 3;
    for (; i < shifted_end; i += 4) {
      sum -= coefficients_[i] * x[rows_[i]] + coefficients_[i + 1] * x[rows_[i + 1]] +
             coefficients_[i + 2] * x[rows_[i + 2]] + coefficients_[i + 3] * x[rows_[i + 3]];
    }
    if (i < i_end) {
      sum -= coefficients_[i] * x[rows_[i]];
      if (i + 1 < i_end) {
        sum -= coefficients_[i + 1] * x[rows_[i + 1]];
        if (i + 2 < i_end) sum -= coefficients_[i + 2] * x[rows_[i + 2]];
      }
    }
    return all_diagonal_coefficients_are_one_ ? sum : sum / diagonal_coefficients_[col];
  }
  Fractional TransposeLowerOutput(const Fractional* x, int col) const {
    Fractional sum = x[col];
    int64_t i = starts_[col + 1] - 1;
    const int64_t i_end = starts_[col];
    const int64_t shifted_end = i_end + 3;
    for (; i >= shifted_end; i -= 4) {
      sum -= coefficients_[i] * x[rows_[i]] + coefficients_[i - 1] * x[rows_[i - 1]] +
             coefficients_[i - 2] * x[rows_[i - 2]] + coefficients_[i - 3] * x[rows_[i - 3]];
    }
    if (i >= i_end) {
      sum -= coefficients_[i] * x[rows_[i]];
      if (i >= i_end + 1) {
        sum -= coefficients_[i - 1] * x[rows_[i - 1]];
        if (i >= i_end + 2) sum -= coefficients_[i - 2] * x[rows_[i - 2]];
      }
    }
    return all_diagonal_coefficients_are_one_ ? sum : sum / diagonal_coefficients_[col];
  }
  // Runs of consecutive columns that read no row of their own run, in the
  // loop's order (forward: TransposeUpperSolve; backward: TransposeLowerSolve):
  // a long run's outputs are independent, the host pool computes them
  // (MILP_HOST_TRI_PAR=0: never). Built on first use after a change.
  bool ParallelTransposeSolve(bool forward, std::vector<Fractional>* rhs) const;

  // sparse.cc:848-897 (grouped 4-term subtraction)
  void TransposeUpperSolve(std::vector<Fractional>* rhs) const {
    if (ParallelTransposeSolve(true, rhs)) return;
    Fractional* x = rhs->data();
    const int end = num_cols_;
    const bool ones = all_diagonal_coefficients_are_one_;
    int64_t i = starts_[first_non_identity_column_];
    for (int col = first_non_identity_column_; col < end; ++col) {
      Fractional sum = x[col];
      const int64_t i_end = starts_[col + 1];
      const int64_t shifted_end = i_end - 3;
      for (; i < shifted_end; i += 4) {
        sum -= coefficients_[i] * x[rows_[i]] +
               coefficients_[i + 1] * x[rows_[i + 1]] +
               coefficients_[i + 2] * x[rows_[i + 2]] +
               coefficients_[i + 3] * x[rows_[i + 3]];
      }
      if (i < i_end) {
        sum -= coefficients_[i] * x[rows_[i]];
        if (i + 1 < i_end) {
          sum -= coefficients_[i + 1] * x[rows_[i + 1]];
          if (i + 2 < i_end) sum -= coefficients_[i + 2] * x[rows_[i + 2]];
        }
        i = i_end;
      }
      x[col] = ones ? sum : sum / diagonal_coefficients_[col];
    }
  }
  // sparse.cc:899-955
  void TransposeLowerSolve(std::vector<Fractional>* rhs) const {
    if (ParallelTransposeSolve(false, rhs)) return;
    Fractional* x = rhs->data();
    const int end = first_non_identity_column_;
    int col = num_cols_ - 1;
    while (col >= end && x[col] == 0.0) --col;
    const bool ones = all_diagonal_coefficients_are_one_;
    int64_t i = starts_[col + 1] - 1;
    for (; col >= end; --col) {
      Fractional sum = x[col];
      const int64_t i_end = starts_[col];
      const int64_t shifted_end = i_end + 3;
      for (; i >= shifted_end; i -= 4) {
        sum -= coefficients_[i] * x[rows_[i]] +
               coefficients_[i - 1] * x[rows_[i - 1]] +
               coefficients_[i - 2] * x[rows_[i - 2]] +
               coefficients_[i - 3] * x[rows_[i - 3]];
      }
      if (i >= i_end) {
        sum -= coefficients_[i] * x[rows_[i]];
        if (i >= i_end + 1) {
          sum -= coefficients_[i - 1] * x[rows_[i - 1]];
          if (i >= i_end + 2) sum -= coefficients_[i - 2] * x[rows_[i - 2]];
        }
        i = i_end - 1;
      }
      x[col] = ones ? sum : sum / diagonal_coefficients_[col];
    }
  }
  // sparse.cc:967-986
  void HyperSparseSolve(std::vector<Fractional>* rhs, std::vector<int>* nz) const {
    Fractional* x = rhs->data();
    const bool ones = all_diagonal_coefficients_are_one_;
    int new_size = 0;
    for (size_t k = 0; k < nz->size(); ++k) {
      const int row = (*nz)[k];
      if (x[row] == 0.0) continue;
      const Fractional coeff = ones ? x[row] : x[row] / diagonal_coefficients_[row];
      x[row] = coeff;
      for (int64_t i = starts_[row]; i < starts_[row + 1]; ++i)
        x[rows_[i]] -= coeff * coefficients_[i];
      (*nz)[new_size++] = row;
    }
    nz->resize(new_size);
  }
  // sparse.cc:1000-1022
  void HyperSparseSolveWithReversedNonZeros(std::vector<Fractional>* rhs,
                                            std::vector<int>* nz) const {
    Fractional* x = rhs->data();
    const bool ones = all_diagonal_coefficients_are_one_;
    int new_start = static_cast<int>(nz->size());
    for (int k = static_cast<int>(nz->size()) - 1; k >= 0; --k) {
      const int row = (*nz)[k];
      if (x[row] == 0.0) continue;
      const Fractional coeff = ones ? x[row] : x[row] / diagonal_coefficients_[row];
      x[row] = coeff;
      for (int64_t i = starts_[row]; i < starts_[row + 1]; ++i)
        x[rows_[i]] -= coeff * coefficients_[i];
      (*nz)[--new_start] = row;
    }
    nz->erase(nz->begin(), nz->begin() + new_start);
  }
  // sparse.cc:1036-1072
  void TransposeHyperSparseSolve(std::vector<Fractional>* rhs,
                                 std::vector<int>* nz) const {
    Fractional* x = rhs->data();
    const bool ones = all_diagonal_coefficients_are_one_;
    int new_size = 0;
    for (size_t k = 0; k < nz->size(); ++k) {
      const int row = (*nz)[k];
      Fractional sum = x[row];
      int64_t i = starts_[row];
      const int64_t i_end = starts_[row + 1];
      const int64_t shifted_end = i_end - 3;
      for (; i < shifted_end; i += 4) {
        sum -= coefficients_[i] * x[rows_[i]] +
               coefficients_[i + 1] * x[rows_[i + 1]] +
               coefficients_[i + 2] * x[rows_[i + 2]] +
               coefficients_[i + 3] * x[rows_[i + 3]];
      }
      if (i < i_end) {
        sum -= coefficients_[i] * x[rows_[i]];
        if (i + 1 < i_end) {
          sum -= coefficients_[i + 1] * x[rows_[i + 1]];
          if (i + 2 < i_end) sum -= coefficients_[i + 2] * x[rows_[i + 2]];
        }
      }
      x[row] = ones ? sum : sum / diagonal_coefficients_[row];
      if (sum != 0.0) (*nz)[new_size++] = row;
    }
    nz->resize(new_size);
  }
  // sparse.cc:1086-1128
  void TransposeHyperSparseSolveWithReversedNonZeros(
      std::vector<Fractional>* rhs, std::vector<int>* nz) const {
    Fractional* x = rhs->data();
    const bool ones = all_diagonal_coefficients_are_one_;
    int new_start = static_cast<int>(nz->size());
    for (int k = static_cast<int>(nz->size()) - 1; k >= 0; --k) {
      const int row = (*nz)[k];
      Fractional sum = x[row];
      int64_t i = starts_[row + 1] - 1;
      const int64_t i_end = starts_[row];
      const int64_t shifted_end = i_end + 3;
      for (; i >= shifted_end; i -= 4) {
        sum -= coefficients_[i] * x[rows_[i]] +
               coefficients_[i - 1] * x[rows_[i - 1]] +
               coefficients_[i - 2] * x[rows_[i - 2]] +
               coefficients_[i - 3] * x[rows_[i - 3]];
      }
      if (i >= i_end) {
        sum -= coefficients_[i] * x[rows_[i]];
        if (i >= i_end + 1) {
          sum -= coefficients_[i - 1] * x[rows_[i - 1]];
          if (i >= i_end + 2) sum -= coefficients_[i - 2] * x[rows_[i - 2]];
        }
      }
      x[row] = ones ? sum : sum / diagonal_coefficients_[row];
      if (sum != 0.0) (*nz)[--new_start] = row;
    }
    nz->erase(nz->begin(), nz->begin() + new_start);
  }

  // sparse.cc:1130-1170
  void PermutedLowerSolve(const SparseColumn& rhs, const std::vector<int>& row_perm,
                          const std::vector<int>& partial_inverse_row_perm,
                          SparseColumn* lower, SparseColumn* upper) const;
  // sparse.cc:1172-1232
  void PermutedLowerSparseSolve(const ColumnView& rhs,
                                const std::vector<int>& row_perm,
                                SparseColumn* lower_column,
                                SparseColumn* upper_column) {
    PermutedComputeRowsToConsider(rhs, row_perm, &lower_column_rows_,
                                  &upper_column_rows_);
    scratch_.resize(num_rows_, 0.0);
    for (int64_t i = 0; i < rhs.n; ++i) scratch_[rhs.rows[i]] = rhs.coefs[i];
    num_fp_operations_ = 0;
    lower_column->Clear();
    upper_column->Reserve(upper_column->num_entries() +
                          static_cast<int64_t>(upper_column_rows_.size()));
    for (int k = static_cast<int>(upper_column_rows_.size()) - 1; k >= 0; --k) {
      const int permuted_row = upper_column_rows_[k];
      const Fractional pivot = scratch_[permuted_row];
      if (pivot == 0.0) continue;
      scratch_[permuted_row] = 0.0;
      const int row_as_col = row_perm[permuted_row];
      upper_column->SetCoefficient(permuted_row, pivot);
      num_fp_operations_ += 1 + ColumnNumEntries(row_as_col);
      for (int64_t i = starts_[row_as_col]; i < starts_[row_as_col + 1]; ++i)
        scratch_[rows_[i]] -= coefficients_[i] * pivot;
    }
    lower_column->Reserve(static_cast<int64_t>(lower_column_rows_.size()));
    for (const int permuted_row : lower_column_rows_) {
      const Fractional pivot = scratch_[permuted_row];
      scratch_[permuted_row] = 0.0;
      lower_column->SetCoefficient(permuted_row, pivot);
    }
  }
  int64_t NumFpOperationsInLastPermutedLowerSparseSolve() const {
    return num_fp_operations_;
  }
  // sparse.cc:1258-1365 (DFS topological order with pruning).
  void PermutedComputeRowsToConsider(const ColumnView& rhs,
                                     const std::vector<int>& row_perm,
                                     std::vector<int>* lower_rows,
                                     std::vector<int>* upper_rows) {
    std::vector<char>& stored_ = stored_slots_[g_lu_slot];
    stored_.resize(num_rows_, false);
    marked_.resize(num_rows_, false);
    lower_rows->clear();
    upper_rows->clear();
    nodes_to_explore_.clear();
    for (int64_t k = 0; k < rhs.n; ++k) {
      const int r = rhs.rows[k];
      const int col = row_perm[r];
      if (col < 0) {
        stored_[r] = true;
        lower_rows->push_back(r);
      } else {
        nodes_to_explore_.push_back(r);
      }
    }
    while (!nodes_to_explore_.empty()) {
      const int row = nodes_to_explore_.back();
      if (row < 0) {
        nodes_to_explore_.pop_back();
        const int explored_row = nodes_to_explore_.back();
        nodes_to_explore_.pop_back();
        stored_[explored_row] = true;
        upper_rows->push_back(explored_row);
        const int col = row_perm[explored_row];
        int64_t i = starts_[col];
        int64_t end = pruned_ends_[col];
        while (i < end) {
          const int entry_row = rows_[i];
          if (!marked_[entry_row]) {
            --end;
            std::swap(rows_[i], rows_[end]);
            std::swap(coefficients_[i], coefficients_[end]);
          } else {
            marked_[entry_row] = false;
            ++i;
          }
        }
        pruned_ends_[col] = end;
        continue;
      }
      if (stored_[row]) {
        nodes_to_explore_.pop_back();
        continue;
      }
      const int col = row_perm[row];
      if (col < 0) {
        stored_[row] = true;
        lower_rows->push_back(row);
        nodes_to_explore_.pop_back();
        continue;
      }
      nodes_to_explore_.push_back(kInvalidRow);
      const int64_t end = pruned_ends_[col];
      for (int64_t i = starts_[col]; i < end; ++i) {
        const int entry_row = rows_[i];
        if (!stored_[entry_row]) nodes_to_explore_.push_back(entry_row);
        marked_[entry_row] = true;
      }
    }
    for (const int r : *lower_rows) stored_[r] = false;
    for (const int r : *upper_rows) stored_[r] = false;
  }
  // sparse.cc:1445-1492 (the ratio arguments are ignored upstream).
  void ComputeRowsToConsiderInSortedOrder(std::vector<int>* nz) const {
    if (nz->empty()) return;
    std::vector<char>& stored_ = stored_slots_[g_lu_slot];
    const int sparsity_threshold = static_cast<int>(0.025 * num_rows_);
    const int num_ops_threshold = static_cast<int>(0.05 * num_rows_);
    int num_ops = static_cast<int>(nz->size());
    if (num_ops > sparsity_threshold) {
      nz->clear();
      return;
    }
    stored_.resize(num_rows_, false);
    for (const int r : *nz) stored_[r] = true;
    for (size_t k = 0; k < nz->size(); ++k) {
      const int row = (*nz)[k];
      for (int64_t i = starts_[row]; i < starts_[row + 1]; ++i) {
        ++num_ops;
        const int er = rows_[i];
        if (!stored_[er]) {
          nz->push_back(er);
          stored_[er] = true;
        }
      }
      if (num_ops > num_ops_threshold) break;
    }
    for (const int r : *nz) stored_[r] = false;
    if (num_ops > num_ops_threshold) {
      nz->clear();
    } else {
      std::sort(nz->begin(), nz->end());
    }
  }
  // sparse.cc:1498-1522
  Fractional ComputeInverseInfinityNormUpperBound() const {
    if (first_non_identity_column_ == num_cols_) return 1.0;
    const bool is_upper = IsUpperTriangular();
    std::vector<Fractional> est(num_rows_, 1.0);
    for (int k = 0; k < num_cols_; ++k) {
      const int col = is_upper ? num_cols_ - 1 - k : k;
      const Fractional coeff = est[col] / std::fabs(diagonal_coefficients_[col]);
      est[col] = coeff;
      for (int64_t i = starts_[col]; i < starts_[col + 1]; ++i)
        est[rows_[i]] += coeff * std::fabs(coefficients_[i]);
    }
    return *std::max_element(est.begin(), est.end());
  }

  std::vector<Fractional> diagonal_coefficients_;
  int first_non_identity_column_ = 0;
  bool all_diagonal_coefficients_are_one_ = true;
  std::vector<int64_t> pruned_ends_;

 private:
  // ParallelTransposeSolve's runs per direction (0 forward, 1 backward):
  // [begin, end) column ranges of the long independent runs, in loop order.
  // Built once per factorization under a lock by the first solve that needs
  // them; read without it by the solver thread and the tau worker, so the
  // ready flag is an acquire/release atomic (copies start not ready).
  struct ReadyFlag {
    std::atomic<bool> v{false};
    ReadyFlag() = default;
    ReadyFlag(const ReadyFlag&) {}
    ReadyFlag& operator=(const ReadyFlag&) {
      v.store(false, std::memory_order_release);
      return *this;
    }
    ReadyFlag& operator=(bool b) {
      v.store(b, std::memory_order_release);
      return *this;
    }
    operator bool() const { return v.load(std::memory_order_acquire); }
  };
  mutable ReadyFlag par_ready_[2];
  mutable std::vector<int> par_runs_[2];
  // Forward solve's dense tail [par_tail_, n): per column, the end of its
  // leading groups of four that read rows < par_tail_ only (-1: no tail).
  mutable int par_tail_ = -1;
  mutable std::vector<int64_t> par_split_;
  mutable std::vector<char> stored_slots_[2];
  std::vector<char> marked_;
  std::vector<int> nodes_to_explore_;
  int64_t num_fp_operations_ = 0;
  std::vector<int> lower_column_rows_;
  std::vector<int> upper_column_rows_;
  std::vector<Fractional> scratch_;
};

// ---------------------------------------------------------------------------
// markowitz.cc:495-718 MatrixNonZeroPattern.
class MatrixNonZeroPattern {
 public:
  void Clear() {
    row_degree_.clear();
    col_degree_.clear();
    row_non_zero_.clear();
    deleted_columns_.clear();
    bool_scratchpad_.clear();
    num_non_deleted_columns_ = 0;
  }
  void Reset(int num_rows, int num_cols) {
    row_degree_.assign(num_rows, 0);
    col_degree_.assign(num_cols, 0);
    row_non_zero_.clear();
    row_non_zero_.resize(num_rows);
    deleted_columns_.assign(num_cols, false);
    bool_scratchpad_.assign(num_cols, false);
    num_non_deleted_columns_ = num_cols;
  }
  void InitializeFromMatrixSubset(const CompactSparseMatrixView& b,
                                  const std::vector<int>& row_perm,
                                  const std::vector<int>& col_perm,
                                  std::vector<int>* singleton_columns,
                                  std::vector<int>* singleton_rows) {
    const int num_cols = b.num_cols();
    const int num_rows = b.num_rows();
    Reset(num_rows, num_cols);
    singleton_columns->clear();
    singleton_rows->clear();
    for (int col = 0; col < num_cols; ++col) {
      if (col_perm[col] != kInvalidCol) {
        deleted_columns_[col] = true;
        --num_non_deleted_columns_;
        continue;
      }
      const ColumnView c = b.column(col);
      for (int64_t i = 0; i < c.n; ++i) ++row_degree_[c.rows[i]];
    }
    for (int row = 0; row < num_rows; ++row) {
      if (row_perm[row] == kInvalidRow) {
        row_non_zero_[row].reserve(row_degree_[row]);
        if (row_degree_[row] == 1) singleton_rows->push_back(row);
      } else {
        row_degree_[row] = 0;
      }
    }
    for (int col = 0; col < num_cols; ++col) {
      if (col_perm[col] != kInvalidCol) continue;
      int32_t col_degree = 0;
      const ColumnView c = b.column(col);
      for (int64_t i = 0; i < c.n; ++i) {
        const int row = c.rows[i];
        if (row_perm[row] == kInvalidRow) {
          ++col_degree;
          row_non_zero_[row].push_back(col);
        }
      }
      col_degree_[col] = col_degree;
      if (col_degree == 1) singleton_columns->push_back(col);
    }
  }
  void AddEntry(int row, int col) {
    ++row_degree_[row];
    ++col_degree_[col];
    row_non_zero_[row].push_back(col);
  }
  int32_t DecreaseColDegree(int col) { return --col_degree_[col]; }
  int32_t DecreaseRowDegree(int row) { return --row_degree_[row]; }
  void DeleteRowAndColumn(int pivot_row, int pivot_col) {
    deleted_columns_[pivot_col] = true;
    --num_non_deleted_columns_;
    row_degree_[pivot_row] = 0;
  }
  bool IsColumnDeleted(int col) const { return deleted_columns_[col]; }
  void RemoveDeletedColumnsFromRow(int row) {
    auto& ref = row_non_zero_[row];
    int new_index = 0;
    const int end = static_cast<int>(ref.size());
    for (int i = 0; i < end; ++i) {
      const int col = ref[i];
      if (!deleted_columns_[col]) ref[new_index++] = col;
    }
    ref.resize(new_index);
  }
  int GetFirstNonDeletedColumnFromRow(int row) const {
    for (const int col : row_non_zero_[row])
      if (!IsColumnDeleted(col)) return col;
    return kInvalidCol;
  }
  void Update(int pivot_row, int pivot_col, const SparseColumn& column) {
    const int max_row_degree = num_non_deleted_columns_ + 1;
    RemoveDeletedColumnsFromRow(pivot_row);
    for (const int col : row_non_zero_[pivot_row]) {
      DecreaseColDegree(col);
      bool_scratchpad_[col] = false;
    }
    for (int64_t k = 0; k < column.num_entries(); ++k) {
      const int row = column.rows[k];
      if (row == pivot_row) continue;
      if (column.coefs[k] == 0.0 || row_degree_[row] == max_row_degree) continue;
      const int kDeletionThreshold = 4;
      if (static_cast<int64_t>(row_non_zero_[row].size()) >
          row_degree_[row] + kDeletionThreshold) {
        RemoveDeletedColumnsFromRow(row);
      }
      MergeInto(pivot_row, row);
    }
  }
  int32_t ColDegree(int col) const { return col_degree_[col]; }
  int32_t RowDegree(int row) const { return row_degree_[row]; }
  const std::vector<int>& RowNonZero(int row) const { return row_non_zero_[row]; }

 private:
  void MergeInto(int pivot_row, int row) {
    for (const int col : row_non_zero_[row]) bool_scratchpad_[col] = true;
    auto& non_zero = row_non_zero_[row];
    const int old_size = static_cast<int>(non_zero.size());
    for (const int col : row_non_zero_[pivot_row]) {
      if (bool_scratchpad_[col]) {
        bool_scratchpad_[col] = false;
      } else {
        non_zero.push_back(col);
        ++col_degree_[col];
      }
    }
    row_degree_[row] += static_cast<int>(non_zero.size()) - old_size;
  }

  std::vector<std::vector<int>> row_non_zero_;
  std::vector<int32_t> row_degree_;
  std::vector<int32_t> col_degree_;
  std::vector<char> deleted_columns_;
  std::vector<char> bool_scratchpad_;
  int num_non_deleted_columns_ = 0;
};

// markowitz.cc:719-768
class ColumnPriorityQueue {
 public:
  void Clear() {
    col_degree_.clear();
    col_index_.clear();
    col_by_degree_.clear();
  }
  void Reset(int max_degree, int num_cols) {
    Clear();
    col_degree_.assign(num_cols, 0);
    col_index_.assign(num_cols, -1);
    col_by_degree_.resize(max_degree + 1);
    min_degree_ = max_degree + 1;
  }
  void PushOrAdjust(int col, int32_t degree) {
    const int32_t old_degree = col_degree_[col];
    if (degree != old_degree) {
      const int32_t old_index = col_index_[col];
      if (old_index != -1) {
        col_by_degree_[old_degree][old_index] = col_by_degree_[old_degree].back();
        col_index_[col_by_degree_[old_degree].back()] = old_index;
        col_by_degree_[old_degree].pop_back();
      }
      if (degree > 0) {
        col_index_[col] = static_cast<int32_t>(col_by_degree_[degree].size());
        col_degree_[col] = degree;
        col_by_degree_[degree].push_back(col);
        min_degree_ = std::min(min_degree_, degree);
      } else {
        col_index_[col] = -1;
        col_degree_[col] = 0;
      }
    }
  }
  int Pop() {
    while (true) {
      if (min_degree_ == static_cast<int32_t>(col_by_degree_.size())) return kInvalidCol;
      if (!col_by_degree_[min_degree_].empty()) break;
      min_degree_++;
    }
    const int col = col_by_degree_[min_degree_].back();
    col_by_degree_[min_degree_].pop_back();
    col_index_[col] = -1;
    col_degree_[col] = 0;
    return col;
  }

 private:
  std::vector<int32_t> col_index_;
  std::vector<int32_t> col_degree_;
  std::vector<std::vector<int>> col_by_degree_;
  int32_t min_degree_ = 0;
};

// markowitz.cc:769-803 (memory reuse has no numerical effect).
class SparseMatrixWithReusableColumnMemory {
 public:
  void Reset(int num_cols) {
    mapping_.assign(num_cols, -1);
    free_columns_.clear();
    columns_.clear();
  }
  const SparseColumn& column(int col) const {
    if (mapping_[col] == -1) return empty_;
    return columns_[mapping_[col]];
  }
  SparseColumn* mutable_column(int col) {
    if (mapping_[col] != -1) return &columns_[mapping_[col]];
    int idx;
    if (free_columns_.empty()) {
      idx = static_cast<int>(columns_.size());
      columns_.emplace_back();
    } else {
      idx = free_columns_.back();
      free_columns_.pop_back();
    }
    mapping_[col] = idx;
    return &columns_[idx];
  }
  void ClearAndReleaseColumn(int col) {
    free_columns_.push_back(mapping_[col]);
    columns_[mapping_[col]].Clear();
    mapping_[col] = -1;
  }
  void Clear() {
    mapping_.clear();
    free_columns_.clear();
    columns_.clear();
  }

 private:
  SparseColumn empty_;
  std::vector<int> mapping_;
  std::vector<int> free_columns_;
  std::vector<SparseColumn> columns_;
};

struct LuParameters {
  double markowitz_singularity_threshold = 1e-15;
  int markowitz_zlatev_parameter = 3;
  double lu_factorization_pivot_threshold = 0.01;
};

// markowitz.cc:14-494
class Markowitz {
 public:
  Status ComputeLU(const CompactSparseMatrixView& b, std::vector<int>* row_perm,
                   std::vector<int>* col_perm, TriangularMatrix* lower,
                   TriangularMatrix* upper);
  Status ComputeRowAndColumnPermutation(const CompactSparseMatrixView& b,
                                        std::vector<int>* row_perm,
                                        std::vector<int>* col_perm);
  void Clear();
  double DeterministicTimeOfLastFactorization() const {
    return DeterministicTimeForFpOperations(num_fp_operations_);
  }
  void SetParameters(const LuParameters& p) { parameters_ = p; }
  const LuParameters& parameters() const { return parameters_; }
  // The operation count of another object's last factorization (an adopted
  // factorization reports the same deterministic time).
  void CopyStatsFrom(const Markowitz& o) { num_fp_operations_ = o.num_fp_operations_; }

 private:
  void ExtractSingletonColumns(const CompactSparseMatrixView& b,
                               std::vector<int>* row_perm,
                               std::vector<int>* col_perm, int* index);
  void ExtractResidualSingletonColumns(const CompactSparseMatrixView& b,
                                       std::vector<int>* row_perm,
                                       std::vector<int>* col_perm, int* index);
  const SparseColumn& ComputeColumn(const std::vector<int>& row_perm, int col);
  int64_t FindPivot(const std::vector<int>& row_perm,
                    const std::vector<int>& col_perm, int* pivot_row,
                    int* pivot_col, Fractional* pivot_coefficient);
  void UpdateDegree(int col, int degree);
  void RemoveRowFromResidualMatrix(int pivot_row, int pivot_col);
  void RemoveColumnFromResidualMatrix(int pivot_row, int pivot_col);
  void UpdateResidualMatrix(int pivot_row, int pivot_col);

  const CompactSparseMatrixView* basis_matrix_ = nullptr;
  SparseMatrixWithReusableColumnMemory permuted_lower_;
  SparseMatrixWithReusableColumnMemory permuted_upper_;
  TriangularMatrix lower_;
  TriangularMatrix upper_;
  std::vector<char> permuted_lower_column_needs_solve_;
  MatrixNonZeroPattern residual_matrix_non_zero_;
  ColumnPriorityQueue col_by_degree_;
  bool contains_only_singleton_columns_ = true;
  bool is_col_by_degree_initialized_ = false;
  std::vector<int> examined_col_;
  std::vector<int> singleton_column_;
  std::vector<int> singleton_row_;
  LuParameters parameters_;
  int64_t num_fp_operations_ = 0;
};

// lu_factorization.{h,cc}
class LuFactorization {
  friend struct SdualBridge;

 public:
  void Clear();
  Status ComputeFactorization(const CompactSparseMatrixView& b);
  std::vector<int> ComputeInitialBasis(const CompactSparseMatrix& matrix,
                                       const std::vector<int>& candidates);
  double DeterministicTimeOfLastFactorization() const {
    return markowitz_.DeterministicTimeOfLastFactorization();
  }
  Fractional RightSolveSquaredNorm(const ColumnView& a) const;
  Fractional DualEdgeSquaredNorm(int row) const;
  void RightSolveLWithPermutedInput(const std::vector<Fractional>& a,
                                    ScatteredVector* x) const;
  void RightSolveLForColumnView(const ColumnView& b, ScatteredVector* x) const;
  void RightSolveLWithNonZeros(ScatteredVector* x) const;
  void RightSolveLForScatteredColumn(const ScatteredVector& b,
                                     ScatteredVector* x) const;
  void LeftSolveUWithNonZeros(ScatteredVector* y) const;
  void RightSolveUWithNonZeros(ScatteredVector* x) const;
  // The U solves of two vectors of the same factorization (the direction on
  // this thread's scratch, tau on slot 1's), in one device launch when both
  // take the dense path; else one after the other. Same bits as two calls.
  void RightSolveUWithNonZerosPair(ScatteredVector* x, ScatteredVector* tau) const;
  void RightSolveUAfterRows(ScatteredVector* x) const;
  // The speculative flip FTRAN's U solve (engine, BasisFactorization::
  // SpecFlipLaunch): RightSolveUWithNonZeros' steps with the dense solve
  // launched on the device's own stream for it. 1: launched (Finish
  // completes x), 0: solved here (identity or hypersparse), -1: the device
  // declined a dense solve (x is not solved; the caller drops it).
  int StartRightSolveUAsync(ScatteredVector* x) const;
  void FinishRightSolveUAsync(ScatteredVector* x) const;
  void DropRightSolveUAsync() const;
  bool LeftSolveLWithNonZeros(ScatteredVector* y,
                              ScatteredVector* result_before_permutation) const;
  int LeftSolveUForUnitRow(int col, ScatteredVector* y) const;
  const SparseColumn& GetColumnOfU(int col) const;
  int64_t NumberOfEntries() const {
    return is_identity_factorization_
               ? 0
               : lower_.num_entries() + upper_.num_entries();
  }
  Fractional ComputeInverseInfinityNormUpperBound() const {
    return lower_.ComputeInverseInfinityNormUpperBound() *
           upper_.ComputeInverseInfinityNormUpperBound();
  }
  const std::vector<int>& GetColumnPermutation() const { return col_perm_; }
  // lu_factorization.cc:102-122, dense solves (product-form path only).
  void RightSolve(std::vector<Fractional>* x) const;
  void LeftSolve(std::vector<Fractional>* y) const;
  void SetColumnPermutationToIdentity() {
    col_perm_.clear();
    inverse_col_perm_.clear();
  }
  void SetParameters(const LuParameters& p) { markowitz_.SetParameters(p); }
  const LuParameters& parameters() const { return markowitz_.parameters(); }
  bool IsIdentityFactorization() const { return is_identity_factorization_; }
  // This object becomes a copy of o's factorization (the factors, their
  // transposes, the permutations and the last factorization's operation
  // count) under a fresh factorization key: what ComputeFactorization of
  // the same basis matrix with the same parameters would have produced.
  void AdoptFactorizationOf(const LuFactorization& o);
  // Dense U solves of the solver's thread go to this device (engine
  // substitution, bit-identical; see device_solver.h).
  void SetDeviceSolver(DeviceSolver* d) { device_solver_ = d; }
  bool HasDeviceSolver() const { return device_solver_ != nullptr; }
  // lower_.LowerSolveStartingAt(start, x), on the device when it takes it.
  void DenseLowerSolve(int start, std::vector<Fractional>* x) const;
  void DenseSolve(TriKind kind, const TriangularMatrix& t, int start,
                  std::vector<Fractional>* x) const;

  const std::vector<int>& inverse_col_perm() const { return inverse_col_perm_; }
  // Exposed for the factor-structure parity tests.
  const TriangularMatrix& lower() const { return lower_; }
  const TriangularMatrix& upper() const { return upper_; }
  const std::vector<int>& row_perm() const { return row_perm_; }

 private:
  template <typename Column>
  void RightSolveLInternal(const Column& b, ScatteredVector* x) const;
  void ComputeTransposeUpper() { transpose_upper_.PopulateFromTranspose(upper_); }
  void ComputeTransposeLower() const {
    transpose_lower_.PopulateFromTranspose(lower_);
  }

  bool is_identity_factorization_ = true;
  TriangularMatrix lower_;
  TriangularMatrix upper_;
  TriangularMatrix transpose_upper_;
  mutable TriangularMatrix transpose_lower_;
  std::vector<int> col_perm_;
  std::vector<int> inverse_col_perm_;
  std::vector<int> row_perm_;
  std::vector<int> inverse_row_perm_;
  mutable std::vector<Fractional> dense_column_scratchpad_;
  mutable std::vector<Fractional> dense_zero_scratchpad_slots_[2];
  std::vector<Fractional>& DenseZeroScratch() const {
    return dense_zero_scratchpad_slots_[g_lu_slot];
  }
  mutable std::vector<int> non_zero_rows_;
  mutable SparseColumn column_of_upper_;
  Markowitz markowitz_;
  DeviceSolver* device_solver_ = nullptr;
  // Unique per factorization (process-wide), so that a device copy of U is
  // never mistaken for the U of another factorization or handle.
  uint64_t factorization_key_ = 0;
};

// rank_one_update.h:30-148
class RankOneUpdateElementaryMatrix {
  friend struct SdualBridge;

 public:
  // u_storage: where u lives when not in `storage` (engine: the speculative
  // flip FTRAN's copy of the next update, BasisFactorization::SpecFlipLaunch).
  RankOneUpdateElementaryMatrix(const CompactSparseMatrix* storage, int u_index,
                                int v_index, Fractional u_dot_v,
                                const CompactSparseMatrix* u_storage = nullptr)
      : storage_(storage), u_storage_(u_storage != nullptr ? u_storage : storage),
        u_index_(u_index), v_index_(v_index), mu_(1.0 + u_dot_v) {}
  bool IsSingular() const { return mu_ == 0.0; }
  void RightSolve(std::vector<Fractional>* x) const {
    const Fractional multiplier =
        -storage_->ColumnScalarProduct(v_index_, x->data()) / mu_;
    u_storage_->ColumnAddMultipleToDenseColumn(u_index_, multiplier, x->data());
  }
  void RightSolveWithNonZeros(ScatteredVector* x) const {
    const Fractional multiplier =
        -storage_->ColumnScalarProduct(v_index_, x->values.data()) / mu_;
    if (multiplier != 0.0)
      u_storage_->ColumnAddMultipleToSparseScatteredColumn(u_index_, multiplier, x);
  }
  void LeftSolve(std::vector<Fractional>* y) const {
    const Fractional multiplier =
        -u_storage_->ColumnScalarProduct(u_index_, y->data()) / mu_;
    storage_->ColumnAddMultipleToDenseColumn(v_index_, multiplier, y->data());
  }
  void LeftSolveWithNonZeros(ScatteredVector* y) const {
    const Fractional multiplier =
        -u_storage_->ColumnScalarProduct(u_index_, y->values.data()) / mu_;
    if (multiplier != 0.0)
      storage_->ColumnAddMultipleToSparseScatteredColumn(v_index_, multiplier, y);
  }
  int64_t num_entries() const {
    return u_storage_->ColumnNumEntries(u_index_) +
           storage_->ColumnNumEntries(v_index_);
  }
  int u_index() const { return u_index_; }
  int v_index() const { return v_index_; }
  Fractional mu() const { return mu_; }

 private:
  const CompactSparseMatrix* storage_;
  const CompactSparseMatrix* u_storage_;
  int u_index_;
  int v_index_;
  Fractional mu_;
};

// rank_one_update.h:150-246
class RankOneUpdateFactorization {
  friend struct SdualBridge;

 public:
  void Clear() {
    elementary_matrices_.clear();
    num_entries_ = 0;
  }
  void Update(const RankOneUpdateElementaryMatrix& m) {
    elementary_matrices_.push_back(m);
    num_entries_ += m.num_entries();
  }
  void LeftSolve(std::vector<Fractional>* y) const {
    for (int i = static_cast<int>(elementary_matrices_.size()) - 1; i >= 0; --i)
      elementary_matrices_[i].LeftSolve(y);
    BumpTime();
  }
  void LeftSolveWithNonZeros(ScatteredVector* y) const {
    if (y->non_zeros.empty()) {
      LeftSolve(&y->values);
      return;
    }
    y->RepopulateSparseMask();
    bool use_dense = y->ShouldUseDenseIteration(hypersparse_ratio_);
    for (int i = static_cast<int>(elementary_matrices_.size()) - 1; i >= 0; --i) {
      if (use_dense) {
        elementary_matrices_[i].LeftSolve(&y->values);
      } else {
        elementary_matrices_[i].LeftSolveWithNonZeros(y);
        use_dense = y->ShouldUseDenseIteration(hypersparse_ratio_);
      }
    }
    y->ClearSparseMask();
    y->ClearNonZerosIfTooDense(hypersparse_ratio_);
    BumpTime();
  }
  void RightSolve(std::vector<Fractional>* d) const {
    for (size_t i = 0; i < elementary_matrices_.size(); ++i)
      elementary_matrices_[i].RightSolve(d);
    BumpTime();
  }
  void RightSolveWithNonZeros(ScatteredVector* d) const {
    if (d->non_zeros.empty()) {
      RightSolve(&d->values);
      return;
    }
    d->RepopulateSparseMask();
    bool use_dense = d->ShouldUseDenseIteration(hypersparse_ratio_);
    for (size_t i = 0; i < elementary_matrices_.size(); ++i) {
      if (use_dense) {
        elementary_matrices_[i].RightSolve(&d->values);
      } else {
        elementary_matrices_[i].RightSolveWithNonZeros(d);
        use_dense = d->ShouldUseDenseIteration(hypersparse_ratio_);
      }
    }
    d->ClearSparseMask();
    d->ClearNonZerosIfTooDense(hypersparse_ratio_);
    BumpTime();
  }
  // RightSolveWithNonZeros split in two calls (engine: the speculative flip
  // FTRAN applies the matrix of the next update later, once it is known):
  // Begin applies the current matrices, End one more and finishes as the
  // loop above finishes. Same steps in the same order, so the same bits as
  // RightSolveWithNonZeros over all of them; neither call bumps (the caller
  // applies BumpTime() where the serial solve would have).
  struct SplitSolve {
    bool dense = false;      // d->non_zeros was empty: RightSolve's dense loop
    bool use_dense = false;  // the sparse loop's state after Begin
  };
  void RightSolveBegin(ScatteredVector* d, SplitSolve* st) const {
    st->dense = d->non_zeros.empty();
    if (st->dense) {
      for (const auto& m : elementary_matrices_) m.RightSolve(&d->values);
      return;
    }
    d->RepopulateSparseMask();
    st->use_dense = d->ShouldUseDenseIteration(hypersparse_ratio_);
    for (const auto& m : elementary_matrices_) {
      if (st->use_dense) {
        m.RightSolve(&d->values);
      } else {
        m.RightSolveWithNonZeros(d);
        st->use_dense = d->ShouldUseDenseIteration(hypersparse_ratio_);
      }
    }
  }
  void RightSolveEnd(ScatteredVector* d, const SplitSolve& st,
                     const RankOneUpdateElementaryMatrix& last) const {
    if (st.dense) {
      last.RightSolve(&d->values);
      return;
    }
    if (st.use_dense) {
      last.RightSolve(&d->values);
    } else {
      last.RightSolveWithNonZeros(d);
    }
    d->ClearSparseMask();
    d->ClearNonZerosIfTooDense(hypersparse_ratio_);
  }
  int64_t num_entries() const { return num_entries_; }
  // A solve on the tau worker defers its bump; the solver's thread applies
  // it (or drops it, if the result is discarded) in program order.
  void BumpTime() const {
    if (g_lu_slot != 0) {
      ++deferred_bumps_;
      return;
    }
    dtime_ += DeterministicTimeForFpOperations(num_entries_);
  }
  void TakeDeferredBumps(bool apply) const {
    for (; deferred_bumps_ > 0; --deferred_bumps_) {
      if (apply) dtime_ += DeterministicTimeForFpOperations(num_entries_);
    }
  }
  double DeterministicTimeSinceLastReset() const { return dtime_; }
  void ResetDeterministicTime() { dtime_ = 0.0; }
  int size() const { return static_cast<int>(elementary_matrices_.size()); }

 private:
  mutable double dtime_ = 0.0;
  mutable int deferred_bumps_ = 0;
  double hypersparse_ratio_ = 0.05;
  int64_t num_entries_ = 0;
  std::vector<RankOneUpdateElementaryMatrix> elementary_matrices_;
};

// basis_representation.cc:176-627 (middle-product-form path).
// basis_representation.h:55-141, .cc:25-176: product-form (eta) updates,
// used instead of the middle-product form when
// use_middle_product_form_update is false.
class EtaMatrix {
  friend struct SdualBridge;

 public:
  EtaMatrix(int eta_col, const ScatteredVector& direction);
  void LeftSolve(std::vector<Fractional>* y) const;
  void RightSolve(std::vector<Fractional>* d) const;
  void SparseLeftSolve(std::vector<Fractional>* y, std::vector<int>* pos) const;

 private:
  int eta_col_;
  Fractional eta_col_coefficient_;
  std::vector<Fractional> eta_coeff_;
  SparseColumn sparse_eta_coeff_;  // entries in direction.non_zeros order
  EtaMatrix() = default;  // the device segment's etas (sdual_bridge.inc)
};

class EtaFactorization {
  friend struct SdualBridge;

 public:
  void Clear() { eta_matrix_.clear(); }
  void Update(int /*entering_col*/, int leaving_variable_row,
              const ScatteredVector& direction) {
    eta_matrix_.emplace_back(new EtaMatrix(leaving_variable_row, direction));
  }
  void LeftSolve(std::vector<Fractional>* y) const {
    for (int i = static_cast<int>(eta_matrix_.size()) - 1; i >= 0; --i)
      eta_matrix_[i]->LeftSolve(y);
  }
  void SparseLeftSolve(std::vector<Fractional>* y, std::vector<int>* pos) const {
    for (int i = static_cast<int>(eta_matrix_.size()) - 1; i >= 0; --i)
      eta_matrix_[i]->SparseLeftSolve(y, pos);
  }
  void RightSolve(std::vector<Fractional>* d) const {
    for (size_t i = 0; i < eta_matrix_.size(); ++i) eta_matrix_[i]->RightSolve(d);
  }

 private:
  std::vector<std::unique_ptr<EtaMatrix>> eta_matrix_;
};

class BasisFactorization {
  friend struct SdualBridge;
  friend struct SdualHooks;

 public:
  BasisFactorization(const CompactSparseMatrix* matrix, const std::vector<int>* basis);
  ~BasisFactorization();
  BasisFactorization(const BasisFactorization&) = delete;
  BasisFactorization& operator=(const BasisFactorization&) = delete;

  // Tau FTRAN off the solver's thread (engine scheduling, no Glop
  // counterpart). The dual loop knows rho, the only input of
  // RightSolveForTau, right after the BTRAN; the worker computes tau then,
  // while the update row, ratio test and direction FTRAN run. The next
  // RightSolveForTau(rho) takes the result; any other use of the
  // factorization first waits for the worker and drops it. The solve is the
  // same code on a private scratch copy, and its deterministic-time bumps are
  // applied when it is taken, so results and timing match the serial order.
  // kTauDeferred: the worker does tau's L and etas only; its U solve waits
  // for the direction's (one two-vector device launch, MILP_TRI_PAIR).
  enum class AsyncKind { kNone, kTau, kLeftSolve, kTauDeferred };
  void StartAsyncTau(const ScatteredVector& rho) const;
  // Small bases: tau on the calling thread, overlapped with the GPU update row.
  bool InlineTauEnabled() const;
  void ComputeTauNow(const ScatteredVector& rho) const;
  // The same for a caller's BTRAN (the primal loop's B^-T d): job runs
  // LeftSolve on the worker; TakeAsync(ticket) waits for it and applies its
  // bumps, and returns false if it was dropped (then the caller solves).
  uint64_t StartAsyncLeftSolve(std::function<void()> job) const;
  bool TakeAsync(uint64_t ticket) const;
  // Waits for and discards any worker job / the job of one ticket.
  void DropAsync() const;
  void DropAsync(uint64_t ticket) const {
    if (async_kind_ != AsyncKind::kNone && ticket == async_ticket_) DropAsync();
  }
  bool AsyncEnabled() const;
  void SetParameters(int refactorization_period, bool dynamic_period,
                     const LuParameters& lu, bool use_middle_product_form_update = true) {
    use_middle_product_form_update_ = use_middle_product_form_update;
    DropAsync();
    max_num_updates_ = refactorization_period;
    dynamic_period_ = dynamic_period;
    lu_factorization_.SetParameters(lu);
  }
  void Clear();
  Status Initialize();
  std::vector<int> ComputeInitialBasis(const std::vector<int>& candidates);
  bool IsRefactorized() const { return num_updates_ == 0; }
  Status Refactorize();
  Status ForceRefactorization();
  Status Update(int entering_col, int leaving_variable_row,
                const ScatteredVector& direction);
  void LeftSolve(ScatteredVector* y) const;
  void RightSolve(ScatteredVector* d) const;
  const std::vector<Fractional>& RightSolveForTau(const ScatteredVector& a) const;
  void LeftSolveForUnitRow(int j, ScatteredVector* y) const;
  void TemporaryLeftSolveForUnitRow(int j, ScatteredVector* y) const;
  void RightSolveForProblemColumn(int col, ScatteredVector* d) const;
  Fractional RightSolveSquaredNorm(const ColumnView& a) const;
  Fractional DualEdgeSquaredNorm(int row) const;
  bool IsIdentityBasis() const;
  Fractional ComputeInfinityNormConditionNumberUpperBound() const;
  double DeterministicTime() const { return deterministic_time_; }
  int NumUpdates() const { return num_updates_; }
  // Run counters (bench.py window statistics): LU factorizations computed
  // by this object and the host wall time spent in them.
  int64_t NumFactorizations() const { return num_factorizations_; }
  double FactorizationSeconds() const { return factorization_seconds_; }
  int GetNumberOfRows() const { return compact_matrix_.num_rows(); }
  const std::vector<int>& GetColumnPermutation() const {
    return lu_factorization_.GetColumnPermutation();
  }
  void SetColumnPermutationToIdentity() {
    DropAsync();
    lu_factorization_.SetColumnPermutationToIdentity();
  }
  void SetLuParameters(const LuParameters& lu) {
    DropAsync();
    lu_factorization_.SetParameters(lu);
  }
  const LuFactorization& lu() const { return lu_factorization_; }
  void SetDeviceSolver(DeviceSolver* d) { lu_factorization_.SetDeviceSolver(d); }

  // basis_representation.cc:607-624 (public: replayed by the GPU paths).
  void BumpDeterministicTimeForSolve(int64_t num_entries) const;
  // A content key of the current factorization: the basis, the LU's
  // permutations and entry counts (engine, no Glop counterpart). Handles
  // that loaded the same matrix with the same LU parameters and hold equal
  // keys hold the same factorization (Markowitz is deterministic).
  uint64_t FactorizationContentKey() const;
  const std::vector<int>& basis() const { return basis_; }
  // Factorizations shared by the handles of one batch call (LuShareCache,
  // engine only): a fresh factorization of a basis the cache holds adopts
  // the cached factors instead of running Markowitz.
  void SetLuShareCache(struct LuShareCache* c) { lu_share_ = c; }

  // Speculative flip FTRAN (engine scheduling, no Glop counterpart). The
  // next iteration's MakeBoxedVariableDualFeasible (revised_simplex.cc:
  // 2391-2437) RightSolves the bound flips' value changes against the basis
  // after this iteration's pivot. The dual loop predicts the flips right
  // after the ratio test and hands their scattered changes to SpecFlipBegin,
  // which runs L and the current etas on them. The direction's FTRAN then
  // builds the MPF update the pivot will make (its u column exactly as
  // MiddleProductFormUpdate builds it, into a scratch storage), applies it
  // and launches the U solve on a stream of its own, behind the rest of the
  // iteration (SpecFlipLaunch). SpecFlipTake hands the result over at the
  // next iteration's top when the factorization is the one it was computed
  // for (one more update, no refactorization), with the deterministic-time
  // bumps RightSolve makes there; the caller has checked the flips. The
  // vector it returns in *out is RightSolve's, bit for bit. Begin takes *f
  // (leaving an all-zero vector there) unless it returns false (PFI path).
  bool SpecFlipBegin(ScatteredVector* f, int entering_col, int leaving_row) const;
  bool SpecFlipTake(ScatteredVector* out) const;
  void SpecFlipDrop() const;  // waits for a launched solve; no-op when idle
  bool SpecFlipPending() const { return spec_state_ != SpecState::kIdle; }

 private:
  Status ComputeFactorization();
  Status MiddleProductFormUpdate(int entering_col, int leaving_variable_row);
  // MiddleProductFormUpdate's u column (basis_representation.cc:272-293):
  // the right pool's column minus U's column of the leaving row, appended to
  // *out through the all-zero scratch; returns u.v (v: the left pool's column).
  Fractional MpfColumn(int right_index, int leaving_row, int left_index,
                       std::vector<Fractional>* scratch, std::vector<int>* scratch_nz,
                       CompactSparseMatrix* out, int* u_index) const;
  void SpecFlipLaunch() const;
  enum class SpecState { kIdle, kArmed, kInflight, kDone };
  mutable SpecState spec_state_ = SpecState::kIdle;
  mutable ScatteredVector spec_vec_;  // all zero when idle
  mutable RankOneUpdateFactorization::SplitSolve spec_split_;
  mutable int spec_entering_ = -1;
  mutable int spec_leaving_ = -1;
  mutable int spec_updates_ = 0;
  mutable int64_t spec_factorizations_ = 0;
  mutable CompactSparseMatrix spec_storage_;
  // The u column SpecFlipLaunch built, when it went straight into storage_
  // (no worker reading storage_ then): MiddleProductFormUpdate of the same
  // pivot on the same factorization takes it instead of rebuilding it.
  struct SpecMpf {
    bool valid = false;
    int entering = -1, leaving = -1, right = -1, left = -1, updates = 0, u_index = -1;
    int64_t factorizations = 0;
    Fractional dot = 0.0;
  };
  mutable SpecMpf spec_mpf_;
  mutable std::vector<Fractional> spec_scratch_;
  mutable std::vector<int> spec_scratch_nz_;

  uint64_t StartAsync(AsyncKind kind, std::function<void()> job) const;
  void WaitAsync() const;
  void SyncForUnitRow() const;
  bool TauFusionEnabled() const;
  void FinishDeferredTauU() const;  // tau's U solve alone (slot 1), if still pending
  mutable bool tau_u_pending_ = false;
  void ComputeTauInto(bool can_be_optimized, const ScatteredVector& a,
                      ScatteredVector* out) const;

  const CompactSparseMatrix& compact_matrix_;
  const std::vector<int>& basis_;
  struct AsyncWorker;
  mutable std::unique_ptr<AsyncWorker> async_;
  mutable AsyncKind async_kind_ = AsyncKind::kNone;
  mutable uint64_t async_ticket_ = 0;
  mutable uint64_t tau_ticket_ = 0;
  mutable const ScatteredVector* async_input_ = nullptr;
  mutable ScatteredVector async_tau_;
  mutable std::vector<int64_t> deferred_solve_entries_;
  int async_min_rows_ = 16384;
  bool inline_tau_ = true;  // MILP_INLINE_TAU=off disables ComputeTauNow's use
  bool fuse_tau_ = true;    // MILP_TRI_PAIR=0: tau's U solve on the worker, not with the direction's
  mutable bool tau_is_computed_ = false;
  mutable bool tau_computation_can_be_optimized_ = false;
  mutable ScatteredVector tau_;
  int max_num_updates_ = 64;
  bool dynamic_period_ = true;
  int num_updates_ = 0;
  int64_t num_factorizations_ = 0;
  double factorization_seconds_ = 0.0;
  mutable std::vector<int> left_pool_mapping_;
  mutable std::vector<int> right_pool_mapping_;
  mutable CompactSparseMatrix storage_;
  mutable CompactSparseMatrix right_storage_;
  std::vector<Fractional> scratchpad_;
  std::vector<int> scratchpad_non_zeros_;
  RankOneUpdateFactorization rank_one_factorization_;
  EtaFactorization eta_factorization_;
  bool use_middle_product_form_update_ = true;
  LuFactorization lu_factorization_;
  double last_factorization_deterministic_time_ = 0.0;
  mutable double deterministic_time_ = 0.0;
  struct LuShareCache* lu_share_ = nullptr;
};

// Factorizations of one batch call's handles (mi_lp_batch_solve_bounds: the
// children of a node load the same matrix and start from the same basis),
// keyed by the basis matrix's columns, its size and the LU parameters.
// An entry also keeps its basis, compared exactly on a hit (the key is a
// hash); the batch call shares the cache only between handles whose loaded
// matrices have the same fingerprint.
struct LuShareCache {
  struct Entry {
    uint64_t key;
    std::vector<int> basis;
    std::shared_ptr<const LuFactorization> lu;
  };
  std::mutex mu;
  std::vector<Entry> entries;
  static constexpr size_t kMaxEntries = 4;
  std::shared_ptr<const LuFactorization> Find(uint64_t key, const std::vector<int>& basis) {
    std::lock_guard<std::mutex> l(mu);
    for (const auto& e : entries) {
      if (e.key == key && e.basis == basis) return e.lu;
    }
    return nullptr;
  }
  void Insert(uint64_t key, const std::vector<int>& basis, const LuFactorization& lu) {
    {
      std::lock_guard<std::mutex> l(mu);
      if (entries.size() >= kMaxEntries) return;
      for (const auto& e : entries) {
        if (e.key == key && e.basis == basis) return;
      }
    }
    auto copy = std::make_shared<LuFactorization>();
    copy->AdoptFactorizationOf(lu);
    std::lock_guard<std::mutex> l(mu);
    if (entries.size() < kMaxEntries) entries.push_back(Entry{key, basis, std::move(copy)});
  }
};

}  // namespace milp

#endif  // MILP_LU_H_
