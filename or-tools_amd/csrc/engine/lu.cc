// Host basis factorization of the MI355X simplex engine (see lu.h).
#include "lu.h"

#include <chrono>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>

namespace milp {

double g_ftran_ms[kFtPieces] = {};
const bool g_ftran_timing = std::getenv("MILP_PHASE_TIMING") != nullptr;

// ---------------------------------------------------------------------------
// Markowitz (markowitz.cc:14-494)
// MILP_LU_TIMING=1: wall time of the factorization's stages, summed over the
// process and printed at exit.
namespace {
struct LuStageTimes {
  static inline const bool on = std::getenv("MILP_LU_TIMING") != nullptr;
  static constexpr int kStages = 6;
  double ms[kStages] = {};
  int64_t count = 0;
  ~LuStageTimes() {
    if (!on || count == 0) return;
    static const char* const kNames[kStages] = {"singleton columns", "residual singletons",
                                                "residual matrix init", "markowitz loop",
                                                "row permutation", "transposes"};
    std::fprintf(stderr, "[lu timing] %lld factorizations\n", static_cast<long long>(count));
    for (int i = 0; i < kStages; ++i) {
      std::fprintf(stderr, "[lu timing]   %-22s %9.3f ms total, %.3f ms each\n", kNames[i], ms[i],
                   ms[i] / count);
    }
  }
};
LuStageTimes g_lu_times;
struct LuLap {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void Lap(int stage) {
    if (!LuStageTimes::on) return;
    const auto now = std::chrono::steady_clock::now();
    g_lu_times.ms[stage] += std::chrono::duration<double, std::milli>(now - t).count();
    t = now;
  }
};
}  // namespace

Status Markowitz::ComputeRowAndColumnPermutation(const CompactSparseMatrixView& b,
                                                 std::vector<int>* row_perm,
                                                 std::vector<int>* col_perm) {
  Clear();
  const int num_rows = b.num_rows();
  const int num_cols = b.num_cols();
  col_perm->assign(num_cols, kInvalidCol);
  row_perm->assign(num_rows, kInvalidRow);
  if (b.IsEmpty()) return Status::OK();
  basis_matrix_ = &b;
  lower_.Reset(num_rows, num_cols);
  upper_.Reset(num_rows, num_cols);
  permuted_lower_.Reset(num_cols);
  permuted_upper_.Reset(num_cols);
  permuted_lower_column_needs_solve_.assign(num_cols, false);
  contains_only_singleton_columns_ = true;

  int index = 0;
  LuLap lap;
  ExtractSingletonColumns(b, row_perm, col_perm, &index);
  lap.Lap(0);
  ExtractResidualSingletonColumns(b, row_perm, col_perm, &index);
  lap.Lap(1);
  residual_matrix_non_zero_.InitializeFromMatrixSubset(
      b, *row_perm, *col_perm, &singleton_column_, &singleton_row_);
  lap.Lap(2);

  const int end_index = std::min(num_rows, num_cols);
  const Fractional singularity_threshold =
      parameters_.markowitz_singularity_threshold;
  while (index < end_index) {
    Fractional pivot_coefficient = 0.0;
    int pivot_row = kInvalidRow;
    int pivot_col = kInvalidCol;
    const int64_t min_markowitz = FindPivot(*row_perm, *col_perm, &pivot_row,
                                            &pivot_col, &pivot_coefficient);
    if (pivot_row == kInvalidRow || pivot_col == kInvalidCol ||
        std::fabs(pivot_coefficient) <= singularity_threshold) {
      return Status(Status::ERROR_LU, "The matrix is singular!");
    }
    const int pivot_col_degree = residual_matrix_non_zero_.ColDegree(pivot_col);
    residual_matrix_non_zero_.DeleteRowAndColumn(pivot_row, pivot_col);
    if (min_markowitz == 0) {
      if (pivot_col_degree == 1) {
        RemoveRowFromResidualMatrix(pivot_row, pivot_col);
      } else {
        RemoveColumnFromResidualMatrix(pivot_row, pivot_col);
      }
    } else {
      UpdateResidualMatrix(pivot_row, pivot_col);
    }
    if (contains_only_singleton_columns_) {
      lower_.AddDiagonalOnlyColumn(1.0);
      upper_.AddTriangularColumn(b.column(pivot_col), pivot_row);
    } else {
      lower_.AddAndNormalizeTriangularColumn(permuted_lower_.column(pivot_col),
                                             pivot_row, pivot_coefficient);
      permuted_lower_.ClearAndReleaseColumn(pivot_col);
      upper_.AddTriangularColumnWithGivenDiagonalEntry(
          permuted_upper_.column(pivot_col), pivot_row, pivot_coefficient);
      permuted_upper_.ClearAndReleaseColumn(pivot_col);
    }
    (*col_perm)[pivot_col] = index;
    (*row_perm)[pivot_row] = index;
    ++index;
  }
  num_fp_operations_ += 10 * lower_.num_entries();
  num_fp_operations_ += 10 * upper_.num_entries();
  lap.Lap(3);
  return Status::OK();
}

Status Markowitz::ComputeLU(const CompactSparseMatrixView& b,
                            std::vector<int>* row_perm, std::vector<int>* col_perm,
                            TriangularMatrix* lower, TriangularMatrix* upper) {
  lower_.Swap(lower);
  upper_.Swap(upper);
  MILP_RETURN_IF_ERROR(ComputeRowAndColumnPermutation(b, row_perm, col_perm));
  LuLap lap;
  lower_.ApplyRowPermutationToNonDiagonalEntries(*row_perm);
  upper_.ApplyRowPermutationToNonDiagonalEntries(*row_perm);
  lap.Lap(4);
  lower_.Swap(lower);
  upper_.Swap(upper);
  return Status::OK();
}

void Markowitz::Clear() {
  permuted_lower_.Clear();
  permuted_upper_.Clear();
  residual_matrix_non_zero_.Clear();
  col_by_degree_.Clear();
  examined_col_.clear();
  num_fp_operations_ = 0;
  is_col_by_degree_initialized_ = false;
}

namespace {
struct MatrixEntry {
  int row;
  int col;
  Fractional coefficient;
  bool operator<(const MatrixEntry& o) const {
    return (row == o.row) ? col < o.col : row < o.row;
  }
};
}  // namespace

void Markowitz::ExtractSingletonColumns(const CompactSparseMatrixView& b,
                                        std::vector<int>* row_perm,
                                        std::vector<int>* col_perm, int* index) {
  std::vector<MatrixEntry> collected;
  const int num_cols = b.num_cols();
  const int num_rows = b.num_rows();
  for (int col = 0; col < num_cols; ++col) {
    const ColumnView c = b.column(col);
    if (c.n == 1) {
      collected.push_back(MatrixEntry{c.GetFirstRow(), col, c.GetFirstCoefficient()});
    }
  }
  // markowitz.cc sorts the entries by (row, col). The keys are distinct and
  // the entries were collected by increasing column, so a stable counting
  // sort by row gives that order in O(entries) instead of O(e log e) (a
  // third of a config-5 refactorization).
  std::vector<int> row_start(num_rows + 1, 0);
  for (const MatrixEntry& e : collected) ++row_start[e.row + 1];
  for (int r = 0; r < num_rows; ++r) row_start[r + 1] += row_start[r];
  std::vector<MatrixEntry> singleton_entries(collected.size());
  for (const MatrixEntry& e : collected) singleton_entries[row_start[e.row]++] = e;
  for (const MatrixEntry e : singleton_entries) {
    if ((*row_perm)[e.row] == kInvalidRow) {
      (*col_perm)[e.col] = *index;
      (*row_perm)[e.row] = *index;
      lower_.AddDiagonalOnlyColumn(1.0);
      upper_.AddDiagonalOnlyColumn(e.coefficient);
      ++(*index);
    }
  }
}

namespace {
bool IsResidualSingletonColumn(const ColumnView& c,
                               const std::vector<int>& row_perm, int* row) {
  int residual_degree = 0;
  for (int64_t i = 0; i < c.n; ++i) {
    if (row_perm[c.rows[i]] != kInvalidRow) continue;
    ++residual_degree;
    if (residual_degree > 1) return false;
    *row = c.rows[i];
  }
  return residual_degree == 1;
}
}  // namespace

void Markowitz::ExtractResidualSingletonColumns(const CompactSparseMatrixView& b,
                                                std::vector<int>* row_perm,
                                                std::vector<int>* col_perm,
                                                int* index) {
  const int num_cols = b.num_cols();
  int row = kInvalidRow;
  for (int col = 0; col < num_cols; ++col) {
    if ((*col_perm)[col] != kInvalidCol) continue;
    const ColumnView c = b.column(col);
    if (!IsResidualSingletonColumn(c, *row_perm, &row)) continue;
    (*col_perm)[col] = *index;
    (*row_perm)[row] = *index;
    lower_.AddDiagonalOnlyColumn(1.0);
    upper_.AddTriangularColumn(c, row);
    ++(*index);
  }
}

const SparseColumn& Markowitz::ComputeColumn(const std::vector<int>& row_perm,
                                             int col) {
  const bool first_time = permuted_lower_.column(col).IsEmpty() &&
                          permuted_upper_.column(col).IsEmpty();
  SparseColumn* lower_column = permuted_lower_.mutable_column(col);
  if (permuted_lower_column_needs_solve_[col]) {
    // Note: when not first_time, the input is a copy of lower_column since the
    // solve overwrites it (Glop passes ColumnView(*lower_column) and clears
    // lower_column only after copying its values into the scratchpad).
    if (first_time) {
      lower_.PermutedLowerSparseSolve(basis_matrix_->column(col), row_perm,
                                      lower_column,
                                      permuted_upper_.mutable_column(col));
    } else {
      const SparseColumn input = *lower_column;
      lower_.PermutedLowerSparseSolve(input.view(), row_perm, lower_column,
                                      permuted_upper_.mutable_column(col));
    }
    permuted_lower_column_needs_solve_[col] = false;
    num_fp_operations_ += lower_.NumFpOperationsInLastPermutedLowerSparseSolve();
    return *lower_column;
  }
  if (lower_column->num_entries() == residual_matrix_non_zero_.ColDegree(col)) {
    return *lower_column;
  }
  if (first_time) {
    const ColumnView c = basis_matrix_->column(col);
    num_fp_operations_ += c.n;
    lower_column->Reserve(c.n);
    for (int64_t i = 0; i < c.n; ++i)
      lower_column->SetCoefficient(c.rows[i], c.coefs[i]);
  }
  num_fp_operations_ += lower_column->num_entries();
  lower_column->MoveTaggedEntriesTo(row_perm, permuted_upper_.mutable_column(col));
  return *lower_column;
}

int64_t Markowitz::FindPivot(const std::vector<int>& row_perm,
                             const std::vector<int>& col_perm, int* pivot_row,
                             int* pivot_col, Fractional* pivot_coefficient) {
  while (!singleton_column_.empty()) {
    const int col = singleton_column_.back();
    singleton_column_.pop_back();
    if (residual_matrix_non_zero_.ColDegree(col) != 1) continue;
    if (contains_only_singleton_columns_) {
      *pivot_col = col;
      const ColumnView c = basis_matrix_->column(col);
      for (int64_t i = 0; i < c.n; ++i) {
        if (row_perm[c.rows[i]] == kInvalidRow) {
          *pivot_row = c.rows[i];
          *pivot_coefficient = c.coefs[i];
          break;
        }
      }
      return 0;
    }
    const SparseColumn& column = ComputeColumn(row_perm, col);
    if (column.IsEmpty()) continue;
    *pivot_col = col;
    *pivot_row = column.GetFirstRow();
    *pivot_coefficient = column.GetFirstCoefficient();
    return 0;
  }
  contains_only_singleton_columns_ = false;

  while (!singleton_row_.empty()) {
    const int row = singleton_row_.back();
    singleton_row_.pop_back();
    if (row_perm[row] != kInvalidRow) continue;
    if (residual_matrix_non_zero_.RowDegree(row) != 1) continue;
    const int col = residual_matrix_non_zero_.GetFirstNonDeletedColumnFromRow(row);
    if (col == kInvalidCol) continue;
    const SparseColumn& column = ComputeColumn(row_perm, col);
    if (column.IsEmpty()) continue;
    *pivot_col = col;
    *pivot_row = row;
    *pivot_coefficient = column.LookUpCoefficient(row);
    return 0;
  }

  if (!is_col_by_degree_initialized_) {
    is_col_by_degree_initialized_ = true;
    const int num_cols = static_cast<int>(col_perm.size());
    col_by_degree_.Reset(static_cast<int>(row_perm.size()), num_cols);
    for (int col = 0; col < num_cols; ++col) {
      if (col_perm[col] != kInvalidCol) continue;
      UpdateDegree(col, residual_matrix_non_zero_.ColDegree(col));
    }
  }

  int64_t min_markowitz_number = std::numeric_limits<int64_t>::max();
  examined_col_.clear();
  const int num_columns_to_examine = parameters_.markowitz_zlatev_parameter;
  const Fractional threshold = parameters_.lu_factorization_pivot_threshold;
  while (static_cast<int>(examined_col_.size()) < num_columns_to_examine) {
    const int col = col_by_degree_.Pop();
    if (col == kInvalidCol) break;
    if (col_perm[col] != kInvalidCol) continue;
    const int col_degree = residual_matrix_non_zero_.ColDegree(col);
    examined_col_.push_back(col);
    const int64_t markowitz_lower_bound = col_degree - 1;
    if (min_markowitz_number < markowitz_lower_bound) break;
    const SparseColumn& column = ComputeColumn(row_perm, col);
    Fractional max_magnitude = 0.0;
    for (int64_t k = 0; k < column.num_entries(); ++k)
      max_magnitude = std::max(max_magnitude, std::fabs(column.coefs[k]));
    if (max_magnitude == 0.0) {
      examined_col_.pop_back();
      continue;
    }
    const Fractional skip_threshold = threshold * max_magnitude;
    for (int64_t k = 0; k < column.num_entries(); ++k) {
      const Fractional magnitude = std::fabs(column.coefs[k]);
      if (magnitude < skip_threshold) continue;
      const int row_degree = residual_matrix_non_zero_.RowDegree(column.rows[k]);
      const int64_t markowitz_number =
          static_cast<int64_t>(col_degree - 1) * (row_degree - 1);
      if (markowitz_number < min_markowitz_number ||
          ((markowitz_number == min_markowitz_number) &&
           magnitude > std::fabs(*pivot_coefficient))) {
        min_markowitz_number = markowitz_number;
        *pivot_col = col;
        *pivot_row = column.rows[k];
        *pivot_coefficient = column.coefs[k];
      }
    }
  }
  for (const int col : examined_col_) {
    if (col != *pivot_col) {
      col_by_degree_.PushOrAdjust(col, residual_matrix_non_zero_.ColDegree(col));
    }
  }
  return min_markowitz_number;
}

void Markowitz::UpdateDegree(int col, int degree) {
  if (degree == 1) {
    singleton_column_.push_back(col);
  } else {
    col_by_degree_.PushOrAdjust(col, degree);
  }
}

void Markowitz::RemoveRowFromResidualMatrix(int pivot_row, int /*pivot_col*/) {
  if (is_col_by_degree_initialized_) {
    for (const int col : residual_matrix_non_zero_.RowNonZero(pivot_row)) {
      if (residual_matrix_non_zero_.IsColumnDeleted(col)) continue;
      UpdateDegree(col, residual_matrix_non_zero_.DecreaseColDegree(col));
    }
  } else {
    for (const int col : residual_matrix_non_zero_.RowNonZero(pivot_row)) {
      if (residual_matrix_non_zero_.IsColumnDeleted(col)) continue;
      if (residual_matrix_non_zero_.DecreaseColDegree(col) == 1) {
        singleton_column_.push_back(col);
      }
    }
  }
}

void Markowitz::RemoveColumnFromResidualMatrix(int /*pivot_row*/, int pivot_col) {
  const SparseColumn& c = permuted_lower_.column(pivot_col);
  for (int64_t k = 0; k < c.num_entries(); ++k) {
    const int row = c.rows[k];
    if (residual_matrix_non_zero_.DecreaseRowDegree(row) == 1) {
      singleton_row_.push_back(row);
    }
  }
}

void Markowitz::UpdateResidualMatrix(int pivot_row, int pivot_col) {
  const SparseColumn& pivot_column = permuted_lower_.column(pivot_col);
  residual_matrix_non_zero_.Update(pivot_row, pivot_col, pivot_column);
  for (const int col : residual_matrix_non_zero_.RowNonZero(pivot_row)) {
    UpdateDegree(col, residual_matrix_non_zero_.ColDegree(col));
    permuted_lower_column_needs_solve_[col] = true;
  }
  RemoveColumnFromResidualMatrix(pivot_row, pivot_col);
}

// ---------------------------------------------------------------------------
// LuFactorization (lu_factorization.cc)
namespace {
uint64_t NextFactorizationKey() {
  static std::atomic<uint64_t> next{1};
  return next.fetch_add(1, std::memory_order_relaxed);
}
}  // namespace

void LuFactorization::Clear() {
  factorization_key_ = NextFactorizationKey();
  lower_.Reset(0, 0);
  upper_.Reset(0, 0);
  transpose_upper_.Reset(0, 0);
  transpose_lower_.Reset(0, 0);
  is_identity_factorization_ = true;
  col_perm_.clear();
  row_perm_.clear();
  inverse_row_perm_.clear();
  inverse_col_perm_.clear();
}

namespace {
void PopulateFromInverse(const std::vector<int>& inverse, std::vector<int>* out) {
  out->assign(inverse.size(), 0);
  for (size_t i = 0; i < inverse.size(); ++i) (*out)[inverse[i]] = static_cast<int>(i);
}
}  // namespace

Status LuFactorization::ComputeFactorization(const CompactSparseMatrixView& b) {
  Clear();
  if (b.num_rows() != b.num_cols()) {
    return Status(Status::ERROR_LU, "Not a square matrix!!");
  }
  MILP_RETURN_IF_ERROR(
      markowitz_.ComputeLU(b, &row_perm_, &col_perm_, &lower_, &upper_));
  LuLap lap;
  PopulateFromInverse(col_perm_, &inverse_col_perm_);
  PopulateFromInverse(row_perm_, &inverse_row_perm_);
  ComputeTransposeUpper();
  ComputeTransposeLower();
  lap.Lap(5);
  if (LuStageTimes::on) ++g_lu_times.count;
  is_identity_factorization_ = false;
  return Status::OK();
}

void LuFactorization::AdoptFactorizationOf(const LuFactorization& o) {
  Clear();  // a fresh factorization key
  is_identity_factorization_ = o.is_identity_factorization_;
  lower_ = o.lower_;
  upper_ = o.upper_;
  transpose_upper_ = o.transpose_upper_;
  transpose_lower_ = o.transpose_lower_;
  col_perm_ = o.col_perm_;
  inverse_col_perm_ = o.inverse_col_perm_;
  row_perm_ = o.row_perm_;
  inverse_row_perm_ = o.inverse_row_perm_;
  markowitz_.CopyStatsFrom(o.markowitz_);
}

std::vector<int> LuFactorization::ComputeInitialBasis(
    const CompactSparseMatrix& matrix, const std::vector<int>& candidates) {
  CompactSparseMatrixView view{&matrix, &candidates};
  (void)markowitz_.ComputeRowAndColumnPermutation(view, &row_perm_, &col_perm_);
  std::vector<int> basis;
  for (int row = 0; row < matrix.num_rows(); ++row) {
    if (row_perm_[row] == kInvalidRow) {
      basis.push_back(matrix.num_cols() + (row - matrix.num_rows()));
    }
  }
  for (size_t i = 0; i < col_perm_.size(); ++i) {
    if (col_perm_[i] != kInvalidCol) basis.push_back(candidates[i]);
  }
  return basis;
}

namespace {
// lp_utils.h:240-277. The zero scratchpad is all zeros between uses (every
// user leaves it so, as upstream DCHECKs), which keeps the sparse permute
// O(nnz) instead of O(m). MILP_CHECK_SCRATCH=1 verifies the invariant.
bool CheckScratchEnabled() {
  static const bool on = [] {
    const char* e = std::getenv("MILP_CHECK_SCRATCH");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}
void CheckAllZero(const std::vector<Fractional>& v) {
  if (!CheckScratchEnabled()) return;
  for (const Fractional x : v) {
    if (x != 0.0) {
      std::fprintf(stderr, "zero scratchpad invariant violated\n");
      std::abort();
    }
  }
}
void PermuteWithScratchpad(const std::vector<int>& perm, std::vector<Fractional>* zero_scratchpad,
                           std::vector<Fractional>* io) {
  CheckAllZero(*zero_scratchpad);
  const size_t size = io->size();
  zero_scratchpad->swap(*io);
  io->resize(size, 0.0);
  for (size_t i = 0; i < size; ++i) {
    const Fractional v = (*zero_scratchpad)[i];
    if (v != 0.0) (*io)[perm[i]] = v;
  }
  zero_scratchpad->assign(size, 0.0);
}
void PermuteWithKnownNonZeros(const std::vector<int>& perm,
                              std::vector<Fractional>* zero_scratchpad,
                              std::vector<Fractional>* output, std::vector<int>* non_zeros) {
  CheckAllZero(*zero_scratchpad);
  zero_scratchpad->swap(*output);
  output->resize(zero_scratchpad->size(), 0.0);
  for (int& ref : *non_zeros) {
    const Fractional v = (*zero_scratchpad)[ref];
    (*zero_scratchpad)[ref] = 0.0;
    const int p = perm[ref];
    (*output)[p] = v;
    ref = p;
  }
  CheckAllZero(*zero_scratchpad);
}

Fractional ComputeSquaredNormAndResetToZero(const std::vector<int>& nz,
                                            std::vector<Fractional>* column) {
  Fractional sum = 0.0;
  if (nz.empty()) {
    sum = SquaredNorm(*column);
    column->clear();
  } else {
    for (const int row : nz) {
      sum += Square((*column)[row]);
      (*column)[row] = 0.0;
    }
  }
  return sum;
}
}  // namespace

// lu_factorization.cc:128-156
Fractional LuFactorization::RightSolveSquaredNorm(const ColumnView& a) const {
  if (is_identity_factorization_) return SquaredNorm(a);
  non_zero_rows_.clear();
  DenseZeroScratch().resize(lower_.num_rows(), 0.0);
  for (int64_t i = 0; i < a.n; ++i) {
    const int permuted_row = row_perm_[a.rows[i]];
    DenseZeroScratch()[permuted_row] = a.coefs[i];
    non_zero_rows_.push_back(permuted_row);
  }
  lower_.ComputeRowsToConsiderInSortedOrder(&non_zero_rows_);
  if (non_zero_rows_.empty()) {
    DenseLowerSolve(0, &DenseZeroScratch());
  } else {
    lower_.HyperSparseSolve(&DenseZeroScratch(), &non_zero_rows_);
    upper_.ComputeRowsToConsiderInSortedOrder(&non_zero_rows_);
  }
  if (non_zero_rows_.empty()) {
    DenseSolve(TriKind::kUpper, upper_, 0, &DenseZeroScratch());
  } else {
    upper_.HyperSparseSolveWithReversedNonZeros(&DenseZeroScratch(),
                                                &non_zero_rows_);
  }
  return ComputeSquaredNormAndResetToZero(non_zero_rows_, &DenseZeroScratch());
}

// lu_factorization.cc:158-186
Fractional LuFactorization::DualEdgeSquaredNorm(int row) const {
  if (is_identity_factorization_) return 1.0;
  const int permuted_row = col_perm_.empty() ? row : col_perm_[row];
  non_zero_rows_.clear();
  DenseZeroScratch().resize(lower_.num_rows(), 0.0);
  DenseZeroScratch()[permuted_row] = 1.0;
  non_zero_rows_.push_back(permuted_row);
  transpose_upper_.ComputeRowsToConsiderInSortedOrder(&non_zero_rows_);
  if (non_zero_rows_.empty()) {
    transpose_upper_.LowerSolveStartingAt(permuted_row, &DenseZeroScratch());
  } else {
    transpose_upper_.HyperSparseSolve(&DenseZeroScratch(), &non_zero_rows_);
    transpose_lower_.ComputeRowsToConsiderInSortedOrder(&non_zero_rows_);
  }
  if (non_zero_rows_.empty()) {
    transpose_lower_.UpperSolve(&DenseZeroScratch());
  } else {
    transpose_lower_.HyperSparseSolveWithReversedNonZeros(&DenseZeroScratch(),
                                                          &non_zero_rows_);
  }
  return ComputeSquaredNormAndResetToZero(non_zero_rows_, &DenseZeroScratch());
}

// The dense L loop of every FTRAN: on the device (same bits: outputs below
// `start` receive nothing in the host loop either), else on the host.
void LuFactorization::DenseLowerSolve(int start, std::vector<Fractional>* x) const {
  if (device_solver_ == nullptr || g_in_overlap ||
      !device_solver_->LowerSolve(lower_, factorization_key_, x)) {
    lower_.LowerSolveStartingAt(start, x);
  }
}

// Every other dense loop of the solves: on the device when it takes them
// (same bits, device_solver.h), else the host loop.
void LuFactorization::DenseSolve(TriKind kind, const TriangularMatrix& t, int start,
                                 std::vector<Fractional>* x) const {
  if (device_solver_ != nullptr && !g_in_overlap &&
      device_solver_->Solve(kind, t, factorization_key_, start, x)) {
    return;
  }
  switch (kind) {
    case TriKind::kUpperT:
    case TriKind::kLowerT:
      t.TransposeLowerSolve(x);
      break;
    case TriKind::kUpperTUp:
      t.TransposeUpperSolve(x);
      break;
    case TriKind::kLower:
    case TriKind::kUnitRow:
      t.LowerSolveStartingAt(start, x);
      break;
    case TriKind::kUpper:
      t.UpperSolve(x);
      break;
  }
}

// lu_factorization.cc:200-212
void LuFactorization::RightSolveLWithPermutedInput(const std::vector<Fractional>& /*a*/,
                                                   ScatteredVector* x) const {
  if (!is_identity_factorization_) {
    lower_.ComputeRowsToConsiderInSortedOrder(&x->non_zeros);
    if (x->non_zeros.empty()) {
      DenseLowerSolve(0, &x->values);
    } else {
      lower_.HyperSparseSolve(&x->values, &x->non_zeros);
    }
  }
}

// lu_factorization.cc:214-243
template <typename Column>
void LuFactorization::RightSolveLInternal(const Column& b, ScatteredVector* x) const {
  int first_column_to_consider = x->size();
  const int limit = lower_.GetFirstNonIdentityColumn();
  for (size_t k = 0; k < b.rows_size(); ++k) {
    const int permuted_row = row_perm_[b.row(k)];
    (*x)[permuted_row] = b.coef(k);
    x->non_zeros.push_back(permuted_row);
    const int col = permuted_row;
    if (col < limit || lower_.ColumnIsDiagonalOnly(col)) continue;
    first_column_to_consider = std::min(first_column_to_consider, col);
  }
  lower_.ComputeRowsToConsiderInSortedOrder(&x->non_zeros);
  x->non_zeros_are_sorted = true;
  if (x->non_zeros.empty()) {
    DenseLowerSolve(first_column_to_consider, &x->values);
  } else {
    lower_.HyperSparseSolve(&x->values, &x->non_zeros);
  }
}

namespace {
struct ColumnViewAdapter {
  const ColumnView& c;
  size_t rows_size() const { return static_cast<size_t>(c.n); }
  int row(size_t k) const { return c.rows[k]; }
  Fractional coef(size_t k) const { return c.coefs[k]; }
};
// Iteration over a ScatteredVector = iteration over its non-zero list.
struct ScatteredAdapter {
  const ScatteredVector& v;
  size_t rows_size() const { return v.non_zeros.size(); }
  int row(size_t k) const { return v.non_zeros[k]; }
  Fractional coef(size_t k) const { return v.values[v.non_zeros[k]]; }
};
}  // namespace

// lu_factorization.cc:245-258
void LuFactorization::RightSolveLForColumnView(const ColumnView& b,
                                               ScatteredVector* x) const {
  x->non_zeros.clear();
  if (is_identity_factorization_) {
    for (int64_t i = 0; i < b.n; ++i) {
      (*x)[b.rows[i]] = b.coefs[i];
      x->non_zeros.push_back(b.rows[i]);
    }
    return;
  }
  RightSolveLInternal(ColumnViewAdapter{b}, x);
}

// lu_factorization.cc:260-277
void LuFactorization::RightSolveLWithNonZeros(ScatteredVector* x) const {
  if (is_identity_factorization_) return;
  if (x->non_zeros.empty()) {
    PermuteWithScratchpad(row_perm_, &DenseZeroScratch(), &x->values);
    DenseLowerSolve(0, &x->values);
    return;
  }
  PermuteWithKnownNonZeros(row_perm_, &DenseZeroScratch(), &x->values, &x->non_zeros);
  lower_.ComputeRowsToConsiderInSortedOrder(&x->non_zeros);
  x->non_zeros_are_sorted = true;
  if (x->non_zeros.empty()) {
    DenseLowerSolve(0, &x->values);
  } else {
    lower_.HyperSparseSolve(&x->values, &x->non_zeros);
  }
}

// lu_factorization.cc:279-296
void LuFactorization::RightSolveLForScatteredColumn(const ScatteredVector& b,
                                                    ScatteredVector* x) const {
  x->non_zeros.clear();
  if (is_identity_factorization_) {
    *x = b;
    return;
  }
  if (b.non_zeros.empty()) {
    *x = b;
    RightSolveLWithNonZeros(x);
    return;
  }
  RightSolveLInternal(ScatteredAdapter{b}, x);
}

// lu_factorization.cc:298-312
void LuFactorization::LeftSolveUWithNonZeros(ScatteredVector* y) const {
  if (is_identity_factorization_) return;
  transpose_upper_.ComputeRowsToConsiderInSortedOrder(&y->non_zeros);
  y->non_zeros_are_sorted = true;
  if (y->non_zeros.empty()) {
    DenseSolve(TriKind::kUpperTUp, upper_, 0, &y->values);
  } else {
    upper_.TransposeHyperSparseSolve(&y->values, &y->non_zeros);
  }
}

void LuFactorization::RightSolveUWithNonZerosPair(ScatteredVector* x,
                                                  ScatteredVector* tau) const {
  if (is_identity_factorization_) return;
  {
    FtranTimer t(kFtURows);
    upper_.ComputeRowsToConsiderInSortedOrder(&x->non_zeros);
  }
  x->non_zeros_are_sorted = true;
  {
    LuSlotGuard slot(1);
    upper_.ComputeRowsToConsiderInSortedOrder(&tau->non_zeros);
    tau->non_zeros_are_sorted = true;
  }
  if (x->non_zeros.empty() && tau->non_zeros.empty() && device_solver_ != nullptr &&
      device_solver_->SolvePair(TriKind::kUpperT, transpose_upper_, factorization_key_,
                                &x->values, &tau->values)) {
    return;
  }
  RightSolveUAfterRows(x);
  LuSlotGuard slot(1);
  RightSolveUAfterRows(tau);
}

// lu_factorization.cc:314-331
void LuFactorization::RightSolveUWithNonZeros(ScatteredVector* x) const {
  if (is_identity_factorization_) return;
  {
    FtranTimer t(kFtURows);
    upper_.ComputeRowsToConsiderInSortedOrder(&x->non_zeros);
  }
  x->non_zeros_are_sorted = true;
  RightSolveUAfterRows(x);
}

void LuFactorization::RightSolveUAfterRows(ScatteredVector* x) const {
  if (x->non_zeros.empty()) {
    // The dense U solve: on the device (the solver's thread and the tau
    // worker each with its own stream), same result bits.
    if (device_solver_ == nullptr ||
        !device_solver_->TransposeLowerSolve(transpose_upper_, factorization_key_,
                                             &x->values)) {
      g_overlap.Run();
      FtranTimer t(kFtUHost);
      transpose_upper_.TransposeLowerSolve(&x->values);
    }
  } else {
    g_overlap.Run();
    FtranTimer t(kFtUHost);
    transpose_upper_.TransposeHyperSparseSolveWithReversedNonZeros(
        &x->values, &x->non_zeros);
  }
}

int LuFactorization::StartRightSolveUAsync(ScatteredVector* x) const {
  if (is_identity_factorization_) return 0;
  upper_.ComputeRowsToConsiderInSortedOrder(&x->non_zeros);
  x->non_zeros_are_sorted = true;
  if (!x->non_zeros.empty()) {
    transpose_upper_.TransposeHyperSparseSolveWithReversedNonZeros(&x->values, &x->non_zeros);
    return 0;
  }
  if (device_solver_ != nullptr &&
      device_solver_->StartAsyncU(transpose_upper_, factorization_key_, x->values)) {
    return 1;
  }
  return -1;
}

void LuFactorization::FinishRightSolveUAsync(ScatteredVector* x) const {
  device_solver_->FinishAsyncU(&x->values);
}

void LuFactorization::DropRightSolveUAsync() const {
  if (device_solver_ != nullptr) device_solver_->DropAsyncU();
}

// lu_factorization.cc:333-399
bool LuFactorization::LeftSolveLWithNonZeros(
    ScatteredVector* y, ScatteredVector* result_before_permutation) const {
  if (is_identity_factorization_) return false;
  std::vector<Fractional>* x = &y->values;
  std::vector<int>* nz = &y->non_zeros;
  transpose_lower_.ComputeRowsToConsiderInSortedOrder(nz);
  y->non_zeros_are_sorted = true;
  if (nz->empty()) {
    DenseSolve(TriKind::kLowerT, lower_, 0, x);
  } else {
    lower_.TransposeHyperSparseSolveWithReversedNonZeros(x, nz);
  }
  if (result_before_permutation == nullptr) {
    if (nz->empty()) {
      PermuteWithScratchpad(inverse_row_perm_, &DenseZeroScratch(), x);
    } else {
      PermuteWithKnownNonZeros(inverse_row_perm_, &DenseZeroScratch(), x, nz);
    }
    return false;
  }
  // ClearAndResizeVectorWithNonZeros(x->size(), result_before_permutation)
  ClearAndResizeVectorWithNonZeros(static_cast<int>(x->size()),
                                   result_before_permutation);
  x->swap(result_before_permutation->values);
  if (nz->empty()) {
    for (size_t row = 0; row < inverse_row_perm_.size(); ++row) {
      const Fractional value = result_before_permutation->values[row];
      if (value != 0.0) (*x)[inverse_row_perm_[row]] = value;
    }
  } else {
    nz->swap(result_before_permutation->non_zeros);
    nz->reserve(result_before_permutation->non_zeros.size());
    for (const int row : result_before_permutation->non_zeros) {
      const Fractional value = result_before_permutation->values[row];
      const int permuted_row = inverse_row_perm_[row];
      (*x)[permuted_row] = value;
      nz->push_back(permuted_row);
    }
    y->non_zeros_are_sorted = false;
  }
  return true;
}

// lu_factorization.cc:405-436
int LuFactorization::LeftSolveUForUnitRow(int col, ScatteredVector* y) const {
  if (is_identity_factorization_) {
    (*y)[col] = 1.0;
    y->non_zeros.push_back(col);
    return col;
  }
  const int permuted_col = col_perm_.empty() ? col : col_perm_[col];
  (*y)[permuted_col] = 1.0;
  y->non_zeros.push_back(permuted_col);
  if (transpose_upper_.ColumnIsDiagonalOnly(permuted_col)) {
    (*y)[permuted_col] /= transpose_upper_.GetDiagonalCoefficient(permuted_col);
  } else {
    transpose_upper_.ComputeRowsToConsiderInSortedOrder(&y->non_zeros);
    y->non_zeros_are_sorted = true;
    if (y->non_zeros.empty()) {
      DenseSolve(TriKind::kUnitRow, transpose_upper_, permuted_col, &y->values);
    } else {
      transpose_upper_.HyperSparseSolve(&y->values, &y->non_zeros);
    }
  }
  return permuted_col;
}

// lu_factorization.cc:438-447
const SparseColumn& LuFactorization::GetColumnOfU(int col) const {
  if (is_identity_factorization_) {
    column_of_upper_.Clear();
    column_of_upper_.SetCoefficient(col, 1.0);
    return column_of_upper_;
  }
  upper_.CopyColumnToSparseColumn(col_perm_.empty() ? col : col_perm_[col],
                                  &column_of_upper_);
  return column_of_upper_;
}

// lu_factorization.cc:102-122 with permutation.h:200-235 (ApplyPermutation,
// ApplyInversePermutation: an empty permutation copies).
namespace {
void ApplyPermutationTo(const std::vector<int>& perm, const std::vector<Fractional>& b,
                        std::vector<Fractional>* result) {
  if (perm.empty()) {
    *result = b;
    return;
  }
  result->resize(b.size(), b.back());
  for (size_t i = 0; i < perm.size(); ++i) (*result)[perm[i]] = b[i];
}
void ApplyInversePermutationTo(const std::vector<int>& perm, const std::vector<Fractional>& b,
                               std::vector<Fractional>* result) {
  if (perm.empty()) {
    *result = b;
    return;
  }
  result->resize(b.size(), b.back());
  for (size_t i = 0; i < perm.size(); ++i) (*result)[i] = b[perm[i]];
}
}  // namespace

void LuFactorization::RightSolve(std::vector<Fractional>* x) const {
  if (is_identity_factorization_) return;
  ApplyPermutationTo(row_perm_, *x, &dense_column_scratchpad_);
  DenseLowerSolve(0, &dense_column_scratchpad_);
  DenseSolve(TriKind::kUpper, upper_, 0, &dense_column_scratchpad_);
  ApplyPermutationTo(inverse_col_perm_, dense_column_scratchpad_, x);
}

void LuFactorization::LeftSolve(std::vector<Fractional>* y) const {
  if (is_identity_factorization_) return;
  ApplyInversePermutationTo(inverse_col_perm_, *y, &dense_column_scratchpad_);
  DenseSolve(TriKind::kUpperTUp, upper_, 0, &dense_column_scratchpad_);
  DenseSolve(TriKind::kLowerT, lower_, 0, &dense_column_scratchpad_);
  ApplyInversePermutationTo(row_perm_, dense_column_scratchpad_, y);
}

// basis_representation.cc:25-125 (EtaMatrix, kSparseThreshold 0.5).
EtaMatrix::EtaMatrix(int eta_col, const ScatteredVector& direction)
    : eta_col_(eta_col), eta_col_coefficient_(direction[eta_col]) {
  eta_coeff_ = direction.values;
  eta_coeff_[eta_col_] = 0.0;
  if (static_cast<double>(direction.non_zeros.size()) < 0.5 * eta_coeff_.size()) {
    for (const int row : direction.non_zeros) {
      if (row == eta_col) continue;
      sparse_eta_coeff_.AddEntry(row, eta_coeff_[row]);
    }
  }
}

void EtaMatrix::LeftSolve(std::vector<Fractional>* y) const {
  Fractional y_value = (*y)[eta_col_];
  if (!sparse_eta_coeff_.IsEmpty()) {
    for (int64_t i = 0; i < sparse_eta_coeff_.num_entries(); ++i) {
      y_value -= (*y)[sparse_eta_coeff_.rows[i]] * sparse_eta_coeff_.coefs[i];
    }
  } else {
    const size_t n = eta_coeff_.size();
    for (size_t row = 0; row < n; ++row) y_value -= (*y)[row] * eta_coeff_[row];
  }
  (*y)[eta_col_] = y_value / eta_col_coefficient_;
}

void EtaMatrix::RightSolve(std::vector<Fractional>* d) const {
  if ((*d)[eta_col_] == 0.0) return;
  const Fractional coeff = (*d)[eta_col_] / eta_col_coefficient_;
  if (!sparse_eta_coeff_.IsEmpty()) {
    for (int64_t i = 0; i < sparse_eta_coeff_.num_entries(); ++i) {
      (*d)[sparse_eta_coeff_.rows[i]] -= sparse_eta_coeff_.coefs[i] * coeff;
    }
  } else {
    const size_t n = eta_coeff_.size();
    for (size_t row = 0; row < n; ++row) (*d)[row] -= eta_coeff_[row] * coeff;
  }
  (*d)[eta_col_] = coeff;
}

void EtaMatrix::SparseLeftSolve(std::vector<Fractional>* y, std::vector<int>* pos) const {
  Fractional y_value = (*y)[eta_col_];
  bool is_eta_col_in_pos = false;
  const int size = static_cast<int>(pos->size());
  for (int i = 0; i < size; ++i) {
    const int col = (*pos)[i];
    if (col == eta_col_) {
      is_eta_col_in_pos = true;
      continue;
    }
    y_value -= (*y)[col] * eta_coeff_[col];
  }
  (*y)[eta_col_] = y_value / eta_col_coefficient_;
  if (!is_eta_col_in_pos) pos->push_back(eta_col_);
}

// ---------------------------------------------------------------------------
// BasisFactorization (basis_representation.cc:176-627)

// One worker thread, one job at a time (the tau FTRAN).
struct BasisFactorization::AsyncWorker {
  AsyncWorker() : thread([this]() { Loop(); }) {}
  ~AsyncWorker() {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    thread.join();
  }
  void Submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> l(mu);
      job = std::move(f);
      busy = true;
    }
    cv.notify_all();
  }
  void Wait() {
    std::unique_lock<std::mutex> l(mu);
    done_cv.wait(l, [&]() { return !busy; });
  }
  void Loop() {
    g_lu_slot = 1;
    std::unique_lock<std::mutex> l(mu);
    while (true) {
      cv.wait(l, [&]() { return stop || static_cast<bool>(job); });
      if (stop) return;
      std::function<void()> f = std::move(job);
      job = nullptr;
      l.unlock();
      f();
      l.lock();
      busy = false;
      done_cv.notify_all();
    }
  }
  std::mutex mu;
  std::condition_variable cv;
  std::condition_variable done_cv;
  std::function<void()> job;
  bool busy = false;
  bool stop = false;
  std::thread thread;
};

BasisFactorization::BasisFactorization(const CompactSparseMatrix* matrix,
                                       const std::vector<int>* basis)
    : compact_matrix_(*matrix), basis_(*basis) {
  if (const char* e = std::getenv("MILP_ASYNC_SOLVES")) {
    if (std::strcmp(e, "off") == 0) async_min_rows_ = -1;
    if (std::strcmp(e, "force") == 0) async_min_rows_ = 0;
  }
  if (const char* e = std::getenv("MILP_INLINE_TAU")) inline_tau_ = std::strcmp(e, "off") != 0;
  if (const char* e = std::getenv("MILP_TRI_PAIR")) fuse_tau_ = std::atoi(e) != 0;
}

BasisFactorization::~BasisFactorization() {
  if (async_) async_->Wait();
}

bool BasisFactorization::AsyncEnabled() const {
  // The product-form path solves through one shared dense scratchpad.
  return use_middle_product_form_update_ && async_min_rows_ >= 0 &&
         compact_matrix_.num_rows() >= async_min_rows_;
}

uint64_t BasisFactorization::StartAsync(AsyncKind kind, std::function<void()> job) const {
  DropAsync();
  if (!async_) async_.reset(new AsyncWorker());
  async_kind_ = kind;
  async_->Submit(std::move(job));
  return ++async_ticket_;
}

bool BasisFactorization::TakeAsync(uint64_t ticket) const {
  if (async_kind_ == AsyncKind::kNone || ticket != async_ticket_) return false;
  if (async_) async_->Wait();
  if (async_kind_ == AsyncKind::kTauDeferred) FinishDeferredTauU();
  async_kind_ = AsyncKind::kNone;
  async_input_ = nullptr;
  // The worker's deterministic-time bumps land now, where the serial solve
  // would have made them.
  rank_one_factorization_.TakeDeferredBumps(true);
  for (const int64_t n : deferred_solve_entries_) BumpDeterministicTimeForSolve(n);
  deferred_solve_entries_.clear();
  return true;
}

void BasisFactorization::DropAsync() const {
  if (async_kind_ == AsyncKind::kNone) return;
  if (async_) async_->Wait();
  tau_u_pending_ = false;
  async_kind_ = AsyncKind::kNone;
  async_input_ = nullptr;
  rank_one_factorization_.TakeDeferredBumps(false);
  deferred_solve_entries_.clear();
}

void BasisFactorization::WaitAsync() const {
  if (async_kind_ != AsyncKind::kNone && async_) async_->Wait();
}

// The body of RightSolveForTau (basis_representation.cc:374-398) into *out,
// without the flag updates.
void BasisFactorization::ComputeTauInto(bool can_be_optimized, const ScatteredVector& a,
                                        ScatteredVector* out) const {
  if (can_be_optimized) {
    lu_factorization_.RightSolveLWithPermutedInput(a.values, out);
  } else {
    ClearAndResizeVectorWithNonZeros(compact_matrix_.num_rows(), out);
    lu_factorization_.RightSolveLForScatteredColumn(a, out);
  }
  rank_one_factorization_.RightSolveWithNonZeros(out);
  lu_factorization_.RightSolveUWithNonZeros(out);
  BumpDeterministicTimeForSolve(static_cast<int64_t>(out->NumNonZerosEstimate()));
}

bool BasisFactorization::TauFusionEnabled() const {
  return fuse_tau_ && AsyncEnabled() && lu_factorization_.HasDeviceSolver();
}

// tau's U solve, alone, on slot 1 (the pending half of a deferred tau), with
// the bump ComputeTauInto makes after it (deferred like the others).
void BasisFactorization::FinishDeferredTauU() const {
  if (!tau_u_pending_) return;
  LuSlotGuard slot(1);
  lu_factorization_.RightSolveUWithNonZeros(&async_tau_);
  BumpDeterministicTimeForSolve(static_cast<int64_t>(async_tau_.NumNonZerosEstimate()));
  tau_u_pending_ = false;
}

void BasisFactorization::StartAsyncTau(const ScatteredVector& rho) const {
  DropAsync();
  if (TauFusionEnabled()) {
    // tau = B^-1 rho (dual_edge_norms.cc:134-141) against the factorization
    // the direction is solved with next: L and the etas on the worker (slot
    // 1, bumps deferred), the U solve together with the direction's
    // (RightSolveForProblemColumn), taken in RightSolveForTau.
    const bool can_be_optimized = tau_computation_can_be_optimized_;
    tau_ticket_ = StartAsync(AsyncKind::kTauDeferred, [this, can_be_optimized, &rho]() {
      if (can_be_optimized) {
        async_tau_ = tau_;
        lu_factorization_.RightSolveLWithPermutedInput(rho.values, &async_tau_);
      } else {
        ClearAndResizeVectorWithNonZeros(compact_matrix_.num_rows(), &async_tau_);
        lu_factorization_.RightSolveLForScatteredColumn(rho, &async_tau_);
      }
      rank_one_factorization_.RightSolveWithNonZeros(&async_tau_);
      tau_u_pending_ = true;  // read by the solver's thread after Wait
    });
    async_input_ = &rho;
    return;
  }
  if (!AsyncEnabled()) return;
  const bool can_be_optimized = tau_computation_can_be_optimized_;
  tau_ticket_ = StartAsync(AsyncKind::kTau, [this, can_be_optimized, &rho]() {
    // The permuted intermediate of the last BTRAN is copied, not consumed:
    // a discarded result leaves tau_ as the serial code would.
    if (can_be_optimized) async_tau_ = tau_;
    ComputeTauInto(can_be_optimized, rho, &async_tau_);
  });
  async_input_ = &rho;
}

// Below the worker-thread size the same tau is computed on the calling thread
// while the GPU computes the update row (the caller launches it first): the
// result and its deferred deterministic-time bumps are handed over through
// the same slot and ticket as the worker's, so TakeAsync/DropAsync behave
// identically (solve scratch slot 1, bumps applied when taken).
bool BasisFactorization::InlineTauEnabled() const {
  return inline_tau_ && use_middle_product_form_update_ && !AsyncEnabled();
}

void BasisFactorization::ComputeTauNow(const ScatteredVector& rho) const {
  DropAsync();
  const bool can_be_optimized = tau_computation_can_be_optimized_;
  async_kind_ = AsyncKind::kTau;
  tau_ticket_ = ++async_ticket_;
  const int saved_slot = g_lu_slot;
  g_lu_slot = 1;
  if (can_be_optimized) async_tau_ = tau_;
  ComputeTauInto(can_be_optimized, rho, &async_tau_);
  g_lu_slot = saved_slot;
  async_input_ = &rho;
}

uint64_t BasisFactorization::StartAsyncLeftSolve(std::function<void()> job) const {
  DropAsync();
  if (!AsyncEnabled()) return 0;
  return StartAsync(AsyncKind::kLeftSolve, std::move(job));
}

// A BTRAN for a unit row reads and extends the left pool (storage_): a
// pending tau was not taken and is dropped; a pending left solve (which
// reads storage_) is waited for and kept.
void BasisFactorization::SyncForUnitRow() const {
  if (async_kind_ == AsyncKind::kLeftSolve) {
    WaitAsync();
  } else {
    DropAsync();
  }
}

void BasisFactorization::Clear() {
  DropAsync();
  SpecFlipDrop();
  spec_mpf_.valid = false;
  num_updates_ = 0;
  tau_computation_can_be_optimized_ = false;
  lu_factorization_.Clear();
  rank_one_factorization_.Clear();
  eta_factorization_.Clear();
  storage_.Reset(compact_matrix_.num_rows());
  right_storage_.Reset(compact_matrix_.num_rows());
  left_pool_mapping_.clear();
  right_pool_mapping_.clear();
}

Status BasisFactorization::Initialize() {
  DropAsync();
  Clear();
  if (IsIdentityBasis()) return Status::OK();
  return ComputeFactorization();
}

std::vector<int> BasisFactorization::ComputeInitialBasis(
    const std::vector<int>& candidates) {
  DropAsync();
  std::vector<int> basis =
      lu_factorization_.ComputeInitialBasis(compact_matrix_, candidates);
  deterministic_time_ += lu_factorization_.DeterministicTimeOfLastFactorization();
  return basis;
}

Status BasisFactorization::Refactorize() {
  if (IsRefactorized()) return Status::OK();
  return ForceRefactorization();
}

Status BasisFactorization::ForceRefactorization() {
  DropAsync();
  Clear();
  return ComputeFactorization();
}

Status BasisFactorization::ComputeFactorization() {
  CompactSparseMatrixView basis_matrix{&compact_matrix_, &basis_};
  const auto t0 = std::chrono::steady_clock::now();
  uint64_t share_key = 0;
  std::shared_ptr<const LuFactorization> shared;
  if (lu_share_ != nullptr) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
    mix(static_cast<uint64_t>(compact_matrix_.num_rows()));
    mix(static_cast<uint64_t>(compact_matrix_.num_cols()));
    for (const int c : basis_) mix(static_cast<uint32_t>(c));
    const LuParameters& p = lu_factorization_.parameters();
    uint64_t bits;
    std::memcpy(&bits, &p.lu_factorization_pivot_threshold, 8);
    mix(bits);
    std::memcpy(&bits, &p.markowitz_singularity_threshold, 8);
    mix(bits);
    mix(static_cast<uint64_t>(p.markowitz_zlatev_parameter));
    share_key = h | 1;
    shared = lu_share_->Find(share_key, basis_);
  }
  Status status;
  if (shared != nullptr) {
    lu_factorization_.AdoptFactorizationOf(*shared);
  } else {
    status = lu_factorization_.ComputeFactorization(basis_matrix);
    if (share_key != 0 && status.ok()) lu_share_->Insert(share_key, basis_, lu_factorization_);
  }
  ++num_factorizations_;
  factorization_seconds_ +=
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  last_factorization_deterministic_time_ =
      lu_factorization_.DeterministicTimeOfLastFactorization();
  deterministic_time_ += last_factorization_deterministic_time_;
  rank_one_factorization_.ResetDeterministicTime();
  return status;
}

// basis_representation.cc:258-302
Status BasisFactorization::MiddleProductFormUpdate(int entering_col,
                                                   int leaving_variable_row) {
  const int right_index = entering_col < static_cast<int>(right_pool_mapping_.size())
                              ? right_pool_mapping_[entering_col]
                              : kInvalidCol;
  const int left_index =
      leaving_variable_row < static_cast<int>(left_pool_mapping_.size())
          ? left_pool_mapping_[leaving_variable_row]
          : kInvalidCol;
  if (right_index == kInvalidCol || left_index == kInvalidCol) {
    return ForceRefactorization();
  }
  int u_index = 0;
  Fractional scalar_product = 0.0;
  const SpecMpf& sm = spec_mpf_;
  if (sm.valid && sm.entering == entering_col && sm.leaving == leaving_variable_row &&
      sm.right == right_index && sm.left == left_index &&
      sm.factorizations == num_factorizations_ && sm.updates + 1 == num_updates_) {
    // Built by the speculative flip FTRAN from the same columns (SpecFlipLaunch).
    u_index = sm.u_index;
    scalar_product = sm.dot;
  } else {
    scalar_product = MpfColumn(right_index, leaving_variable_row, left_index, &scratchpad_,
                               &scratchpad_non_zeros_, &storage_, &u_index);
  }
  spec_mpf_.valid = false;
  RankOneUpdateElementaryMatrix m(&storage_, u_index, left_index, scalar_product);
  if (m.IsSingular()) {
    return Status(Status::ERROR_LU, "Degenerate rank-one update.");
  }
  rank_one_factorization_.Update(m);
  return Status::OK();
}

Fractional BasisFactorization::MpfColumn(int right_index, int leaving_row, int left_index,
                                         std::vector<Fractional>* scratch,
                                         std::vector<int>* scratch_nz, CompactSparseMatrix* out,
                                         int* u_index) const {
  scratch->resize(right_storage_.num_rows(), 0.0);
  const ColumnView rc = right_storage_.column(right_index);
  for (int64_t i = 0; i < rc.n; ++i) {
    (*scratch)[rc.rows[i]] = rc.coefs[i];
    scratch_nz->push_back(rc.rows[i]);
  }
  const SparseColumn& column_of_u = lu_factorization_.GetColumnOfU(leaving_row);
  for (int64_t k = 0; k < column_of_u.num_entries(); ++k) {
    (*scratch)[column_of_u.rows[k]] -= column_of_u.coefs[k];
    scratch_nz->push_back(column_of_u.rows[k]);
  }
  const Fractional scalar_product = storage_.ColumnScalarProduct(left_index, scratch->data());
  *u_index = out->AddAndClearColumnWithNonZeros(scratch, scratch_nz);
  return scalar_product;
}

// ---- speculative flip FTRAN (lu.h, BasisFactorization::SpecFlipBegin) ----
bool BasisFactorization::SpecFlipBegin(ScatteredVector* f, int entering_col,
                                       int leaving_row) const {
  SpecFlipDrop();
  if (!use_middle_product_form_update_) return false;
  std::swap(spec_vec_, *f);  // *f gets the idle (all-zero) vector
  spec_entering_ = entering_col;
  spec_leaving_ = leaving_row;
  spec_updates_ = num_updates_;
  spec_factorizations_ = num_factorizations_;
  spec_state_ = SpecState::kArmed;
  return true;
}

// Inside the direction's FTRAN (after its right-pool append, while its U
// solve runs on the device): the update UpdateAndPivot will make, applied
// to the flip vector, then the flip vector's U solve.
void BasisFactorization::SpecFlipLaunch() const {
  if (spec_state_ != SpecState::kArmed) return;
  const int right_index = spec_entering_ < static_cast<int>(right_pool_mapping_.size())
                              ? right_pool_mapping_[spec_entering_]
                              : kInvalidCol;
  const int left_index = spec_leaving_ < static_cast<int>(left_pool_mapping_.size())
                             ? left_pool_mapping_[spec_leaving_]
                             : kInvalidCol;
  if (right_index == kInvalidCol || left_index == kInvalidCol) {
    SpecFlipDrop();
    return;
  }
  // RightSolve (basis_representation.cc:358-372): L and the etas it has now
  // (none changed since the ratio test), while the device solves the
  // direction's U; their dense loops stay on the host (g_in_overlap).
  lu_factorization_.RightSolveLWithNonZeros(&spec_vec_);
  rank_one_factorization_.RightSolveBegin(&spec_vec_, &spec_split_);
  // u goes straight into storage_ (where MiddleProductFormUpdate would put
  // it) unless a worker may be reading storage_ now; an unused column there
  // is never referenced and goes with the next refactorization's Clear.
  const bool into_storage =
      async_kind_ == AsyncKind::kNone || async_kind_ == AsyncKind::kTauDeferred;
  CompactSparseMatrix* out = into_storage ? &storage_ : &spec_storage_;
  if (!into_storage) spec_storage_.Reset(compact_matrix_.num_rows());
  int u_index = 0;
  const Fractional dot = MpfColumn(right_index, spec_leaving_, left_index, &spec_scratch_,
                                   &spec_scratch_nz_, out, &u_index);
  if (into_storage) {
    spec_mpf_ = SpecMpf{true, spec_entering_, spec_leaving_, right_index, left_index,
                        num_updates_, u_index, num_factorizations_, dot};
  }
  const RankOneUpdateElementaryMatrix next(&storage_, u_index, left_index, dot, out);
  if (next.IsSingular()) {
    SpecFlipDrop();
    return;
  }
  rank_one_factorization_.RightSolveEnd(&spec_vec_, spec_split_, next);
  const int r = lu_factorization_.StartRightSolveUAsync(&spec_vec_);
  if (r < 0) {
    SpecFlipDrop();
    return;
  }
  spec_state_ = r == 1 ? SpecState::kInflight : SpecState::kDone;
}

bool BasisFactorization::SpecFlipTake(ScatteredVector* out) const {
  if (spec_state_ != SpecState::kInflight && spec_state_ != SpecState::kDone) {
    SpecFlipDrop();
    return false;
  }
  if (num_factorizations_ != spec_factorizations_ || num_updates_ != spec_updates_ + 1) {
    SpecFlipDrop();
    return false;
  }
  if (spec_state_ == SpecState::kInflight) {
    spec_state_ = SpecState::kDone;
    lu_factorization_.FinishRightSolveUAsync(&spec_vec_);
  }
  spec_state_ = SpecState::kIdle;
  std::swap(*out, spec_vec_);  // spec_vec_ takes the caller's all-zero vector
  out->SortNonZerosIfNeeded();
  // RightSolve's bumps, in its order: the etas', then the solve's.
  rank_one_factorization_.BumpTime();
  BumpDeterministicTimeForSolve(static_cast<int64_t>(out->NumNonZerosEstimate()));
  return true;
}

void BasisFactorization::SpecFlipDrop() const {
  if (spec_state_ == SpecState::kIdle) return;
  if (spec_state_ == SpecState::kInflight) lu_factorization_.DropRightSolveUAsync();
  spec_state_ = SpecState::kIdle;
  std::fill(spec_vec_.values.begin(), spec_vec_.values.end(), 0.0);
  spec_vec_.non_zeros.clear();
  spec_vec_.non_zeros_are_sorted = false;
  spec_vec_.is_non_zero.assign(spec_vec_.values.size(), false);
}

// basis_representation.cc:304-340
Status BasisFactorization::Update(int entering_col, int leaving_variable_row,
                                  const ScatteredVector& direction) {
  DropAsync();
  if (num_updates_ >= max_num_updates_) {
    if (!dynamic_period_) return ForceRefactorization();
    if (last_factorization_deterministic_time_ <
        rank_one_factorization_.DeterministicTimeSinceLastReset()) {
      return ForceRefactorization();
    }
  }
  ++num_updates_;
  if (use_middle_product_form_update_) {
    MILP_RETURN_IF_ERROR(MiddleProductFormUpdate(entering_col, leaving_variable_row));
  } else {
    eta_factorization_.Update(entering_col, leaving_variable_row, direction);
  }
  tau_computation_can_be_optimized_ = false;
  return Status::OK();
}

// basis_representation.cc:342-356
void BasisFactorization::LeftSolve(ScatteredVector* y) const {
  if (!use_middle_product_form_update_) {
    y->non_zeros.clear();
    eta_factorization_.LeftSolve(&y->values);
    lu_factorization_.LeftSolve(&y->values);
    BumpDeterministicTimeForSolve(static_cast<int64_t>(y->NumNonZerosEstimate()));
    return;
  }
  lu_factorization_.LeftSolveUWithNonZeros(y);
  rank_one_factorization_.LeftSolveWithNonZeros(y);
  lu_factorization_.LeftSolveLWithNonZeros(y, nullptr);
  y->SortNonZerosIfNeeded();
  BumpDeterministicTimeForSolve(static_cast<int64_t>(y->NumNonZerosEstimate()));
}

thread_local OverlapWork g_overlap;
thread_local bool g_in_overlap = false;
void OverlapWork::Run() {
  if (!f) return;
  std::function<void()> g = std::move(f);
  f = nullptr;
  struct Flag {
    Flag() { g_in_overlap = true; }
    ~Flag() { g_in_overlap = false; }
  } flag;
  g();
}

bool TriangularMatrix::ParallelTransposeSolve(bool forward, std::vector<Fractional>* rhs) const {
  // Opt-in (MILP_HOST_TRI_PAR=1): on the MI355X box the gain on config 2's
  // late window stayed within the noise and config 5's window read -9 % / +3 %
  // in two A/Bs (scripts/gpu_r04_tripar.sh).
  static const bool enabled = [] {
    const char* e = std::getenv("MILP_HOST_TRI_PAR");
    return e != nullptr && std::atoi(e) != 0;
  }();
  constexpr int kMinRun = 2048;
  const int n = num_cols_;
  const int fni = first_non_identity_column_;
  // (A dense tail can be short: a kernel of a few hundred columns behind
  // thousands of identity columns.)
  if (!enabled || n - fni < 64 || HostPool::Get().threads() <= 1) return false;
  const int d = forward ? 0 : 1;
  if (!par_ready_[d]) {
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    if (!par_ready_[d]) {
      std::vector<int>& runs = par_runs_[d];
      runs.clear();
      int64_t long_entries = 0;
      if (forward) {
        // Column c reads rows r < c (and rows below fni, final): a run
        // [a, b) reads no row of its own iff every column's largest row < a.
        int a = fni;
        while (a < n) {
          int b = a + 1;
          while (b < n) {
            int mx = -1;
            for (int64_t i = starts_[b]; i < starts_[b + 1]; ++i) mx = std::max(mx, rows_[i]);
            if (mx >= a) break;
            ++b;
          }
          if (b - a >= kMinRun) {
            runs.push_back(a);
            runs.push_back(b);
            long_entries += starts_[b] - starts_[a];
          }
          a = b;
        }
        // A dense tail: the trailing columns holding at least n/4 entries
        // each. Their leading groups of four that read rows below the tail
        // only are final when the tail starts: that part of each column's
        // subtraction chain is computed for all tail columns at once.
        par_tail_ = -1;
        int t = n;
        while (t > fni && starts_[t] - starts_[t - 1] >= n / 4) --t;
        if (n - t >= 64) {
          par_split_.assign(n - t, 0);
          int64_t pre = 0;
          for (int c = t; c < n; ++c) {
            const int64_t i0 = starts_[c], i1 = starts_[c + 1];
            int64_t i = i0;
            while (i + 3 < i1 && rows_[i] < t && rows_[i + 1] < t && rows_[i + 2] < t &&
                   rows_[i + 3] < t) {
              i += 4;
            }
            par_split_[c - t] = i;
            pre += i - i0;
          }
          if (pre >= (1 << 16)) {
            par_tail_ = t;
            // Runs past the tail's start would race with it: cut them there.
            std::vector<int> kept;
            for (size_t r = 0; r < runs.size(); r += 2) {
              const int rb = runs[r], re = std::min(runs[r + 1], t);
              if (re - rb >= kMinRun) {
                kept.push_back(rb);
                kept.push_back(re);
              }
            }
            runs.swap(kept);
            long_entries = std::max<int64_t>(long_entries, 1 << 16);  // the tail pays
          }
        }
      } else {
        // Column c reads rows r > c: a run from a down to b reads no row of
        // its own iff every column's smallest row > a.
        int a = n - 1;
        while (a >= fni) {
          int b = a - 1;
          while (b >= fni) {
            int mn = n;
            for (int64_t i = starts_[b]; i < starts_[b + 1]; ++i) mn = std::min(mn, rows_[i]);
            if (mn <= a) break;
            --b;
          }
          if (a - b >= kMinRun) {
            runs.push_back(b + 1);  // [b + 1, a + 1)
            runs.push_back(a + 1);
            long_entries += starts_[a + 1] - starts_[b + 1];
          }
          a = b;
        }
      }
      if (long_entries < (1 << 16)) runs.clear();
      static const bool debug = std::getenv("MILP_HOST_TRI_PAR_DEBUG") != nullptr;
      if (debug) {
        int cols = 0;
        for (size_t r = 0; r < runs.size(); r += 2) cols += runs[r + 1] - runs[r];
        std::fprintf(stderr, "[tri par] %s n %d fni %d: %zu runs, %d columns, %lld entries, tail %d\n",
                     forward ? "forward" : "backward", n, fni, runs.size() / 2, cols,
                     static_cast<long long>(long_entries), forward ? par_tail_ : -1);
      }
      par_ready_[d] = true;
    }
  }
  const std::vector<int>& runs = par_runs_[d];
  if (runs.empty() && !(forward && par_tail_ >= fni)) return false;
  Fractional* x = rhs->data();
  auto run_parallel = [&](int b, int e) {
    ParallelRanges(e - b, 512, 1, [&](int, int64_t lo, int64_t hi) {
      for (int64_t k = lo; k < hi; ++k) {
        const int col = b + static_cast<int>(k);
        x[col] = forward ? TransposeUpperOutput(x, col) : TransposeLowerOutput(x, col);
      }
    });
  };
  if (forward) {
    size_t r = 0;
    int col = fni;
    const int tail = par_tail_ >= fni ? par_tail_ : n;
    while (col < tail) {
      if (r < runs.size() && runs[r] == col) {
        run_parallel(runs[r], runs[r + 1]);
        col = runs[r + 1];
        r += 2;
      } else {
        x[col] = TransposeUpperOutput(x, col);
        ++col;
      }
    }
    if (tail < n) {
      // The chains' final-only prefixes (sum = x[c], then the loop's own
      // grouped subtractions up to the split), in parallel; then each column
      // in order continues its chain exactly where the loop would be.
      // Per thread: the solver thread and the tau worker solve concurrently.
      thread_local std::vector<Fractional> prefix;
      prefix.resize(n - tail);
      Fractional* pre = prefix.data();
      ParallelRanges(n - tail, 64, 1, [&](int, int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi; ++k) {
          const int c = tail + static_cast<int>(k);
          Fractional sum = x[c];
          const int64_t split = par_split_[k];
          for (int64_t i = starts_[c]; i < split; i += 4) {
            sum -= coefficients_[i] * x[rows_[i]] + coefficients_[i + 1] * x[rows_[i + 1]] +
                   coefficients_[i + 2] * x[rows_[i + 2]] +
                   coefficients_[i + 3] * x[rows_[i + 3]];
          }
          pre[k] = sum;
        }
      });
      for (int c = tail; c < n; ++c) {
        Fractional sum = pre[c - tail];
        int64_t i = par_split_[c - tail];
        const int64_t i_end = starts_[c + 1];
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
        x[c] = all_diagonal_coefficients_are_one_ ? sum : sum / diagonal_coefficients_[c];
      }
    }
    return true;
  }
  // Backward: the loop starts at the last non-zero input (the columns above
  // it keep their zero).
  int col = n - 1;
  while (col >= fni && x[col] == 0.0) --col;
  size_t r = 0;
  while (r < runs.size() && runs[r] > col) r += 2;  // runs entirely above the start
  while (col >= fni) {
    if (r < runs.size() && runs[r + 1] - 1 >= col && runs[r] <= col) {
      const int lo = runs[r];
      run_parallel(lo, col + 1);  // the part of the run at or below col
      col = lo - 1;
      r += 2;
    } else {
      x[col] = TransposeLowerOutput(x, col);
      --col;
      while (r < runs.size() && runs[r] > col) r += 2;
    }
  }
  return true;
}

// basis_representation.cc:358-372
void BasisFactorization::RightSolve(ScatteredVector* d) const {
  if (!use_middle_product_form_update_) {
    d->non_zeros.clear();
    lu_factorization_.RightSolve(&d->values);
    eta_factorization_.RightSolve(&d->values);
    BumpDeterministicTimeForSolve(static_cast<int64_t>(d->NumNonZerosEstimate()));
    return;
  }
  FtranTimer t(kFtL);
  lu_factorization_.RightSolveLWithNonZeros(d);
  t.Lap(kFtEtas);
  rank_one_factorization_.RightSolveWithNonZeros(d);
  t.Lap(kFtU);
  lu_factorization_.RightSolveUWithNonZeros(d);
  d->SortNonZerosIfNeeded();
  BumpDeterministicTimeForSolve(static_cast<int64_t>(d->NumNonZerosEstimate()));
}

// basis_representation.cc:374-398
const std::vector<Fractional>& BasisFactorization::RightSolveForTau(
    const ScatteredVector& a) const {
  if ((async_kind_ == AsyncKind::kTau || async_kind_ == AsyncKind::kTauDeferred) &&
      async_input_ == &a && TakeAsync(tau_ticket_)) {
    std::swap(tau_, async_tau_);
    tau_computation_can_be_optimized_ = false;
    tau_is_computed_ = true;
    return tau_.values;
  }
  DropAsync();
  if (!use_middle_product_form_update_) {
    tau_.non_zeros.clear();
    tau_.values = a.values;
    lu_factorization_.RightSolve(&tau_.values);
    eta_factorization_.RightSolve(&tau_.values);
    tau_is_computed_ = true;
    BumpDeterministicTimeForSolve(static_cast<int64_t>(tau_.NumNonZerosEstimate()));
    return tau_.values;
  }
  if (tau_computation_can_be_optimized_) {
    tau_computation_can_be_optimized_ = false;
    lu_factorization_.RightSolveLWithPermutedInput(a.values, &tau_);
  } else {
    ClearAndResizeVectorWithNonZeros(compact_matrix_.num_rows(), &tau_);
    lu_factorization_.RightSolveLForScatteredColumn(a, &tau_);
  }
  rank_one_factorization_.RightSolveWithNonZeros(&tau_);
  lu_factorization_.RightSolveUWithNonZeros(&tau_);
  tau_is_computed_ = true;
  BumpDeterministicTimeForSolve(static_cast<int64_t>(tau_.NumNonZerosEstimate()));
  return tau_.values;
}

// basis_representation.cc:400-453
void BasisFactorization::LeftSolveForUnitRow(int j, ScatteredVector* y) const {
  SyncForUnitRow();
  ClearAndResizeVectorWithNonZeros(compact_matrix_.num_rows(), y);
  if (!use_middle_product_form_update_) {
    (*y)[j] = 1.0;
    y->non_zeros.push_back(j);
    eta_factorization_.SparseLeftSolve(&y->values, &y->non_zeros);
    lu_factorization_.LeftSolve(&y->values);
    BumpDeterministicTimeForSolve(static_cast<int64_t>(y->NumNonZerosEstimate()));
    return;
  }
  if (j >= static_cast<int>(left_pool_mapping_.size())) {
    left_pool_mapping_.resize(j + 1, kInvalidCol);
  }
  if (left_pool_mapping_[j] == kInvalidCol) {
    const int start = lu_factorization_.LeftSolveUForUnitRow(j, y);
    if (y->non_zeros.empty()) {
      left_pool_mapping_[j] = storage_.AddDenseColumnPrefix(y->values, start);
    } else {
      left_pool_mapping_[j] = storage_.AddDenseColumnWithNonZeros(y->values, y->non_zeros);
    }
  } else {
    storage_.ColumnCopyToClearedDenseColumnWithNonZeros(left_pool_mapping_[j],
                                                        &y->values, &y->non_zeros);
  }
  rank_one_factorization_.LeftSolveWithNonZeros(y);
  if (tau_is_computed_) {
    tau_computation_can_be_optimized_ =
        lu_factorization_.LeftSolveLWithNonZeros(y, &tau_);
  } else {
    tau_computation_can_be_optimized_ = false;
    lu_factorization_.LeftSolveLWithNonZeros(y, nullptr);
  }
  tau_is_computed_ = false;
  y->SortNonZerosIfNeeded();
  BumpDeterministicTimeForSolve(static_cast<int64_t>(y->NumNonZerosEstimate()));
}

// basis_representation.cc:455-466
void BasisFactorization::TemporaryLeftSolveForUnitRow(int j, ScatteredVector* y) const {
  SyncForUnitRow();
  ClearAndResizeVectorWithNonZeros(compact_matrix_.num_rows(), y);
  lu_factorization_.LeftSolveUForUnitRow(j, y);
  lu_factorization_.LeftSolveLWithNonZeros(y, nullptr);
  y->SortNonZerosIfNeeded();
  BumpDeterministicTimeForSolve(static_cast<int64_t>(y->NumNonZerosEstimate()));
}

// basis_representation.cc:468-501
void BasisFactorization::RightSolveForProblemColumn(int col, ScatteredVector* d) const {
  ClearAndResizeVectorWithNonZeros(compact_matrix_.num_rows(), d);
  if (!use_middle_product_form_update_) {
    const ColumnView c = compact_matrix_.column(col);  // ColumnCopyToClearedDenseColumn
    d->values.resize(compact_matrix_.num_rows(), 0.0);
    for (int64_t i = 0; i < c.n; ++i) d->values[c.rows[i]] = c.coefs[i];
    lu_factorization_.RightSolve(&d->values);
    eta_factorization_.RightSolve(&d->values);
    BumpDeterministicTimeForSolve(static_cast<int64_t>(d->NumNonZerosEstimate()));
    return;
  }
  FtranTimer t(kFtL);
  lu_factorization_.RightSolveLForColumnView(compact_matrix_.column(col), d);
  if (g_trace_ftran) g_ftran_hash[0] = TraceHashVector(d->values, d->non_zeros);
  t.Lap(kFtEtas);
  rank_one_factorization_.RightSolveWithNonZeros(d);
  if (g_trace_ftran) g_ftran_hash[1] = TraceHashVector(d->values, d->non_zeros);
  t.Lap(kFtU);
  if (col >= static_cast<int>(right_pool_mapping_.size())) {
    right_pool_mapping_.resize(col + 1, kInvalidCol);
  }
  // A thrown device error must not leave the append armed for a later solve.
  struct Disarm {
    ~Disarm() { g_overlap.f = nullptr; }
  } disarm;
  // The speculative flip FTRAN of this pivot (SpecFlipBegin) takes the
  // update built from this column: it runs right after the append.
  const bool spec = spec_state_ == SpecState::kArmed && spec_entering_ == col;
  if (spec_state_ == SpecState::kArmed && !spec) SpecFlipDrop();
  if (d->non_zeros.empty()) {
    // Appended while the device solves U (the column is the vector before U;
    // g_overlap runs before anything overwrites it).
    const int slot_col = col;
    g_overlap.f = [this, slot_col, d, spec]() {
      right_pool_mapping_[slot_col] = right_storage_.AddDenseColumn(d->values);
      if (spec) SpecFlipLaunch();
    };
  } else {
    FtranTimer pool_timer(kFtUPool);
    std::sort(d->non_zeros.begin(), d->non_zeros.end());
    right_pool_mapping_[col] =
        right_storage_.AddDenseColumnWithNonZeros(d->values, d->non_zeros);
    if (spec) g_overlap.f = [this]() { SpecFlipLaunch(); };
  }
  if (async_kind_ == AsyncKind::kTauDeferred && async_) async_->Wait();  // tau's L, etas
  if (async_kind_ == AsyncKind::kTauDeferred && tau_u_pending_) {
    // The direction's and tau's U solves together; tau's bump deferred.
    lu_factorization_.RightSolveUWithNonZerosPair(d, &async_tau_);
    LuSlotGuard slot(1);
    BumpDeterministicTimeForSolve(static_cast<int64_t>(async_tau_.NumNonZerosEstimate()));
    tau_u_pending_ = false;
  } else {
    lu_factorization_.RightSolveUWithNonZeros(d);
  }
  g_overlap.Run();  // nothing solved U (identity factorization)
  d->SortNonZerosIfNeeded();
  if (g_trace_ftran) g_ftran_hash[2] = TraceHashVector(d->values, d->non_zeros);
  BumpDeterministicTimeForSolve(static_cast<int64_t>(d->NumNonZerosEstimate()));
}

Fractional BasisFactorization::RightSolveSquaredNorm(const ColumnView& a) const {
  BumpDeterministicTimeForSolve(a.n);
  return lu_factorization_.RightSolveSquaredNorm(a);
}

uint64_t BasisFactorization::FactorizationContentKey() const {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
  mix(static_cast<uint64_t>(compact_matrix_.num_rows()));
  mix(static_cast<uint64_t>(compact_matrix_.num_cols()));
  for (const int c : basis_) mix(static_cast<uint32_t>(c));
  const LuFactorization& lu = lu_factorization_;
  mix(lu.IsIdentityFactorization() ? 1 : 0);
  mix(static_cast<uint64_t>(lu.NumberOfEntries()));
  mix(0x9e3779b97f4a7c15ull);
  for (const int c : lu.row_perm()) mix(static_cast<uint32_t>(c));
  mix(0x9e3779b97f4a7c15ull);
  for (const int c : lu.GetColumnPermutation()) mix(static_cast<uint32_t>(c));
  return h;
}

Fractional BasisFactorization::DualEdgeSquaredNorm(int row) const {
  BumpDeterministicTimeForSolve(1);
  return lu_factorization_.DualEdgeSquaredNorm(row);
}

// basis_representation.cc:520-531
bool BasisFactorization::IsIdentityBasis() const {
  const int num_rows = compact_matrix_.num_rows();
  for (int row = 0; row < num_rows; ++row) {
    const int col = basis_[row];
    const ColumnView c = compact_matrix_.column(col);
    if (c.n != 1) return false;
    if (c.rows[0] != row || c.coefs[0] != 1.0) return false;
  }
  return true;
}

// basis_representation.cc:595-601
Fractional BasisFactorization::ComputeInfinityNormConditionNumberUpperBound() const {
  if (IsIdentityBasis()) return 1.0;
  BumpDeterministicTimeForSolve(compact_matrix_.num_rows());
  CompactSparseMatrixView basis_matrix{&compact_matrix_, &basis_};
  return basis_matrix.ComputeInfinityNorm() *
         lu_factorization_.ComputeInverseInfinityNormUpperBound();
}

// basis_representation.cc:607-624
void BasisFactorization::BumpDeterministicTimeForSolve(int64_t num_entries) const {
  if (g_lu_slot != 0) {  // tau worker: applied when the result is taken
    deferred_solve_entries_.push_back(num_entries);
    return;
  }
  if (compact_matrix_.num_rows() == 0) return;
  const double density = static_cast<double>(num_entries) /
                         static_cast<double>(compact_matrix_.num_rows());
  deterministic_time_ +=
      density * DeterministicTimeForFpOperations(lu_factorization_.NumberOfEntries()) +
      DeterministicTimeForFpOperations(rank_one_factorization_.num_entries());
}

}  // namespace milp
