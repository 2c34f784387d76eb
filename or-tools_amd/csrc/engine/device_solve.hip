// DeviceLp: dense triangular solves of the basis factorization (see
// device_solver.h and kernels/tri_solve.hip).
//
// Glop's FTRAN ends with U x = b (lu_factorization.cc:314-331). When the
// result is too dense for the hypersparse path it runs
// TriangularMatrix::TransposeLowerSolve (sparse.cc:899-955) on U's transpose:
// a gather over every row. On config 5 (m = 100 000) that is most of the
// host time of an iteration, twice per iteration (direction, bound flips).
// U changes only at refactorization, so its level schedule is built and
// uploaded once per factorization; each solve then moves the right-hand side
// in, runs one single-CU kernel and moves the result out.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../kernels/kernel_args.h"
#include "device_lp.h"
#include "host_pool.h"
#include "lu.h"

namespace milp {

namespace {
inline hipStream_t Stream(void* p) { return reinterpret_cast<hipStream_t>(p); }

struct SolveCallTimer {
  mi_lp_kernel_stats* stats;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit SolveCallTimer(mi_lp_kernel_stats* s) : stats(s) {}
  ~SolveCallTimer() {
    stats->call_ms[MI_K_TRI_SOLVE] +=
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
            .count();
  }
};

template <typename T>
void Grow(T** p, size_t* cap_elems, size_t need, const char* what) {
  if (*p != nullptr && *cap_elems >= need) return;
  if (*p != nullptr) (void)hipFree(*p);
  *p = nullptr;
  const size_t n = std::max<size_t>(need, 1) + need / 4;
  if (hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)) != hipSuccess) {
    throw DeviceError(std::string("hipMalloc (") + what + ")");
  }
  *cap_elems = n;
}

}  // namespace

void DeviceLp::FreeTriBuffers() {
  for (void* p : {static_cast<void*>(d_tri_level_start_), static_cast<void*>(d_tri_work_row_),
                  static_cast<void*>(d_tri_work_begin_),
                  static_cast<void*>(d_tri_entry_row_), static_cast<void*>(d_tri_entry_coef_),
                  static_cast<void*>(d_tri_diag_), static_cast<void*>(d_tri_x_)}) {
    if (p != nullptr) (void)hipFree(p);
  }
  d_tri_level_start_ = d_tri_work_row_ = d_tri_work_begin_ = d_tri_entry_row_ = nullptr;
  d_tri_entry_coef_ = d_tri_diag_ = d_tri_x_ = nullptr;
  if (d_tri_clock_ != nullptr) (void)hipFree(d_tri_clock_);
  d_tri_clock_ = nullptr;
  if (h_tri_x_ != nullptr) (void)hipHostFree(h_tri_x_);
  if (h_tri_stage_ != nullptr) (void)hipHostFree(h_tri_stage_);
  h_tri_x_ = nullptr;
  h_tri_stage_ = nullptr;
  tri_stage_bytes_ = 0;
  tri_key_ = 0;
  tri_ok_ = false;
  tri_caps_ = TriCaps();
}

// Level schedule of t's TransposeLowerSolve: output c (a column of t, rows
// first_non_identity .. num_cols-1) depends on the rows of its entries, all
// > c. level(c) = 0 without entries, else 1 + the deepest entry. Outputs
// with no entries and a unit diagonal are the identity and are not listed.
void DeviceLp::BuildTriSchedule(const TriangularMatrix& t, uint64_t key) {
  tri_key_ = key;
  tri_ok_ = false;
  const int nc = t.num_cols();
  const int fni = t.GetFirstNonIdentityColumn();
  tri_rows_ = nc;
  tri_first_col_ = fni;
  tri_ones_ = t.all_diagonal_coefficients_are_one_;
  const int64_t nnz = t.starts_[nc] - t.starts_[0];
  if (nnz >= (int64_t{1} << 31)) return;
  std::vector<int32_t> level(nc, 0);
  int depth = 0;
  int num_work = 0;
  for (int c = nc - 1; c >= fni; --c) {
    int l = 0;
    for (int64_t i = t.starts_[c]; i < t.starts_[c + 1]; ++i) {
      l = std::max(l, level[t.rows_[i]] + 1);
    }
    level[c] = l;
    depth = std::max(depth, l);
    if (l > 0 || !tri_ones_) ++num_work;
  }
  // Counting sort by level; inside a level, descending c (the host order).
  std::vector<int32_t> level_start(depth + 2, 0);
  for (int c = nc - 1; c >= fni; --c) {
    if (level[c] > 0 || !tri_ones_) ++level_start[level[c] + 1];
  }
  for (int l = 0; l <= depth; ++l) level_start[l + 1] += level_start[l];
  tri_work_ = num_work;
  tri_level_width_.resize(depth + 1);
  for (int l = 0; l <= depth; ++l) tri_level_width_[l] = level_start[l + 1] - level_start[l];
  if (const char* d = std::getenv("MILP_TRI_DEBUG")) tri_debug_left_ = std::atoi(d);
  // Levels that hold listed outputs (level 0 is empty when every diagonal is 1).
  tri_levels_ = depth + 1;
  // Staging layout: level_start | work_row | work_begin | entry_row | (pad)
  // entry_coef | diag.
  const size_t off_work = size_t(depth + 2) * 4;
  const size_t off_begin = off_work + size_t(num_work) * 4;
  const size_t off_entry = off_begin + size_t(num_work + 1) * 4;
  const size_t off_coef = (off_entry + size_t(nnz) * 4 + 7) / 8 * 8;
  const size_t off_diag = off_coef + size_t(nnz) * 8;
  const size_t bytes = off_diag + (tri_ones_ ? 0 : size_t(num_work) * 8);
  if (tri_stage_bytes_ < bytes) {
    if (h_tri_stage_ != nullptr) (void)hipHostFree(h_tri_stage_);
    h_tri_stage_ = nullptr;
    Check(hipHostMalloc(&h_tri_stage_, bytes + bytes / 4), "pin");
    tri_stage_bytes_ = bytes + bytes / 4;
  }
  char* st = static_cast<char*>(h_tri_stage_);
  int32_t* lstart = reinterpret_cast<int32_t*>(st);
  std::copy(level_start.begin(), level_start.end(), lstart);
  int32_t* work_row = reinterpret_cast<int32_t*>(st + off_work);
  int32_t* work_begin = reinterpret_cast<int32_t*>(st + off_begin);
  int32_t* entry_row = reinterpret_cast<int32_t*>(st + off_entry);
  double* entry_coef = reinterpret_cast<double*>(st + off_coef);
  double* diag = reinterpret_cast<double*>(st + off_diag);
  std::vector<int32_t> next(level_start.begin(), level_start.end() - 1);
  std::vector<int32_t> pos_of(nc, -1);
  for (int c = nc - 1; c >= fni; --c) {
    if (level[c] == 0 && tri_ones_) continue;
    const int k = next[level[c]]++;
    work_row[k] = c;
    pos_of[c] = k;
  }
  // Entries of each listed output in evaluation order: the host walks the
  // column from its last entry down (sparse.cc:908-955).
  int32_t e = 0;
  for (int k = 0; k < num_work; ++k) {
    const int c = work_row[k];
    work_begin[k] = e;
    for (int64_t i = t.starts_[c + 1] - 1; i >= t.starts_[c]; --i) {
      entry_row[e] = t.rows_[i];
      entry_coef[e] = t.coefficients_[i];
      ++e;
    }
    if (!tri_ones_) diag[k] = t.diagonal_coefficients_[c];
  }
  work_begin[num_work] = e;
  // Prefix counts by output row, for the byte accounting of a solve that
  // stops at `top`.
  tri_rows_upto_.assign(nc + 1, 0);
  tri_entries_upto_.assign(nc + 1, 0);
  for (int c = 0; c < nc; ++c) {
    const bool listed = pos_of[c] >= 0;
    tri_rows_upto_[c + 1] = tri_rows_upto_[c] + (listed ? 1 : 0);
    tri_entries_upto_[c + 1] =
        tri_entries_upto_[c] + (listed ? t.starts_[c + 1] - t.starts_[c] : 0);
  }
  TriCaps& caps = tri_caps_;
  Grow(&d_tri_level_start_, &caps.levels, size_t(depth) + 2, "tri levels");
  Grow(&d_tri_work_row_, &caps.work, num_work, "tri work");
  Grow(&d_tri_work_begin_, &caps.begin, size_t(num_work) + 1, "tri begin");
  Grow(&d_tri_entry_row_, &caps.entries, size_t(nnz), "tri entries");
  Grow(&d_tri_entry_coef_, &caps.coefs, size_t(nnz), "tri coefs");
  if (!tri_ones_) Grow(&d_tri_diag_, &caps.diag, num_work, "tri diag");
  if (caps.x < size_t(nc) || h_tri_x_ == nullptr) {
    Grow(&d_tri_x_, &caps.x, nc, "tri x");
    if (h_tri_x_ != nullptr) (void)hipHostFree(h_tri_x_);
    h_tri_x_ = nullptr;
    Check(hipHostMalloc(reinterpret_cast<void**>(&h_tri_x_), caps.x * sizeof(double)), "pin");
  }
  Upload(d_tri_level_start_, lstart, size_t(depth + 2) * 4);
  Upload(d_tri_work_row_, work_row, size_t(num_work) * 4);
  Upload(d_tri_work_begin_, work_begin, size_t(num_work + 1) * 4);
  Upload(d_tri_entry_row_, entry_row, size_t(nnz) * 4);
  Upload(d_tri_entry_coef_, entry_coef, size_t(nnz) * 8);
  if (!tri_ones_) Upload(d_tri_diag_, diag, size_t(num_work) * 8);
  // The staging buffer is reused by the next build: wait for the copies.
  Check(hipStreamSynchronize(Stream(stream_)), "sync");
  tri_ok_ = true;
}

bool DeviceLp::TransposeLowerSolve(const TriangularMatrix& t, uint64_t key,
                                   std::vector<double>* x) {
  if (tri_mode_ == 2) return false;
  const int nc = t.num_cols();
  if (tri_mode_ == 0 && nc < tri_min_rows_) return false;
  if (static_cast<int>(x->size()) < nc) return false;
  SolveCallTimer timer(&stats_);
  if (tri_key_ != key) BuildTriSchedule(t, key);
  if (!tri_ok_) return false;
  double* xv = x->data();
  const int fni = tri_first_col_;
  // sparse.cc:908-912: the host loop starts at the last non-zero.
  int top = nc - 1;
  while (top >= fni && xv[top] == 0.0) --top;
  if (top < fni) return true;
  if (tri_rows_upto_[top + 1] - tri_rows_upto_[fni] == 0) return true;  // identity part only
  // Outputs c >= fni read rows > c only: x[fni..nc) in, x[fni..top] out.
  const size_t in = size_t(nc - fni);
  CopyHost(h_tri_x_ + fni, xv + fni, in * sizeof(double));
  Upload(d_tri_x_ + fni, h_tri_x_ + fni, in * sizeof(double));
  milp_kernels::TriSolveArgs a;
  a.level_start = d_tri_level_start_;
  a.num_levels = tri_levels_;
  a.work_row = d_tri_work_row_;
  a.work_begin = d_tri_work_begin_;
  a.entry_row = d_tri_entry_row_;
  a.entry_coef = d_tri_entry_coef_;
  a.diag = tri_ones_ ? nullptr : d_tri_diag_;
  a.x = d_tri_x_;
  a.num_work = tri_work_;
  a.num_rows = nc;
  a.top = top;
  a.clock = nullptr;
  // MILP_TRI_DEBUG=k: per-level wall clock of the first k solves after each
  // schedule build, printed to stderr with the level widths.
  const bool debug = tri_debug_left_ > 0;
  if (debug) {
    if (d_tri_clock_ == nullptr) {
      Check(hipMalloc(reinterpret_cast<void**>(&d_tri_clock_), 65536 * sizeof(uint64_t)),
            "hipMalloc");
    }
    if (tri_levels_ + 1 < 65536) a.clock = d_tri_clock_;
  }
  BeginKernel(MI_K_TRI_SOLVE);
  Check(milp_launch::tri_transpose_lower(a, Stream(stream_)), "tri_transpose_lower");
  const double rows = tri_rows_upto_[top + 1] - tri_rows_upto_[fni];
  const double entries =
      static_cast<double>(tri_entries_upto_[top + 1] - tri_entries_upto_[fni]);
  // Per computed output: its list slot (4 + 4 B), x in and out (16 B), the
  // diagonal (8 B) unless unit; per entry: row and value (12 B) and the
  // gathered x (8 B).
  EndKernel(MI_K_TRI_SOLVE, rows * (24.0 + (tri_ones_ ? 0.0 : 8.0)) + entries * 20.0);
  const size_t out = size_t(top - fni + 1);
  if (a.clock != nullptr) {
    --tri_debug_left_;
    std::vector<uint64_t> clk(tri_levels_ + 1);
    Check(hipMemcpy(clk.data(), d_tri_clock_, clk.size() * sizeof(uint64_t),
                    hipMemcpyDeviceToHost), "D2H");
    std::fprintf(stderr, "[tri] rows %d work %d levels %d top %d: total %.1f us; per level (us/width):",
                 nc, tri_work_, tri_levels_, top, (clk.back() - clk[0]) / 100.0);
    for (int l = 0; l < tri_levels_; ++l) {
      std::fprintf(stderr, " %.2f/%d", (clk[l + 1] - clk[l]) / 100.0,
                   tri_level_width_[l]);
    }
    std::fprintf(stderr, "\n");
  }
  Download(h_tri_x_ + fni, d_tri_x_ + fni, out * sizeof(double));
  CopyHost(xv + fni, h_tri_x_ + fni, out * sizeof(double));
  return true;
}

}  // namespace milp
