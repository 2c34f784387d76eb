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

}  // namespace

void DeviceLp::TriReserve(int which, size_t bytes) {
  TriBuffer& b = tri_buf_[which];
  if (b.ptr != nullptr && b.bytes >= bytes) return;
  if (b.ptr != nullptr) (void)hipFree(b.ptr);
  b.ptr = nullptr;
  b.bytes = 0;
  const size_t n = std::max<size_t>(bytes, 16) + bytes / 4;
  Check(hipMalloc(&b.ptr, n), "hipMalloc (triangular solve)");
  b.bytes = n;
}

void DeviceLp::FreeTriBuffers() {
  for (TriBuffer& b : tri_buf_) {
    if (b.ptr != nullptr) (void)hipFree(b.ptr);
    b = TriBuffer();
  }
  if (d_tri_clock_ != nullptr) (void)hipFree(d_tri_clock_);
  d_tri_clock_ = nullptr;
  if (tri_graph_exec_ != nullptr) {
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(tri_graph_exec_));
  }
  tri_graph_exec_ = nullptr;
  tri_graph_ready_ = false;
  if (h_tri_top_ != nullptr) (void)hipHostFree(h_tri_top_);
  h_tri_top_ = nullptr;
  if (h_tri_x_ != nullptr) (void)hipHostFree(h_tri_x_);
  if (h_tri_stage_ != nullptr) (void)hipHostFree(h_tri_stage_);
  h_tri_x_ = nullptr;
  h_tri_x_elems_ = 0;
  h_tri_stage_ = nullptr;
  tri_stage_bytes_ = 0;
  tri_key_ = 0;
  tri_ok_ = false;
}

// Level schedule of t's TransposeLowerSolve: output c (a column of t, rows
// first_non_identity .. num_cols-1) depends on the rows of its entries, all
// > c. level(c) = 0 without entries, else 1 + the deepest entry. Outputs
// with no entries and a unit diagonal are the identity and are not listed.
// Positions: the listed outputs by level (descending c inside a level, the
// host order), then the other rows >= first_non_identity (read, never
// written). Entries refer to positions.
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
  const int num_pos = nc - fni;
  // Counting sort by level.
  std::vector<int32_t> level_start(depth + 2, 0);
  for (int c = nc - 1; c >= fni; --c) {
    if (level[c] > 0 || !tri_ones_) ++level_start[level[c] + 1];
  }
  for (int l = 0; l <= depth; ++l) level_start[l + 1] += level_start[l];
  tri_work_ = num_work;
  tri_pos_ = num_pos;
  tri_levels_ = depth + 1;
  tri_level_width_.resize(depth + 1);
  for (int l = 0; l <= depth; ++l) tri_level_width_[l] = level_start[l + 1] - level_start[l];
  // Launch segments: each wide level alone over the chip, each run of narrow
  // levels as one single-CU launch (tri_solve.hip).
  tri_segments_.clear();
  for (int l = 0; l <= depth;) {
    const int w = tri_level_width_[l];
    if (w == 0) {
      ++l;
      continue;
    }
    if (w > tri_wide_level_) {
      tri_segments_.push_back(-l - 1);
      tri_segments_.push_back(std::min(1024, (w + 255) / 256));
      ++l;
      continue;
    }
    int e = l;
    while (e <= depth && tri_level_width_[e] <= tri_wide_level_) ++e;
    tri_segments_.push_back(l);
    tri_segments_.push_back(e);
    l = e;
  }
  if (const char* d = std::getenv("MILP_TRI_DEBUG")) tri_debug_left_ = std::atoi(d);
  // Positions.
  std::vector<int32_t> pos_row(num_pos);
  std::vector<int32_t> pos_of(nc, -1);
  {
    std::vector<int32_t> next(level_start.begin(), level_start.end() - 1);
    int tail = num_work;
    for (int c = nc - 1; c >= fni; --c) {
      const int k = (level[c] > 0 || !tri_ones_) ? next[level[c]]++ : tail++;
      pos_row[k] = c;
      pos_of[c] = k;
    }
  }
  int64_t num_ovf = 0;
  for (int k = 0; k < num_work; ++k) {
    const int c = pos_row[k];
    const int64_t n = t.starts_[c + 1] - t.starts_[c];
    if (n > 4) num_ovf += n;
  }
  // Staging layout, 16-byte aligned pieces.
  auto al = [](size_t b) { return (b + 15) / 16 * 16; };
  const size_t b_levels = al(size_t(depth + 2) * 4);
  const size_t b_row = al(size_t(num_work) * 4);
  const size_t b_n = al(size_t(num_work) * 4);
  const size_t b_entry = size_t(num_work) * 16;
  const size_t b_value = size_t(num_work) * 32;
  const size_t b_diag = tri_ones_ ? 0 : al(size_t(num_work) * 8);
  const size_t b_ovf_pos = al(size_t(num_ovf) * 4);
  const size_t b_ovf_val = al(size_t(num_ovf) * 8);
  const size_t b_pos_row = al(size_t(num_pos) * 4);
  const size_t sizes[kTriNumStaged] = {b_levels, b_row,     b_n,       b_entry,  b_value,
                                       b_diag,   b_ovf_pos, b_ovf_val, b_pos_row};
  size_t offs[kTriNumStaged];
  size_t bytes = 0;
  for (int b = 0; b < kTriNumStaged; ++b) {
    offs[b] = bytes;
    bytes += sizes[b];
  }
  if (tri_stage_bytes_ < bytes) {
    if (h_tri_stage_ != nullptr) (void)hipHostFree(h_tri_stage_);
    h_tri_stage_ = nullptr;
    Check(hipHostMalloc(&h_tri_stage_, bytes + bytes / 4 + 16), "pin");
    tri_stage_bytes_ = bytes + bytes / 4 + 16;
  }
  char* st = static_cast<char*>(h_tri_stage_);
  int32_t* lstart = reinterpret_cast<int32_t*>(st + offs[kTriLevels]);
  int32_t* rec_row = reinterpret_cast<int32_t*>(st + offs[kTriRecRow]);
  int32_t* rec_n = reinterpret_cast<int32_t*>(st + offs[kTriRecN]);
  int32_t* rec_entry = reinterpret_cast<int32_t*>(st + offs[kTriRecEntry]);
  double* rec_value = reinterpret_cast<double*>(st + offs[kTriRecValue]);
  double* diag = reinterpret_cast<double*>(st + offs[kTriDiag]);
  int32_t* ovf_pos = reinterpret_cast<int32_t*>(st + offs[kTriOvfPos]);
  double* ovf_value = reinterpret_cast<double*>(st + offs[kTriOvfValue]);
  std::copy(level_start.begin(), level_start.end(), lstart);
  std::copy(pos_row.begin(), pos_row.end(), reinterpret_cast<int32_t*>(st + offs[kTriPosRow]));
  // Entries of each listed output in evaluation order: the host walks the
  // column from its last entry down (sparse.cc:908-955).
  int64_t o = 0;
  for (int k = 0; k < num_work; ++k) {
    const int c = pos_row[k];
    const int64_t b = t.starts_[c], e = t.starts_[c + 1];
    const int n = static_cast<int>(e - b);
    rec_row[k] = c;
    rec_n[k] = n;
    if (n <= 4) {
      for (int j = 0; j < 4; ++j) {
        rec_entry[4 * k + j] = j < n ? pos_of[t.rows_[e - 1 - j]] : 0;
        rec_value[4 * k + j] = j < n ? t.coefficients_[e - 1 - j] : 0.0;
      }
    } else {
      rec_entry[4 * k] = static_cast<int32_t>(o);
      rec_entry[4 * k + 1] = rec_entry[4 * k + 2] = rec_entry[4 * k + 3] = 0;
      for (int j = 0; j < 4; ++j) rec_value[4 * k + j] = 0.0;
      for (int64_t i = e - 1; i >= b; --i) {
        ovf_pos[o] = pos_of[t.rows_[i]];
        ovf_value[o] = t.coefficients_[i];
        ++o;
      }
    }
    if (!tri_ones_) diag[k] = t.diagonal_coefficients_[c];
  }
  // Prefix counts by output row, for the byte accounting of a solve that
  // stops at `top`.
  tri_rows_upto_.assign(nc + 1, 0);
  tri_entries_upto_.assign(nc + 1, 0);
  for (int c = 0; c < nc; ++c) {
    const bool listed = c >= fni && pos_of[c] < num_work;
    tri_rows_upto_[c + 1] = tri_rows_upto_[c] + (listed ? 1 : 0);
    tri_entries_upto_[c + 1] =
        tri_entries_upto_[c] + (listed ? t.starts_[c + 1] - t.starts_[c] : 0);
  }
  for (int b = 0; b < kTriNumStaged; ++b) {
    if (sizes[b] == 0) continue;
    TriReserve(b, sizes[b]);
    Upload(tri_buf_[b].ptr, st + offs[b], sizes[b]);
  }
  TriReserve(kTriX, size_t(nc) * 8);
  TriReserve(kTriY, size_t(std::max(num_pos, 1)) * 8);
  if (h_tri_x_elems_ < size_t(nc)) {
    if (h_tri_x_ != nullptr) (void)hipHostFree(h_tri_x_);
    h_tri_x_ = nullptr;
    h_tri_x_elems_ = size_t(nc) + size_t(nc) / 4;
    Check(hipHostMalloc(reinterpret_cast<void**>(&h_tri_x_), h_tri_x_elems_ * sizeof(double)),
          "pin");
  }
  TriReserve(kTriTop, 16);
  if (h_tri_top_ == nullptr) {
    Check(hipHostMalloc(reinterpret_cast<void**>(&h_tri_top_), 64), "pin");
  }
  // The staging buffer is reused by the next build: wait for the copies.
  Check(hipStreamSynchronize(Stream(stream_)), "sync");
  tri_ok_ = true;
  tri_graph_ready_ = false;  // captured at the first solve of this factorization
}

milp_kernels::TriSolveArgs DeviceLp::TriArgs() const {
  milp_kernels::TriSolveArgs a;
  a.level_start = static_cast<const int32_t*>(tri_buf_[kTriLevels].ptr);
  a.rec_row = static_cast<const int32_t*>(tri_buf_[kTriRecRow].ptr);
  a.rec_n = static_cast<const int32_t*>(tri_buf_[kTriRecN].ptr);
  a.rec_entry = static_cast<const int4*>(tri_buf_[kTriRecEntry].ptr);
  a.rec_value = static_cast<const double2*>(tri_buf_[kTriRecValue].ptr);
  a.diag = tri_ones_ ? nullptr : static_cast<const double*>(tri_buf_[kTriDiag].ptr);
  a.ovf_pos = static_cast<const int32_t*>(tri_buf_[kTriOvfPos].ptr);
  a.ovf_value = static_cast<const double*>(tri_buf_[kTriOvfValue].ptr);
  a.pos_row = static_cast<const int32_t*>(tri_buf_[kTriPosRow].ptr);
  a.x = static_cast<double*>(tri_buf_[kTriX].ptr);
  a.y = static_cast<double*>(tri_buf_[kTriY].ptr);
  a.top = static_cast<const int*>(tri_buf_[kTriTop].ptr);
  a.num_work = tri_work_;
  a.num_pos = tri_pos_;
  a.num_levels = tri_levels_;
  a.clock = nullptr;
  return a;
}

// One solve = copy in (x[fni..nc), top), the launches of the segment plan,
// copy out (x[fni..nc)). Without debugging the launches are captured once per
// factorization into a HIP graph and replayed with one launch: the plan has
// tens of kernels, whose individual launches would cost more host time than
// their GPU time.
void DeviceLp::TriCopyIn() {
  const int fni = tri_first_col_;
  const size_t in = size_t(tri_rows_ - fni);
  double* d_x = static_cast<double*>(tri_buf_[kTriX].ptr);
  Upload(d_x + fni, h_tri_x_ + fni, in * sizeof(double));
  Upload(tri_buf_[kTriTop].ptr, h_tri_top_, sizeof(int));
}

void DeviceLp::TriCopyOut() {
  const int fni = tri_first_col_;
  const size_t in = size_t(tri_rows_ - fni);
  double* d_x = static_cast<double*>(tri_buf_[kTriX].ptr);
  Check(hipMemcpyAsync(h_tri_x_ + fni, d_x + fni, in * sizeof(double), hipMemcpyDeviceToHost,
                       Stream(stream_)),
        "D2H");
}

void DeviceLp::EnqueueTriKernels(const milp_kernels::TriSolveArgs& a) {
  Check(milp_launch::tri_transpose_lower(a, tri_segments_.data(),
                                         static_cast<int>(tri_segments_.size() / 2),
                                         Stream(stream_)),
        "tri_transpose_lower");
}

void DeviceLp::CaptureTriGraph() {
  if (tri_graph_exec_ != nullptr) {
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(tri_graph_exec_));
    tri_graph_exec_ = nullptr;
  }
  hipGraph_t graph = nullptr;
  Check(hipStreamBeginCapture(Stream(stream_), hipStreamCaptureModeThreadLocal), "capture");
  EnqueueTriKernels(TriArgs());
  Check(hipStreamEndCapture(Stream(stream_), &graph), "capture end");
  hipGraphExec_t exec = nullptr;
  const hipError_t e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  Check(e, "graph instantiate");
  tri_graph_exec_ = exec;
  tri_graph_ready_ = true;
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
  // Outputs c >= fni read rows > c only: x[fni..nc) in and out.
  const size_t in = size_t(nc - fni);
  CopyHost(h_tri_x_ + fni, xv + fni, in * sizeof(double));
  *h_tri_top_ = top;
  const double rows = tri_rows_upto_[top + 1] - tri_rows_upto_[fni];
  const double entries =
      static_cast<double>(tri_entries_upto_[top + 1] - tri_entries_upto_[fni]);
  // Per computed output: its record (row, count: 8 B), its value in and out
  // (16 B), the diagonal (8 B) unless unit; per entry: position and value
  // (12 B) and the value it reads (8 B). The permutes in and out: 8 B in, 8 B
  // out and the 4-B row index per position, both ways.
  const double bytes = rows * (24.0 + (tri_ones_ ? 0.0 : 8.0)) + entries * 20.0 +
                       double(tri_pos_) * 20.0 + rows * 20.0;
  if (tri_debug_left_ > 0) {
    // MILP_TRI_DEBUG=k: per-level wall clock of the first k solves after each
    // schedule build (single-CU segments), printed with the level widths.
    milp_kernels::TriSolveArgs a = TriArgs();
    if (d_tri_clock_ == nullptr) {
      Check(hipMalloc(reinterpret_cast<void**>(&d_tri_clock_), 65536 * sizeof(uint64_t)),
            "hipMalloc");
    }
    Check(hipMemsetAsync(d_tri_clock_, 0, 65536 * sizeof(uint64_t), Stream(stream_)), "memset");
    if (tri_levels_ + 1 < 65536) a.clock = d_tri_clock_;
    TriCopyIn();
    BeginKernel(MI_K_TRI_SOLVE);
    EnqueueTriKernels(a);
    EndKernel(MI_K_TRI_SOLVE, bytes);
    TriCopyOut();
    Synchronize();
    --tri_debug_left_;
    std::vector<uint64_t> clk(tri_levels_ + 1);
    Check(hipMemcpy(clk.data(), d_tri_clock_, clk.size() * sizeof(uint64_t),
                    hipMemcpyDeviceToHost), "D2H");
    std::fprintf(stderr, "[tri] rows %d work %d levels %d segments %zu top %d; per level (us/width):",
                 nc, tri_work_, tri_levels_, tri_segments_.size() / 2, top);
    for (int l = 0; l < tri_levels_; ++l) {
      const bool ok = clk[l] != 0 && clk[l + 1] >= clk[l];
      std::fprintf(stderr, " %.2f/%d", ok ? (clk[l + 1] - clk[l]) / 100.0 : -1.0,
                   tri_level_width_[l]);
    }
    std::fprintf(stderr, "\n");
  } else {
    if (!tri_graph_ready_) CaptureTriGraph();
    TriCopyIn();
    BeginKernel(MI_K_TRI_SOLVE);  // events around the graph: the kernels only
    Check(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(tri_graph_exec_), Stream(stream_)),
          "graph launch");
    EndKernel(MI_K_TRI_SOLVE, bytes);
    TriCopyOut();
    Synchronize();
  }
  CopyHost(xv + fni, h_tri_x_ + fni, size_t(top - fni + 1) * sizeof(double));
  return true;
}

}  // namespace milp
