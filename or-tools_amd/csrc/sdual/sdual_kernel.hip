// Device dual simplex segment on gfx950: one workgroup runs the phase-II dual
// loop of one LP (sdual_core.h) over its arena in HBM until the loop needs the
// host (SdExit). DeviceLp owns the arena, a pinned staging image and the
// transfers; RevisedSimplex (engine/simplex.cc) packs and unpacks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <thread>

#include "../engine/device_lp.h"
#include "../engine/fibers.h"
#include "sdual_core.h"

namespace milp {
namespace {
inline hipStream_t Stream(void* p) { return reinterpret_cast<hipStream_t>(p); }
}  // namespace

// One thread walks Glop's loop; the header lives in the arena.
__global__ __launch_bounds__(64) void sdual_segment_kernel(sdual::Lp* lp) {
  if (threadIdx.x == 0) sdual::sd_run(*lp);
}

void DeviceLp::SdualReserve(size_t bytes, int rows, int64_t lu_cap) {
  if (bytes > sdual_cap_) {
    const size_t cap = std::max(bytes + bytes / 4, static_cast<size_t>(1) << 20);
    if (sdual_arena_ != nullptr) {
      Check(hipStreamSynchronize(Stream(stream_)), "sdual sync");
      Check(hipFree(sdual_arena_), "hipFree");
      Check(hipHostFree(sdual_staging_), "hipHostFree");
      sdual_arena_ = nullptr;
      sdual_staging_ = nullptr;
    }
    Check(hipMalloc(&sdual_arena_, cap), "hipMalloc sdual arena");
    Check(hipHostMalloc(&sdual_staging_, cap, hipHostMallocDefault), "hipHostMalloc sdual");
    sdual_cap_ = cap;
  }
  const size_t basis_off = 256;
  const size_t image_off = basis_off + ((sizeof(int32_t) * static_cast<size_t>(rows) + 255) & ~size_t{255});
  const size_t mb_bytes = image_off + static_cast<size_t>(lu_cap);
  if (mb_bytes > sdual_mb_cap_) {
    if (sdual_mb_block_ != nullptr) Check(hipHostFree(sdual_mb_block_), "hipHostFree mailbox");
    const size_t cap = mb_bytes + mb_bytes / 4;
    Check(hipHostMalloc(&sdual_mb_block_, cap, hipHostMallocMapped | hipHostMallocCoherent),
          "hipHostMalloc mailbox");
    Check(hipHostGetDevicePointer(&sdual_mb_device_, sdual_mb_block_, 0), "mailbox pointer");
    sdual_mb_cap_ = cap;
  }
  char* base = static_cast<char*>(sdual_mb_block_);
  sdual_mb_ = reinterpret_cast<sdual::Mailbox*>(base);
  sdual_mb_basis_ = reinterpret_cast<int32_t*>(base + basis_off);
  sdual_mb_image_ = base + image_off;
  std::memset(base, 0, sizeof(sdual::Mailbox));
  sdual_mb_->image_cap = lu_cap;
}

void DeviceLp::SdualMailboxDevice(sdual::Mailbox** mb, int32_t** basis, char** image) const {
  char* d = static_cast<char*>(sdual_mb_device_);
  const char* h = static_cast<const char*>(sdual_mb_block_);
  *mb = reinterpret_cast<sdual::Mailbox*>(d);
  *basis = reinterpret_cast<int32_t*>(d + (reinterpret_cast<const char*>(sdual_mb_basis_) - h));
  *image = d + (sdual_mb_image_ - h);
}

void DeviceLp::SdualFree() {
  if (sdual_arena_ != nullptr) {
    (void)hipStreamSynchronize(Stream(stream_));
    (void)hipFree(sdual_arena_);
    (void)hipHostFree(sdual_staging_);
  }
  if (sdual_mb_block_ != nullptr) (void)hipHostFree(sdual_mb_block_);
  sdual_arena_ = nullptr;
  sdual_staging_ = nullptr;
  sdual_cap_ = 0;
  sdual_mb_block_ = nullptr;
  sdual_mb_cap_ = 0;
}

void DeviceLp::SdualMatrix(const int64_t** starts, const int32_t** rows, const double** vals,
                           const int64_t** t_starts, const int32_t** t_cols,
                           const double** t_vals) const {
  *starts = d_starts_;
  *rows = d_rows_;
  *vals = d_vals_;
  *t_starts = d_t_starts_;
  *t_cols = d_t_cols_;
  *t_vals = d_t_vals_;
}

void DeviceLp::SdualRun(size_t bytes, const double* arena_coeff, int n, void (*serve)(void*),
                        void* ctx) {
  DeviceOp("sdual segment");
  if (batch_pending_) WaitSmallBatch();
  BeginKernel(MI_K_SDUAL);
  Check(hipMemcpyAsync(sdual_arena_, sdual_staging_, bytes, hipMemcpyHostToDevice,
                       Stream(stream_)),
        "sdual H2D");
  hipLaunchKernelGGL(sdual_segment_kernel, dim3(1), dim3(64), 0, Stream(stream_),
                     reinterpret_cast<sdual::Lp*>(sdual_arena_));
  Check(hipGetLastError(), "sdual launch");
  // The segment's last update row becomes the device copy that later device
  // update-row reads see (update_row.cc coefficient_, non-listed positions
  // included).
  if (d_coeff_ != nullptr && n > 0) {
    Check(hipMemcpyAsync(d_coeff_, arena_coeff, sizeof(double) * static_cast<size_t>(n),
                         hipMemcpyDeviceToDevice, Stream(stream_)),
          "sdual coefficients");
  }
  Check(hipMemcpyAsync(sdual_staging_, sdual_arena_, bytes, hipMemcpyDeviceToHost,
                       Stream(stream_)),
        "sdual D2H");
  EndKernel(MI_K_SDUAL, 2.0 * static_cast<double>(bytes));
  // Answer factorization requests until the stream (kernel, copies) is done.
  int32_t* flag = &sdual_mb_->flag;
  while (true) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == 1) {
      DeviceOp("sdual factorization request");
      serve(ctx);
      __atomic_store_n(flag, 2, __ATOMIC_RELEASE);
      continue;
    }
    const hipError_t q = hipStreamQuery(Stream(stream_));
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) Check(q, "sdual segment");
    if (InFiber()) {
      FiberYield();
      RestoreDevice();
    } else {
      std::this_thread::yield();
    }
  }
  DeviceOp("sdual segment done");
}

}  // namespace milp
