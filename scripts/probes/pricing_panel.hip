// Measured note for SURVEY's MFMA pricing panel ("MFMA"):
// A^T Y for k right-hand sides over a dense m x n block (config 2's shape),
// three ways, on one MI355X:
//   exact1  k single-vector passes in Glop's ColumnScalarProduct order (four
//           strided chains r1..r4 over the rows, ((r1 + r2) + r3) + r4, a
//           product and a sum rounded separately) -- what the engine does now;
//   exactk  one pass, the same order for all k vectors at once (A read once);
//   mfma    v_mfma_f64_16x16x4_f64 tiles (16 columns x 16 vectors, 4 rows
//           per instruction).
// Prints each variant's time per panel, its HBM rate, and how many of the
// n*k results differ bitwise from exact1's (and the largest difference in
// ulps). Layout here: A row-major (lanes of a wave read consecutive columns
// of one row), not the engine's chain-major block; the A reads are the cost.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o pricing_panel pricing_panel.hip
//   ./pricing_panel [m] [n] [k]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

constexpr int kMaxK = 16;

// Glop's four chains: wave c of a 256-thread workgroup accumulates rows
// r = c, c + 4, ... of 64 consecutive columns (one per lane) for every
// vector; the chains meet in LDS and fold as ((r1 + r2) + r3) + r4.
template <int K>
__global__ __launch_bounds__(256) void exact_kernel(const double* __restrict__ a,
                                                    const double* __restrict__ y, int m, int n,
                                                    double* __restrict__ out) {
  __shared__ double part[4][K][64];
  const int lane = threadIdx.x & 63;
  const int chain = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  double acc[K];
#pragma unroll
  for (int j = 0; j < K; ++j) acc[j] = 0.0;
  if (col < n) {
    for (int r = chain; r < m; r += 4) {
      const double v = a[static_cast<int64_t>(r) * n + col];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const double p = __dmul_rn(v, y[static_cast<int64_t>(j) * m + r]);
        acc[j] = __dadd_rn(acc[j], p);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < K; ++j) part[chain][j][lane] = acc[j];
  __syncthreads();
  if (chain == 0 && col < n) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const double s = __dadd_rn(__dadd_rn(__dadd_rn(part[0][j][lane], part[1][j][lane]),
                                           part[2][j][lane]),
                                 part[3][j][lane]);
      out[static_cast<int64_t>(j) * n + col] = s;
    }
  }
}

// One wave per 16 columns x 16 vectors: per 4 rows one MFMA, lane l holding
// A[r0 + (l >> 4)][c0 + (l & 15)] and Y[r0 + (l >> 4)][l & 15]; the result
// D[c0 + (l >> 4) + 4 i][l & 15] in register i.
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void mfma_kernel(const double* __restrict__ a,
                                                   const double* __restrict__ y, int m, int n,
                                                   double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int c0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
  if (c0 >= n) return;
  const int kk = lane >> 4;
  const int ci = lane & 15;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int r0 = 0; r0 < m; r0 += 4) {
    const int r = r0 + kk;
    const double av = (r < m && c0 + ci < n) ? a[static_cast<int64_t>(r) * n + c0 + ci] : 0.0;
    const double yv = r < m ? y[static_cast<int64_t>(ci) * m + r] : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, yv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = c0 + kk + 4 * i;
    if (col < n) out[static_cast<int64_t>(ci) * n + col] = acc[i];
  }
}

static uint64_t lcg(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return s >> 11;
}

int main(int argc, char** argv) {
  const int m = argc > 1 ? std::atoi(argv[1]) : 10000;
  const int n = argc > 2 ? std::atoi(argv[2]) : 50000;
  const int k = kMaxK;
  std::vector<double> ha(static_cast<size_t>(m) * n), hy(static_cast<size_t>(k) * m);
  uint64_t s = 20261018;
  for (auto& v : ha) v = static_cast<double>(lcg(s)) / 9007199254740992.0 * 2.0 - 1.0;
  for (auto& v : hy) v = static_cast<double>(lcg(s)) / 9007199254740992.0 * 2.0 - 1.0;
  double *a, *y, *y1, *o1, *ok, *om;
  const size_t abytes = ha.size() * sizeof(double);
  CHECK(hipMalloc(&a, abytes));
  CHECK(hipMalloc(&y, hy.size() * sizeof(double)));
  CHECK(hipMalloc(&y1, static_cast<size_t>(m) * sizeof(double)));
  CHECK(hipMalloc(&o1, static_cast<size_t>(k) * n * sizeof(double)));
  CHECK(hipMalloc(&ok, static_cast<size_t>(k) * n * sizeof(double)));
  CHECK(hipMalloc(&om, static_cast<size_t>(k) * n * sizeof(double)));
  CHECK(hipMemcpy(a, ha.data(), abytes, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(y, hy.data(), hy.size() * sizeof(double), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int blocks_e = (n + 63) / 64;
  const int blocks_m = (n / 16 + 3) / 4 + 1;
  auto time = [&](auto launch, int reps) {
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return static_cast<double>(ms) / reps;
  };
  // exact1: k passes of the one-vector kernel (vector j copied to y1 first is
  // not needed: the kernel takes y + j * m).
  const double t1 = time([&] {
    for (int j = 0; j < k; ++j) {
      exact_kernel<1><<<blocks_e, 256>>>(a, y + static_cast<size_t>(j) * m, m, n,
                                         o1 + static_cast<size_t>(j) * n);
    }
  }, 5);
  const double tk = time([&] { exact_kernel<kMaxK><<<blocks_e, 256>>>(a, y, m, n, ok); }, 5);
  const double tm = time([&] { mfma_kernel<<<blocks_m, 256>>>(a, y, m, n, om); }, 5);
  CHECK(hipGetLastError());
  std::vector<double> r1(static_cast<size_t>(k) * n), rk(r1.size()), rm(r1.size());
  CHECK(hipMemcpy(r1.data(), o1, r1.size() * 8, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(rk.data(), ok, rk.size() * 8, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(rm.data(), om, rm.size() * 8, hipMemcpyDeviceToHost));
  auto diff = [&](const std::vector<double>& x, int64_t* count, double* max_ulp) {
    *count = 0;
    *max_ulp = 0;
    for (size_t i = 0; i < x.size(); ++i) {
      if (std::memcmp(&x[i], &r1[i], 8) == 0) continue;
      ++*count;
      const double ulp = std::fabs(x[i] - r1[i]) / std::ldexp(1.0, std::ilogb(r1[i]) - 52);
      if (ulp > *max_ulp) *max_ulp = ulp;
    }
  };
  int64_t ck, cm;
  double uk, um;
  diff(rk, &ck, &uk);
  diff(rm, &cm, &um);
  const double gb = static_cast<double>(abytes) / 1e9;
  std::printf("{\"m\": %d, \"n\": %d, \"k\": %d, \"A_GB\": %.3f,\n", m, n, k, gb);
  std::printf(" \"exact1_ms\": %.3f, \"exact1_GBps\": %.0f,\n", t1, k * gb / (t1 * 1e-3));
  std::printf(" \"exactk_ms\": %.3f, \"exactk_GBps\": %.0f, \"exactk_bitwise_differences\": %lld,\n",
              tk, gb / (tk * 1e-3), static_cast<long long>(ck));
  std::printf(" \"mfma_ms\": %.3f, \"mfma_GBps\": %.0f, \"mfma_bitwise_differences\": %lld, "
              "\"mfma_max_ulps\": %.1f, \"results\": %zu}\n",
              tm, gb / (tm * 1e-3), static_cast<long long>(cm), um, r1.size());
  return 0;
}
