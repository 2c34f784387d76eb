// Device-resident dual simplex segment: the algorithms.
//
// One restatement, compiled twice: by g++ into the host engine (the CPU
// checks and MILP_SDUAL=host) and by hipcc into the gfx950 kernel
// (sdual_kernel.hip). Each function follows the Glop function named in its
// comment with the same floating-point evaluation order, so the device run is
// bit-identical to the host engine and to the oracle. Compiled with
// -ffp-contract=off everywhere.
#ifndef MILP_SDUAL_CORE_H_
#define MILP_SDUAL_CORE_H_

#include "sdual_state.h"

#if !defined(__HIPCC__)
#include <cmath>
#endif

namespace sdual {

constexpr int kInvalid = -1;
// lp_types.h VariableStatus / VariableType
constexpr int8_t kBasic = 0, kFixedValue = 1, kAtLower = 2, kAtUpper = 3, kFree = 4;
constexpr int8_t kUnconstrained = 0, kLowerBounded = 1, kUpperBounded = 2, kBoxed = 3,
                 kFixedVariable = 4;

SD_INLINE f64 sd_inf() { return __builtin_inf(); }
SD_INLINE f64 sd_dbl_max() { return 1.7976931348623157e308; }
SD_INLINE f64 sd_fabs(f64 v) { return __builtin_fabs(v); }
SD_INLINE f64 sd_sqrt(f64 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_sqrt(v);
#else
  return std::sqrt(v);
#endif
}
// std::max / std::min exactly (NaN and signed-zero behaviour included).
SD_INLINE f64 sd_max(f64 a, f64 b) { return (a < b) ? b : a; }
SD_INLINE f64 sd_min(f64 a, f64 b) { return (b < a) ? b : a; }
SD_INLINE f64 sq(f64 v) { return v * v; }
SD_INLINE f64 dt_ops(int64_t n) { return 2e-9 * static_cast<f64>(n); }

// ---- the wave ----
// On the device all 64 lanes of the workgroup's single wave walk the loop
// together: scalar work is executed redundantly (same addresses, same values,
// so the memory system serves them once), and loops whose iterations are
// independent are split over the lanes, followed by sd_sync(). On the host
// there is one lane.
SD_INLINE int sd_lane() {
#if defined(__HIP_DEVICE_COMPILE__)
  return static_cast<int>(threadIdx.x);
#else
  return 0;
#endif
}
SD_INLINE int sd_lanes() {
#if defined(__HIP_DEVICE_COMPILE__)
  return static_cast<int>(blockDim.x);
#else
  return 1;
#endif
}
SD_INLINE void sd_sync() {
#if defined(__HIP_DEVICE_COMPILE__)
  __threadfence_block();
  __syncthreads();
#endif
}
// Maximum over the lanes (exact: no rounding; values are finite).
SD_INLINE f64 sd_wave_max(f64 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  for (int off = 32; off > 0; off >>= 1) {
    const f64 o = __shfl_xor(v, off, 64);
    v = (v < o) ? o : v;
  }
#endif
  return v;
}
SD_INLINE int sd_wave_min_int(int v) {
#if defined(__HIP_DEVICE_COMPILE__)
  for (int off = 32; off > 0; off >>= 1) {
    const int o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
#endif
  return v;
}
// Positions i in [0, n) with keep(i), in increasing order, into out; returns
// the count (ballot + prefix popcount per 64-wide chunk).
// sd_ordered_compact_map: the values map(i) of those positions instead.
template <typename Keep, typename Map>
SD_INLINE int sd_ordered_compact_map(int n, int32_t* out, Keep keep, Map map) {
#if defined(__HIP_DEVICE_COMPILE__)
  int count = 0;
  const int lane = sd_lane();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  // Four chunks per round: their keep() tests (loads) are all issued before
  // the first write, so a round waits on one memory trip instead of four;
  // the chunks are then written in order.
  for (int base = 0; base < n; base += 256) {
    bool k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = base + 64 * u + lane;
      k[u] = i < n && keep(i);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t mask = __ballot(k[u]);
      if (k[u]) out[count + __popcll(mask & below)] = map(base + 64 * u + lane);
      count += __popcll(mask);
    }
  }
  sd_sync();
  return count;
#else
  int count = 0;
  for (int i = 0; i < n; ++i) {
    if (keep(i)) out[count++] = map(i);
  }
  return count;
#endif
}
template <typename Keep>
SD_INLINE int sd_ordered_compact(int n, int32_t* out, Keep keep) {
  return sd_ordered_compact_map(n, out, keep, [](int i) { return i; });
}
SD_INLINE int64_t sd_wave_sum_i64(int64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
#endif
  return v;
}

template <typename T>
SD_INLINE void sd_fill(T* p, int64_t n, T v) {
  for (int64_t i = sd_lane(); i < n; i += sd_lanes()) p[i] = v;
  sd_sync();
}

// The workgroup's LDS scratch (sdual_kernel.hip: after the staging area):
// 256 products or chain sums, then one chunk of rank-one step metadata.
struct SdScratch {
  f64 red[256];
  int64_t meta[64 * 4];
  f64 mu[64];
};
constexpr int kSdScratchDoubles = static_cast<int>(sizeof(SdScratch) / sizeof(f64));

#if defined(__HIP_DEVICE_COMPILE__)
// Explicit address spaces for the hot loops: the arena's arrays are global
// memory (AS 1), the workgroup's scratch LDS (AS 3). Typed pointers let the
// compiler issue global_load / ds_read (partial waits, several loads in
// flight) instead of flat accesses, and know that the two never alias.
#define SD_G(T, p) ((__attribute__((address_space(1))) T*)(p))
#define SD_L(T, p) ((__attribute__((address_space(3))) T*)(p))
typedef __attribute__((address_space(1))) f64 g_f64;
typedef __attribute__((address_space(3))) f64 l_f64;
typedef __attribute__((address_space(1))) const int32_t gc_i32;
typedef __attribute__((address_space(1))) const int64_t gc_i64;
typedef __attribute__((address_space(1))) const f64 gc_f64;
typedef __attribute__((address_space(3))) int64_t l_i64;
// Whether a generic pointer addresses the workgroup's LDS (the solves'
// working vector lives there, SdLdsVec).
__device__ inline bool sd_is_lds(const void* p) { return __builtin_amdgcn_is_shared(p); }


// Lane j's accumulator chain of an ordered dot: acc += red[j], red[j + 4],
// ... (groups terms, in order). The LDS reads go out eight at a time ahead of
// the additions (a plain loop waits on each read before its add); the
// additions keep their order, so the sum is bit for bit the loop's.
__device__ inline f64 sd_chain_sum(l_f64* red, int lane, int groups, f64 acc) {
  int g = 0;
  for (; g + 8 <= groups; g += 8) {
    f64 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = red[lane + 4 * (g + u)];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; g < groups; ++g) acc += red[lane + 4 * g];
  return acc;
}
// red[0 .. cnt) added in order onto sum (one lane), the reads eight ahead.
__device__ inline f64 sd_seq_sum(l_f64* red, int cnt, f64 sum) {
  int j = 0;
  for (; j + 8 <= cnt; j += 8) {
    f64 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = red[j + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) sum += v[u];
  }
  for (; j < cnt; ++j) sum += red[j];
  return sum;
}

// ColumnScalarProduct (sparse.h:514-542) of entries [b, e) of a column
// (rows/coefs) against x, on the lanes: up to 256 products are computed
// together (their loads in flight at once) and written to LDS, then lane
// j < 4 adds the products of entries j, j + 4, ... in order (Glop's
// accumulator r_{j+1}); the four sums are folded as ((r1 + r2) + r3) + r4
// and the tail entries added in order. Same roundings as the sequential loop.
template <typename XP>
__device__ inline f64 sd_ordered_dot(gc_i32* rows, gc_f64* coefs, int64_t b, int64_t e, XP x,
                                     l_f64* red) {
  const int lane = sd_lane();
  const int64_t len = e - b;
  const int64_t body = len & ~int64_t{3};
  f64 acc = 0.0;
  f64 tail[3] = {0.0, 0.0, 0.0};
  // Rounds of up to 256 entries cover the body and the (up to three) tail
  // entries; the tail products are read back before the chain sums reuse red.
  for (int64_t base = 0; base < len; base += 256) {
    const int64_t n = len - base < 256 ? len - base : 256;
    f64 p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t k = base + u * 64 + lane;
      p[u] = 0.0;
      if (u * 64 + lane < n) p[u] = coefs[b + k] * x[rows[b + k]];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) red[u * 64 + lane] = p[u];
    sd_sync();
    const int64_t nb = body - base < n ? (body - base > 0 ? body - base : 0) : n;
    if (lane < 4) acc = sd_chain_sum(red, lane, static_cast<int>(nb >> 2), acc);
    for (int64_t t = body > base ? body : base; t < base + n; ++t) tail[t - body] = red[t - base];
    sd_sync();
  }
  if (lane < 4) red[lane] = acc;
  sd_sync();
  f64 result = red[0] + red[1] + red[2] + red[3];
  sd_sync();
  for (int64_t t = body; t < len; ++t) result += tail[t - body];
  return result;
}
#endif

// ---- Bitset64 ----
SD_INLINE bool bit_get(const uint64_t* w, int i) { return (w[i >> 6] >> (i & 63)) & 1; }
SD_INLINE void bit_set(uint64_t* w, int i) { w[i >> 6] |= (1ull << (i & 63)); }
SD_INLINE void bit_clear(uint64_t* w, int i) { w[i >> 6] &= ~(1ull << (i & 63)); }
SD_INLINE void bit_put(uint64_t* w, int i, bool v) {
  if (v) bit_set(w, i); else bit_clear(w, i);
}
SD_INLINE int sd_ctz(uint64_t v) { return __builtin_ctzll(v); }

// ---- std::mt19937_64, libstdc++ state layout ----
SD_INLINE uint64_t mt_next(Lp& s) {
  const int n = 312, mm = 156;
  const uint64_t upper = ~((1ull << 31) - 1), lower = (1ull << 31) - 1;
  if (s.mti >= 312) {
    for (int k = 0; k < n - mm; ++k) {
      const uint64_t y = (s.mt[k] & upper) | (s.mt[k + 1] & lower);
      s.mt[k] = s.mt[k + mm] ^ (y >> 1) ^ ((y & 1) ? 0xb5026f5aa96619e9ull : 0);
    }
    for (int k = n - mm; k < n - 1; ++k) {
      const uint64_t y = (s.mt[k] & upper) | (s.mt[k + 1] & lower);
      s.mt[k] = s.mt[k + (mm - n)] ^ (y >> 1) ^ ((y & 1) ? 0xb5026f5aa96619e9ull : 0);
    }
    const uint64_t y = (s.mt[n - 1] & upper) | (s.mt[0] & lower);
    s.mt[n - 1] = s.mt[mm - 1] ^ (y >> 1) ^ ((y & 1) ? 0xb5026f5aa96619e9ull : 0);
    s.mti = 0;
  }
  uint64_t z = s.mt[s.mti++];
  z ^= (z >> 29) & 0x5555555555555555ull;
  z ^= (z << 17) & 0x71d67fffeda60000ull;
  z ^= (z << 37) & 0xfff7eee000000000ull;
  z ^= (z >> 43);
  return z;
}

SD_INLINE void mul64(uint64_t a, uint64_t b, uint64_t* hi, uint64_t* lo) {
#if defined(__HIP_DEVICE_COMPILE__)
  *hi = __umul64hi(a, b);
  *lo = a * b;
#else
  const unsigned __int128 p = static_cast<unsigned __int128>(a) * b;
  *hi = static_cast<uint64_t>(p >> 64);
  *lo = static_cast<uint64_t>(p);
#endif
}

// std::uniform_int_distribution<int>(0, hi)(mt19937_64): libstdc++ (GCC 11)
// takes _S_nd<unsigned __int128> (Lemire) for a full 64-bit generator.
SD_INLINE int uniform_int(Lp& s, int hi) {
  const uint64_t range = static_cast<uint64_t>(hi) + 1;
  uint64_t ph, pl;
  mul64(mt_next(s), range, &ph, &pl);
  if (pl < range) {
    const uint64_t threshold = (0ull - range) % range;
    while (pl < threshold) mul64(mt_next(s), range, &ph, &pl);
  }
  return static_cast<int>(ph);
}

// absl::Bernoulli as restated by the oracle (oracle_simplex.h AbslBernoulli).
SD_INLINE bool bernoulli(Lp& s, f64 p) {
  const f64 kP32 = 4294967296.0;
  while (true) {
    const uint64_t c = static_cast<uint64_t>(static_cast<int64_t>(p * kP32));
    const uint32_t v = static_cast<uint32_t>(mt_next(s));
    if (v != c) return v < c;
    const f64 q = static_cast<f64>(c) / kP32;
    const f64 here = (p - q) * kP32;
    if (here == 0) return false;
    p = here;
  }
}

// std::sort of distinct-or-not ints: any correct sort gives the same result.
SD_INLINE void sort_ints(int32_t* a, int n) {
  if (n < 2) return;
  if (n <= 24) {
    for (int i = 1; i < n; ++i) {
      const int32_t v = a[i];
      int j = i - 1;
      while (j >= 0 && a[j] > v) {
        a[j + 1] = a[j];
        --j;
      }
      a[j + 1] = v;
    }
    return;
  }
  // heap sort
  for (int start = (n - 2) / 2; start >= 0; --start) {
    int root = start;
    while (2 * root + 1 < n) {
      int child = 2 * root + 1;
      if (child + 1 < n && a[child] < a[child + 1]) ++child;
      if (a[root] < a[child]) {
        const int32_t t = a[root]; a[root] = a[child]; a[child] = t;
        root = child;
      } else {
        break;
      }
    }
  }
  for (int end = n - 1; end > 0; --end) {
    const int32_t t = a[0]; a[0] = a[end]; a[end] = t;
    int root = 0;
    while (2 * root + 1 < end) {
      int child = 2 * root + 1;
      if (child + 1 < end && a[child] < a[child + 1]) ++child;
      if (a[root] < a[child]) {
        const int32_t u = a[root]; a[root] = a[child]; a[child] = u;
        root = child;
      } else {
        break;
      }
    }
  }
}

// Sorts n distinct values of [0, range) in increasing order (the result of
// any correct sort). flags: `range` bytes, zero on entry and on exit. On the
// device: up to 128 values by rank (each lane counts the smaller values via
// shuffles), more by marking the flags and compacting [0, range) in order
// (ballot prefix counts, four 64-position chunks per round).
SD_INLINE void sort_distinct(int32_t* a, int n, int range, char* flags) {
  if (n < 2) return;
#if defined(__HIP_DEVICE_COMPILE__)
  sd_sync();  // the list and the flags were last written by every lane
  const int lane = sd_lane();
  if (__builtin_amdgcn_is_shared(flags) && range <= 64 * 256) {
    // Flags in LDS: mark, then lane j scans its block of range / 64
    // positions, counts, takes its offset from a wave prefix sum and writes
    // its positions in order (clearing the flags).
    __attribute__((address_space(3))) char* f = SD_L(char, flags);
    for (int k = lane; k < n; k += 64) f[a[k]] = 1;
    sd_sync();
    const int per = (range + 63) / 64;
    const int lo = lane * per;
    const int hi = lo + per < range ? lo + per : range;
    int count = 0;
    for (int i = lo; i < hi; ++i) count += f[i] != 0;
    int incl = count;
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(incl, off, 64);
      if (lane >= off) incl += t;
    }
    int pos = incl - count;
    for (int i = lo; i < hi; ++i) {
      if (f[i] != 0) {
        a[pos++] = i;
        f[i] = 0;
      }
    }
    sd_sync();
    return;
  }
  if (n <= 128) {
    const int32_t kNone = 0x7fffffff;
    const int32_t v0 = lane < n ? a[lane] : kNone;
    const int32_t v1 = lane + 64 < n ? a[lane + 64] : kNone;
    int r0 = 0, r1 = 0;
    for (int j = 0; j < 64; ++j) {
      const int32_t x0 = __shfl(v0, j, 64), x1 = __shfl(v1, j, 64);
      r0 += (x0 < v0) + (x1 < v0);
      r1 += (x0 < v1) + (x1 < v1);
    }
    sd_sync();
    if (lane < n) a[r0] = v0;
    if (lane + 64 < n) a[r1] = v1;
    sd_sync();
    return;
  }
  for (int k = lane; k < n; k += 64) flags[a[k]] = 1;
  sd_sync();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int count = 0;
  for (int base = 0; base < range; base += 256) {
    bool f[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = base + 64 * u + lane;
      f[u] = i < range && flags[i] != 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = base + 64 * u + lane;
      const uint64_t m = __ballot(f[u]);
      if (f[u]) {
        a[count + __popcll(m & below)] = i;
        flags[i] = 0;
      }
      count += __popcll(m);
    }
  }
  sd_sync();
#else
  (void)range;
  (void)flags;
  sort_ints(a, n);
#endif
}

// ---- ScatteredVector helpers (scattered_vector.h, lp_utils.h) ----
SD_INLINE bool vec_dense(const Vec& v, f64 ratio) {
  if (v.nnz == 0) return true;
  return static_cast<f64>(v.nnz) > ratio * static_cast<f64>(v.size);
}
// The list holds distinct positions: loops over it split over the lanes.
SD_INLINE void vec_clear_mask(Vec& v) {
  if (vec_dense(v, 0.8)) {
    sd_fill<char>(v.mask, v.size, 0);
  } else {
    for (int k = sd_lane(); k < v.nnz; k += sd_lanes()) v.mask[v.nz[k]] = 0;
    sd_sync();
  }
}
SD_INLINE void vec_repopulate_mask(Vec& v) {
  vec_clear_mask(v);
  for (int k = sd_lane(); k < v.nnz; k += sd_lanes()) v.mask[v.nz[k]] = 1;
  sd_sync();
}
SD_INLINE void vec_clear_nz_if_too_dense(Vec& v, f64 ratio) {
  if (vec_dense(v, ratio)) {
    vec_clear_mask(v);
    v.nnz = 0;
  }
}
SD_INLINE void vec_add(Vec& v, int i, f64 value) {
  v.values[i] += value;
  if (!v.mask[i] && value != 0.0) {
    v.mask[i] = 1;
    v.nz[v.nnz++] = i;
    v.sorted = 0;
  }
}
SD_INLINE void vec_sort_if_needed(Vec& v, char* flags) {
  if (!v.sorted) {
    sort_distinct(v.nz, v.nnz, v.size, flags);
    v.sorted = 1;
  }
}
SD_INLINE int64_t vec_nnz_estimate(const Vec& v) { return v.nnz == 0 ? v.size : v.nnz; }
// lp_utils.h:281-299 (the size is always m here).
SD_INLINE void vec_clear_and_resize(Vec& v, int size) {
  if (v.nnz != 0 && static_cast<f64>(v.nnz) < 0.05 * static_cast<f64>(size)) {
    for (int k = sd_lane(); k < v.nnz; k += sd_lanes()) v.values[v.nz[k]] = 0.0;
    for (int i = v.size + sd_lane(); i < size; i += sd_lanes()) v.values[i] = 0.0;
    sd_sync();
  } else {
    sd_fill<f64>(v.values, size, 0.0);
  }
  v.size = size;
  v.nnz = 0;
}
SD_INLINE void vec_copy(Vec& dst, const Vec& src) {  // *x = b
  for (int i = sd_lane(); i < src.size; i += sd_lanes()) {
    dst.values[i] = src.values[i];
    dst.mask[i] = src.mask[i];
  }
  for (int k = sd_lane(); k < src.nnz; k += sd_lanes()) dst.nz[k] = src.nz[k];
  sd_sync();
  dst.size = src.size;
  dst.nnz = src.nnz;
  dst.sorted = src.sorted;
}
// lp_utils.cc:62-75 and :46-54
SD_INLINE f64 dense_squared_norm(const f64* c, int n) {
  f64 sum = 0.0;
  int r = 0;
  const int blocks = n / 4;
  for (int b = 0; b < blocks; ++b) {
    sum += sq(c[r]) + sq(c[r + 1]) + sq(c[r + 2]) + sq(c[r + 3]);
    r += 4;
  }
  while (r < n) {
    sum += sq(c[r]);
    ++r;
  }
  return sum;
}
#if defined(__HIP_DEVICE_COMPILE__)
// SquaredNorm of a ScatteredVector (lp_utils.h: blocks of four in order for
// a dense vector, the listed entries in order otherwise) on the lanes: up to
// 256 terms (a block's ((a + b) + c) + d, or one square) are computed
// together and lane 0 adds them in order; the result is broadcast.
__device__ inline f64 vec_squared_norm_dev(const Vec& v, f64* lds_scratch) {
  l_f64* red = SD_L(f64, reinterpret_cast<SdScratch*>(lds_scratch)->red);
  const int lane = sd_lane();
  const bool dense = vec_dense(v, 0.8);
  const f64* c = v.values;
  const int n = dense ? v.size / 4 : v.nnz;
  f64 sum = 0.0;
  for (int base = 0; base < n; base += 256) {
    const int cnt = n - base < 256 ? n - base : 256;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = base + 64 * u + lane;
      f64 term = 0.0;
      if (64 * u + lane < cnt) {
        if (dense) {
          const int r = 4 * j;
          term = sq(c[r]) + sq(c[r + 1]) + sq(c[r + 2]) + sq(c[r + 3]);
        } else {
          term = sq(c[v.nz[j]]);
        }
      }
      red[64 * u + lane] = term;
    }
    sd_sync();
    if (lane == 0) sum = sd_seq_sum(red, cnt, sum);
    sd_sync();
  }
  if (lane == 0) {
    if (dense) {
      for (int r = 4 * n; r < v.size; ++r) sum += sq(c[r]);
    }
    red[0] = sum;
  }
  sd_sync();
  const f64 result = red[0];
  sd_sync();
  return result;
}
#endif
SD_INLINE f64 vec_squared_norm(const Vec& v) {
  if (vec_dense(v, 0.8)) return dense_squared_norm(v.values, v.size);
  f64 sum = 0.0;
  for (int k = 0; k < v.nnz; ++k) sum += sq(v.values[v.nz[k]]);
  return sum;
}

// ---- CompactSparseMatrix column ops ----
// sparse.h:514-542
template <typename M>
SD_INLINE f64 col_dot(const M& a, int col, const f64* v) {
  int64_t i = a.starts[col];
  const int64_t end = a.starts[col + 1];
  const int64_t shifted_end = end - 3;
  f64 r1 = 0.0, r2 = 0.0, r3 = 0.0, r4 = 0.0;
  for (; i < shifted_end; i += 4) {
    r1 += a.coefs[i] * v[a.rows[i]];
    r2 += a.coefs[i + 1] * v[a.rows[i + 1]];
    r3 += a.coefs[i + 2] * v[a.rows[i + 2]];
    r4 += a.coefs[i + 3] * v[a.rows[i + 3]];
  }
  f64 result = r1 + r2 + r3 + r4;
  if (i < end) {
    result += a.coefs[i] * v[a.rows[i]];
    if (i + 1 < end) {
      result += a.coefs[i + 1] * v[a.rows[i + 1]];
      if (i + 2 < end) result += a.coefs[i + 2] * v[a.rows[i + 2]];
    }
  }
  return result;
}
template <typename M>
SD_INLINE int64_t col_entries(const M& a, int col) {
  return a.starts[col + 1] - a.starts[col];
}
// col_dot with the products on the lanes: lane j < 4 keeps accumulator
// r_{j+1} and adds the products of entries j, j + 4, j + 8, ... in order, so
// the sums round exactly as the sequential loop's.
template <typename M>
SD_INLINE f64 col_dot_par(const M& a, int col, const f64* v, f64* lds_scratch) {
#if defined(__HIP_DEVICE_COMPILE__)
  l_f64* red = SD_L(f64, reinterpret_cast<SdScratch*>(lds_scratch)->red);
  if (sd_is_lds(v)) {
    return sd_ordered_dot(SD_G(const int32_t, a.rows), SD_G(const f64, a.coefs), a.starts[col],
                          a.starts[col + 1], SD_L(const f64, v), red);
  }
  return sd_ordered_dot(SD_G(const int32_t, a.rows), SD_G(const f64, a.coefs), a.starts[col],
                        a.starts[col + 1], SD_G(const f64, v), red);
#else
  (void)lds_scratch;
  return col_dot(a, col, v);
#endif
}
// sparse.h:389-399
template <typename M>
SD_INLINE void col_add_dense(const M& a, int col, f64 mult, f64* dense) {
  if (mult == 0.0) return;
  // A column's rows are distinct: the lanes split it.
  for (int64_t i = a.starts[col] + sd_lane(); i < a.starts[col + 1]; i += sd_lanes())
    dense[a.rows[i]] += mult * a.coefs[i];
  sd_sync();
}
// sparse.h:403-413
// The lanes take 64 entries at a time (a column's rows are distinct); the new
// positions join the list in entry order (ballot prefix counts).
template <typename M>
SD_INLINE void col_add_scattered(const M& a, int col, f64 mult, Vec& c) {
  if (mult == 0.0) return;
#if defined(__HIP_DEVICE_COMPILE__)
  const int64_t e = a.starts[col + 1];
  const int lane = sd_lane();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int nnz = c.nnz;
  for (int64_t base = a.starts[col]; base < e; base += 64) {
    const int64_t i = base + lane;
    bool fresh = false;
    int row = 0;
    if (i < e) {
      row = a.rows[i];
      const f64 value = mult * a.coefs[i];
      c.values[row] += value;
      fresh = !c.mask[row] && value != 0.0;
      if (fresh) c.mask[row] = 1;
    }
    const uint64_t fresh_mask = __ballot(fresh);
    if (fresh) c.nz[nnz + __popcll(fresh_mask & below)] = row;
    nnz += __popcll(fresh_mask);
  }
  sd_sync();
  if (nnz != c.nnz) c.sorted = 0;
  c.nnz = nnz;
#else
  for (int64_t i = a.starts[col]; i < a.starts[col + 1]; ++i)
    vec_add(c, a.rows[i], mult * a.coefs[i]);
#endif
}

// ---- growing storage (sparse.cc:576-623) ----
// Appends the nonzeros among positions pos(k), k < count, in k order as a
// new column (ballot prefix counts give each lane its slot); clear: zero the
// appended values in d. `pos` null: position k itself. A list that may
// repeat a position (the MPF scratch) goes through the sequential loop: its
// first occurrence takes the value and clears it.
SD_INLINE int store_append(Store& st, f64* d, const int32_t* pos, int first, int count, bool clear) {
  int64_t e = st.starts[st.num_cols];
#if defined(__HIP_DEVICE_COMPILE__)
  if (clear) {
    for (int k = first; k < count; ++k) {
      const int r = pos != nullptr ? pos[k] : k;
      const f64 v = d[r];
      if (v != 0.0) {
        st.rows[e] = r;
        st.coefs[e] = v;
        d[r] = 0.0;
        ++e;
      }
    }
    st.starts[st.num_cols + 1] = e;
    return st.num_cols++;
  }
  const int lane = sd_lane();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int base = first; base < count; base += 64) {
    const int k = base + lane;
    int r = 0;
    f64 v = 0.0;
    if (k < count) {
      r = pos != nullptr ? pos[k] : k;
      v = d[r];
    }
    const bool keep = v != 0.0;
    const uint64_t mask = __ballot(keep);
    if (keep) {
      const int64_t at = e + __popcll(mask & below);
      st.rows[at] = r;
      st.coefs[at] = v;
    }
    e += __popcll(mask);
  }
  sd_sync();
#else
  for (int k = first; k < count; ++k) {
    const int r = pos != nullptr ? pos[k] : k;
    const f64 v = d[r];
    if (v != 0.0) {
      st.rows[e] = r;
      st.coefs[e] = v;
      if (clear) d[r] = 0.0;
      ++e;
    }
  }
#endif
  st.starts[st.num_cols + 1] = e;
  return st.num_cols++;
}
SD_INLINE int store_add_dense_prefix(Store& st, const f64* d, int n, int start) {
  return store_append(st, const_cast<f64*>(d), nullptr, start, n, false);
}
SD_INLINE int store_add_dense_nz(Store& st, const f64* d, int n, const int32_t* nz, int nnz) {
  if (nnz == 0) return store_add_dense_prefix(st, d, n, 0);
  return store_append(st, const_cast<f64*>(d), nz, 0, nnz, false);
}
SD_INLINE int store_add_and_clear(Store& st, f64* col, int32_t* nz, int* nnz) {
  const int index = store_append(st, col, nz, 0, *nnz, true);
  *nnz = 0;
  return index;
}
// ColumnCopyToClearedDenseColumnWithNonZeros (sparse.h:440-455)
SD_INLINE void store_copy_to_vec(const Store& st, int col, Vec& v) {
  const int64_t b = st.starts[col];
  const int count = static_cast<int>(st.starts[col + 1] - b);
  for (int k = sd_lane(); k < count; k += sd_lanes()) {
    v.values[st.rows[b + k]] = st.coefs[b + k];
    v.nz[k] = st.rows[b + k];
  }
  sd_sync();
  v.nnz = count;
}

SD_INLINE uint64_t sd_now() {
#if defined(__HIP_DEVICE_COMPILE__)
  return wall_clock64();
#else
  return 0;
#endif
}
// Sub-phase timers (MILP_SDUAL_PROFILE): slots 9-11 count the dense
// triangular scatters, the dense transposed gathers and the rank-one
// products inside the loop phases that call them.
struct SdSubTimer {
  uint64_t* slot;
  uint64_t t0;
  SD_HD explicit SdSubTimer(uint64_t* p) : slot(p), t0(sd_now()) {}
  SD_HD ~SdSubTimer() { *slot += sd_now() - t0; }
};

// ---- TriangularMatrix solves (sparse.cc:776-1128) ----
SD_INLINE void tri_lower_solve_from(const Tri& t, int start, f64* x) {
  const int begin = start > t.first_non_identity ? start : t.first_non_identity;
  const int end = t.num_cols;
  const bool ones = t.all_ones;
  for (int col = begin; col < end; ++col) {
    const f64 value = x[col];
    if (value == 0.0) continue;
    const f64 coeff = ones ? value : value / t.diag[col];
    if (!ones) x[col] = coeff;
    for (int64_t i = t.starts[col]; i < t.starts[col + 1]; ++i)
      x[t.rows[i]] -= coeff * t.coefs[i];
  }
}
SD_INLINE void tri_upper_solve(const Tri& t, f64* x) {
  const int end = t.first_non_identity;
  const bool ones = t.all_ones;
  for (int col = t.num_cols - 1; col >= end; --col) {
    const f64 value = x[col];
    if (value == 0.0) continue;
    const f64 coeff = ones ? value : value / t.diag[col];
    if (!ones) x[col] = coeff;
    for (int64_t i = t.starts[col + 1] - 1; i >= t.starts[col]; --i)
      x[t.rows[i]] -= coeff * t.coefs[i];
  }
}
// One column of TransposeUpperSolve / TransposeLowerSolve
// (sparse.cc:872-947): the entries in the sequential code's order and
// grouping of four, so that a column computes the same value wherever it runs.
SD_INLINE f64 tri_tu_column(const Tri& t, const f64* x, int col) {
  f64 sum = x[col];
  int64_t i = t.starts[col];
  const int64_t i_end = t.starts[col + 1];
  const int64_t shifted_end = i_end - 3;
  for (; i < shifted_end; i += 4) {
    sum -= t.coefs[i] * x[t.rows[i]] + t.coefs[i + 1] * x[t.rows[i + 1]] +
           t.coefs[i + 2] * x[t.rows[i + 2]] + t.coefs[i + 3] * x[t.rows[i + 3]];
  }
  if (i < i_end) {
    sum -= t.coefs[i] * x[t.rows[i]];
    if (i + 1 < i_end) {
      sum -= t.coefs[i + 1] * x[t.rows[i + 1]];
      if (i + 2 < i_end) sum -= t.coefs[i + 2] * x[t.rows[i + 2]];
    }
  }
  return t.all_ones ? sum : sum / t.diag[col];
}
SD_INLINE f64 tri_tl_column(const Tri& t, const f64* x, int col) {
  f64 sum = x[col];
  int64_t i = t.starts[col + 1] - 1;
  const int64_t i_end = t.starts[col];
  const int64_t shifted_end = i_end + 3;
  for (; i >= shifted_end; i -= 4) {
    sum -= t.coefs[i] * x[t.rows[i]] + t.coefs[i - 1] * x[t.rows[i - 1]] +
           t.coefs[i - 2] * x[t.rows[i - 2]] + t.coefs[i - 3] * x[t.rows[i - 3]];
  }
  if (i >= i_end) {
    sum -= t.coefs[i] * x[t.rows[i]];
    if (i >= i_end + 1) {
      sum -= t.coefs[i - 1] * x[t.rows[i - 1]];
      if (i >= i_end + 2) sum -= t.coefs[i - 2] * x[t.rows[i - 2]];
    }
  }
  return t.all_ones ? sum : sum / t.diag[col];
}
// A level schedule pays when the levels are few against the columns.
SD_INLINE bool tri_use_levels(const Tri& t) {
  return t.num_levels >= 0 && 4 * t.num_levels <= t.num_cols - t.first_non_identity;
}
#if defined(__HIP_DEVICE_COMPILE__)
// One column of tri_tu_column (kUpper) / tri_tl_column with typed pointers:
// the four entries of a group load together.
template <bool kUpper, typename XP>
__device__ inline f64 tri_column_dev(gc_i32* rows, gc_f64* coefs, int64_t b, int64_t e, XP x,
                                     int col) {
  f64 sum = x[col];
  if (kUpper) {
    int64_t i = b;
    for (; i < e - 3; i += 4) {
      sum -= coefs[i] * x[rows[i]] + coefs[i + 1] * x[rows[i + 1]] +
             coefs[i + 2] * x[rows[i + 2]] + coefs[i + 3] * x[rows[i + 3]];
    }
    if (i < e) {
      sum -= coefs[i] * x[rows[i]];
      if (i + 1 < e) {
        sum -= coefs[i + 1] * x[rows[i + 1]];
        if (i + 2 < e) sum -= coefs[i + 2] * x[rows[i + 2]];
      }
    }
  } else {
    int64_t i = e - 1;
    for (; i >= b + 3; i -= 4) {
      sum -= coefs[i] * x[rows[i]] + coefs[i - 1] * x[rows[i - 1]] +
             coefs[i - 2] * x[rows[i - 2]] + coefs[i - 3] * x[rows[i - 3]];
    }
    if (i >= b) {
      sum -= coefs[i] * x[rows[i]];
      if (i >= b + 1) {
        sum -= coefs[i - 1] * x[rows[i - 1]];
        if (i >= b + 2) sum -= coefs[i - 2] * x[rows[i - 2]];
      }
    }
  }
  return sum;
}
// A lane's next column of a level sweep, fetched ahead: its entry range,
// the first group of four entries in the order tri_column_dev takes them
// (from the start for kUpper, from the end otherwise) and the diagonal.
struct SdColPf {
  int col;
  int64_t b, e;
  int r[4];
  f64 c[4];
  f64 diag;
};
template <bool kUpper>
__device__ inline void tri_fetch_col(gc_i32* order, gc_i64* starts, gc_i32* rows, gc_f64* coefs,
                                     gc_f64* diag, bool ones, int k, SdColPf* p) {
  p->col = order[k];
  p->b = starts[p->col];
  p->e = starts[p->col + 1];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = kUpper ? p->b + u : p->e - 1 - u;
    const bool in = kUpper ? i < p->e : i >= p->b;
    p->r[u] = in ? rows[i] : 0;
    p->c[u] = in ? coefs[i] : 0.0;
  }
  p->diag = ones ? 1.0 : diag[p->col];
}
// tri_column_dev with the first group of entries from a prefetch.
template <bool kUpper, typename XP>
__device__ inline f64 tri_column_pf(gc_i32* rows, gc_f64* coefs, const SdColPf& p, XP x) {
  const int64_t b = p.b, e = p.e;
  f64 sum = x[p.col];
  if (e - b >= 4) {
    sum -= p.c[0] * x[p.r[0]] + p.c[1] * x[p.r[1]] + p.c[2] * x[p.r[2]] + p.c[3] * x[p.r[3]];
    if (kUpper) {
      int64_t i = b + 4;
      // Whole groups with the next group's entries loaded while the current
      // one is subtracted (same expression and order per group).
      if (i < e - 3) {
        int r[4];
        f64 c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          r[u] = rows[i + u];
          c[u] = coefs[i + u];
        }
        for (; i < e - 3; i += 4) {
          int nr[4] = {0, 0, 0, 0};
          f64 nc[4] = {0.0, 0.0, 0.0, 0.0};
          if (i + 4 < e - 3) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              nr[u] = rows[i + 4 + u];
              nc[u] = coefs[i + 4 + u];
            }
          }
          sum -= c[0] * x[r[0]] + c[1] * x[r[1]] + c[2] * x[r[2]] + c[3] * x[r[3]];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            r[u] = nr[u];
            c[u] = nc[u];
          }
        }
      }
      if (i < e) {
        sum -= coefs[i] * x[rows[i]];
        if (i + 1 < e) {
          sum -= coefs[i + 1] * x[rows[i + 1]];
          if (i + 2 < e) sum -= coefs[i + 2] * x[rows[i + 2]];
        }
      }
    } else {
      int64_t i = e - 5;
      if (i >= b + 3) {
        int r[4];
        f64 c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          r[u] = rows[i - u];
          c[u] = coefs[i - u];
        }
        for (; i >= b + 3; i -= 4) {
          int nr[4] = {0, 0, 0, 0};
          f64 nc[4] = {0.0, 0.0, 0.0, 0.0};
          if (i - 4 >= b + 3) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              nr[u] = rows[i - 4 - u];
              nc[u] = coefs[i - 4 - u];
            }
          }
          sum -= c[0] * x[r[0]] + c[1] * x[r[1]] + c[2] * x[r[2]] + c[3] * x[r[3]];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            r[u] = nr[u];
            c[u] = nc[u];
          }
        }
      }
      if (i >= b) {
        sum -= coefs[i] * x[rows[i]];
        if (i >= b + 1) {
          sum -= coefs[i - 1] * x[rows[i - 1]];
          if (i >= b + 2) sum -= coefs[i - 2] * x[rows[i - 2]];
        }
      }
    }
  } else {
    const int64_t len = e - b;
    if (len > 0) {
      sum -= p.c[0] * x[p.r[0]];
      if (len > 1) {
        sum -= p.c[1] * x[p.r[1]];
        if (len > 2) sum -= p.c[2] * x[p.r[2]];
      }
    }
  }
  return sum;
}
// The level sweep with each lane's next-level column (bounds, first four
// entries, diagonal: read-only schedule and factor data) loaded while the
// current level computes, so a level mostly waits on x in LDS.
template <bool kUpper, typename XP>
__device__ inline void tri_level_sweep_dev(const Tri& t, XP x, int last) {
  gc_i64* starts = SD_G(const int64_t, t.starts);
  gc_i32* rows = SD_G(const int32_t, t.rows);
  gc_f64* coefs = SD_G(const f64, t.coefs);
  gc_f64* diag = SD_G(const f64, t.diag);
  gc_i32* order = SD_G(const int32_t, t.lv_order);
  gc_i32* lvs = SD_G(const int32_t, t.lv_starts);
  const bool ones = t.all_ones;
  const int lane = sd_lane();
  const int levels = t.num_levels;
  if (levels <= 0) return;
  int le = lvs[1];
  int k = lvs[0] + lane;
  SdColPf cur;
  if (k < le) tri_fetch_col<kUpper>(order, starts, rows, coefs, diag, ones, k, &cur);
  for (int l = 0; l < levels; ++l) {
    const int le2 = l + 1 < levels ? lvs[l + 2] : le;
    const int k2 = le + lane;
    SdColPf nxt;
    if (k2 < le2) tri_fetch_col<kUpper>(order, starts, rows, coefs, diag, ones, k2, &nxt);
    while (k < le) {
      if (kUpper || cur.col <= last) {
        const f64 sum = tri_column_pf<kUpper>(rows, coefs, cur, x);
        x[cur.col] = ones ? sum : sum / cur.diag;
      }
      k += 64;
      if (k < le) tri_fetch_col<kUpper>(order, starts, rows, coefs, diag, ones, k, &cur);
    }
    sd_sync();
    le = le2;
    k = k2;
    cur = nxt;
  }
}
#endif
// Columns of each level split over the lanes, a barrier between levels:
// every column reads only finished columns, so the results are those of the
// sequential sweep.
SD_INLINE void tri_level_sweep_upper(const Tri& t, f64* x) {
  for (int l = 0; l < t.num_levels; ++l) {
    for (int k = t.lv_starts[l] + sd_lane(); k < t.lv_starts[l + 1]; k += sd_lanes()) {
      const int col = t.lv_order[k];
      x[col] = tri_tu_column(t, x, col);
    }
    sd_sync();
  }
}
SD_INLINE void tri_level_sweep_lower(const Tri& t, f64* x, int last) {
  for (int l = 0; l < t.num_levels; ++l) {
    for (int k = t.lv_starts[l] + sd_lane(); k < t.lv_starts[l + 1]; k += sd_lanes()) {
      const int col = t.lv_order[k];
      if (col <= last) x[col] = tri_tl_column(t, x, col);
    }
    sd_sync();
  }
}
// The dense vector of a level sweep in LDS when it fits: each level then
// waits on one round trip (its entries) instead of three.
SD_INLINE f64* sd_stage_in(f64* lds, int cap, const f64* x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (sd_is_lds(x)) return const_cast<f64*>(x);  // already the LDS working vector
#endif
  if (lds == nullptr || n > cap) return nullptr;
#if defined(__HIP_DEVICE_COMPILE__)
  l_f64* l = SD_L(f64, lds);
  gc_f64* g = SD_G(const f64, x);
#pragma unroll 8
  for (int i = sd_lane(); i < n; i += 64) l[i] = g[i];
#else
  for (int i = sd_lane(); i < n; i += sd_lanes()) lds[i] = x[i];
#endif
  sd_sync();
  return lds;
}
SD_INLINE void sd_stage_out(const f64* lds, f64* x, int n) {
  if (lds == x) return;
#if defined(__HIP_DEVICE_COMPILE__)
  // The staging area is left all zero (the LDS working vector's invariant).
  l_f64* l = SD_L(f64, const_cast<f64*>(lds));
  g_f64* g = SD_G(f64, x);
#pragma unroll 8
  for (int i = sd_lane(); i < n; i += 64) {
    g[i] = l[i];
    l[i] = 0.0;
  }
#else
  for (int i = sd_lane(); i < n; i += sd_lanes()) x[i] = lds[i];
#endif
  sd_sync();
}
SD_INLINE void tri_transpose_upper_solve(const Tri& t, f64* x, f64* lds = nullptr, int cap = 0) {
  if (tri_use_levels(t)) {
    if (f64* v = sd_stage_in(lds, cap, x, t.num_cols)) {
#if defined(__HIP_DEVICE_COMPILE__)
      tri_level_sweep_dev<true>(t, SD_L(f64, v), t.num_cols);
#else
      tri_level_sweep_upper(t, v);
#endif
      sd_stage_out(v, x, t.num_cols);
      return;
    }
    tri_level_sweep_upper(t, x);
    return;
  }
  for (int col = t.first_non_identity; col < t.num_cols; ++col) x[col] = tri_tu_column(t, x, col);
}
// The last column with a nonzero value (the sequential code's skip of the
// trailing zeros), end - 1 when there is none.
SD_INLINE int tri_last_nonzero(const f64* x, int end, int num_cols) {
#if defined(__HIP_DEVICE_COMPILE__)
  for (int top = num_cols - 1; top >= end; top -= 64) {
    const int col = top - sd_lane();
    const uint64_t mask = __ballot(col >= end && x[col] != 0.0);
    if (mask != 0) return top - (__builtin_ctzll(mask));
  }
  return end - 1;
#else
  int col = num_cols - 1;
  while (col >= end && x[col] == 0.0) --col;
  return col;
#endif
}
SD_INLINE void tri_transpose_lower_solve(const Tri& t, f64* x, f64* lds = nullptr, int cap = 0) {
  const int end = t.first_non_identity;
  const int last = tri_last_nonzero(x, end, t.num_cols);
  if (last < end) return;
  if (tri_use_levels(t)) {
    // Columns above `last` are read (zeros of either sign) but not written.
    if (f64* v = sd_stage_in(lds, cap, x, t.num_cols)) {
#if defined(__HIP_DEVICE_COMPILE__)
      tri_level_sweep_dev<false>(t, SD_L(f64, v), last);
#else
      tri_level_sweep_lower(t, v, last);
#endif
      sd_stage_out(v, x, last + 1);
      if (v != x) {  // entries above `last` were read only: clear their staged copies
        for (int i = last + 1 + sd_lane(); i < t.num_cols; i += sd_lanes()) v[i] = 0.0;
        sd_sync();
      }
      return;
    }
    tri_level_sweep_lower(t, x, last);
    return;
  }
  for (int col = last; col >= end; --col) x[col] = tri_tl_column(t, x, col);
}
#if defined(__HIP_DEVICE_COMPILE__)
// Hypersparse solves over a non-zero list (sparse.cc:957-1128) on the
// device: the next listed column's bounds, first entries and diagonal load
// while the current one computes (read-only factor data; the list entries
// ahead of the loop are never rewritten before they are read).
// kScatter: HyperSparseSolve / ...WithReversedNonZeros (a column scatter,
// split over the lanes); else TransposeHyperSparseSolve / ...Reversed (a
// grouped dot, tri_column_pf's order). kRev: the list from its end, kept rows
// gathered at its end and moved to the front (erase_prefix).
struct SdHyperPf {
  int row;
  int64_t b, e;
  int r;
  f64 c;
  f64 diag;
};
template <bool kScatter, bool kRev, typename XP>
__device__ inline void tri_hyper_dev(const Tri& t, XP x, int32_t* nz, int* nnz) {
  gc_i64* starts = SD_G(const int64_t, t.starts);
  gc_i32* rows = SD_G(const int32_t, t.rows);
  gc_f64* coefs = SD_G(const f64, t.coefs);
  gc_f64* diag = SD_G(const f64, t.diag);
  __attribute__((address_space(1))) int32_t* nzg = SD_G(int32_t, nz);
  const bool ones = t.all_ones;
  const int lane = sd_lane();
  const int n = *nnz;
  int out = kRev ? n : 0;
  if (kScatter) {
    auto fetch = [&](int k, SdHyperPf* p) {
      p->row = nzg[k];
      p->b = starts[p->row];
      p->e = starts[p->row + 1];
      const int64_t i = p->b + lane;
      p->r = i < p->e ? rows[i] : 0;
      p->c = i < p->e ? coefs[i] : 0.0;
      p->diag = ones ? 1.0 : diag[p->row];
    };
    SdHyperPf cur;
    if (n > 0) fetch(kRev ? n - 1 : 0, &cur);
    for (int j = 0; j < n; ++j) {
      const int k = kRev ? n - 1 - j : j;
      SdHyperPf nxt;
      if (j + 1 < n) fetch(kRev ? k - 1 : k + 1, &nxt);
      const f64 v = x[cur.row];
      if (v != 0.0) {
        const f64 coeff = ones ? v : v / cur.diag;
        x[cur.row] = coeff;
        if (cur.b + lane < cur.e) x[cur.r] -= coeff * cur.c;
        // The rest of the column (distinct rows): four chunks' loads at once.
        for (int64_t i0 = cur.b + 64 + lane; i0 < cur.e; i0 += 256) {
          int r[4];
          f64 c[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + 64 * u;
            r[u] = i < cur.e ? rows[i] : 0;
            c[u] = i < cur.e ? coefs[i] : 0.0;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (i0 + 64 * u < cur.e) x[r[u]] -= coeff * c[u];
          }
        }
        sd_sync();
        if (kRev) {
          nzg[--out] = cur.row;
        } else {
          nzg[out++] = cur.row;
        }
      }
      cur = nxt;
    }
  } else {
    // transposed: kRev walks the list backwards with the lower-triangle
    // (backward) grouping, as TransposeHyperSparseSolveWithReversedNonZeros.
    constexpr bool kForward = !kRev;
    gc_i32* order = nzg;
    SdColPf cur;
    if (n > 0) tri_fetch_col<kForward>(order, starts, rows, coefs, diag, ones, kRev ? n - 1 : 0, &cur);
    for (int j = 0; j < n; ++j) {
      const int k = kRev ? n - 1 - j : j;
      SdColPf nxt;
      if (j + 1 < n) tri_fetch_col<kForward>(order, starts, rows, coefs, diag, ones, kRev ? k - 1 : k + 1, &nxt);
      const f64 sum = tri_column_pf<kForward>(rows, coefs, cur, x);
      x[cur.col] = ones ? sum : sum / cur.diag;
      sd_sync();
      if (sum != 0.0) {
        if (kRev) {
          nzg[--out] = cur.col;
        } else {
          nzg[out++] = cur.col;
        }
      }
      cur = nxt;
    }
  }
  sd_sync();
  if (kRev) {
    // erase_prefix: the kept rows [out, n) to the front, chunk by chunk in
    // increasing order (a chunk's sources lie at or after its targets).
    const int cnt = n - out;
    for (int c0 = 0; c0 < cnt; c0 += 64) {
      const int k = c0 + lane;
      const int v = k < cnt ? nzg[out + k] : 0;
      sd_sync();
      if (k < cnt) nzg[k] = v;
      sd_sync();
    }
    *nnz = cnt;
  } else {
    *nnz = out;
  }
}
template <bool kScatter, bool kRev>
__device__ inline void tri_hyper_dispatch(const Tri& t, f64* x, int32_t* nz, int* nnz) {
  if (sd_is_lds(x)) {
    tri_hyper_dev<kScatter, kRev>(t, SD_L(f64, x), nz, nnz);
  } else {
    tri_hyper_dev<kScatter, kRev>(t, SD_G(f64, x), nz, nnz);
  }
}
#endif
// A column's scatter over its (distinct) rows is split over the lanes.
SD_INLINE void tri_scatter_column(const Tri& t, int col, f64 coeff, f64* x) {
  for (int64_t i = t.starts[col] + sd_lane(); i < t.starts[col + 1]; i += sd_lanes())
    x[t.rows[i]] -= coeff * t.coefs[i];
  sd_sync();
}
SD_INLINE void tri_hyper_solve(const Tri& t, f64* x, int32_t* nz, int* nnz) {
#if defined(__HIP_DEVICE_COMPILE__)
  tri_hyper_dispatch<true, false>(t, x, nz, nnz);
  return;
#endif
  const bool ones = t.all_ones;
  int new_size = 0;
  for (int k = 0; k < *nnz; ++k) {
    const int row = nz[k];
    if (x[row] == 0.0) continue;
    const f64 coeff = ones ? x[row] : x[row] / t.diag[row];
    x[row] = coeff;
    tri_scatter_column(t, row, coeff, x);
    nz[new_size++] = row;
  }
  *nnz = new_size;
}
SD_INLINE void erase_prefix(int32_t* nz, int* nnz, int new_start) {
  const int n = *nnz - new_start;
  for (int k = 0; k < n; ++k) nz[k] = nz[new_start + k];
  *nnz = n;
}
SD_INLINE void tri_hyper_solve_rev(const Tri& t, f64* x, int32_t* nz, int* nnz) {
#if defined(__HIP_DEVICE_COMPILE__)
  tri_hyper_dispatch<true, true>(t, x, nz, nnz);
  return;
#endif
  const bool ones = t.all_ones;
  int new_start = *nnz;
  for (int k = *nnz - 1; k >= 0; --k) {
    const int row = nz[k];
    if (x[row] == 0.0) continue;
    const f64 coeff = ones ? x[row] : x[row] / t.diag[row];
    x[row] = coeff;
    tri_scatter_column(t, row, coeff, x);
    nz[--new_start] = row;
  }
  erase_prefix(nz, nnz, new_start);
}
SD_INLINE void tri_transpose_hyper_solve(const Tri& t, f64* x, int32_t* nz, int* nnz) {
#if defined(__HIP_DEVICE_COMPILE__)
  tri_hyper_dispatch<false, false>(t, x, nz, nnz);
  return;
#endif
  const bool ones = t.all_ones;
  int new_size = 0;
  for (int k = 0; k < *nnz; ++k) {
    const int row = nz[k];
    f64 sum = x[row];
    int64_t i = t.starts[row];
    const int64_t i_end = t.starts[row + 1];
    const int64_t shifted_end = i_end - 3;
    for (; i < shifted_end; i += 4) {
      sum -= t.coefs[i] * x[t.rows[i]] + t.coefs[i + 1] * x[t.rows[i + 1]] +
             t.coefs[i + 2] * x[t.rows[i + 2]] + t.coefs[i + 3] * x[t.rows[i + 3]];
    }
    if (i < i_end) {
      sum -= t.coefs[i] * x[t.rows[i]];
      if (i + 1 < i_end) {
        sum -= t.coefs[i + 1] * x[t.rows[i + 1]];
        if (i + 2 < i_end) sum -= t.coefs[i + 2] * x[t.rows[i + 2]];
      }
    }
    x[row] = ones ? sum : sum / t.diag[row];
    if (sum != 0.0) nz[new_size++] = row;
  }
  *nnz = new_size;
}
SD_INLINE void tri_transpose_hyper_solve_rev(const Tri& t, f64* x, int32_t* nz, int* nnz) {
#if defined(__HIP_DEVICE_COMPILE__)
  tri_hyper_dispatch<false, true>(t, x, nz, nnz);
  return;
#endif
  const bool ones = t.all_ones;
  int new_start = *nnz;
  for (int k = *nnz - 1; k >= 0; --k) {
    const int row = nz[k];
    f64 sum = x[row];
    int64_t i = t.starts[row + 1] - 1;
    const int64_t i_end = t.starts[row];
    const int64_t shifted_end = i_end + 3;
    for (; i >= shifted_end; i -= 4) {
      sum -= t.coefs[i] * x[t.rows[i]] + t.coefs[i - 1] * x[t.rows[i - 1]] +
             t.coefs[i - 2] * x[t.rows[i - 2]] + t.coefs[i - 3] * x[t.rows[i - 3]];
    }
    if (i >= i_end) {
      sum -= t.coefs[i] * x[t.rows[i]];
      if (i >= i_end + 1) {
        sum -= t.coefs[i - 1] * x[t.rows[i - 1]];
        if (i >= i_end + 2) sum -= t.coefs[i - 2] * x[t.rows[i - 2]];
      }
    }
    x[row] = ones ? sum : sum / t.diag[row];
    if (sum != 0.0) nz[--new_start] = row;
  }
  erase_prefix(nz, nnz, new_start);
}
// sparse.cc:1445-1492 (ComputeRowsToConsiderInSortedOrder; the ratio
// arguments are ignored upstream).
SD_INLINE void tri_rows_to_consider(const Tri& t, int32_t* nz, int* nnz, char* stored) {
  if (*nnz == 0) return;
  const int sparsity_threshold = static_cast<int>(0.025 * t.num_rows);
  const int num_ops_threshold = static_cast<int>(0.05 * t.num_rows);
  int num_ops = *nnz;
  if (num_ops > sparsity_threshold) {
    *nnz = 0;
    return;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  // A column's entries (distinct rows) on the lanes; its new rows join the
  // list in entry order (ballot prefix counts), as the sequential loop appends.
  // The next listed row's bounds and first 64 entries load while the current
  // one is expanded (when it is already listed).
  const int lane = sd_lane();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  gc_i64* tst = SD_G(const int64_t, t.starts);
  gc_i32* trows = SD_G(const int32_t, t.rows);
  int n = *nnz;
  {
    // The listed rows are expanded first, in order: if their entries alone
    // take the count past the threshold, so does the sequential loop (the
    // list is then dropped: the caller takes the dense path).
    int64_t entries = 0;
    for (int k = lane; k < n; k += 64) entries += tst[nz[k] + 1] - tst[nz[k]];
    entries = sd_wave_sum_i64(entries);
    if (num_ops + entries > num_ops_threshold) {
      *nnz = 0;
      return;
    }
  }
  for (int k = lane; k < n; k += 64) stored[nz[k]] = 1;
  sd_sync();
  int64_t pb = 0, pe = 0;
  int per = 0;
  bool have = false;
  auto fetch = [&](int k) {
    const int row = nz[k];
    pb = tst[row];
    pe = tst[row + 1];
    per = pb + lane < pe ? trows[pb + lane] : 0;
    have = true;
  };
  if (n > 0) fetch(0);
  for (int k = 0; k < n; ++k) {
    if (!have) fetch(k);
    const int64_t b = pb, e = pe;
    const int first_er = per;
    have = false;
    if (k + 1 < n) fetch(k + 1);
    for (int64_t base = b; base < e; base += 64) {
      const int64_t i = base + lane;
      bool fresh = false;
      int er = 0;
      if (i < e) {
        er = base == b ? first_er : trows[i];
        fresh = !stored[er];
      }
      const uint64_t m = __ballot(fresh);
      if (fresh) {
        nz[n + __popcll(m & below)] = er;
        stored[er] = 1;
      }
      n += __popcll(m);
    }
    num_ops += static_cast<int>(e - b);
    sd_sync();
    if (num_ops > num_ops_threshold) break;
  }
  *nnz = n;
  for (int k = lane; k < n; k += 64) stored[nz[k]] = 0;
  sd_sync();
#else
  for (int k = 0; k < *nnz; ++k) stored[nz[k]] = 1;
  for (int k = 0; k < *nnz; ++k) {
    const int row = nz[k];
    for (int64_t i = t.starts[row]; i < t.starts[row + 1]; ++i) {
      ++num_ops;
      const int er = t.rows[i];
      if (!stored[er]) {
        nz[(*nnz)++] = er;
        stored[er] = 1;
      }
    }
    if (num_ops > num_ops_threshold) break;
  }
  for (int k = 0; k < *nnz; ++k) stored[nz[k]] = 0;
#endif
  if (num_ops > num_ops_threshold) {
    *nnz = 0;
  } else {
    sort_distinct(nz, *nnz, t.num_rows, stored);
  }
}
SD_INLINE int64_t tri_num_entries(const Tri& t) {
  return static_cast<int64_t>(t.num_cols) + t.ncoefs;
}

// ---- LuFactorization (lu_factorization.cc:200-454) ----
// lp_utils.h:240-277. `values` and the zero scratchpad swap buffers.
SD_INLINE void permute_with_scratchpad(Lp& s, const int32_t* perm, Vec& io) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (sd_is_lds(io.values)) {
    // The working vector stays in LDS: its values go through the (all-zero)
    // global scratchpad and come back permuted; the scratchpad ends zero.
    l_f64* w = SD_L(f64, io.values);
    g_f64* z = SD_G(f64, s.zero_scratch);
    gc_i32* pg = SD_G(const int32_t, perm);
    const int size = io.size;
    for (int i = sd_lane(); i < size; i += 64) {
      z[i] = w[i];
      w[i] = 0.0;
    }
    sd_sync();
    for (int i0 = sd_lane(); i0 < size; i0 += 512) {
      f64 v[8];
      int p[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 64 * u;
        v[u] = i < size ? z[i] : 0.0;
        p[u] = i < size ? pg[i] : 0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 64 * u;
        if (v[u] != 0.0) {
          w[p[u]] = v[u];  // a permutation: distinct targets
          z[i] = 0.0;
        }
      }
    }
    sd_sync();
    return;
  }
#endif
  f64* old = io.values;
  io.values = s.zero_scratch;
  s.zero_scratch = old;
  const int size = io.size;
  sd_fill<f64>(io.values, size, 0.0);  // resize(size, 0.0) of an all-zero buffer
#if defined(__HIP_DEVICE_COMPILE__)
  {
    gc_f64* src = SD_G(const f64, s.zero_scratch);
    gc_i32* pg = SD_G(const int32_t, perm);
    g_f64* dst = SD_G(f64, io.values);
    // Eight chunks at a time, every load before any store.
    for (int i0 = sd_lane(); i0 < size; i0 += 512) {
      f64 v[8];
      int p[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 64 * u;
        v[u] = i < size ? src[i] : 0.0;
        p[u] = i < size ? pg[i] : 0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (v[u] != 0.0) dst[p[u]] = v[u];  // a permutation: distinct targets
      }
    }
  }
#else
  for (int i = sd_lane(); i < size; i += sd_lanes()) {
    const f64 v = s.zero_scratch[i];
    if (v != 0.0) io.values[perm[i]] = v;  // a permutation: distinct targets
  }
#endif
  sd_sync();
  sd_fill<f64>(s.zero_scratch, size, 0.0);
}
SD_INLINE void permute_with_known_nz(Lp& s, const int32_t* perm, Vec& io) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (sd_is_lds(io.values)) {
    // In LDS: every listed value is read (into the global scratchpad, at its
    // position) and cleared before any is written at its permuted position.
    l_f64* w = SD_L(f64, io.values);
    g_f64* z = SD_G(f64, s.zero_scratch);
    gc_i32* pg = SD_G(const int32_t, perm);
    __attribute__((address_space(1))) int32_t* nz = SD_G(int32_t, io.nz);
    const int n = io.nnz;
    for (int k = sd_lane(); k < n; k += 64) {
      const int ref = nz[k];
      z[ref] = w[ref];
      w[ref] = 0.0;
    }
    sd_sync();
    for (int k0 = sd_lane(); k0 < n; k0 += 256) {
      int ref[4], p[4];
      f64 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) ref[u] = k0 + 64 * u < n ? nz[k0 + 64 * u] : -1;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (ref[u] >= 0) {
          v[u] = z[ref[u]];
          p[u] = pg[ref[u]];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (ref[u] >= 0) {
          z[ref[u]] = 0.0;
          w[p[u]] = v[u];
          nz[k0 + 64 * u] = p[u];
        }
      }
    }
    sd_sync();
    return;
  }
#endif
  f64* old = io.values;
  io.values = s.zero_scratch;
  s.zero_scratch = old;
#if defined(__HIP_DEVICE_COMPILE__)
  {
    g_f64* zs = SD_G(f64, s.zero_scratch);
    gc_i32* pg = SD_G(const int32_t, perm);
    g_f64* dst = SD_G(f64, io.values);
    __attribute__((address_space(1))) int32_t* nz = SD_G(int32_t, io.nz);
    const int n = io.nnz;
    // Four chunks at a time, every load before any store (distinct positions).
    for (int k0 = sd_lane(); k0 < n; k0 += 256) {
      int ref[4], p[4];
      f64 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) ref[u] = k0 + 64 * u < n ? nz[k0 + 64 * u] : -1;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (ref[u] >= 0) {
          v[u] = zs[ref[u]];
          p[u] = pg[ref[u]];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (ref[u] >= 0) {
          zs[ref[u]] = 0.0;
          dst[p[u]] = v[u];
          nz[k0 + 64 * u] = p[u];
        }
      }
    }
  }
#else
  for (int k = sd_lane(); k < io.nnz; k += sd_lanes()) {  // distinct positions
    const int ref = io.nz[k];
    const f64 v = s.zero_scratch[ref];
    s.zero_scratch[ref] = 0.0;
    const int p = perm[ref];
    io.values[p] = v;
    io.nz[k] = p;
  }
#endif
  sd_sync();
}
SD_INLINE void lu_right_solve_l_permuted_input(Lp& s, Vec& x) {
  if (s.is_identity) return;
  { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.lower, x.nz, &x.nnz, s.stored); }
  if (x.nnz == 0) {
    {
      SdSubTimer t_(&s.phase_ticks[9]);
      tri_lower_solve_from(s.lower, 0, x.values);
    }
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[17]); tri_hyper_solve(s.lower, x.values, x.nz, &x.nnz); }
  }
}
// RightSolveLInternal (lu_factorization.cc:214-243); the rhs is a matrix
// column (rows/coefs/n) or a scattered vector's list.
SD_INLINE void lu_right_solve_l_internal(Lp& s, const int32_t* brows, const f64* bcoefs,
                                          const f64* bvalues, int bn, Vec& x) {
  int first = x.size;
  const int limit = s.lower.first_non_identity;
  const int base = x.nnz;
  for (int k = sd_lane(); k < bn; k += sd_lanes()) {  // distinct rows
    const int r = brows[k];
    const int permuted_row = s.row_perm[r];
    x.values[permuted_row] = bcoefs != nullptr ? bcoefs[k] : bvalues[r];
    x.nz[base + k] = permuted_row;
    const int col = permuted_row;
    if (col < limit || s.lower.starts[col + 1] == s.lower.starts[col]) continue;
    first = first < col ? first : col;
  }
  first = sd_wave_min_int(first);
  x.nnz = base + bn;
  sd_sync();
  { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.lower, x.nz, &x.nnz, s.stored); }
  x.sorted = 1;
  if (x.nnz == 0) {
    {
      SdSubTimer t_(&s.phase_ticks[9]);
      tri_lower_solve_from(s.lower, first, x.values);
    }
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[17]); tri_hyper_solve(s.lower, x.values, x.nz, &x.nnz); }
  }
}
SD_INLINE void lu_right_solve_l_for_column(Lp& s, int col, Vec& x) {
  x.nnz = 0;
  const int64_t b = s.A.starts[col], e = s.A.starts[col + 1];
  if (s.is_identity) {
    for (int64_t i = b; i < e; ++i) {
      x.values[s.A.rows[i]] = s.A.coefs[i];
      x.nz[x.nnz++] = s.A.rows[i];
    }
    return;
  }
  lu_right_solve_l_internal(s, s.A.rows + b, s.A.coefs + b, nullptr, static_cast<int>(e - b), x);
}
SD_INLINE void lu_right_solve_l_with_nz(Lp& s, Vec& x) {
  if (s.is_identity) return;
  if (x.nnz == 0) {
    { SdSubTimer t_x_(&s.phase_ticks[22]); permute_with_scratchpad(s, s.row_perm, x); }
    {
      SdSubTimer t_(&s.phase_ticks[9]);
      tri_lower_solve_from(s.lower, 0, x.values);
    }
    return;
  }
  { SdSubTimer t_x_(&s.phase_ticks[22]); permute_with_known_nz(s, s.row_perm, x); }
  { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.lower, x.nz, &x.nnz, s.stored); }
  x.sorted = 1;
  if (x.nnz == 0) {
    {
      SdSubTimer t_(&s.phase_ticks[9]);
      tri_lower_solve_from(s.lower, 0, x.values);
    }
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[17]); tri_hyper_solve(s.lower, x.values, x.nz, &x.nnz); }
  }
}
SD_INLINE void lu_right_solve_l_for_scattered(Lp& s, const Vec& b, Vec& x) {
  x.nnz = 0;
  if (s.is_identity) {
    vec_copy(x, b);
    return;
  }
  if (b.nnz == 0) {
    vec_copy(x, b);
    lu_right_solve_l_with_nz(s, x);
    return;
  }
  lu_right_solve_l_internal(s, b.nz, nullptr, b.values, b.nnz, x);
}
SD_INLINE void lu_right_solve_u_with_nz(Lp& s, Vec& x) {
  if (s.is_identity) return;
  { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.upper, x.nz, &x.nnz, s.stored); }
  x.sorted = 1;
  if (x.nnz == 0) {
    {
      SdSubTimer t_(&s.phase_ticks[10]);
      tri_transpose_lower_solve(s.tupper, x.values, s.lds, s.lds_doubles);
    }
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[17]); tri_transpose_hyper_solve_rev(s.tupper, x.values, x.nz, &x.nnz); }
  }
}
// LeftSolveLWithNonZeros (lu_factorization.cc:333-399); `before` is tau_
// (result_before_permutation) or null. Returns true when `before` was filled.
SD_INLINE bool lu_left_solve_l_with_nz(Lp& s, Vec& y, Vec* before) {
  if (s.is_identity) return false;
  { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.tlower, y.nz, &y.nnz, s.stored); }
  y.sorted = 1;
  if (y.nnz == 0) {
    {
      SdSubTimer t_(&s.phase_ticks[10]);
      tri_transpose_lower_solve(s.lower, y.values, s.lds, s.lds_doubles);
    }
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[17]); tri_transpose_hyper_solve_rev(s.lower, y.values, y.nz, &y.nnz); }
  }
  if (before == nullptr) {
    if (y.nnz == 0) {
      { SdSubTimer t_x_(&s.phase_ticks[22]); permute_with_scratchpad(s, s.inv_row_perm, y); }
    } else {
      { SdSubTimer t_x_(&s.phase_ticks[22]); permute_with_known_nz(s, s.inv_row_perm, y); }
    }
    return false;
  }
  vec_clear_and_resize(*before, y.size);
  {  // x->swap(result_before_permutation->values)
    f64* t = y.values;
    y.values = before->values;
    before->values = t;
    const int sz = y.size;
    y.size = before->size;
    before->size = sz;
  }
  if (y.nnz == 0) {
    for (int row = sd_lane(); row < s.m; row += sd_lanes()) {
      const f64 value = before->values[row];
      if (value != 0.0) y.values[s.inv_row_perm[row]] = value;
    }
    sd_sync();
  } else {
    {  // nz->swap(result_before_permutation->non_zeros)
      int32_t* t = y.nz;
      y.nz = before->nz;
      before->nz = t;
      const int n = y.nnz;
      y.nnz = before->nnz;
      before->nnz = n;
    }
    // nz is the cleared list of `before` (vec_clear_and_resize)
    for (int k = sd_lane(); k < before->nnz; k += sd_lanes()) {  // distinct rows
      const int row = before->nz[k];
      const f64 value = before->values[row];
      const int permuted_row = s.inv_row_perm[row];
      y.values[permuted_row] = value;
      y.nz[k] = permuted_row;
    }
    sd_sync();
    y.nnz = before->nnz;
    y.sorted = 0;
  }
  return true;
}
// LeftSolveUForUnitRow (lu_factorization.cc:405-436)
SD_INLINE int lu_left_solve_u_unit_row(Lp& s, int col, Vec& y) {
  if (s.is_identity) {
    y.values[col] = 1.0;
    y.nz[y.nnz++] = col;
    return col;
  }
  const int pc = s.col_perm_empty ? col : s.col_perm[col];
  y.values[pc] = 1.0;
  y.nz[y.nnz++] = pc;
  if (s.tupper.starts[pc + 1] == s.tupper.starts[pc]) {
    y.values[pc] /= s.tupper.diag[pc];
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.tupper, y.nz, &y.nnz, s.stored); }
    y.sorted = 1;
    if (y.nnz == 0) {
      {
        SdSubTimer t_(&s.phase_ticks[9]);
        tri_lower_solve_from(s.tupper, pc, y.values);
      }
    } else {
      { SdSubTimer t_x_(&s.phase_ticks[17]); tri_hyper_solve(s.tupper, y.values, y.nz, &y.nnz); }
    }
  }
  return pc;
}
// GetColumnOfU (lu_factorization.cc:438-447) with SparseVector::CleanUp.
SD_INLINE void lu_column_of_u(Lp& s, int col) {
  s.n_col_u = 0;
  if (s.is_identity) {
    s.col_u_rows[0] = col;
    s.col_u_coefs[0] = 1.0;
    s.n_col_u = 1;
    return;
  }
  const int c = s.col_perm_empty ? col : s.col_perm[col];
  const Tri& u = s.upper;
  int n = 0;
  for (int64_t i = u.starts[c]; i < u.starts[c + 1]; ++i) {
    s.col_u_rows[n] = u.rows[i];
    s.col_u_coefs[n] = u.coefs[i];
    ++n;
  }
  s.col_u_rows[n] = c;
  s.col_u_coefs[n] = u.diag[c];
  ++n;
  // stable insertion sort by row
  for (int i = 1; i < n; ++i) {
    const int32_t r = s.col_u_rows[i];
    const f64 v = s.col_u_coefs[i];
    int j = i - 1;
    while (j >= 0 && s.col_u_rows[j] > r) {
      s.col_u_rows[j + 1] = s.col_u_rows[j];
      s.col_u_coefs[j + 1] = s.col_u_coefs[j];
      --j;
    }
    s.col_u_rows[j + 1] = r;
    s.col_u_coefs[j + 1] = v;
  }
  int out = 0;
  for (int i = 0; i < n; ++i) {
    if (s.col_u_coefs[i] == 0.0) continue;
    if (i + 1 == n || s.col_u_rows[i] != s.col_u_rows[i + 1]) {
      s.col_u_rows[out] = s.col_u_rows[i];
      s.col_u_coefs[out] = s.col_u_coefs[i];
      ++out;
    }
  }
  s.n_col_u = out;
}
SD_INLINE int64_t lu_number_of_entries(const Lp& s) {
  return s.is_identity ? 0 : tri_num_entries(s.lower) + tri_num_entries(s.upper);
}

// ---- RankOneUpdateFactorization (rank_one_update.h:30-246) ----
#if defined(__HIP_DEVICE_COMPILE__)
// ColumnScalarProduct as sd_ordered_dot, with the column's first 256
// entries already in registers (pr/pc: entry base + 64u + lane).
template <typename XP>
__device__ inline f64 sd_ordered_dot_pf(gc_i32* rows, gc_f64* coefs, int64_t b, int64_t e, XP x,
                                        l_f64* red, const int* pr, const f64* pc) {
  const int lane = sd_lane();
  const int64_t len = e - b;
  const int64_t body = len & ~int64_t{3};
  f64 acc = 0.0;
  f64 tail[3] = {0.0, 0.0, 0.0};
  for (int64_t base = 0; base < len; base += 256) {
    const int64_t n = len - base < 256 ? len - base : 256;
    f64 p[4];
    if (base == 0) {
#pragma unroll
      for (int u = 0; u < 4; ++u) p[u] = u * 64 + lane < n ? pc[u] * x[pr[u]] : 0.0;
    } else {
      int r[4];
      f64 c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t k = b + base + u * 64 + lane;
        const bool in = u * 64 + lane < n;
        r[u] = in ? rows[k] : 0;
        c[u] = in ? coefs[k] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) p[u] = u * 64 + lane < n ? c[u] * x[r[u]] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) red[u * 64 + lane] = p[u];
    sd_sync();
    const int64_t nb = body - base < n ? (body - base > 0 ? body - base : 0) : n;
    if (lane < 4) acc = sd_chain_sum(red, lane, static_cast<int>(nb >> 2), acc);
    for (int64_t t = body > base ? body : base; t < base + n; ++t) tail[t - body] = red[t - base];
    sd_sync();
  }
  if (lane < 4) red[lane] = acc;
  sd_sync();
  f64 result = red[0] + red[1] + red[2] + red[3];
  sd_sync();
  for (int64_t t = body; t < len; ++t) result += tail[t - body];
  return result;
}
// The first entries of step k's columns (k's bounds staged in meta).
__device__ inline void r1_fetch(l_i64* meta, int k, gc_i32* rows, gc_f64* coefs, int* pr, f64* pc,
                                int* ar, f64* ac) {
  const int lane = sd_lane();
  const int64_t db = meta[4 * k], de = meta[4 * k + 1];
  const int64_t ab = meta[4 * k + 2], ae = meta[4 * k + 3];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t i = db + 64 * u + lane;
    pr[u] = i < de ? rows[i] : 0;
    pc[u] = i < de ? coefs[i] : 0.0;
  }
  *ar = ab + lane < ae ? rows[ab + lane] : 0;
  *ac = ab + lane < ae ? coefs[ab + lane] : 0.0;
}
// Steps k = 0 .. count-1 of a rank-one solve (RankOneUpdateFactorization::
// RightSolveWithNonZeros / LeftSolveWithNonZeros, rank_one_update.h:196-246):
// update i = first + k (right) or first - k (left), x += mult * add_col with
// mult = -(dot_col . x) / mu (right: dot v_i, add u_i; left: dot u_i, add
// v_i). While the vector is sparse (dense == false) the add is Glop's
// scattered add (new positions join the list in entry order, the mask marks
// them) and the 5% density test follows every step; once dense, plain adds
// for the remaining steps. A 64-step chunk's column bounds and mu are staged
// in LDS; the next step's first 256 dot entries and 64 add entries are
// loaded while the current step computes.
template <typename XP>
__device__ inline void r1_run_dev(Lp& s, Vec& d, XP x, int first, int count, bool left,
                                  bool dense) {
  const Store& st = s.storage;
  const int lane = sd_lane();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  SdScratch* sc = reinterpret_cast<SdScratch*>(s.lds_scratch);
  l_f64* red = SD_L(f64, sc->red);
  l_i64* meta = SD_L(int64_t, sc->meta);
  l_f64* mus = SD_L(f64, sc->mu);
  gc_i64* starts = SD_G(const int64_t, st.starts);
  gc_i32* rows = SD_G(const int32_t, st.rows);
  gc_f64* coefs = SD_G(const f64, st.coefs);
  gc_i32* ru = SD_G(const int32_t, s.r1_u);
  gc_i32* rv = SD_G(const int32_t, s.r1_v);
  gc_f64* rmu = SD_G(const f64, s.r1_mu);
  for (int c0 = 0; c0 < count; c0 += 64) {
    if (c0 + lane < count) {
      const int i = left ? first - (c0 + lane) : first + (c0 + lane);
      const int dcol = left ? ru[i] : rv[i];
      const int acol = left ? rv[i] : ru[i];
      meta[4 * lane + 0] = starts[dcol];
      meta[4 * lane + 1] = starts[dcol + 1];
      meta[4 * lane + 2] = starts[acol];
      meta[4 * lane + 3] = starts[acol + 1];
      mus[lane] = rmu[i];
    }
    sd_sync();
    const int steps = count - c0 < 64 ? count - c0 : 64;
    int pr[4], ar;
    f64 pc[4], ac;
    r1_fetch(meta, 0, rows, coefs, pr, pc, &ar, &ac);
    for (int k = 0; k < steps; ++k) {
      const int64_t db = meta[4 * k], de = meta[4 * k + 1];
      const int64_t ab = meta[4 * k + 2], ae = meta[4 * k + 3];
      const f64 mu = mus[k];
      int nr[4] = {0, 0, 0, 0}, nar = 0;
      f64 nc[4] = {0.0, 0.0, 0.0, 0.0}, nac = 0.0;
      if (k + 1 < steps) r1_fetch(meta, k + 1, rows, coefs, nr, nc, &nar, &nac);
      const f64 dot = sd_ordered_dot_pf(rows, coefs, db, de, x, red, pr, pc);
      const f64 mult = -dot / mu;
      if (mult != 0.0) {
        if (dense) {  // col_add_dense: a column's rows are distinct
          if (ab + lane < ae) x[ar] += mult * ac;
          for (int64_t e0 = ab + 64 + lane; e0 < ae; e0 += 256) {
            int r[4];
            f64 c[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int64_t e = e0 + 64 * u;
              r[u] = e < ae ? rows[e] : 0;
              c[u] = e < ae ? coefs[e] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (e0 + 64 * u < ae) x[r[u]] += mult * c[u];
            }
          }
        } else {  // col_add_scattered (sparse.h:403-413)
          int nnz = d.nnz;
          for (int64_t base = ab; base < ae; base += 64) {
            const int64_t i = base + lane;
            bool fresh = false;
            int row = 0;
            if (i < ae) {
              row = base == ab ? ar : rows[i];
              const f64 value = mult * (base == ab ? ac : coefs[i]);
              x[row] += value;
              fresh = !d.mask[row] && value != 0.0;
              if (fresh) d.mask[row] = 1;
            }
            const uint64_t fresh_mask = __ballot(fresh);
            if (fresh) d.nz[nnz + __popcll(fresh_mask & below)] = row;
            nnz += __popcll(fresh_mask);
          }
          sd_sync();
          if (nnz != d.nnz) d.sorted = 0;
          d.nnz = nnz;
        }
      }
      if (!dense) dense = vec_dense(d, 0.05);
      sd_sync();
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        pr[u] = nr[u];
        pc[u] = nc[u];
      }
      ar = nar;
      ac = nac;
    }
  }
}
SD_INLINE void r1_run(Lp& s, Vec& d, int first, int count, bool left, bool dense) {
  if (count <= 0) return;
  if (sd_is_lds(d.values)) {
    r1_run_dev(s, d, SD_L(f64, d.values), first, count, left, dense);
  } else {
    r1_run_dev(s, d, SD_G(f64, d.values), first, count, left, dense);
  }
}
#else
SD_INLINE void r1_dense_steps(Lp& s, f64* x, int first, int count, bool left) {
  for (int k = 0; k < count; ++k) {
    const int i = left ? first - k : first + k;
    const int dcol = left ? s.r1_u[i] : s.r1_v[i];
    const int acol = left ? s.r1_v[i] : s.r1_u[i];
    const f64 mult = -col_dot(s.storage, dcol, x) / s.r1_mu[i];
    col_add_dense(s.storage, acol, mult, x);
  }
}
#endif
#if defined(__HIP_DEVICE_COMPILE__)
SD_INLINE void r1_right_solve_nz(Lp& s, Vec& d) {
  SdSubTimer t_(&s.phase_ticks[11]);
  if (d.nnz == 0) {
    r1_run(s, d, 0, s.r1_count, false, true);
  } else {
    vec_repopulate_mask(d);
    r1_run(s, d, 0, s.r1_count, false, vec_dense(d, 0.05));
    vec_clear_mask(d);
    vec_clear_nz_if_too_dense(d, 0.05);
  }
  s.r1_dtime += dt_ops(s.r1_num_entries);
}
SD_INLINE void r1_left_solve_nz(Lp& s, Vec& y) {
  SdSubTimer t_(&s.phase_ticks[11]);
  if (y.nnz == 0) {
    r1_run(s, y, s.r1_count - 1, s.r1_count, true, true);
  } else {
    vec_repopulate_mask(y);
    r1_run(s, y, s.r1_count - 1, s.r1_count, true, vec_dense(y, 0.05));
    vec_clear_mask(y);
    vec_clear_nz_if_too_dense(y, 0.05);
  }
  s.r1_dtime += dt_ops(s.r1_num_entries);
}
#else
SD_INLINE void r1_right_solve_dense(Lp& s, f64* x) {
  r1_dense_steps(s, x, 0, s.r1_count, false);
  s.r1_dtime += dt_ops(s.r1_num_entries);
}
SD_INLINE void r1_right_solve_nz(Lp& s, Vec& d) {
  SdSubTimer t_(&s.phase_ticks[11]);
  if (d.nnz == 0) {
    r1_right_solve_dense(s, d.values);
    return;
  }
  vec_repopulate_mask(d);
  bool use_dense = vec_dense(d, 0.05);
  for (int i = 0; i < s.r1_count; ++i) {
    if (use_dense) {  // stays dense for the remaining updates
      r1_dense_steps(s, d.values, i, s.r1_count - i, false);
      break;
    }
    const f64 mult = -col_dot_par(s.storage, s.r1_v[i], d.values, s.lds_scratch) / s.r1_mu[i];
    if (mult != 0.0) col_add_scattered(s.storage, s.r1_u[i], mult, d);
    use_dense = vec_dense(d, 0.05);
  }
  vec_clear_mask(d);
  vec_clear_nz_if_too_dense(d, 0.05);
  s.r1_dtime += dt_ops(s.r1_num_entries);
}
SD_INLINE void r1_left_solve_dense(Lp& s, f64* y) {
  r1_dense_steps(s, y, s.r1_count - 1, s.r1_count, true);
  s.r1_dtime += dt_ops(s.r1_num_entries);
}
SD_INLINE void r1_left_solve_nz(Lp& s, Vec& y) {
  SdSubTimer t_(&s.phase_ticks[11]);
  if (y.nnz == 0) {
    r1_left_solve_dense(s, y.values);
    return;
  }
  vec_repopulate_mask(y);
  bool use_dense = vec_dense(y, 0.05);
  for (int i = s.r1_count - 1; i >= 0; --i) {
    if (use_dense) {  // stays dense for the remaining updates
      r1_dense_steps(s, y.values, i, i + 1, true);
      break;
    }
    const f64 mult = -col_dot_par(s.storage, s.r1_u[i], y.values, s.lds_scratch) / s.r1_mu[i];
    if (mult != 0.0) col_add_scattered(s.storage, s.r1_v[i], mult, y);
    use_dense = vec_dense(y, 0.05);
  }
  vec_clear_mask(y);
  vec_clear_nz_if_too_dense(y, 0.05);
  s.r1_dtime += dt_ops(s.r1_num_entries);
}

#endif
// The working vector of one BasisFactorization solve in LDS (device, when
// m fits the workgroup's staging area): the vector's values are moved into
// the LDS buffer for the solve (copy_in) and back into its global buffer at
// the end, so that every step of the solve (L, rank-one updates, U, their
// permutes and level sweeps) reads and writes LDS. The solve may hand the
// buffer to tau (LeftSolveLWithNonZeros' swap) or to the zero scratchpad (a
// permute's swap); whoever holds it at the end gets the saved global buffer
// with the same contents. The LDS buffer is all zero between solves.
struct SdLdsVec {
  Lp& s;
  Vec& v;
  f64* saved = nullptr;
  SD_HD SdLdsVec(Lp& lp, Vec& vec, bool copy_in) : s(lp), v(vec) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (s.lds == nullptr || s.lds_busy || s.m > s.lds_doubles) return;
    s.lds_busy = 1;
    saved = v.values;
    l_f64* w = SD_L(f64, s.lds);
    if (copy_in) {
      gc_f64* g = SD_G(const f64, saved);
#pragma unroll 8
      for (int i = sd_lane(); i < s.m; i += 64) w[i] = g[i];
      sd_sync();
    }
    v.values = s.lds;
#else
    (void)copy_in;
#endif
  }
  SD_HD ~SdLdsVec() {
#if defined(__HIP_DEVICE_COMPILE__)
    if (saved == nullptr) return;
    f64* w = s.lds;
    l_f64* wl = SD_L(f64, w);
    g_f64* g = SD_G(f64, saved);
    const int m = s.m;
    if (s.zero_scratch == w) {  // the buffer is zero (a permute cleared it)
      for (int i = sd_lane(); i < m; i += 64) g[i] = 0.0;
      s.zero_scratch = saved;
    } else {
      f64** owner = v.values == w ? &v.values : &s.tau.values;
      for (int i = sd_lane(); i < m; i += 64) {
        g[i] = wl[i];
        wl[i] = 0.0;
      }
      *owner = saved;
    }
    sd_sync();
    s.lds_busy = 0;
#endif
  }
};

// ---- EtaFactorization (basis_representation.cc:25-176, PFI path) ----
// The loops are sequential in Glop's order (a running sum, or scatters
// whose order fixes nothing but are kept), on every lane of the wave.
SD_INLINE void eta_left_solve_one(const Lp& s, int k, f64* y) {
  const int c = s.eta_col[k];
  f64 y_value = y[c];
  const int64_t b = s.eta_sp_starts[k], e = s.eta_sp_starts[k + 1];
  if (b != e) {
    for (int64_t i = b; i < e; ++i) y_value -= y[s.eta_sp_rows[i]] * s.eta_sp_coefs[i];
  } else {
    const f64* coeff = s.eta_dense + static_cast<int64_t>(k) * s.m;
    for (int row = 0; row < s.m; ++row) y_value -= y[row] * coeff[row];
  }
  sd_sync();
  y[c] = y_value / s.eta_piv[k];
  sd_sync();
}
SD_INLINE void eta_right_solve_one(const Lp& s, int k, f64* d) {
  const int c = s.eta_col[k];
  if (d[c] == 0.0) return;
  const f64 coeff = d[c] / s.eta_piv[k];
  const int64_t b = s.eta_sp_starts[k], e = s.eta_sp_starts[k + 1];
  sd_sync();
  // The rows of one eta are distinct (and differ from its column): the
  // lanes split them.
  if (b != e) {
    for (int64_t i = b + sd_lane(); i < e; i += sd_lanes()) {
      d[s.eta_sp_rows[i]] -= s.eta_sp_coefs[i] * coeff;
    }
  } else {
    const f64* ec = s.eta_dense + static_cast<int64_t>(k) * s.m;
    for (int row = sd_lane(); row < s.m; row += sd_lanes()) d[row] -= ec[row] * coeff;
  }
  sd_sync();
  d[c] = coeff;
  sd_sync();
}
SD_INLINE void eta_left_solve(const Lp& s, f64* y) {
  for (int k = s.eta_count - 1; k >= 0; --k) eta_left_solve_one(s, k, y);
}
SD_INLINE void eta_right_solve(const Lp& s, f64* d) {
  for (int k = 0; k < s.eta_count; ++k) eta_right_solve_one(s, k, d);
}
// SparseLeftSolve: y's positions in `pos` (the eta column joins the list).
SD_INLINE void eta_sparse_left_solve(const Lp& s, f64* y, int32_t* pos, int* npos) {
  for (int k = s.eta_count - 1; k >= 0; --k) {
    const int c = s.eta_col[k];
    const f64* coeff = s.eta_dense + static_cast<int64_t>(k) * s.m;
    f64 y_value = y[c];
    bool in_pos = false;
    const int size = *npos;
    for (int i = 0; i < size; ++i) {
      const int col = pos[i];
      if (col == c) {
        in_pos = true;
        continue;
      }
      y_value -= y[col] * coeff[col];
    }
    sd_sync();
    y[c] = y_value / s.eta_piv[k];
    if (!in_pos) pos[(*npos)++] = c;
    sd_sync();
  }
}
// EtaFactorization::Update: EtaMatrix(leaving_row, direction).
SD_INLINE void eta_update(Lp& s, int leaving_row, const Vec& dir) {
  const int k = s.eta_count;
  f64* ec = s.eta_dense + static_cast<int64_t>(k) * s.m;
  for (int row = sd_lane(); row < s.m; row += sd_lanes()) ec[row] = dir.values[row];
  sd_sync();
  s.eta_col[k] = leaving_row;
  s.eta_piv[k] = dir.values[leaving_row];
  ec[leaving_row] = 0.0;
  int64_t e = s.eta_sp_starts[k];
  if (static_cast<f64>(dir.nnz) < 0.5 * static_cast<f64>(s.m)) {
    for (int i = 0; i < dir.nnz; ++i) {
      const int row = dir.nz[i];
      if (row == leaving_row) continue;
      s.eta_sp_rows[e] = row;
      s.eta_sp_coefs[e] = ec[row];
      ++e;
    }
  }
  s.eta_sp_starts[k + 1] = e;
  s.eta_count = k + 1;
  sd_sync();
}
// LuFactorization::RightSolve / LeftSolve on dense vectors
// (lu_factorization.cc:135-156): permute into the scratchpad, the two
// triangular loops, permute back.
SD_INLINE void lu_right_solve_dense(Lp& s, f64* x) {
  if (s.is_identity) return;
  f64* t = s.pfi_scratch;
  for (int i = sd_lane(); i < s.m; i += sd_lanes()) t[s.row_perm[i]] = x[i];
  sd_sync();
  tri_lower_solve_from(s.lower, 0, t);
  sd_sync();
  tri_upper_solve(s.upper, t);
  sd_sync();
  for (int i = sd_lane(); i < s.m; i += sd_lanes()) {
    x[s.col_perm_empty ? i : s.inv_col_perm[i]] = t[i];
  }
  sd_sync();
}
SD_INLINE void lu_left_solve_dense(Lp& s, f64* y) {
  if (s.is_identity) return;
  f64* t = s.pfi_scratch;
  for (int i = sd_lane(); i < s.m; i += sd_lanes()) {
    t[i] = y[s.col_perm_empty ? i : s.inv_col_perm[i]];
  }
  sd_sync();
  tri_transpose_upper_solve(s.upper, t);
  sd_sync();
  tri_transpose_lower_solve(s.lower, t);
  sd_sync();
  for (int i = sd_lane(); i < s.m; i += sd_lanes()) y[i] = t[s.row_perm[i]];
  sd_sync();
}

// ---- BasisFactorization (basis_representation.cc:304-624, MPF path) ----
SD_INLINE void bf_bump(Lp& s, int64_t num_entries) {
  if (s.m == 0) return;
  const f64 density = static_cast<f64>(num_entries) / static_cast<f64>(s.m);
  s.bf_dtime += density * dt_ops(lu_number_of_entries(s)) + dt_ops(s.r1_num_entries);
}
SD_INLINE void bf_right_solve(Lp& s, Vec& d) {
  if (!s.mpf) {  // RightSolve, PFI (basis_representation.cc:358-372)
    d.nnz = 0;
    lu_right_solve_dense(s, d.values);
    eta_right_solve(s, d.values);
    bf_bump(s, vec_nnz_estimate(d));
    return;
  }
  SdLdsVec lds_(s, d, true);
  lu_right_solve_l_with_nz(s, d);
  r1_right_solve_nz(s, d);
  lu_right_solve_u_with_nz(s, d);
  vec_sort_if_needed(d, s.stored);
  bf_bump(s, vec_nnz_estimate(d));
}
// LeftSolveUWithNonZeros (lu_factorization.cc:298-312)
SD_INLINE void lu_left_solve_u_with_nz(Lp& s, Vec& y) {
  if (s.is_identity) return;
  { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.tupper, y.nz, &y.nnz, s.stored); }
  y.sorted = 1;
  if (y.nnz == 0) {
    {
      SdSubTimer t_(&s.phase_ticks[10]);
      tri_transpose_upper_solve(s.upper, y.values, s.lds, s.lds_doubles);
    }
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[17]); tri_transpose_hyper_solve(s.upper, y.values, y.nz, &y.nnz); }
  }
}
// BasisFactorization::LeftSolve (basis_representation.cc:342-356, MPF)
SD_INLINE void bf_left_solve(Lp& s, Vec& y) {
  if (!s.mpf) {  // LeftSolve, PFI (:342-356)
    y.nnz = 0;
    eta_left_solve(s, y.values);
    lu_left_solve_dense(s, y.values);
    bf_bump(s, vec_nnz_estimate(y));
    return;
  }
  SdLdsVec lds_(s, y, true);
  lu_left_solve_u_with_nz(s, y);
  r1_left_solve_nz(s, y);
  lu_left_solve_l_with_nz(s, y, nullptr);
  vec_sort_if_needed(y, s.stored);
  bf_bump(s, vec_nnz_estimate(y));
}
// LuFactorization::DualEdgeSquaredNorm (lu_factorization.cc:158-186) with
// BasisFactorization's bump (basis_representation.cc).
SD_INLINE f64 bf_dual_edge_squared_norm(Lp& s, int row) {
  bf_bump(s, 1);
  if (s.is_identity) return 1.0;
  const int pr = s.col_perm_empty ? row : s.col_perm[row];
  int32_t* nz = s.dp.equiv;  // non_zero_rows_ scratch
  int nnz = 0;
  f64* z = s.zero_scratch;
  z[pr] = 1.0;
  nz[nnz++] = pr;
  { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.tupper, nz, &nnz, s.stored); }
  if (nnz == 0) {
    {
      SdSubTimer t_(&s.phase_ticks[9]);
      tri_lower_solve_from(s.tupper, pr, z);
    }
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[17]); tri_hyper_solve(s.tupper, z, nz, &nnz); }
    { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.tlower, nz, &nnz, s.stored); }
  }
  if (nnz == 0) {
    {
      SdSubTimer t_(&s.phase_ticks[9]);
      tri_upper_solve(s.tlower, z);
    }
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[17]); tri_hyper_solve_rev(s.tlower, z, nz, &nnz); }
  }
  f64 sum = 0.0;
  if (nnz == 0) {
    sum = dense_squared_norm(z, s.m);
    for (int i = 0; i < s.m; ++i) z[i] = 0.0;
  } else {
    for (int k = 0; k < nnz; ++k) {
      sum += sq(z[nz[k]]);
      z[nz[k]] = 0.0;
    }
  }
  return sum;
}
SD_INLINE const f64* bf_right_solve_for_tau(Lp& s, const Vec& a) {
  SdSubTimer t_sub_(&s.phase_ticks[30]);
  if (!s.mpf) {  // RightSolveForTau, PFI (:374-398)
    s.tau.nnz = 0;
    for (int i = sd_lane(); i < a.size; i += sd_lanes()) s.tau.values[i] = a.values[i];
    sd_sync();
    s.tau.size = a.size;
    lu_right_solve_dense(s, s.tau.values);
    eta_right_solve(s, s.tau.values);
    s.tau_is_computed = 1;
    bf_bump(s, vec_nnz_estimate(s.tau));
    return s.tau.values;
  }
  {
  SdLdsVec lds_(s, s.tau, s.tau_can_opt != 0);
  if (s.tau_can_opt) {
    s.tau_can_opt = 0;
    lu_right_solve_l_permuted_input(s, s.tau);
  } else {
    vec_clear_and_resize(s.tau, s.m);
    lu_right_solve_l_for_scattered(s, a, s.tau);
  }
  r1_right_solve_nz(s, s.tau);
  lu_right_solve_u_with_nz(s, s.tau);
  }
  s.tau_is_computed = 1;
  bf_bump(s, vec_nnz_estimate(s.tau));
  return s.tau.values;
}
SD_INLINE void bf_left_solve_for_unit_row(Lp& s, int j, Vec& y) {
  if (!s.mpf) {  // LeftSolveForUnitRow, PFI (:400-453)
    vec_clear_and_resize(y, s.m);
    y.values[j] = 1.0;
    y.nz[y.nnz++] = j;
    eta_sparse_left_solve(s, y.values, y.nz, &y.nnz);
    lu_left_solve_dense(s, y.values);
    bf_bump(s, vec_nnz_estimate(y));
    return;
  }
  SdLdsVec lds_(s, y, false);
  vec_clear_and_resize(y, s.m);
  if (s.left_pool[j] == kInvalid) {
    const int start = lu_left_solve_u_unit_row(s, j, y);
    if (y.nnz == 0) {
      { SdSubTimer t_x_(&s.phase_ticks[18]); s.left_pool[j] = store_add_dense_prefix(s.storage, y.values, y.size, start); }
    } else {
      { SdSubTimer t_x_(&s.phase_ticks[18]); s.left_pool[j] = store_add_dense_nz(s.storage, y.values, y.size, y.nz, y.nnz); }
    }
  } else {
    store_copy_to_vec(s.storage, s.left_pool[j], y);
  }
  r1_left_solve_nz(s, y);
  if (s.tau_is_computed) {
    s.tau_can_opt = lu_left_solve_l_with_nz(s, y, &s.tau) ? 1 : 0;
  } else {
    s.tau_can_opt = 0;
    lu_left_solve_l_with_nz(s, y, nullptr);
  }
  s.tau_is_computed = 0;
  vec_sort_if_needed(y, s.stored);
  bf_bump(s, vec_nnz_estimate(y));
}
SD_INLINE void bf_right_solve_for_column(Lp& s, int col, Vec& d) {
  if (!s.mpf) {  // RightSolveForProblemColumn, PFI (:468-501)
    vec_clear_and_resize(d, s.m);
    for (int64_t i = s.A.starts[col] + sd_lane(); i < s.A.starts[col + 1]; i += sd_lanes()) {
      d.values[s.A.rows[i]] = s.A.coefs[i];
    }
    sd_sync();
    lu_right_solve_dense(s, d.values);
    eta_right_solve(s, d.values);
    bf_bump(s, vec_nnz_estimate(d));
    return;
  }
  SdLdsVec lds_(s, d, false);
  vec_clear_and_resize(d, s.m);
  lu_right_solve_l_for_column(s, col, d);
  r1_right_solve_nz(s, d);
  if (d.nnz == 0) {
    { SdSubTimer t_x_(&s.phase_ticks[18]); s.right_pool[col] = store_add_dense_prefix(s.right_storage, d.values, d.size, 0); }
  } else {
    sort_distinct(d.nz, d.nnz, d.size, s.stored);
    { SdSubTimer t_x_(&s.phase_ticks[18]); s.right_pool[col] = store_add_dense_nz(s.right_storage, d.values, d.size, d.nz, d.nnz); }
  }
  lu_right_solve_u_with_nz(s, d);
  vec_sort_if_needed(d, s.stored);
  bf_bump(s, vec_nnz_estimate(d));
}

// ---- DynamicMaximum (pricing.h:152-345) ----
// HeapLess: a.value > b.value (min-heap); libstdc++ make_heap restated.
SD_INLINE void dp_push_heap(Lp& s, DynMax& d, int hole, int top, int vi, f64 vv) {
  int parent = (hole - 1) / 2;
  while (hole > top && d.tops_val[parent] > vv) {
    d.tops_idx[hole] = d.tops_idx[parent];
    d.tops_val[hole] = d.tops_val[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  d.tops_idx[hole] = vi;
  d.tops_val[hole] = vv;
}
SD_INLINE void dp_adjust_heap(Lp& s, DynMax& d, int hole, int len, int vi, f64 vv) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (d.tops_val[second] > d.tops_val[second - 1]) second--;
    d.tops_idx[hole] = d.tops_idx[second];
    d.tops_val[hole] = d.tops_val[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    d.tops_idx[hole] = d.tops_idx[second - 1];
    d.tops_val[hole] = d.tops_val[second - 1];
    hole = second - 1;
  }
  dp_push_heap(s, d, hole, top, vi, vv);
}
SD_INLINE void dp_make_heap(Lp& s, DynMax& d) {
  const int len = d.ntops;
  if (len < 2) return;
  int parent = (len - 2) / 2;
  while (true) {
    const int vi = d.tops_idx[parent];
    const f64 vv = d.tops_val[parent];
    dp_adjust_heap(s, d, parent, len, vi, vv);
    if (parent == 0) return;
    parent--;
  }
}
SD_INLINE void dp_update_top_k(Lp& s, DynMax& d, int position, f64 value) {
  const int k = 31;
  if (d.ntops < k) {
    d.tops_idx[d.ntops] = position;
    d.tops_val[d.ntops] = value;
    ++d.ntops;
    if (d.ntops == k) {
      dp_make_heap(s, d);
      d.threshold = d.tops_val[0];
    }
    return;
  }
  if (value == d.tops_val[0]) {
    if (bernoulli(s, 0.5)) d.tops_idx[0] = position;
    return;
  }
  int i = 0;
  const int limit = k / 2;
  for (; i < limit;) {
    const int left = 2 * i + 1;
    const int right = left + 1;
    const f64 lv = d.tops_val[left];
    const f64 rv = d.tops_val[right];
    if (lv > rv) {
      if (value <= rv) break;
      d.tops_idx[i] = d.tops_idx[right];
      d.tops_val[i] = d.tops_val[right];
      i = right;
    } else {
      if (value <= lv) break;
      d.tops_idx[i] = d.tops_idx[left];
      d.tops_val[i] = d.tops_val[left];
      i = left;
    }
  }
  d.tops_idx[i] = position;
  d.tops_val[i] = value;
  d.threshold = d.tops_val[0];
}
SD_INLINE void dp_clear_and_resize(Lp& s, DynMax& d, int n) {
  d.ntops = 0;
  d.threshold = -sd_inf();
  for (int i = d.size + sd_lane(); i < n; i += sd_lanes()) d.values[i] = 0.0;
  d.size = n;
  const int words = (n + 63) / 64;
  for (int w = sd_lane(); w < words; w += sd_lanes()) d.cand[w] = 0;
  sd_sync();
}
SD_INLINE void dp_start_dense_updates(Lp& s, DynMax& d) {
  d.ntops = 0;
  d.threshold = sd_inf();
}
SD_INLINE void dp_dense_add_or_update(Lp& s, DynMax& d, int position, f64 value) {
  bit_set(d.cand, position);
  d.values[position] = value;
}
SD_INLINE void dp_add_or_update(Lp& s, DynMax& d, int position, f64 value) {
  bit_set(d.cand, position);
  d.values[position] = value;
  if (value >= d.threshold) dp_update_top_k(s, d, position, value);
}
SD_INLINE void dp_remove(Lp& s, DynMax& d, int position) { bit_clear(d.cand, position); }
SD_INLINE int dp_randomize(Lp& s, DynMax& d, int best, int n_equiv) {
  if (n_equiv == 0) return best;
  d.equiv[n_equiv++] = best;
  return d.equiv[uniform_int(s, n_equiv - 1)];
}
SD_INLINE int dp_get_maximum(Lp& s, DynMax& d) {
  SdSubTimer t_sub_(&s.phase_ticks[27]);
  f64 best_value = -sd_inf();
  int best_position = -1;
  int n_equiv = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  const int lane = sd_lane();
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  if (d.ntops != 0) {
    // The tops on the lanes (at most 31): the kept ones (still candidates
    // with an unchanged value) compacted in order; the maximum's first
    // occurrence is the best position, its later ones the equivalent
    // choices in order (the sequential loop's result).
    const int n = d.ntops;
    int idx = 0;
    f64 val = -sd_inf();
    bool kept = false;
    if (lane < n) {
      idx = d.tops_idx[lane];
      val = d.tops_val[lane];
      kept = bit_get(d.cand, idx) && d.values[idx] == val;
    }
    const uint64_t kmask = __ballot(kept);
    const int new_size = __popcll(kmask);
    sd_sync();
    if (kept) {
      const int pos = __popcll(kmask & below);
      d.tops_idx[pos] = idx;
      d.tops_val[pos] = val;
    }
    d.ntops = new_size;
    if (new_size != 0) {
      const f64 top = sd_wave_max(kept ? val : -sd_inf());
      const uint64_t emask = __ballot(kept && val == top);
      const int first = __builtin_ctzll(emask);
      best_position = __shfl(idx, first, 64);
      n_equiv = __popcll(emask) - 1;
      if (((emask >> lane) & 1) && lane != first) {
        d.equiv[__popcll(emask & below) - 1] = idx;
      }
      sd_sync();
      return dp_randomize(s, d, best_position, n_equiv);
    }
    sd_sync();
  }
  // Rescan: 64 positions at a time, candidates below the threshold at the
  // chunk's start skipped on the lanes (the threshold never decreases), the
  // others replayed in order.
  d.threshold = -sd_inf();
  for (int base = 0; base < d.size; base += 64) {
    const int position = base + lane;
    f64 value = 0.0;
    bool cand = false;
    if (position < d.size && bit_get(d.cand, position)) {
      value = d.values[position];
      cand = value >= d.threshold;
    }
    uint64_t mask = __ballot(cand);
    while (mask != 0) {
      const int l = __builtin_ctzll(mask);
      mask &= mask - 1;
      const f64 v = __shfl(value, l, 64);
      if (v < d.threshold) continue;
      dp_update_top_k(s, d, base + l, v);
      if (v >= best_value) {
        if (v == best_value) {
          d.equiv[n_equiv++] = base + l;
          continue;
        }
        n_equiv = 0;
        best_value = v;
        best_position = base + l;
      }
    }
  }
  sd_sync();
  return dp_randomize(s, d, best_position, n_equiv);
#endif
  if (d.ntops != 0) {
    // iterate over a copy of tops_ (the loop compacts in place)
    int32_t cidx[32];
    f64 cval[32];
    const int n = d.ntops;
    for (int k = 0; k < n; ++k) {
      cidx[k] = d.tops_idx[k];
      cval[k] = d.tops_val[k];
    }
    int new_size = 0;
    for (int k = 0; k < n; ++k) {
      const int idx = cidx[k];
      const f64 val = cval[k];
      if (!bit_get(d.cand, idx)) continue;
      if (d.values[idx] != val) continue;
      d.tops_idx[new_size] = idx;
      d.tops_val[new_size] = val;
      ++new_size;
      if (val >= best_value) {
        if (val == best_value) {
          d.equiv[n_equiv++] = idx;
          continue;
        }
        n_equiv = 0;
        best_value = val;
        best_position = idx;
      }
    }
    d.ntops = new_size;
    if (new_size != 0) return dp_randomize(s, d, best_position, n_equiv);
  }
  d.threshold = -sd_inf();
  const int words = (d.size + 63) / 64;
  for (int w = 0; w < words; ++w) {
    uint64_t word = d.cand[w];
    while (word) {
      const int position = w * 64 + sd_ctz(word);
      word &= word - 1;
      if (position >= d.size) break;
      const f64 value = d.values[position];
      if (value < d.threshold) continue;
      dp_update_top_k(s, d, position, value);
      if (value >= best_value) {
        if (value == best_value) {
          d.equiv[n_equiv++] = position;
          continue;
        }
        n_equiv = 0;
        best_value = value;
        best_position = position;
      }
    }
  }
  return dp_randomize(s, d, best_position, n_equiv);
}

// DualEdgeNorms::GetEdgeSquaredNorms (dual_edge_norms.cc:120-132)
SD_INLINE const f64* norms_get(Lp& s) {
  if (s.norms_recompute) {
    for (int row = 0; row < s.m; ++row) s.norms[row] = bf_dual_edge_squared_norm(s, row);
    s.norms_recompute = 0;
  }
  return s.norms;
}

// ---- VariableValues (variable_values.cc) ----
SD_INLINE f64 row_infeasibility(const Lp& s, int col) {
  return sd_max(s.x[col] - s.ub[col], s.lb[col] - s.x[col]);
}
SD_INLINE void vv_recompute_dual_prices(Lp& s, int put_more_importance_on_norm) {
  dp_clear_and_resize(s, s.dp, s.m);
  dp_start_dense_updates(s, s.dp);
  s.put_more_importance_on_norm = put_more_importance_on_norm;
  const f64 tol = s.primal_feasibility_tolerance;
  norms_get(s);
#if defined(__HIP_DEVICE_COMPILE__)
  // Row chunk c is candidate word c (cleared above): its bits are the ballot.
  for (int base = 0; base < s.m; base += 64) {
    const int row = base + sd_lane();
    bool keep = false;
    if (row < s.m) {
      const f64 inf = row_infeasibility(s, s.basis[row]);
      if (inf > tol) {
        keep = true;
        s.dp.values[row] = s.put_more_importance_on_norm ? sd_fabs(inf) / s.norms[row]
                                                         : sq(inf) / s.norms[row];
      }
    }
    const uint64_t word = __ballot(keep);
    if (sd_lane() == 0) s.dp.cand[base >> 6] = word;
  }
  sd_sync();
#else
  for (int row = 0; row < s.m; ++row) {
    const int col = s.basis[row];
    const f64 inf = row_infeasibility(s, col);
    if (inf > tol) {
      dp_dense_add_or_update(s, s.dp, row, s.put_more_importance_on_norm
                                         ? sd_fabs(inf) / s.norms[row]
                                         : sq(inf) / s.norms[row]);
    }
  }
#endif
}
SD_INLINE void vv_update_dual_price(Lp& s, int row) {
  const int col = s.basis[row];
  const f64 inf = row_infeasibility(s, col);
  if (inf > s.primal_feasibility_tolerance) {
    dp_add_or_update(s, s.dp, row, s.put_more_importance_on_norm ? sd_fabs(inf) / s.norms[row]
                                                           : sq(inf) / s.norms[row]);
  } else {
    dp_remove(s, s.dp, row);
  }
}
// UpdateDualPrices(rows); the caller guarantees the norms are current.
SD_INLINE void vv_update_dual_prices(Lp& s, const int32_t* rows, int n) {
  SdSubTimer t_sub_(&s.phase_ticks[19]);
  if (s.dp.size != s.m) {
    vv_recompute_dual_prices(s, s.put_more_importance_on_norm);
    return;
  }
  norms_get(s);
#if defined(__HIP_DEVICE_COMPILE__)
  // 64 rows at a time: the prices, values and candidate bits on the lanes
  // (distinct rows; words shared by lanes take atomic or/and), then the rows
  // that can enter the top-k (price >= the threshold at the chunk's start:
  // the threshold never decreases) replay dp_update_top_k in list order.
  const int lane = sd_lane();
  const f64 tol = s.primal_feasibility_tolerance;
  for (int base = 0; base < n; base += 64) {
    const int k = base + lane;
    int row = 0;
    f64 price = 0.0;
    bool cand = false;
    if (k < n) {
      row = rows[k];
      const f64 inf = row_infeasibility(s, s.basis[row]);
      unsigned long long* word = reinterpret_cast<unsigned long long*>(s.dp.cand + (row >> 6));
      const unsigned long long bit = 1ull << (row & 63);
      if (inf > tol) {
        price = s.put_more_importance_on_norm ? sd_fabs(inf) / s.norms[row] : sq(inf) / s.norms[row];
        s.dp.values[row] = price;
        atomicOr(word, bit);
        cand = price >= s.dp.threshold;
      } else {
        atomicAnd(word, ~bit);
      }
    }
    uint64_t mask = __ballot(cand);
    while (mask != 0) {
      const int l = __builtin_ctzll(mask);
      mask &= mask - 1;
      const int r = __shfl(row, l, 64);
      const f64 p = __shfl(price, l, 64);
      if (p >= s.dp.threshold) dp_update_top_k(s, s.dp, r, p);
    }
  }
  sd_sync();
#else
  for (int k = 0; k < n; ++k) vv_update_dual_price(s, rows[k]);
#endif
}
SD_INLINE void vv_set_nonbasic_from_status(Lp& s, int col) {
  switch (s.vstatus[col]) {
    case kFixedValue:
    case kAtLower:
      s.x[col] = s.lb[col];
      break;
    case kAtUpper:
      s.x[col] = s.ub[col];
      break;
    default:
      break;
  }
}
// UpdateGivenNonBasicVariables(cols, update_basic = true) (:179-227)
SD_INLINE void vv_update_given_nonbasic(Lp& s, const int32_t* cols, int n) {
  Vec& v = s.ia0;
  for (int i = v.size; i < s.m; ++i) v.values[i] = 0.0;  // resize(num_rows, 0.0)
  v.size = s.m;
  vec_clear_mask(v);
  bool use_dense = false;
  for (int k = 0; k < n; ++k) {
    const int col = cols[k];
    const f64 old_value = s.x[col];
    vv_set_nonbasic_from_status(s, col);
    if (use_dense) {
      col_add_dense(s.A, col, s.x[col] - old_value, v.values);
    } else {
      col_add_scattered(s.A, col, s.x[col] - old_value, v);
      use_dense = vec_dense(v, 0.8);
    }
  }
  vec_clear_mask(v);
  vec_clear_nz_if_too_dense(v, 0.8);
  bf_right_solve(s, v);
  if (v.nnz == 0) {
    for (int row = sd_lane(); row < s.m; row += sd_lanes()) {  // distinct basic columns
      s.x[s.basis[row]] -= v.values[row];
      v.values[row] = 0.0;
    }
    sd_sync();
    v.size = s.m;
    vv_recompute_dual_prices(s, 0);  // RecomputeDualPrices() default argument
    return;
  }
  for (int k = sd_lane(); k < v.nnz; k += sd_lanes()) {  // distinct rows
    const int row = v.nz[k];
    s.x[s.basis[row]] -= v.values[row];
    v.values[row] = 0.0;
  }
  sd_sync();
  vv_update_dual_prices(s, v.nz, v.nnz);
  v.nnz = 0;
}

// ---- VariablesInfo (variables_info.cc) ----
SD_INLINE void vi_set_relevance(Lp& s, int col, bool relevance) {
  if (bit_get(s.relevant, col) == relevance) return;
  if (relevance) {
    bit_set(s.relevant, col);
    s.num_entries_relevant += col_entries(s.A, col);
  } else {
    bit_clear(s.relevant, col);
    s.num_entries_relevant -= col_entries(s.A, col);
  }
}
SD_INLINE void vi_to_basic(Lp& s, int col) {
  s.vstatus[col] = kBasic;
  bit_set(s.is_basic, col);
  bit_clear(s.not_basic, col);
  bit_clear(s.can_inc, col);
  bit_clear(s.can_dec, col);
  bit_clear(s.boxed, col);
  vi_set_relevance(s, col, false);
}
SD_INLINE void vi_to_nonbasic(Lp& s, int col, int8_t status) {
  s.vstatus[col] = status;
  bit_clear(s.is_basic, col);
  bit_set(s.not_basic, col);
  bit_put(s.can_inc, col, status == kAtLower || status == kFree);
  bit_put(s.can_dec, col, status == kAtUpper || status == kFree);
  const bool boxed = s.vtype[col] == kBoxed;
  bit_put(s.boxed, col, boxed);
  const bool relevance = status != kFixedValue && (s.boxed_relevant || !boxed);
  vi_set_relevance(s, col, relevance);
}

// ---- UpdateRow (update_row.cc:60-306) ----
SD_INLINE void ur_invalidate(Lp& s) {
  s.left_inv_for = kInvalid;
  s.urow_for = kInvalid;
}
SD_INLINE void ur_compute_unit_row_left_inverse(Lp& s, int leaving_row) {
  if (s.left_inv_for == leaving_row) return;
  s.left_inv_for = leaving_row;
  bf_left_solve_for_unit_row(s, leaving_row, s.rho);
}
#if defined(__HIP_DEVICE_COMPILE__)
// The rows of rho_filtered[c0, c0 + 64) staged in LDS for the row-wise
// update rows: the entry range of row k at meta[4k], meta[4k + 1], its
// multiplier rho[col] at mus[k].
__device__ inline int ur_stage_rows(const Lp& s, int c0, l_i64* meta, l_f64* mus) {
  const int lane = sd_lane();
  const int n = s.n_rho_filtered - c0 < 64 ? s.n_rho_filtered - c0 : 64;
  if (lane < n) {
    const int col = SD_G(const int32_t, s.rho_filtered)[c0 + lane];
    gc_i64* st = SD_G(const int64_t, s.At.starts);
    meta[4 * lane] = st[col];
    meta[4 * lane + 1] = st[col + 1];
    mus[lane] = SD_G(const f64, s.rho.values)[col];
  }
  sd_sync();
  return n;
}
// ComputeUpdatesRowWise (update_row.cc:196-216) with the accumulator in
// LDS (when N fits the staging area and no solve holds it): zero, then each
// filtered row's products added in row order (a row's positions are
// distinct, split over the lanes; the next row's first 64 entries load
// while the current one adds), then the list and the coefficients out.
__device__ inline bool ur_row_wise_lds(Lp& s) {
  if (s.lds == nullptr || s.lds_busy || s.N > s.lds_doubles) return false;
  SdScratch* sc = reinterpret_cast<SdScratch*>(s.lds_scratch);
  l_i64* meta = SD_L(int64_t, sc->meta);
  l_f64* mus = SD_L(f64, sc->mu);
  l_f64* acc = SD_L(f64, s.lds);  // all zero between uses
  gc_i32* rows = SD_G(const int32_t, s.At.rows);
  gc_f64* coefs = SD_G(const f64, s.At.coefs);
  const int lane = sd_lane();
  for (int c0 = 0; c0 < s.n_rho_filtered; c0 += 64) {
    const int n = ur_stage_rows(s, c0, meta, mus);
    int pr = 0;
    f64 pc = 0.0;
    if (meta[0] + lane < meta[1]) {
      pr = rows[meta[0] + lane];
      pc = coefs[meta[0] + lane];
    }
    for (int k = 0; k < n; ++k) {
      const int64_t b = meta[4 * k], e = meta[4 * k + 1];
      const f64 mult = mus[k];
      int nr = 0;
      f64 nc = 0.0;
      if (k + 1 < n && meta[4 * k + 4] + lane < meta[4 * k + 5]) {
        nr = rows[meta[4 * k + 4] + lane];
        nc = coefs[meta[4 * k + 4] + lane];
      }
      if (b + lane < e) acc[pr] += mult * pc;
      for (int64_t i = b + 64 + lane; i < e; i += 64) acc[rows[i]] += mult * coefs[i];
      sd_sync();
      pr = nr;
      pc = nc;
    }
  }
  const f64 drop = s.drop_tolerance;
  const uint64_t* relevant = s.relevant;
  s.n_nzpos = sd_ordered_compact(s.N, s.nzpos, [&](int col) {
    return bit_get(relevant, col) && sd_fabs(acc[col]) > drop;
  });
  g_f64* coeff = SD_G(f64, s.coeff);
  for (int i = lane; i < s.N; i += 64) {
    coeff[i] = acc[i];
    acc[i] = 0.0;
  }
  sd_sync();
  return true;
}
#endif
SD_INLINE void ur_row_wise(Lp& s) {
  SdSubTimer t_sub_(&s.phase_ticks[28]);
#if defined(__HIP_DEVICE_COMPILE__)
  if (ur_row_wise_lds(s)) return;
#endif
  sd_fill<f64>(s.coeff, s.N, 0.0);
  // Rows in list order; a row's entries are distinct positions, so they are
  // split over the lanes (each position keeps its row-by-row order).
  for (int k = 0; k < s.n_rho_filtered; ++k) {
    const int col = s.rho_filtered[k];
    const f64 mult = s.rho.values[col];
    for (int64_t i = s.At.starts[col] + sd_lane(); i < s.At.starts[col + 1]; i += sd_lanes())
      s.coeff[s.At.rows[i]] += mult * s.At.coefs[i];
    sd_sync();
  }
  const f64 drop = s.drop_tolerance;
  const uint64_t* relevant = s.relevant;
  const f64* coeff = s.coeff;
  s.n_nzpos = sd_ordered_compact(s.N, s.nzpos, [&](int col) {
    return bit_get(relevant, col) && sd_fabs(coeff[col]) > drop;
  });
}
// The first touch of a position sets it, later ones add (row by row, a
// row's positions over the lanes); touched positions are flagged in col_flag
// (bytes, so that lanes never share a word) and cleared after the list.
#if defined(__HIP_DEVICE_COMPILE__)
// ComputeUpdatesRowWiseHypersparse (update_row.cc:220-259) with the
// accumulator and the touch flags in LDS: the first touch of a position
// sets it, later ones add; only touched positions are written back (the
// others keep their stale values, as upstream).
__device__ inline bool ur_row_wise_hyper_lds(Lp& s) {
  if (s.lds == nullptr || s.lds_busy ||
      static_cast<int64_t>(s.N) * 9 > static_cast<int64_t>(s.lds_doubles) * 8) {
    return false;
  }
  SdScratch* sc = reinterpret_cast<SdScratch*>(s.lds_scratch);
  l_i64* meta = SD_L(int64_t, sc->meta);
  l_f64* mus = SD_L(f64, sc->mu);
  l_f64* acc = SD_L(f64, s.lds);  // all zero between uses
  __attribute__((address_space(3))) char* flag = SD_L(char, s.lds + s.N);
  gc_i32* rows = SD_G(const int32_t, s.At.rows);
  gc_f64* coefs = SD_G(const f64, s.At.coefs);
  const int lane = sd_lane();
  for (int c0 = 0; c0 < s.n_rho_filtered; c0 += 64) {
    const int n = ur_stage_rows(s, c0, meta, mus);
    int pr = 0;
    f64 pc = 0.0;
    if (meta[0] + lane < meta[1]) {
      pr = rows[meta[0] + lane];
      pc = coefs[meta[0] + lane];
    }
    for (int k = 0; k < n; ++k) {
      const int64_t b = meta[4 * k], e = meta[4 * k + 1];
      const f64 mult = mus[k];
      int nr = 0;
      f64 nc = 0.0;
      if (k + 1 < n && meta[4 * k + 4] + lane < meta[4 * k + 5]) {
        nr = rows[meta[4 * k + 4] + lane];
        nc = coefs[meta[4 * k + 4] + lane];
      }
      for (int64_t i = b + lane; i < e; i += 64) {
        const int pos = i == b + lane ? pr : rows[i];
        const f64 v = mult * (i == b + lane ? pc : coefs[i]);
        if (!flag[pos]) {
          acc[pos] = v;
          flag[pos] = 1;
        } else {
          acc[pos] += v;
        }
      }
      sd_sync();
      pr = nr;
      pc = nc;
    }
  }
  // non_zero_position_set_: the touched positions, relevant ones only.
  for (int w = 0; w < s.nwords; ++w) {
    const int col = w * 64 + lane;
    const uint64_t touched = __ballot(col < s.N && flag[col]);
    if (lane == 0) s.nzset[w] = touched & s.relevant[w];
  }
  sd_sync();
  const f64 drop = s.drop_tolerance;
  const uint64_t* nzset = s.nzset;
  s.n_nzpos = sd_ordered_compact(s.N, s.nzpos, [&](int col) {
    return bit_get(nzset, col) && sd_fabs(acc[col]) > drop;
  });
  g_f64* coeff = SD_G(f64, s.coeff);
  for (int i = lane; i < s.N; i += 64) {
    if (flag[i]) {
      coeff[i] = acc[i];
      acc[i] = 0.0;
      flag[i] = 0;
    }
  }
  sd_sync();
  return true;
}
#endif
SD_INLINE void ur_row_wise_hypersparse(Lp& s) {
  SdSubTimer t_sub_(&s.phase_ticks[28]);
#if defined(__HIP_DEVICE_COMPILE__)
  if (ur_row_wise_hyper_lds(s)) return;
#endif
  for (int k = 0; k < s.n_rho_filtered; ++k) {
    const int col = s.rho_filtered[k];
    const f64 mult = s.rho.values[col];
    for (int64_t i = s.At.starts[col] + sd_lane(); i < s.At.starts[col + 1]; i += sd_lanes()) {
      const int pos = s.At.rows[i];
      const f64 v = mult * s.At.coefs[i];
      if (!s.col_flag[pos]) {
        s.coeff[pos] = v;
        s.col_flag[pos] = 1;
      } else {
        s.coeff[pos] += v;
      }
    }
    sd_sync();
  }
  // non_zero_position_set_: the touched positions, relevant ones only.
  for (int w = 0; w < s.nwords; ++w) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int col = w * 64 + sd_lane();
    const uint64_t touched = __ballot(col < s.N && s.col_flag[col]);
#else
    uint64_t touched = 0;
    for (int b = 0; b < 64 && w * 64 + b < s.N; ++b)
      if (s.col_flag[w * 64 + b]) touched |= 1ull << b;
#endif
    s.nzset[w] = touched & s.relevant[w];
  }
  sd_sync();
  const f64 drop = s.drop_tolerance;
  const uint64_t* nzset = s.nzset;
  const f64* coeff = s.coeff;
  s.n_nzpos = sd_ordered_compact(s.N, s.nzpos, [&](int col) {
    return bit_get(nzset, col) && sd_fabs(coeff[col]) > drop;
  });
  for (int k = 0; k < s.n_rho_filtered; ++k) {
    const int col = s.rho_filtered[k];
    for (int64_t i = s.At.starts[col] + sd_lane(); i < s.At.starts[col + 1]; i += sd_lanes())
      s.col_flag[s.At.rows[i]] = 0;
  }
  sd_sync();
}
SD_INLINE void ur_single_row(Lp& s, int row_as_col) {
  SdSubTimer t_sub_(&s.phase_ticks[28]);
  const f64 drop = s.drop_tolerance;
  const f64 mult = s.rho.values[row_as_col];
  const int64_t b = s.At.starts[row_as_col];
  const int len = static_cast<int>(s.At.starts[row_as_col + 1] - b);
  const int32_t* rows = s.At.rows + b;
  const f64* coefs = s.At.coefs + b;
  const uint64_t* relevant = s.relevant;
  f64* coeff = s.coeff;
  // Entries in row order; a kept entry also writes its product.
  s.n_nzpos = sd_ordered_compact_map(
      len, s.nzpos,
      [&](int k) {
        const int pos = rows[k];
        if (!bit_get(relevant, pos)) return false;
        const f64 v = mult * coefs[k];
        if (!(sd_fabs(v) > drop)) return false;
        coeff[pos] = v;
        return true;
      },
      [&](int k) { return rows[k]; });
}
SD_INLINE void ur_column_wise(Lp& s) {
  SdSubTimer t_sub_(&s.phase_ticks[28]);
  s.n_nzpos = 0;
  const f64 drop = s.drop_tolerance;
  // The dots, one column per lane (a word of the relevance mask per lane);
  // then the list in increasing position order.
  for (int w = sd_lane(); w < s.nwords; w += sd_lanes()) {
    uint64_t word = s.relevant[w];
    while (word) {
      const int col = w * 64 + sd_ctz(word);
      word &= word - 1;
      if (col >= s.N) break;
      const f64 c = col_dot(s.A, col, s.rho.values);
      if (sd_fabs(c) > drop) {
        s.coeff[col] = c;
        s.col_flag[col] = 1;
      }
    }
  }
  sd_sync();
  const uint64_t* relevant = s.relevant;
  const char* flag = s.col_flag;
  s.n_nzpos = sd_ordered_compact(s.N, s.nzpos, [&](int col) {
    return flag[col] && bit_get(relevant, col);
  });
  for (int k = sd_lane(); k < s.n_nzpos; k += sd_lanes()) s.col_flag[s.nzpos[k]] = 0;
  sd_sync();
}
SD_INLINE void ur_compute_update_row(Lp& s, int leaving_row) {
  if (s.urow_for == leaving_row) return;
  s.urow_for = leaving_row;
  ur_compute_unit_row_left_inverse(s, leaving_row);
  if (s.use_transposed_matrix) {
    SdSubTimer t_x_(&s.phase_ticks[29]);
    const f64 drop = s.drop_tolerance;
    const f64* rho = s.rho.values;
    const int32_t* rho_nz = s.rho.nz;
    if (s.rho.nnz == 0) {
      s.n_rho_filtered = sd_ordered_compact(
          s.rho.size, s.rho_filtered, [&](int col) { return sd_fabs(rho[col]) > drop; });
    } else {
      s.n_rho_filtered = sd_ordered_compact_map(
          s.rho.nnz, s.rho_filtered, [&](int k) { return sd_fabs(rho[rho_nz[k]]) > drop; },
          [&](int k) { return rho_nz[k]; });
    }
    int64_t num_row_wise_entries = 0;  // an integer sum: any order
    for (int k = sd_lane(); k < s.n_rho_filtered; k += sd_lanes())
      num_row_wise_entries += col_entries(s.At, s.rho_filtered[k]);
    num_row_wise_entries = sd_wave_sum_i64(num_row_wise_entries);
    if (s.n_rho_filtered == 1) {
      ur_single_row(s, s.rho_filtered[0]);
      s.ur_ops += num_row_wise_entries;
      s.last_alg = 0;
      return;
    }
    const int64_t num_col_wise_entries = s.num_entries_relevant;
    const f64 row_wise = static_cast<f64>(num_row_wise_entries);
    if (row_wise < 0.5 * static_cast<f64>(num_col_wise_entries)) {
      if (row_wise < 1.1 * static_cast<f64>(s.N)) {
        ur_row_wise_hypersparse(s);
        s.ur_ops += 5 * num_row_wise_entries + s.N / 64;
        s.last_alg = 1;
      } else {
        ur_row_wise(s);
        s.ur_ops += num_row_wise_entries + s.m;
        s.last_alg = 2;
      }
    } else {
      ur_column_wise(s);
      s.ur_ops += num_col_wise_entries + s.N;
      s.last_alg = 3;
    }
  } else {
    ur_column_wise(s);
    s.ur_ops += s.num_entries_relevant + s.N;
    s.last_alg = 3;
  }
}

// ---- EnteringVariable::DualChooseEnteringColumn (entering_variable.cc:37-239) ----
// ColWithRatio order: a < b iff (a.ratio == b.ratio ? (a.mag == b.mag ? a.col > b.col
// : a.mag < b.mag) : a.ratio > b.ratio). std::make_heap/pop_heap pop the
// greatest first; the order is total, so any max-heap pops the same sequence.
SD_INLINE bool bp_less(const Lp& s, int a, int b) {
  if (s.bp_ratio[a] == s.bp_ratio[b]) {
    if (s.bp_mag[a] == s.bp_mag[b]) return s.bp_col[a] > s.bp_col[b];
    return s.bp_mag[a] < s.bp_mag[b];
  }
  return s.bp_ratio[a] > s.bp_ratio[b];
}
SD_INLINE void bp_swap(Lp& s, int a, int b) {
  const int32_t c = s.bp_col[a]; s.bp_col[a] = s.bp_col[b]; s.bp_col[b] = c;
  const f64 r = s.bp_ratio[a]; s.bp_ratio[a] = s.bp_ratio[b]; s.bp_ratio[b] = r;
  const f64 g = s.bp_mag[a]; s.bp_mag[a] = s.bp_mag[b]; s.bp_mag[b] = g;
}
SD_INLINE void bp_sift_down(Lp& s, int i, int n) {
  while (true) {
    const int l = 2 * i + 1;
    if (l >= n) return;
    int c = l;
    if (l + 1 < n && bp_less(s, l, l + 1)) c = l + 1;
    if (!bp_less(s, i, c)) return;
    bp_swap(s, i, c);
    i = c;
  }
}
SD_INLINE void ent_dual_choose(Lp& s, bool nothing_to_recompute, f64 cost_variation,
                               int* entering_col) {
  const f64 threshold =
      nothing_to_recompute ? s.minimum_acceptable_pivot : s.ratio_test_zero_threshold;
  f64 variation_magnitude = sd_fabs(cost_variation) - threshold;
  const f64 harris_tolerance = s.harris_tolerance_ratio * s.dual_tol;
  f64 harris_ratio = sd_dbl_max();
  const f64 minimum_delta = s.degenerate_ministep_factor * s.dual_tol;
  s.ent_ops += 10 * static_cast<int64_t>(s.n_nzpos);
  int nbp = 0;
  for (int k = 0; k < s.n_nzpos; ++k) {
    const int col = s.nzpos[k];
    const f64 coeff = (cost_variation > 0.0) ? s.coeff[col] : -s.coeff[col];
    f64 ratio, mag;
    if (bit_get(s.can_dec, col) && coeff > threshold) {
      if (-s.rc[col] > harris_ratio * coeff) continue;
      ratio = -s.rc[col] / coeff;
      mag = coeff;
    } else if (bit_get(s.can_inc, col) && coeff < -threshold) {
      if (s.rc[col] > harris_ratio * -coeff) continue;
      ratio = s.rc[col] / -coeff;
      mag = -coeff;
    } else {
      continue;
    }
    const f64 hr = sd_max(minimum_delta / mag, ratio + harris_tolerance / mag);
    if (hr < harris_ratio) {
      if (bit_get(s.boxed, col)) {
        const f64 delta = (s.ub[col] - s.lb[col]) * mag;
        if (delta >= variation_magnitude) harris_ratio = hr;
      } else {
        harris_ratio = hr;
      }
    }
    s.bp_col[nbp] = col;
    s.bp_ratio[nbp] = ratio;
    s.bp_mag[nbp] = mag;
    ++nbp;
  }
  for (int i = nbp / 2 - 1; i >= 0; --i) bp_sift_down(s, i, nbp);
  harris_ratio = sd_dbl_max();
  *entering_col = kInvalid;
  s.n_flips = 0;
  f64 step = 0.0;
  f64 best_coeff = -1.0;
  int n_equiv = 0;
  while (nbp > 0) {
    const int tcol = s.bp_col[0];
    const f64 tratio = s.bp_ratio[0];
    const f64 tmag = s.bp_mag[0];
    if (tratio > harris_ratio) break;
    bool popped = false;
    if (variation_magnitude > 0.0) {
      if (bit_get(s.boxed, tcol)) {
        variation_magnitude -= (s.ub[tcol] - s.lb[tcol]) * tmag;
        if (variation_magnitude > 0.0) {
          s.flips[s.n_flips++] = tcol;
          popped = true;
        }
      }
    }
    if (!popped) {
      if (tmag >= best_coeff) {
        harris_ratio =
            sd_min(harris_ratio, sd_max(minimum_delta / tmag, tratio + harris_tolerance / tmag));
        if (tmag == best_coeff && tratio == step) {
          s.ent_equiv[n_equiv++] = tcol;
        } else {
          n_equiv = 0;
          best_coeff = tmag;
          *entering_col = tcol;
          step = tratio;
        }
      }
    }
    --nbp;
    if (nbp > 0) {
      bp_swap(s, 0, nbp);
      bp_sift_down(s, 0, nbp);
    }
  }
  if (n_equiv != 0) {
    s.ent_equiv[n_equiv++] = *entering_col;
    *entering_col = s.ent_equiv[uniform_int(s, n_equiv - 1)];
  }
  if (*entering_col == kInvalid) return;
  const f64 pivot_limit = s.minimum_acceptable_pivot;
  if (best_coeff < pivot_limit && s.n_flips != 0) {
    for (int i = s.n_flips - 1; i >= 0; --i) {
      const int col = s.flips[i];
      if (sd_fabs(s.coeff[col]) < pivot_limit) continue;
      *entering_col = col;
      break;
    }
  }
}

// ---- DualEdgeNorms (dual_edge_norms.cc:49-118) ----
SD_INLINE bool den_test_precision(Lp& s, int leaving_row) {
  if (s.norms_recompute) return true;
  f64 leaving;
  {
    SdSubTimer t_x_(&s.phase_ticks[21]);
#if defined(__HIP_DEVICE_COMPILE__)
    leaving = vec_squared_norm_dev(s.rho, s.lds_scratch);
#else
    leaving = vec_squared_norm(s.rho);
#endif
  }
  const f64 old = s.norms[leaving_row];
  const f64 acc = (sd_sqrt(leaving) - sd_sqrt(old)) / sd_sqrt(leaving);
  if (sd_fabs(acc) > s.recompute_edges_norm_threshold) s.norms_recompute = 1;
  s.norms[leaving_row] = leaving;
  return old > 0.25 * leaving;
}
SD_INLINE void den_update_before_pivot(Lp& s, int leaving_row) {
  if (s.norms_recompute) return;
  const f64* tau = bf_right_solve_for_tau(s, s.rho);
  const f64 pivot = s.dir.values[leaving_row];
  const f64 new_leaving = s.norms[leaving_row] / sq(pivot);
  SdSubTimer t_x_(&s.phase_ticks[24]);
  // Element-wise over the direction's distinct rows: split over the lanes.
  for (int k = sd_lane(); k < s.dir.nnz; k += sd_lanes()) {
    const int row = s.dir.nz[k];
    const f64 c = s.dir.values[row];
    s.norms[row] += c * (c * new_leaving - 2.0 / pivot * tau[row]);
    const f64 kLowerBound = 1e-4;
    if (s.norms[row] < kLowerBound) {
      if (row == leaving_row) continue;
      s.norms[row] = kLowerBound;
    }
  }
  sd_sync();
  s.norms[leaving_row] = new_leaving;
}

// ---- ReducedCosts (reduced_costs.cc:172-488) ----
SD_INLINE void rc_shift_cost_if_needed(Lp& s, bool increasing_rc_is_needed, int col) {
  const f64 minimum_delta = s.degenerate_ministep_factor * s.dual_tol;
  if (increasing_rc_is_needed && s.rc[col] <= -minimum_delta) return;
  if (!increasing_rc_is_needed && s.rc[col] >= minimum_delta) return;
  const f64 delta = increasing_rc_is_needed ? minimum_delta : -minimum_delta;
  s.cost_pert[col] -= s.rc[col] + delta;
  s.rc[col] = -delta;
  s.has_cost_shift = 1;
}
SD_INLINE void rc_update_before_pivot(Lp& s, int entering_col, int leaving_row) {
  const int leaving_col = s.basis[leaving_row];
  if (!s.recompute_rc) {
    const f64 entering_rc = s.rc[entering_col];
    if (entering_rc == 0.0) {
      s.rc_precise = 0;
    } else {
      s.rc_recomputed = 0;
      s.rc_precise = 0;
      ur_compute_update_row(s, leaving_row);
      const f64 new_leaving_rc = entering_rc / -s.dir.values[leaving_row];
      SdSubTimer t_x_(&s.phase_ticks[23]);
      for (int k = sd_lane(); k < s.n_nzpos; k += sd_lanes()) {  // distinct positions
        const int col = s.nzpos[k];
        s.rc[col] += new_leaving_rc * s.coeff[col];
      }
      sd_sync();
      s.rc[leaving_col] = new_leaving_rc;
      s.rc[entering_col] = 0.0;
    }
  }
  s.basic_obj[leaving_row] = s.objective[entering_col] + s.cost_pert[entering_col];
  s.recompute_bo_left_inverse = 1;
}

// ---- RevisedSimplex ----
SD_INLINE f64 rs_deterministic_time(const Lp& s) {
  return dt_ops(s.num_update_price_ops) + s.bf_dtime + dt_ops(s.ur_ops) + dt_ops(s.ent_ops) +
         s.rc_dtime + s.primal_norms_dtime;
}
SD_INLINE void rs_advance_deterministic_time(Lp& s) {
  const f64 cur = rs_deterministic_time(s);
  s.tl_det_elapsed += cur - s.last_det_update;
  s.last_det_update = cur;
}
SD_INLINE void rs_compute_direction(Lp& s, int col) {
  bf_right_solve_for_column(s, col, s.dir);
  // The list of a dense result in increasing row order and the infinity norm
  // (a maximum of absolute values: exact in any order).
  f64 norm = 0.0;
  if (s.dir.nnz == 0) {
    const f64* v = s.dir.values;
    s.dir.nnz = sd_ordered_compact(s.m, s.dir.nz, [&](int r) { return v[r] != 0.0; });
    for (int k = sd_lane(); k < s.dir.nnz; k += sd_lanes())
      norm = sd_max(norm, sd_fabs(v[s.dir.nz[k]]));
  } else {
    for (int k = sd_lane(); k < s.dir.nnz; k += sd_lanes())
      norm = sd_max(norm, sd_fabs(s.dir.values[s.dir.nz[k]]));
  }
  s.dir_inf_norm = sd_wave_max(norm);
}
SD_INLINE void rs_make_boxed_dual_feasible(Lp& s) {
  SdSubTimer t_sub_(&s.phase_ticks[31]);
  int n_changed = 0;
  const f64 threshold = s.dual_tol;
  for (int k = 0; k < s.n_flips; ++k) {
    const int col = s.flips[k];
    const f64 rc = s.rc[col];
    const int8_t status = s.vstatus[col];
    if (rc > threshold && status == kAtUpper) {
      vi_to_nonbasic(s, col, kAtLower);
      s.changed_cols[n_changed++] = col;
    } else if (rc < -threshold && status == kAtLower) {
      vi_to_nonbasic(s, col, kAtUpper);
      s.changed_cols[n_changed++] = col;
    }
  }
  if (n_changed != 0) vv_update_given_nonbasic(s, s.changed_cols, n_changed);
}

// ---- ReducedCosts recomputation (reduced_costs.cc:303-439) ----
SD_INLINE void rc_set_recompute_and_notify(Lp& s) {
  s.recompute_rc = 1;
  s.rc_notify = 1;
  s.pp_recompute = 1;  // PrimalPrices::recompute_ watches the reduced costs
}
SD_INLINE void rc_make_precise(Lp& s) {
  if (s.rc_precise) return;
  s.must_refactorize = 1;
  s.recompute_bo_left_inverse = 1;
  rc_set_recompute_and_notify(s);
}
SD_INLINE void rc_clear_and_remove_cost_shifts(Lp& s) {
  s.has_cost_shift = 0;
  sd_fill<f64>(s.cost_pert, s.N, 0.0);
  s.recompute_bo = 1;
  s.recompute_bo_left_inverse = 1;
  s.rc_precise = 0;
  rc_set_recompute_and_notify(s);
}
SD_INLINE void rc_compute_basic_objective(Lp& s) {
  for (int row = sd_lane(); row < s.m; row += sd_lanes()) {
    const int bc = s.basis[row];
    s.basic_obj[row] = s.objective[bc] + s.cost_pert[bc];
  }
  sd_sync();
  s.recompute_bo = 0;
  s.recompute_bo_left_inverse = 1;
}
SD_INLINE void rc_compute_basic_objective_left_inverse(Lp& s) {
  if (s.recompute_bo) rc_compute_basic_objective(s);
  Vec& y = s.bolinv;
  for (int row = sd_lane(); row < s.m; row += sd_lanes()) y.values[row] = s.basic_obj[row];
  sd_sync();
  y.size = s.m;
  y.nnz = 0;
  bf_left_solve(s, y);
  s.recompute_bo_left_inverse = 0;
}
SD_INLINE void rc_compute_reduced_costs(Lp& s) {
  if (s.recompute_bo_left_inverse) rc_compute_basic_objective_left_inverse(s);
  f64 dual_residual_error = 0.0;
  const f64* y = s.bolinv.values;
  for (int col = sd_lane(); col < s.N; col += sd_lanes()) {
    s.rc[col] = s.objective[col] + s.cost_pert[col] - col_dot(s.A, col, y);
  }
  sd_sync();
  // A maximum of absolute values: exact in any order.
  for (int col = sd_lane(); col < s.N; col += sd_lanes()) {
    if (bit_get(s.is_basic, col)) {
      dual_residual_error = sd_max(dual_residual_error, sd_fabs(s.rc[col]));
    }
  }
  dual_residual_error = sd_wave_max(dual_residual_error);
  s.rc_dtime += dt_ops(s.a_num_entries);
  s.recompute_rc = 0;
  s.rc_recomputed = 1;
  s.rc_precise = s.num_updates == 0 ? 1 : 0;
  s.dual_tol = s.dual_feasibility_tolerance;
  if (dual_residual_error > s.dual_tol) s.dual_tol = dual_residual_error;
}
// GetReducedCosts() side effects.
SD_INLINE void rc_get(Lp& s) {
  if (s.num_updates == 0) s.must_refactorize = 0;
  if (s.recompute_rc) rc_compute_reduced_costs(s);
}

// ---- Dual phase I (revised_simplex.cc:2198-2388, entering_variable.cc:241-355) ----
// Glop's dedicated dual feasibility algorithm: the leaving row maximizes
// price^2 / norm over the phase-I prices (dual_pricing_vector_, the right
// solve of the sum of the dual-infeasible columns signed by the direction
// that improves them), the entering column is the phase-I breakpoint test,
// and the prices follow the pivot instead of the primal values.
SD_INLINE bool dp1_is_candidate(f64 price, int8_t type, f64 threshold) {
  if (price == 0.0) return false;
  return type == kBoxed || type == kFixedVariable ||
         (type == kUpperBounded && price < -threshold) ||
         (type == kLowerBounded && price > threshold);
}
// OnDualPriceChange (:2198-2215) for distinct rows in list order: `upd(row,
// &type)` applies the row's price change and names the basic type. On the
// device 64 rows at a time: prices, values and candidate bits on the lanes,
// then the rows that can enter the top-k (value >= the threshold at the
// chunk's start: the threshold never decreases) replay dp_update_top_k in
// list order, as the sequential AddOrUpdate calls do.
template <typename Upd>
SD_INLINE void dp1_rows_changed(Lp& s, const int32_t* rows, int n, const f64* sn, Upd upd) {
  const f64 threshold = s.ratio_test_zero_threshold;
#if defined(__HIP_DEVICE_COMPILE__)
  const int lane = sd_lane();
  for (int base = 0; base < n; base += 64) {
    const int k = base + lane;
    int row = 0;
    f64 value = 0.0;
    bool cand = false;
    if (k < n) {
      row = rows[k];
      int8_t type;
      upd(row, &type);
      const f64 price = s.dpv[row];
      unsigned long long* word = reinterpret_cast<unsigned long long*>(s.dp.cand + (row >> 6));
      const unsigned long long bit = 1ull << (row & 63);
      if (dp1_is_candidate(price, type, threshold)) {
        value = sq(price) / sn[row];
        s.dp.values[row] = value;
        atomicOr(word, bit);
        cand = value >= s.dp.threshold;
      } else {
        atomicAnd(word, ~bit);
      }
    }
    uint64_t mask = __ballot(cand);
    while (mask != 0) {
      const int l = __builtin_ctzll(mask);
      mask &= mask - 1;
      const int r = __shfl(row, l, 64);
      const f64 v = __shfl(value, l, 64);
      if (v >= s.dp.threshold) dp_update_top_k(s, s.dp, r, v);
    }
  }
  sd_sync();
#else
  for (int k = 0; k < n; ++k) {
    const int row = rows[k];
    int8_t type;
    upd(row, &type);
    const f64 price = s.dpv[row];
    if (dp1_is_candidate(price, type, threshold)) {
      dp_add_or_update(s, s.dp, row, sq(price) / sn[row]);
    } else {
      dp_remove(s, s.dp, row);
    }
  }
#endif
}
// DualPhaseIUpdatePrice (:2217-2267), before UpdateAndPivot.
// AreReducedCostsRecomputed(): recomputed, or about to be (reduced_costs.h).
SD_INLINE bool rc_are_recomputed(const Lp& s) { return s.recompute_rc || s.rc_recomputed; }
SD_INLINE void dp1_update_price(Lp& s, int leaving_row, int entering_col) {
  if (rc_are_recomputed(s) || s.norms_recompute || s.dpv_size == 0) return;
  const f64* sn = norms_get(s);
  const f64 step = s.dpv[leaving_row] / s.dir.values[leaving_row];
  dp1_rows_changed(s, s.dir.nz, s.dir.nnz, sn, [&](int row, int8_t* type) {
    s.dpv[row] -= s.dir.values[row] * step;
    *type = s.vtype[s.basis[row]];
  });
  s.dpv[leaving_row] = step;
  s.dpv[leaving_row] -= s.diid[entering_col];
  if (s.diid[entering_col] != 0.0) --s.n_dual_inf;
  s.diid[entering_col] = 0.0;
  s.diid[s.basis[leaving_row]] = 0.0;
  const int32_t one = leaving_row;
  dp1_rows_changed(s, &one, 1, sn, [&](int, int8_t* type) { *type = s.vtype[entering_col]; });
}
// DualPhaseIUpdatePriceOnReducedCostChange (:2269-2333) over `cols` (null:
// the relevant columns in increasing order). The changed columns' signed
// sum is scattered in order into the zero scratchpad (ia0: the host's two
// initially-all-zero scratchpads are both zero between uses), solved with
// B and added to the prices.
SD_INLINE void dp1_update_price_on_rc_change(Lp& s, const int32_t* cols, int n) {
  rc_get(s);  // GetReducedCosts()
  const f64 tol = s.dual_tol;
  Vec& v = s.ia0;
  bool something_to_do = false;
  auto change = [&](int col, f64 sign) {
    const f64 old = s.diid[col];
    if (sign == 0.0) {
      --s.n_dual_inf;
    } else if (old == 0.0) {
      ++s.n_dual_inf;
    }
    if (!something_to_do) {
      for (int i = v.size + sd_lane(); i < s.m; i += sd_lanes()) v.values[i] = 0.0;
      sd_sync();
      v.size = s.m;
      vec_clear_mask(v);
      v.nnz = 0;
      something_to_do = true;
    }
    s.num_update_price_ops += 10 * col_entries(s.A, col);
    col_add_scattered(s.A, col, sign - old, v);
    s.diid[col] = sign;
  };
  auto sign_of = [&](int col) -> f64 {
    const f64 rc = s.rc[col];
    return (bit_get(s.can_inc, col) && rc < -tol)   ? 1.0
           : (bit_get(s.can_dec, col) && rc > tol) ? -1.0
                                                   : 0.0;
  };
  const int count = cols != nullptr ? n : s.N;
#if defined(__HIP_DEVICE_COMPILE__)
  // 64 positions at a time: the signs on the lanes, the changed columns
  // replayed in order (their scatters are order-dependent).
  for (int base = 0; base < count; base += 64) {
    const int k = base + sd_lane();
    int col = -1;
    f64 sign = 0.0;
    if (k < count) {
      col = cols != nullptr ? cols[k] : (bit_get(s.relevant, k) ? k : -1);
      if (col >= 0) sign = sign_of(col);
    }
    uint64_t mask = __ballot(col >= 0 && sign != s.diid[col >= 0 ? col : 0]);
    while (mask != 0) {
      const int l = __builtin_ctzll(mask);
      mask &= mask - 1;
      change(__shfl(col, l, 64), __shfl(sign, l, 64));
    }
  }
#else
  for (int k = 0; k < count; ++k) {
    const int col = cols != nullptr ? cols[k] : k;
    if (cols == nullptr && !bit_get(s.relevant, col)) continue;
    const f64 sign = sign_of(col);
    if (sign != s.diid[col]) change(col, sign);
  }
#endif
  if (!something_to_do) return;
  vec_clear_nz_if_too_dense(v, 0.8);  // ClearNonZerosIfTooDense()
  vec_clear_mask(v);                  // ClearSparseMask()
  const f64* sn = norms_get(s);
  bf_right_solve(s, v);
  if (v.nnz == 0) {
    // DenseAddOrUpdate over the rows with a change (no top-k maintenance).
    dp_start_dense_updates(s, s.dp);
    const f64 threshold = s.ratio_test_zero_threshold;
#if defined(__HIP_DEVICE_COMPILE__)
    for (int base = 0; base < s.m; base += 64) {
      const int row = base + sd_lane();
      bool touched = false, cand = false;
      if (row < s.m && v.values[row] != 0.0) {
        touched = true;
        s.dpv[row] += v.values[row];
        const f64 price = s.dpv[row];
        if (dp1_is_candidate(price, s.vtype[s.basis[row]], threshold)) {
          cand = true;
          s.dp.values[row] = sq(price) / sn[row];
        }
      }
      const uint64_t tmask = __ballot(touched);
      const uint64_t cmask = __ballot(cand);
      if (sd_lane() == 0 && tmask != 0) {
        s.dp.cand[base >> 6] = (s.dp.cand[base >> 6] & ~tmask) | cmask;
      }
    }
    sd_sync();
#else
    for (int row = 0; row < s.m; ++row) {
      if (v.values[row] == 0.0) continue;
      s.dpv[row] += v.values[row];
      const f64 price = s.dpv[row];
      if (dp1_is_candidate(price, s.vtype[s.basis[row]], threshold)) {
        dp_dense_add_or_update(s, s.dp, row, sq(price) / sn[row]);
      } else {
        dp_remove(s, s.dp, row);
      }
    }
#endif
    sd_fill<f64>(v.values, s.m, 0.0);
  } else {
    dp1_rows_changed(s, v.nz, v.nnz, sn, [&](int row, int8_t* type) {
      s.dpv[row] += v.values[row];
      v.values[row] = 0.0;
      *type = s.vtype[s.basis[row]];
    });
  }
  v.nnz = 0;
}
// DualPhaseIChooseLeavingVariableRow (:2335-2388); kInvalid when none.
SD_INLINE int dp1_choose_leaving(Lp& s, f64* cost_variation, f64* target_bound) {
  if (rc_are_recomputed(s) || s.norms_recompute || s.dpv_size == 0) {
    s.n_dual_inf = 0;
    sd_fill<f64>(s.dpv, s.m, 0.0);
    s.dpv_size = s.m;
    dp_clear_and_resize(s, s.dp, s.m);
    sd_fill<f64>(s.diid, s.N, 0.0);
    s.diid_size = s.N;
    dp1_update_price_on_rc_change(s, nullptr, 0);
  } else {
    dp1_update_price_on_rc_change(s, s.nzpos, s.n_nzpos);
  }
  if (s.n_dual_inf == 0) return kInvalid;
  const int row = dp_get_maximum(s, s.dp);
  if (row == kInvalid) return kInvalid;
  *cost_variation = s.dpv[row];
  const int col = s.basis[row];
  *target_bound = *cost_variation < 0.0 ? s.ub[col] : s.lb[col];
  return row;
}
// EnteringVariable::DualPhaseIChooseEnteringColumn (entering_variable.cc:241-355).
SD_INLINE void ent_dual_phase1_choose(Lp& s, bool nothing_to_recompute, f64 cost_variation,
                                      int* entering_col) {
  rc_get(s);  // GetReducedCosts()
  const f64 threshold =
      nothing_to_recompute ? s.minimum_acceptable_pivot : s.ratio_test_zero_threshold;
  const f64 dual_tol = s.dual_tol;
  const f64 harris_tolerance = s.harris_tolerance_ratio * dual_tol;
  const f64 minimum_delta = s.degenerate_ministep_factor * dual_tol;
  s.ent_ops += 10 * static_cast<int64_t>(s.n_nzpos);
  int nbp = 0;
  for (int k = 0; k < s.n_nzpos; ++k) {
    const int col = s.nzpos[k];
    if (sd_fabs(s.coeff[col]) < threshold) continue;
    const f64 coeff = (cost_variation > 0.0) ? s.coeff[col] : -s.coeff[col];
    const f64 rc = s.rc[col];
    f64 ratio;  // the ColWithRatio's reduced_cost argument
    if (sd_fabs(rc) <= dual_tol) {
      if (coeff > 0 && !bit_get(s.can_dec, col)) continue;
      if (coeff < 0 && !bit_get(s.can_inc, col)) continue;
      ratio = coeff * rc > 0.0 ? sd_max(minimum_delta, harris_tolerance - sd_fabs(rc))
                               : sd_fabs(rc) + harris_tolerance;
    } else {
      if (coeff * rc > 0.0) continue;
      ratio = sd_fabs(rc) + harris_tolerance;
    }
    // ColWithRatio(col, reduced_cost, coeff_m): ratio = reduced_cost / coeff_m.
    const f64 mag = sd_fabs(coeff);
    s.bp_col[nbp] = col;
    s.bp_ratio[nbp] = ratio / mag;
    s.bp_mag[nbp] = mag;
    ++nbp;
  }
  for (int i = nbp / 2 - 1; i >= 0; --i) bp_sift_down(s, i, nbp);
  f64 pivot_magnitude = 0.0;
  *entering_col = kInvalid;
  f64 step = -1.0;
  f64 improvement = sd_fabs(cost_variation);
  while (nbp > 0) {
    const int tcol = s.bp_col[0];
    const f64 tratio = s.bp_ratio[0];
    const f64 tmag = s.bp_mag[0];
    if (tratio > step && tmag >= pivot_magnitude) {
      *entering_col = tcol;
      step = tratio;
      pivot_magnitude = tmag;
    }
    improvement -= tmag;
    if (bit_get(s.can_dec, tcol) && bit_get(s.can_inc, tcol) && sd_fabs(s.rc[tcol]) > threshold) {
      improvement -= tmag;
    }
    if (improvement <= 0.0) break;
    --nbp;
    if (nbp > 0) {
      bp_swap(s, 0, nbp);
      bp_sift_down(s, 0, nbp);
    }
  }
}

// ---- factorization (host Markowitz through the mailbox) ----
// Points the LU fields at an image installed at address `b` (`im` is a
// readable copy of its header).
SD_INLINE void sd_install_lu(Lp& s, const LuImage* im, uintptr_t b) {
  auto fix = [&](Tri* t, const Tri& src) {
    *t = src;
    t->starts = reinterpret_cast<int64_t*>(b + reinterpret_cast<uintptr_t>(src.starts));
    t->rows = reinterpret_cast<int32_t*>(b + reinterpret_cast<uintptr_t>(src.rows));
    t->coefs = reinterpret_cast<f64*>(b + reinterpret_cast<uintptr_t>(src.coefs));
    t->diag = reinterpret_cast<f64*>(b + reinterpret_cast<uintptr_t>(src.diag));
    if (src.num_levels >= 0) {
      t->lv_order = reinterpret_cast<int32_t*>(b + reinterpret_cast<uintptr_t>(src.lv_order));
      t->lv_starts = reinterpret_cast<int32_t*>(b + reinterpret_cast<uintptr_t>(src.lv_starts));
    }
  };
  fix(&s.lower, im->lower);
  fix(&s.upper, im->upper);
  fix(&s.tupper, im->tupper);
  fix(&s.tlower, im->tlower);
  s.is_identity = im->is_identity;
  s.col_perm_empty = im->col_perm_empty;
  s.col_perm = reinterpret_cast<int32_t*>(b + im->off_col_perm);
  s.inv_col_perm = reinterpret_cast<int32_t*>(b + im->off_inv_col_perm);
  s.row_perm = reinterpret_cast<int32_t*>(b + im->off_row_perm);
  s.inv_row_perm = reinterpret_cast<int32_t*>(b + im->off_inv_row_perm);
}

#if defined(__HIP_DEVICE_COMPILE__)
// Polls are relaxed (the polled word bypasses the caches, nothing else is
// invalidated); the caller fences once the value changed.
__device__ inline int32_t sd_mb_load(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void sd_mb_store(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
#endif

// ForceRefactorization (basis_representation.cc:228-238): Clear() and a new
// factorization of the current basis. Markowitz runs on the host (the
// mailbox); this side mirrors Clear()'s and ComputeFactorization()'s effects.
// Returns the image status: 0 installed, 1 LU error, 2 computed but too
// large for the arena (the caller hands the LP back).
SD_INLINE int sd_refactorize(Lp& s, int bump) {
  int status;
#if defined(__HIP_DEVICE_COMPILE__)
  for (int r = sd_lane(); r < s.m; r += sd_lanes()) s.mb_basis[r] = s.basis[r];
  sd_sync();
  s.mb->bump = bump;
  __threadfence_system();
  sd_mb_store(&s.mb->flag, 1);
  // The flag sits in host memory: every poll is a PCIe read. One lane polls,
  // backing off from ~3 us to ~27 us (a Markowitz answer takes ~100 us), so
  // that hundreds of waiting waves leave the link to the image copies.
  for (int polls = 0;; ++polls) {
    int32_t f = 0;
    if (sd_lane() == 0) f = sd_mb_load(&s.mb->flag);
    if (__shfl(f, 0, 64) == 2) break;
    const int reps = polls < 4 ? 1 : polls < 12 ? 3 : 8;
    for (int r = 0; r < reps; ++r) __builtin_amdgcn_s_sleep(127);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const LuImage* im = reinterpret_cast<const LuImage*>(s.mb_image);
  status = im->status;
  const f64 dtime = im->last_fact_dtime;
  if (status == 0) {
    // Over PCIe: 16-byte words, eight reads in flight per lane.
    SdSubTimer t_(&s.phase_ticks[12]);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const int64_t words = (im->bytes + 15) / 16;
    const u32x4* src = reinterpret_cast<const u32x4*>(s.mb_image);
    u32x4* dst = reinterpret_cast<u32x4*>(s.lu_region);
    const int lane = sd_lane();
    int64_t w = 0;
    for (; w + 8 * 64 <= words; w += 8 * 64) {
      u32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(src + w + u * 64 + lane);
#pragma unroll
      for (int u = 0; u < 8; ++u) dst[w + u * 64 + lane] = v[u];
    }
    for (w += lane; w < words; w += 64) dst[w] = src[w];
    sd_sync();
  }
  sd_mb_store(&s.mb->flag, 0);
#else
  status = s.lu_service(s.lu_ctx, &s, bump);
  const f64 dtime = reinterpret_cast<const LuImage*>(s.lu_region)->last_fact_dtime;
#endif
  if (bump) {
    f64 t = s.lu_factorization_pivot_threshold * 1.5;
    s.lu_factorization_pivot_threshold = t < 0.9 ? t : 0.9;
  }
  // Clear()
  s.num_updates = 0;
  s.tau_can_opt = 0;
  s.r1_count = 0;
  s.r1_num_entries = 0;
  s.eta_count = 0;  // eta_factorization_.Clear()
  s.storage.num_cols = 0;
  s.storage.starts[0] = 0;
  s.right_storage.num_cols = 0;
  s.right_storage.starts[0] = 0;
  sd_fill<int32_t>(s.left_pool, s.m, kInvalid);
  sd_fill<int32_t>(s.right_pool, s.N, kInvalid);
  // ComputeFactorization()
  s.last_fact_dtime = dtime;
  s.bf_dtime += dtime;
  s.r1_dtime = 0.0;
  ++s.factorizations;
  // Not installed: the host's factorization (and its column permutation) is
  // newer than anything this side holds.
  if (status == 2) s.col_perm_empty = 0;
  if (status == 0) {
    sd_install_lu(s, reinterpret_cast<const LuImage*>(s.lu_region),
                  reinterpret_cast<uintptr_t>(s.lu_region));
  }
  return status;
}

// PermuteBasis (revised_simplex.cc:2475-2502)
SD_INLINE void rs_permute_basis(Lp& s) {
  SdSubTimer t_sub_(&s.phase_ticks[22]);
  if (s.col_perm_empty) return;
  // col_perm is a permutation: every loop writes distinct positions.
  int32_t* tmp = s.changed_cols;
  for (int i = sd_lane(); i < s.m; i += sd_lanes()) tmp[s.col_perm[i]] = s.basis[i];
  sd_sync();
  for (int i = sd_lane(); i < s.m; i += sd_lanes()) s.basis[i] = tmp[i];
  sd_sync();
  f64* ftmp = s.bp_ratio;
  if (s.dpv_size != 0) {
    for (int i = sd_lane(); i < s.m; i += sd_lanes()) ftmp[s.col_perm[i]] = s.dpv[i];
    sd_sync();
    for (int i = sd_lane(); i < s.m; i += sd_lanes()) s.dpv[i] = ftmp[i];
    sd_sync();
  }
  s.recompute_bo = 1;
  s.recompute_bo_left_inverse = 1;
  if (!s.norms_recompute) {
    for (int i = sd_lane(); i < s.m; i += sd_lanes()) ftmp[s.col_perm[i]] = s.norms[i];
    sd_sync();
    for (int i = sd_lane(); i < s.m; i += sd_lanes()) s.norms[i] = ftmp[i];
    sd_sync();
  }
  s.col_perm_empty = 1;
}

// MakeBoxedVariableDualFeasible(GetNonBasicBoxedVariables(), false)
SD_INLINE void rs_make_boxed_dual_feasible_all(Lp& s) {
  const f64 threshold = s.dual_tol;
  rc_get(s);
  for (int w = 0; w < s.nwords; ++w) {
    uint64_t word = s.boxed[w];
    while (word) {
      const int col = w * 64 + sd_ctz(word);
      word &= word - 1;
      if (col >= s.N) break;
      const f64 rc = s.rc[col];
      const int8_t status = s.vstatus[col];
      if (rc > threshold && status == kAtUpper) {
        vi_to_nonbasic(s, col, kAtLower);
        vv_set_nonbasic_from_status(s, col);
      } else if (rc < -threshold && status == kAtLower) {
        vi_to_nonbasic(s, col, kAtUpper);
        vv_set_nonbasic_from_status(s, col);
      }
    }
  }
}
// RecomputeBasicVariableValues (variable_values.cc:101-118)
SD_INLINE void vv_recompute_basic_values(Lp& s) {
  Vec& v = s.vv_scratch;
  v.nnz = 0;
  v.size = s.m;
  // sum over non-basic columns in increasing order of -x_j a_j: per row over
  // the transpose (its entries are in increasing column order), zero
  // multipliers skipped as ColumnAddMultipleToDenseColumn does.
  for (int r = sd_lane(); r < s.m; r += sd_lanes()) {
    f64 acc = 0.0;
    for (int64_t i = s.At.starts[r]; i < s.At.starts[r + 1]; ++i) {
      const int col = s.At.rows[i];
      if (!bit_get(s.not_basic, col)) continue;
      const f64 mult = -s.x[col];
      if (mult == 0.0) continue;
      acc += mult * s.At.coefs[i];
    }
    v.values[r] = acc;
  }
  sd_sync();
  bf_right_solve(s, v);
  for (int row = sd_lane(); row < s.m; row += sd_lanes()) s.x[s.basis[row]] = v.values[row];
  sd_sync();
  dp_clear_and_resize(s, s.dp, 0);  // dual_prices_->Clear()
}
// PreciseScalarProduct(objective_, variable_values_) (lp_utils.h:106-114)
SD_INLINE f64 rs_objective_value(const Lp& s) {
  f64 sum = 0.0, err = 0.0;
  for (int c = 0; c < s.N; ++c) {
    err += s.objective[c] * s.x[c];
    const f64 new_sum = sum + err;
    err += sum - new_sum;
    sum = new_sum;
  }
  return sum;
}

// Room for one more iteration in every fixed-capacity array.
SD_INLINE bool sd_room_for_iteration(const Lp& s) {
  const int64_t need = static_cast<int64_t>(s.m) + 1;
  if (s.storage.num_cols + 3 > s.storage.cap_cols) return false;
  if (s.right_storage.num_cols + 2 > s.right_storage.cap_cols) return false;
  if (s.storage.starts[s.storage.num_cols] + 2 * need > s.storage.cap_entries) return false;
  if (s.right_storage.starts[s.right_storage.num_cols] + need > s.right_storage.cap_entries)
    return false;
  if (s.r1_count + 1 > s.r1_cap) return false;
  if (!s.mpf) {  // one more eta, dense and possibly sparse
    if (s.eta_count + 1 > s.eta_cap) return false;
    if (s.eta_sp_starts[s.eta_count] + s.m / 2 + 1 > s.eta_sp_cap) return false;
  }
  return true;
}

// UpdateAndPivot (revised_simplex.cc:2504-2575) up to the factorization:
// the pivot from the update row (or its ColumnScalarProduct with rho when the
// row is not computed for leaving_row), UpdateBasis, the precision test, then
// the MPF update (basis_representation.cc:258-340) or *refactor = 1
// (ForceRefactorization) / 2 (the same after the LU threshold bump). Returns
// kExitLuError for a degenerate rank-one update, else kExitNone.
SD_INLINE int32_t sd_pivot(Lp& s, int entering_col, int leaving_row, f64 target_bound,
                           int* refactor) {
  *refactor = 0;
  f64 pivot_from_update_row;
  if (s.urow_for == leaving_row) {  // update_row_.IsComputedFor(leaving_row)
    pivot_from_update_row = s.coeff[entering_col];
  } else {
    ur_compute_unit_row_left_inverse(s, leaving_row);
    pivot_from_update_row = col_dot_par(s.A, entering_col, s.rho.values, s.lds_scratch);
  }
  const int lcol = s.basis[leaving_row];
  const int8_t leaving_status = s.lb[lcol] == s.ub[lcol] ? kFixedValue
                                : target_bound == s.lb[lcol] ? kAtLower
                                                             : kAtUpper;
  vi_to_nonbasic(s, lcol, leaving_status);  // UpdateBasis
  s.basis[leaving_row] = entering_col;
  vi_to_basic(s, entering_col);
  ur_invalidate(s);
  const f64 pivot_from_direction = s.dir.values[leaving_row];
  const f64 diff = sd_fabs(pivot_from_update_row - pivot_from_direction);
  s.exit_col = lcol;
  if (diff > s.refactorization_threshold *
                 (1.0 + sd_min(sd_fabs(pivot_from_update_row), sd_fabs(pivot_from_direction)))) {
    *refactor = s.num_updates < 10 ? 2 : 1;
  } else if (s.num_updates >= s.max_updates &&
             (!s.dynamic_period || s.last_fact_dtime < s.r1_dtime)) {
    *refactor = 1;  // BasisFactorization::Update (:304-340)
  } else if (!s.mpf) {
    ++s.num_updates;  // EtaFactorization::Update (PFI)
    eta_update(s, leaving_row, s.dir);
    s.tau_can_opt = 0;
  } else {
    const int right_index = s.right_pool[entering_col];
    const int left_index = s.left_pool[leaving_row];
    ++s.num_updates;
    if (right_index == kInvalid || left_index == kInvalid) {
      *refactor = 1;
    } else {
      // MiddleProductFormUpdate (:258-302)
      SdSubTimer t_x_(&s.phase_ticks[26]);
      // Each column's rows are distinct: the lanes split them; the list
      // entries keep their positions (right column, then U's column).
      {
        const int64_t rb = s.right_storage.starts[right_index];
        const int rn = static_cast<int>(s.right_storage.starts[right_index + 1] - rb);
        const int base = s.n_mpf_scratch_nz;
        for (int k = sd_lane(); k < rn; k += sd_lanes()) {
          const int r = s.right_storage.rows[rb + k];
          s.mpf_scratch[r] = s.right_storage.coefs[rb + k];
          s.mpf_scratch_nz[base + k] = r;
        }
        sd_sync();
        s.n_mpf_scratch_nz = base + rn;
      }
      lu_column_of_u(s, leaving_row);
      {
        const int base = s.n_mpf_scratch_nz;
        for (int k = sd_lane(); k < s.n_col_u; k += sd_lanes()) {
          s.mpf_scratch[s.col_u_rows[k]] -= s.col_u_coefs[k];
          s.mpf_scratch_nz[base + k] = s.col_u_rows[k];
        }
        sd_sync();
        s.n_mpf_scratch_nz = base + s.n_col_u;
      }
      const f64 scalar_product = col_dot_par(s.storage, left_index, s.mpf_scratch, s.lds_scratch);
      const int u_index =
          store_add_and_clear(s.storage, s.mpf_scratch, s.mpf_scratch_nz, &s.n_mpf_scratch_nz);
      const f64 mu = 1.0 + scalar_product;
      if (mu == 0.0) return kExitLuError;
      s.r1_u[s.r1_count] = u_index;
      s.r1_v[s.r1_count] = left_index;
      s.r1_mu[s.r1_count] = mu;
      ++s.r1_count;
      s.r1_num_entries += col_entries(s.storage, u_index) + col_entries(s.storage, left_index);
      s.tau_can_opt = 0;
    }
  }
  return kExitNone;
}

// The phase-II dual loop (revised_simplex.cc:3058-3367), entered after the
// loop-top block, until the loop returns or needs the host. Returns the exit.
// Phase timer (device only): 0 loop top, 1 leaving row, 2 BTRAN, 3 update
// row, 4 ratio test, 5 FTRAN, 6 rc and norm updates with tau, 7 pivot (x,
// basis, MPF), 8 factorization requests.
#define SD_PHASE(k)                          \
  do {                                       \
    const uint64_t now_ = sd_now();          \
    s.phase_ticks[phase_] += now_ - mark_;   \
    mark_ = now_;                            \
    phase_ = (k);                            \
  } while (0)

SD_INLINE int32_t sd_run(Lp& s) {
  s.exit_code = kExitNone;
  s.iterations_done = 0;
  bool at_top = false;  // false: enter after the loop-top block
  uint64_t mark_ = sd_now();
  int phase_ = 0;
  struct Flush {
    Lp& s;
    uint64_t& mark;
    int& phase;
    SD_HD ~Flush() { s.phase_ticks[phase] += sd_now() - mark; }
  } flush_{s, mark_, phase_};
  while (true) {
    SD_PHASE(0);
    if (at_top) {
      if ((s.iteration_cap > 0 && s.iterations_done >= s.iteration_cap) ||
          !sd_room_for_iteration(s)) {
        return s.exit_code = kExitLoopTop;  // s.refactorize carries the flag
      }
      const int old_refactorize = s.refactorize;
      if (!s.refactorize && s.must_refactorize) s.refactorize = 1;
      if (!s.refactorize && s.norms_recompute) s.refactorize = 1;
      // RefactorizeBasisIfNeeded
      if (s.refactorize && s.num_updates != 0) {
        SD_PHASE(8);
        const int st = sd_refactorize(s, 0);
        SD_PHASE(0);
        if (st == 1) return s.exit_code = kExitLuError;
        if (st == 2) {
          s.refactorize = old_refactorize;
          return s.exit_code = kExitResumeTop;
        }
        ur_invalidate(s);
        rs_permute_basis(s);
      }
      s.refactorize = 0;
      if (s.dual_phase1) {
        // Phase I: only MakeReducedCostsPrecise after a factorization.
        if (s.num_updates == 0) rc_make_precise(s);
      } else if (s.num_updates == 0) {
        SdSubTimer t_x_(&s.phase_ticks[20]);
        if (old_refactorize) rc_make_precise(s);
        rs_make_boxed_dual_feasible_all(s);
        vv_recompute_basic_values(s);
        vv_recompute_dual_prices(s, s.dual_price_prioritize_norm);
        if (s.phase_optimization && s.dual_objective_limit != sd_inf() &&
            rs_objective_value(s) > s.dual_objective_limit) {
          s.objective_limit_reached = 1;
          return s.exit_code = kExitObjectiveLimit;
        }
      } else {
        rs_make_boxed_dual_feasible(s);
        s.n_flips = 0;
        vv_update_dual_prices(s, s.dir.nz, s.dir.nnz);
      }
    }
    at_top = true;
    SD_PHASE(1);
    // DualChooseLeavingVariableRow (:2148-2181) / DualPhaseIChooseLeavingVariableRow
    f64 cost_variation = 0.0, target_bound = 0.0;
    int leaving_row;
    if (s.dual_phase1) {
      leaving_row = dp1_choose_leaving(s, &cost_variation, &target_bound);
    } else {
      if (s.dp.size == 0) vv_recompute_dual_prices(s, s.dual_price_prioritize_norm);
      leaving_row = dp_get_maximum(s, s.dp);
    }
    if (leaving_row == kInvalid) {
      if (s.num_updates != 0 || s.has_cost_shift) {
        rc_clear_and_remove_cost_shifts(s);
        s.refactorize = 1;
        continue;
      }
      s.exit_row = kInvalid;
      // Phase I: DUAL_FEASIBLE / DUAL_INFEASIBLE from n_dual_inf (the bridge).
      return s.exit_code = kExitOptimal;
    }
    const int lcol = s.basis[leaving_row];
    if (!s.dual_phase1) {
      const f64 value = s.x[lcol];
      if (value < s.lb[lcol]) {
        cost_variation = s.lb[lcol] - value;
        target_bound = s.lb[lcol];
      } else {
        cost_variation = s.ub[lcol] - value;
        target_bound = s.ub[lcol];
      }
    }
    s.exit_row = leaving_row;
    s.exit_cost_variation = cost_variation;
    s.exit_target_bound = target_bound;

    SD_PHASE(2);
    ur_compute_unit_row_left_inverse(s, leaving_row);
    if (!den_test_precision(s, leaving_row)) {
      if (s.dual_phase1) {
        const f64 price = s.dpv[leaving_row];
        const f64* sn = norms_get(s);
        dp_add_or_update(s, s.dp, leaving_row, sq(price) / sn[leaving_row]);
      } else {
        const int32_t one = leaving_row;
        vv_update_dual_prices(s, &one, 1);
      }
      continue;
    }
    SD_PHASE(3);
    ur_compute_update_row(s, leaving_row);

    SD_PHASE(4);
    int entering_col;
    if (s.dual_phase1) {
      ent_dual_phase1_choose(s, s.rc_precise != 0, cost_variation, &entering_col);
    } else {
      ent_dual_choose(s, s.rc_precise != 0, cost_variation, &entering_col);
    }
    if (entering_col == kInvalid) {
      if (!s.rc_precise) {
        s.refactorize = 1;
        continue;
      }
      return s.exit_code = kExitNoEntering;  // phase I: ABNORMAL (the bridge)
    }
    const f64 entering_coeff = s.coeff[entering_col];
    if (sd_fabs(entering_coeff) < s.dual_small_pivot_threshold && !s.rc_precise) {
      s.refactorize = 1;
      continue;
    }
    SD_PHASE(5);
    rs_compute_direction(s, entering_col);
    if (sd_fabs(s.dir.values[leaving_row]) < s.small_pivot_threshold * s.dir_inf_norm) {
      if (!s.rc_precise) {
        s.refactorize = 1;
        continue;
      }
    }
    rs_advance_deterministic_time(s);
    if (s.num_iterations == s.max_number_of_iterations || s.tl_det_elapsed > s.tl_det_max) {
      return s.exit_code = kExitReturnOk;
    }
    const bool increasing_rc_is_needed = (cost_variation > 0.0) == (entering_coeff > 0.0);
    SD_PHASE(6);
    rc_shift_cost_if_needed(s, increasing_rc_is_needed, entering_col);
    rc_update_before_pivot(s, entering_col, leaving_row);
    den_update_before_pivot(s, leaving_row);
    SD_PHASE(7);
    if (s.dual_phase1) {
      dp1_update_price(s, leaving_row, entering_col);
    } else {
      // ComputeStepToMoveBasicVariableToBound + UpdateOnPivoting
      const f64 primal_step = (s.x[lcol] - target_bound) / s.dir.values[leaving_row];
      {
        SdSubTimer t_x_(&s.phase_ticks[25]);
        for (int k = sd_lane(); k < s.dir.nnz; k += sd_lanes()) {  // distinct basic columns
          const int row = s.dir.nz[k];
          s.x[s.basis[row]] -= s.dir.values[row] * primal_step;
        }
        sd_sync();
      }
      s.x[entering_col] += primal_step;
    }
    // UpdateAndPivot (:2504-2575)
    int refactor = 0;  // 1: ForceRefactorization, 2: the same after the LU threshold bump
    if (sd_pivot(s, entering_col, leaving_row, target_bound, &refactor) != kExitNone) {
      return s.exit_code = kExitLuError;
    }
    if (refactor != 0) {
      SD_PHASE(8);
      const int st = sd_refactorize(s, refactor == 2 ? 1 : 0);
      if (st == 1) return s.exit_code = kExitLuError;
      if (st == 2) return s.exit_code = kExitResumePivot;
      rs_permute_basis(s);  // IsRefactorized() holds after a factorization
    }
    vv_set_nonbasic_from_status(s, lcol);
#if !defined(__HIP_DEVICE_COMPILE__)
    if (s.trace != nullptr) s.trace(&s);
#endif
    ++s.num_iterations;  // OnIterationDone
    ++s.iterations_done;
  }
}

}  // namespace sdual

#include "sprimal_core.h"

#endif  // MILP_SDUAL_CORE_H_
