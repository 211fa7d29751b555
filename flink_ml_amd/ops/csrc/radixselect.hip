// Multi-quantile radix-select histograms (the exact replacement for the
// reference's per-column QuantileSummary aggregate in RobustScaler/Imputer, RobustScaler.java:82,
// 114-140).
//
// Each value maps to an order-preserving unsigned key (fp32 -> u32, fp64 -> u64: sign bit set ->
// flip all bits, else flip the sign bit). One pass histograms the 8-bit digit at `shift` of every
// key whose higher digits equal the prefix selected so far — for Q quantiles of every column at
// once. The host picks the digit holding each target rank and extends the prefix; 4 (fp32) or 8
// (fp64) streaming passes over X give the exact k-th smallest values, with only Q·d·256 counts per
// pass to all-reduce across ranks.
//
// Block = 16 columns × 16 row lanes (256 threads); LDS histogram [Q][16][256] u32 with LDS
// atomics (only lanes of the same column collide: 4 per wave); per-(row chunk) partial histograms
// are written out plainly and summed in chunk order by a second kernel (no global atomics,
// deterministic). NaNs are skipped.
#include "common.h"

namespace {
constexpr int kCols = 16;
constexpr int kRows = 16;
constexpr int kBins = 256;
constexpr int kMaxQ = 4;
constexpr int kUnroll = 8;

template <typename T> struct Key;
template <> struct Key<float> {
  typedef uint32_t U;
  static __device__ __forceinline__ bool ok(float v) { return v == v; }
  static __device__ __forceinline__ float nan() { return __builtin_nanf(""); }
  static __device__ __forceinline__ U get(float v) {
    const uint32_t b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
  }
};
template <> struct Key<double> {
  typedef unsigned long long U;
  static __device__ __forceinline__ bool ok(double v) { return v == v; }
  static __device__ __forceinline__ double nan() { return __builtin_nan(""); }
  static __device__ __forceinline__ U get(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
  }
};

template <typename T>
__global__ __launch_bounds__(256) void radix_hist_kernel(const T* __restrict__ X, long ld, long n, int d,
                                                        const long long* __restrict__ prefix, int Q, int shift,
                                                        int match_all, long rows_per_chunk,
                                                        uint32_t* __restrict__ part) {
  typedef typename Key<T>::U U;
  __shared__ uint32_t h[kMaxQ * kCols * kBins];
  const int tid = threadIdx.x;
  const int lc = tid % kCols, lr = tid / kCols;
  const int c = blockIdx.y * kCols + lc;
  const long chunk = blockIdx.x;
  for (int i = tid; i < Q * kCols * kBins; i += 256) h[i] = 0;
  U pre[kMaxQ];
#pragma unroll
  for (int q = 0; q < kMaxQ; ++q) pre[q] = (q < Q && c < d) ? (U)prefix[(long)q * d + c] : (U)0;
  __syncthreads();
  const int hs = shift + 8;
  if (c < d) {
    const long r0 = chunk * rows_per_chunk;
    long r1 = r0 + rows_per_chunk;
    if (r1 > n) r1 = n;
    // kUnroll independent loads in flight per thread before the LDS atomics that consume them
    for (long r = r0 + lr; r < r1; r += (long)kRows * kUnroll) {
      T v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const long rr = r + (long)u * kRows;
        v[u] = rr < r1 ? X[rr * ld + c] : Key<T>::nan();
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (!Key<T>::ok(v[u])) continue;
        const U key = Key<T>::get(v[u]);
        const int dig = (int)((key >> shift) & 0xFF);
        const U hi = match_all ? (U)0 : (key >> hs);
#pragma unroll
        for (int q = 0; q < kMaxQ; ++q)
          if (q < Q && (match_all || hi == pre[q])) atomicAdd(&h[(q * kCols + lc) * kBins + dig], 1u);
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < Q * kCols * kBins; i += 256) {
    const int q = i / (kCols * kBins), l = (i / kBins) % kCols, bin = i % kBins;
    const int cc = blockIdx.y * kCols + l;
    if (cc < d) part[((chunk * Q + q) * (long)d + cc) * kBins + bin] = h[i];
  }
}

__global__ __launch_bounds__(256) void radix_combine_kernel(const uint32_t* __restrict__ part, long chunks,
                                                           long rec, long long* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rec) return;
  long long s = 0;
  for (long k = 0; k < chunks; ++k) s += part[k * rec + i];
  out[i] = s;
}
}  // namespace

// X [n, d] row-major (stride ld); prefix [Q][d] key bits selected so far (ignored when
// match_all); part scratch [chunks][Q][d][256] u32; out [Q][d][256] int64.
FMLX_API int fmlx_radix_hist(int dtype, const void* X, long ld, long n, int d, const long long* prefix, int Q,
                             int shift, int match_all, long chunks, uint32_t* part, long long* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (Q < 1 || Q > kMaxQ || d < 1 || chunks < 1 || (shift & 7)) return -1;
  const long rpc = (n + chunks - 1) / chunks;
  dim3 grid((unsigned)chunks, (unsigned)((d + kCols - 1) / kCols));
  if (dtype == DT_F32)
    hipLaunchKernelGGL(radix_hist_kernel<float>, grid, dim3(256), 0, s, (const float*)X, ld, n, d, prefix, Q, shift,
                       match_all, rpc, part);
  else if (dtype == DT_F64)
    hipLaunchKernelGGL(radix_hist_kernel<double>, grid, dim3(256), 0, s, (const double*)X, ld, n, d, prefix, Q,
                       shift, match_all, rpc, part);
  else
    return -1;
  const long rec = (long)Q * d * kBins;
  hipLaunchKernelGGL(radix_combine_kernel, dim3((unsigned)((rec + 255) / 256)), dim3(256), 0, s, part, chunks, rec,
                     out);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
