// Column statistics and per-column affine transforms.
//
// Reference hot loops: StandardScaler ComputeMetaOperator (sum, Σx², n — StandardScaler.java:75-140),
// MinMaxScaler min/max (MinMaxScaler.java:88-98), MaxAbsScaler max|x| (MaxAbsScaler.java:78-82),
// VarianceThresholdSelector (sum, Σx², n — VarianceThresholdSelector.java:73), and the per-row
// Model.map functions that scale/offset each coordinate (StandardScalerModel, MinMaxScalerModel,
// MaxAbsScalerModel, RobustScalerModel, ElementwiseProduct).
//
// MI355X design: one pass over the row-major [n, d] matrix; a block owns a contiguous row range
// and each thread owns columns (c = tid, tid + 256, ...), so every row is read as one coalesced
// segment. Accumulation in fp64 registers (exact enough for 10M-row sums); one fp64 partial
// record [sum | sumsq | min | max] per block, combined in block order (deterministic) by a
// second tiny kernel. The affine kernel fuses (x - sub) * mul + add per column.
#include "common.h"

namespace {

template <typename T>
__global__ __launch_bounds__(256) void colstats_partial_kernel(const T* __restrict__ X, long ld, long n, int d,
                                                               long rows_per_block, double* __restrict__ part) {
  const long r0 = (long)blockIdx.x * rows_per_block;
  long r1 = r0 + rows_per_block;
  if (r1 > n) r1 = n;
  double* out = part + (long)blockIdx.x * 4 * d;
  for (int c = threadIdx.x; c < d; c += blockDim.x) {
    double s = 0, q = 0, mn = __builtin_huge_val(), mx = -__builtin_huge_val();
    long r = r0;
    for (; r + 4 <= r1; r += 4) {
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = (double)Ld<T>::f(X[(r + u) * ld + c]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += v[u];
        q += v[u] * v[u];
        mn = v[u] < mn ? v[u] : mn;
        mx = v[u] > mx ? v[u] : mx;
      }
    }
    for (; r < r1; ++r) {
      const double v = (double)Ld<T>::f(X[r * ld + c]);
      s += v;
      q += v * v;
      mn = v < mn ? v : mn;
      mx = v > mx ? v : mx;
    }
    out[c] = s;
    out[d + c] = q;
    out[2 * d + c] = mn;
    out[3 * d + c] = mx;
  }
}

__global__ __launch_bounds__(256) void colstats_combine_kernel(const double* __restrict__ part, int nb, int d,
                                                               double* __restrict__ res) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  double s = 0, q = 0, mn = __builtin_huge_val(), mx = -__builtin_huge_val();
  for (int b = 0; b < nb; ++b) {
    const double* p = part + (long)b * 4 * d;
    s += p[c];
    q += p[d + c];
    mn = p[2 * d + c] < mn ? p[2 * d + c] : mn;
    mx = p[3 * d + c] > mx ? p[3 * d + c] : mx;
  }
  res[c] = s;
  res[d + c] = q;
  res[2 * d + c] = mn;
  res[3 * d + c] = mx;
}

template <typename T, typename O>
__global__ __launch_bounds__(256) void affine_cols_kernel(const T* __restrict__ X, long ld, long n, int d,
                                                          const double* __restrict__ sub,
                                                          const double* __restrict__ mul,
                                                          const double* __restrict__ add, O* __restrict__ out) {
  const long total = n * (long)d;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / d;
    const int c = (int)(i - r * d);
    double v = (double)Ld<T>::f(X[r * ld + c]);
    if (sub) v -= sub[c];
    if (mul) v *= mul[c];
    if (add) v += add[c];
    out[i] = (O)v;
  }
}

template <typename T>
int launch_stats(const void* X, long ld, long n, int d, double* part, int nb, double* res, hipStream_t s) {
  const long rpb = (n + nb - 1) / nb;
  hipLaunchKernelGGL(colstats_partial_kernel<T>, dim3(nb), dim3(256), 0, s, (const T*)X, ld, n, d, rpb, part);
  hipLaunchKernelGGL(colstats_combine_kernel, dim3((d + 255) / 256), dim3(256), 0, s, part, nb, d, res);
  return (int)hipGetLastError();
}

template <typename T, typename O>
int launch_affine(const void* X, long ld, long n, int d, const double* sub, const double* mul, const double* add,
                  void* out, hipStream_t s) {
  long total = n * (long)d;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) return 0;
  hipLaunchKernelGGL((affine_cols_kernel<T, O>), dim3(blocks), dim3(256), 0, s, (const T*)X, ld, n, d, sub, mul, add,
                     (O*)out);
  return (int)hipGetLastError();
}

}  // namespace

// part: scratch [nb][4][d] fp64; res: [4][d] fp64 = sum | sumsq | min | max
FMLX_API int fmlx_colstats(int dtype, const void* X, long ld, long n, int d, double* part, int nb, double* res,
                           void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (nb < 1) return -1;
  if (dtype == DT_F32) return launch_stats<float>(X, ld, n, d, part, nb, res, s);
  if (dtype == DT_F64) return launch_stats<double>(X, ld, n, d, part, nb, res, s);
  if (dtype == DT_BF16) return launch_stats<bf16_t>(X, ld, n, d, part, nb, res, s);
  return -1;
}

// out[r, c] = ((x - sub[c]) * mul[c]) + add[c]   (any of sub/mul/add may be null); out is dense [n, d]
FMLX_API int fmlx_affine_cols(int dtype, int out_dtype, const void* X, long ld, long n, int d, const double* sub,
                              const double* mul, const double* add, void* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DT_F32 && out_dtype == DT_F32) return launch_affine<float, float>(X, ld, n, d, sub, mul, add, out, s);
  if (dtype == DT_F64 && out_dtype == DT_F64)
    return launch_affine<double, double>(X, ld, n, d, sub, mul, add, out, s);
  if (dtype == DT_BF16 && out_dtype == DT_F32)
    return launch_affine<bf16_t, float>(X, ld, n, d, sub, mul, add, out, s);
  if (dtype == DT_F32 && out_dtype == DT_F64)
    return launch_affine<float, double>(X, ld, n, d, sub, mul, add, out, s);
  return -1;
}

// ---- Bucketizer (Bucketizer.java:118-143 with Bucketizer's binarySearch semantics): one pass
// per column instead of searchsorted + ~10 elementwise torch passes. For split points s[0..m):
// pos = the first index with s[pos] >= x; an exact hit maps to pos (the last split to m − 2),
// anything else to pos − 1; NaN and values outside [s[0], s[m−1]] are invalid — counted in
// *ninv, flagged in inv[] (when given) and, with keep_invalid, mapped to bucket m − 1. The splits
// stay in LDS (m <= BKZ_LDS) or are read from global memory.
namespace {
constexpr int BKZ_LDS = 4096;
__global__ __launch_bounds__(256) void bucketize_kernel(const double* __restrict__ x, long n,
                                                        const double* __restrict__ sp, int m, int keep_invalid,
                                                        double* __restrict__ out, unsigned char* __restrict__ inv,
                                                        int* __restrict__ ninv) {
  __shared__ double ls[BKZ_LDS];
  const bool in_lds = m <= BKZ_LDS;
  if (in_lds)
    for (int i = threadIdx.x; i < m; i += blockDim.x) ls[i] = sp[i];
  __syncthreads();
  const double* s = in_lds ? ls : sp;
  int bad = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const double v = x[i];
    int lo = 0, hi = m;  // lower bound: first s[pos] >= v (NaN: no s[mid] < v holds -> 0; flagged below)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s[mid] < v)
        lo = mid + 1;
      else
        hi = mid;
    }
    const int pos = lo;
    const bool exact = pos < m && s[pos] == v;
    const bool invalid = v != v || (!exact && (pos == 0 || pos == m));
    double b = exact ? (double)(pos == m - 1 ? pos - 1 : pos) : (double)(pos - 1);
    if (invalid && keep_invalid) b = (double)(m - 1);
    out[i] = b;
    if (inv) inv[i] = invalid ? 1 : 0;
    bad += invalid ? 1 : 0;
  }
  // per-wave sum, one vector atomic per wave with invalid values
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(ninv, bad);
}
}  // namespace

FMLX_API int fmlx_bucketize(const double* x, long n, const double* splits, int m, int keep_invalid, double* out,
                            unsigned char* inv, int* ninv, void* stream) {
  if (n <= 0) return 0;
  if (x == nullptr || splits == nullptr || m < 1 || out == nullptr || ninv == nullptr) return -1;
  const long want = (n + 255) / 256;
  const int blocks = (int)(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(bucketize_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, n, splits, m, keep_invalid,
                     out, inv, ninv);
  return (int)hipGetLastError();
}

// ---- Imputer mean strategy (Imputer.java:140-170): sum and count of the values that are neither
// NaN nor missingValue, without materialising the filtered column. Block partials in a fixed
// order, then one block folds them in block order: deterministic run to run.
namespace {
constexpr int MSUM_BLOCKS = 1024;
__device__ __forceinline__ void block_sum2(double& a, double& b, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[w] = a;
    sh[nw + w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a = 0.0;
    b = 0.0;
    for (int i = 0; i < nw; ++i) {
      a += sh[i];
      b += sh[nw + i];
    }
  }
}
__global__ __launch_bounds__(256) void masked_sum_kernel(const double* __restrict__ x, long n, double missing,
                                                         int miss_nan, double* __restrict__ part) {
  __shared__ double sh[8];
  double s = 0.0, c = 0.0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const double v = x[i];
    const bool skip = v != v || (!miss_nan && v == missing);
    s += skip ? 0.0 : v;
    c += skip ? 0.0 : 1.0;
  }
  block_sum2(s, c, sh);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s;
    part[2 * blockIdx.x + 1] = c;
  }
}
__global__ __launch_bounds__(256) void fold_pairs_kernel(const double* __restrict__ part, int np, double* __restrict__ out) {
  __shared__ double sh[8];
  double s = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    s += part[2 * i];
    c += part[2 * i + 1];
  }
  block_sum2(s, c, sh);
  if (threadIdx.x == 0) {
    out[0] = s;
    out[1] = c;
  }
}
}  // namespace

// out[2] = (sum, count) of x's entries that are not NaN and (unless miss_nan) != missing;
// part: scratch of 2 * 1024 doubles
FMLX_API int fmlx_masked_sum_f64(const double* x, long n, double missing, int miss_nan, double* part, double* out,
                                 void* stream) {
  if (x == nullptr && n > 0) return -1;
  if (part == nullptr || out == nullptr) return -1;
  const long want = (n + 255) / 256;
  const int blocks = (int)(want < 1 ? 1 : (want < MSUM_BLOCKS ? want : MSUM_BLOCKS));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(masked_sum_kernel, dim3(blocks), dim3(256), 0, st, x, n, missing, miss_nan, part);
  hipLaunchKernelGGL(fold_pairs_kernel, dim3(1), dim3(256), 0, st, part, blocks, out);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
