// Categorical statistics on the device: the (feature, value, label) contingency counts of
// NaiveBayes (LIB/classification/naivebayes/NaiveBayes.java:97-107,293-360) and
// ChiSqTest (K20; LIB/stats/chisqtest/ChiSqTest.java:102-730), and the sorted distinct values /
// value codes behind them. No library sort, unique or bincount.
//
// Integer-valued data (the categorical case: LabeledPointWithWeightGenerator's featureArity /
// labelArity columns, the reference's benchmarks):
//   cs_flags   one pass over a strided [n, d] matrix: min, max and "any non-integer" (per-block
//              partials, then one block; exact, order-free);
//   cs_ihist   integer histogram of one column (labels) over [lo, lo + R): LDS-private counts
//              per block, flushed with integer atomics (exact);
//   cs_hist    counts[j][label][value − vmin] of every element (row-major, coalesced reads): the
//              table is privatised in LDS when it fits (d·L·V ≤ 32K ints: 2M × 100 × 20 values ×
//              10 labels = 20K), integer LDS atomics, one flush per block.
// Any other values: per column the stable 64-bit radix sort (radix.hip fmlx_sort_u64) of the
// ordered value bits with the row ids, then
//   cs_heads   per 4096-entry tile of the sorted columns: the number of distinct-value heads;
//   cs_scan    one block: exclusive prefix of the tile counts (the global distinct ids);
//   cs_codes   per tile: each entry's global distinct id (a block scan of the heads + the tile's
//              carry) → codes[column][row], the distinct values and their columns;
//   cs_chist   counts[code][label] of every (row, column) with integer atomics.
#include "common.h"

namespace {

constexpr int CS_THREADS = 256;
constexpr int CS_WAVES = CS_THREADS / 64;
constexpr int CS_LDS_INTS = 32 * 1024;  // privatised table: 128 KiB of LDS (one block per CU)
constexpr int CS_PER = 16;
constexpr int CS_TILE = CS_THREADS * CS_PER;

// Grid-stride walk over the row-major elements of an [n, d] matrix as (row, column) pairs: one
// 64-bit division at the start, then a constant (row, column) step with a carry — the flat index
// e / d of every element cost a 64-bit integer division each (~1.6 ms of 2M × 100).
struct FlatWalk {
  long i;
  int j;
  long di;
  int dj, d;
  __device__ FlatWalk(long n, int d_, long start, long stride) : d(d_) {
    i = start / d_;
    j = (int)(start - i * d_);
    di = stride / d_;
    dj = (int)(stride - di * d_);
    (void)n;
  }
  __device__ __forceinline__ void next() {
    i += di;
    j += dj;
    if (j >= d) {
      j -= d;
      ++i;
    }
  }
};

template <typename T>
__device__ __forceinline__ double ld_val(const T* X, long ld, long i, int j) {
  return (double)X[i * ld + j];
}

// 16 bytes of T: 4 floats or 2 doubles, loaded with one instruction
template <typename T>
struct Vec16 {
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};
template <typename T>
__device__ __forceinline__ Vec16<T> ld16(const T* p) {
  Vec16<T> r;
  *reinterpret_cast<uint4*>(r.v) = *reinterpret_cast<const uint4*>(p);
  return r;
}

__device__ __forceinline__ void flag_one(double v, double& mn, double& mx, double& non) {
  mn = v < mn ? v : mn;
  mx = v > mx ? v : mx;
  if (v != rint(v) || v - v != 0.0) non = 1.0;  // fractions, NaN (v != v), ±inf (inf − inf = NaN)
}

// part[b] = {min, max, nonint} over the block's elements. Contiguous rows (ld == d, 16-byte
// aligned): one flat stream of 16-byte loads, UNR of them in flight per thread; otherwise a
// (row, column) walk.
template <typename T>
__global__ __launch_bounds__(CS_THREADS) void cs_flags_kernel(const T* __restrict__ X, long ld, long n, int d,
                                                              double* __restrict__ part) {
  __shared__ double smin[CS_WAVES], smax[CS_WAVES], snon[CS_WAVES];
  double mn = __builtin_inf(), mx = -__builtin_inf(), non = 0.0;
  const long gt = (long)blockIdx.x * CS_THREADS + threadIdx.x, gs = (long)gridDim.x * CS_THREADS;
  if (ld == d && (((uintptr_t)X) & 15) == 0) {
    constexpr int VN = Vec16<T>::N, UNR = 4;
    const long total = n * (long)d, nv = total / VN;
    long v = gt;
    for (; v + (UNR - 1) * gs < nv; v += UNR * gs) {
      Vec16<T> q[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) q[u] = ld16(X + (v + u * gs) * VN);
#pragma unroll
      for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int c = 0; c < VN; ++c) flag_one((double)q[u].v[c], mn, mx, non);
    }
    for (; v < nv; v += gs) {
      const Vec16<T> q = ld16(X + v * VN);
#pragma unroll
      for (int c = 0; c < VN; ++c) flag_one((double)q.v[c], mn, mx, non);
    }
    for (long e = nv * VN + gt; e < total; e += gs) flag_one((double)X[e], mn, mx, non);
  } else {
    FlatWalk it(n, d, gt, gs);
    for (; it.i < n; it.next()) flag_one(ld_val(X, ld, it.i, it.j), mn, mx, non);
  }
  for (int off = 32; off > 0; off >>= 1) {
    const double a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64), c = __shfl_xor(non, off, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
    non = c > non ? c : non;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smin[w] = mn;
    smax[w] = mx;
    snon[w] = non;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < CS_WAVES; ++q) {
      mn = smin[q] < mn ? smin[q] : mn;
      mx = smax[q] > mx ? smax[q] : mx;
      non = snon[q] > non ? snon[q] : non;
    }
    part[blockIdx.x * 3 + 0] = mn;
    part[blockIdx.x * 3 + 1] = mx;
    part[blockIdx.x * 3 + 2] = non;
  }
}

__global__ __launch_bounds__(64) void cs_flags_final(const double* __restrict__ part, int nb,
                                                     double* __restrict__ out) {
  double mn = __builtin_inf(), mx = -__builtin_inf(), non = 0.0;
  for (int b = threadIdx.x; b < nb; b += 64) {
    mn = part[b * 3] < mn ? part[b * 3] : mn;
    mx = part[b * 3 + 1] > mx ? part[b * 3 + 1] : mx;
    non = part[b * 3 + 2] > non ? part[b * 3 + 2] : non;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const double a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64), c = __shfl_xor(non, off, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
    non = c > non ? c : non;
  }
  if (threadIdx.x == 0) {
    out[0] = mn;
    out[1] = mx;
    out[2] = non;
  }
}

// counts[v − lo] for the integer values of column X[:, col] (values outside [lo, lo + R) ignored)
template <typename T>
__global__ __launch_bounds__(CS_THREADS) void cs_ihist_kernel(const T* __restrict__ X, long ld, long n, int col,
                                                              long lo, int R, int* __restrict__ counts) {
  extern __shared__ int h[];
  const bool priv = R <= CS_LDS_INTS;
  if (priv)
    for (int i = threadIdx.x; i < R; i += CS_THREADS) h[i] = 0;
  __syncthreads();
  for (long i = (long)blockIdx.x * CS_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * CS_THREADS) {
    const long v = (long)ld_val(X, ld, i, col) - lo;
    if (v >= 0 && v < R) {
      if (priv)
        atomicAdd(&h[v], 1);
      else
        atomicAdd(&counts[v], 1);
    }
  }
  __syncthreads();
  if (priv)
    for (int i = threadIdx.x; i < R; i += CS_THREADS)
      if (h[i]) atomicAdd(&counts[i], h[i]);
}

// counts[(j·L + li[i])·V + (x − vmin)] over every element (li outside [0, L): row skipped).
// Privatised: the block's table lives in LDS with feature j's L·V cells at j·FS, FS = L·V rounded up
// to an odd count, so the 64 lanes of a wave — 64 consecutive elements, i.e. consecutive features —
// hit 64 different banks (an even stride put them on stride·j mod 64: 8 banks at L·V = 200).
// Contiguous rows (ld == d): 16-byte loads of the flat element stream, UNR in flight per thread,
// row = e / d by a 64-bit multiply-high with the host's magic ceil(2^64 / d) (exact for e < 2^32).
template <typename T, bool PRIV>
__global__ __launch_bounds__(CS_THREADS) void cs_hist_kernel(const T* __restrict__ X, long ld, long n, int d,
                                                             const int* __restrict__ li, int L, long vmin, int V,
                                                             int* __restrict__ counts, uint64_t magic, int FS) {
  extern __shared__ int h[];
  const long tsize = (long)d * FS;
  if (PRIV)
    for (long i = threadIdx.x; i < tsize; i += CS_THREADS) h[i] = 0;
  __syncthreads();
  const long LV = (long)L * V;
  auto add = [&](long i, int j, double x) {
    const int l = li[i];
    const long v = (long)x - vmin;
    if (l >= 0 && l < L && v >= 0 && v < V) {
      if (PRIV)
        atomicAdd(&h[(long)j * FS + (long)l * V + v], 1);
      else
        atomicAdd(&counts[(long)j * LV + (long)l * V + v], 1);
    }
  };
  const long gt = (long)blockIdx.x * CS_THREADS + threadIdx.x, gs = (long)gridDim.x * CS_THREADS;
  const long total = n * (long)d;
  if (ld == d && (((uintptr_t)X) & 15) == 0 && total < (1L << 32) && d >= Vec16<T>::N) {
    constexpr int VN = Vec16<T>::N, UNR = 4;
    const long nv = total / VN;
    auto row_of = [&](long e) -> long { return d == 1 ? e : (long)__umul64hi((uint64_t)e, magic); };
    long v = gt;
    for (; v + (UNR - 1) * gs < nv; v += UNR * gs) {
      Vec16<T> q[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) q[u] = ld16(X + (v + u * gs) * VN);
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const long e = (v + u * gs) * VN;
        long i = row_of(e);
        int j = (int)(e - i * d);
#pragma unroll
        for (int c = 0; c < VN; ++c) {
          add(i, j, (double)q[u].v[c]);
          if (++j == d) {
            j = 0;
            ++i;
          }
        }
      }
    }
    for (; v < nv; v += gs) {
      const Vec16<T> q = ld16(X + v * VN);
      const long e = v * VN;
      long i = row_of(e);
      int j = (int)(e - i * d);
#pragma unroll
      for (int c = 0; c < VN; ++c) {
        add(i, j, (double)q.v[c]);
        if (++j == d) {
          j = 0;
          ++i;
        }
      }
    }
    for (long e = nv * VN + gt; e < total; e += gs) {
      const long i = row_of(e);
      add(i, (int)(e - i * d), (double)X[e]);
    }
  } else {
    FlatWalk it(n, d, gt, gs);
    for (; it.i < n; it.next()) add(it.i, it.j, ld_val(X, ld, it.i, it.j));
  }
  __syncthreads();
  if (PRIV)
    for (long i = threadIdx.x; i < tsize; i += CS_THREADS) {
      const int j = (int)(i / FS), r = (int)(i - (long)j * FS);
      if (r < LV && h[i]) atomicAdd(&counts[(long)j * LV + r], h[i]);
    }
}

// ---- general values: ordered keys of columns [j0, j0 + nc), sorted per column ----------------
__device__ __forceinline__ uint64_t asc_key(double v) {
  if (v == 0.0) v = 0.0;  // −0 → +0
  uint64_t b = (uint64_t)__double_as_longlong(v);
  if (v != v) b = 0x7ff8000000000000ull;
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_val(uint64_t k) {
  const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

template <typename T>
__global__ __launch_bounds__(CS_THREADS) void cs_col_keys_kernel(const T* __restrict__ X, long ld, long n, int j0,
                                                                 int nc, uint64_t* __restrict__ keys,
                                                                 uint32_t* __restrict__ rows,
                                                                 unsigned long long* __restrict__ orand) {
  __shared__ unsigned long long so[CS_WAVES], sa[CS_WAVES];
  unsigned long long o = 0, a = ~0ull;
  const long total = n * (long)nc;
  for (long e = (long)blockIdx.x * CS_THREADS + threadIdx.x; e < total; e += (long)gridDim.x * CS_THREADS) {
    const long c = e / n, i = e - c * n;  // column-major output: segment c = column j0 + c
    const uint64_t k = asc_key(ld_val(X, ld, i, j0 + (int)c));
    keys[e] = k;
    rows[e] = (uint32_t)i;
    o |= k;
    a &= k;
  }
  for (int off = 32; off > 0; off >>= 1) {
    o |= __shfl_xor(o, off, 64);
    a &= __shfl_xor(a, off, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    so[w] = o;
    sa[w] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < CS_WAVES; ++q) {
      o |= so[q];
      a &= sa[q];
    }
    atomicOr(orand, o);
    atomicAnd(orand + 1, a);
  }
}

// entry e of the sorted column-major array heads a distinct value: first of its column, or a key
// different from the previous one (NaN equals NaN here: one distinct NaN per column)
__device__ __forceinline__ bool cs_head(const uint64_t* keys, long e, long n) {
  return (e % n) == 0 || keys[e] != keys[e - 1];
}

__global__ __launch_bounds__(CS_THREADS) void cs_heads_kernel(const uint64_t* __restrict__ keys, long total, long n,
                                                              long* __restrict__ tcnt) {
  __shared__ long sh[CS_WAVES];
  const long base = (long)blockIdx.x * CS_TILE;
  long c = 0;
  for (int q = 0; q < CS_PER; ++q) {
    const long e = base + (long)q * CS_THREADS + threadIdx.x;
    if (e < total && cs_head(keys, e, n)) ++c;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < CS_WAVES; ++q) c += sh[q];
    tcnt[blockIdx.x] = c;
  }
}

// one block: tcnt ← exclusive prefix; tcnt[nt] = total distinct
__global__ __launch_bounds__(1024) void cs_scan_kernel(long* __restrict__ tcnt, long nt) {
  __shared__ long s[1024];
  __shared__ long run;
  if (threadIdx.x == 0) run = 0;
  __syncthreads();
  for (long base = 0; base < nt; base += 1024) {
    const long t = base + threadIdx.x;
    s[threadIdx.x] = t < nt ? tcnt[t] : 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      long a = run;
      const long m = nt - base < 1024 ? nt - base : 1024;
      for (long i = 0; i < m; ++i) {
        const long v = s[i];
        s[i] = a;
        a += v;
      }
      run = a;
    }
    __syncthreads();
    if (t < nt) tcnt[t] = s[threadIdx.x];
    __syncthreads();
  }
  if (threadIdx.x == 0) tcnt[nt] = run;
}

// per tile: gid of every entry; codes[c·n + row] = gid − (first gid of column c); distinct values
// / columns at gid (heads only)
__global__ __launch_bounds__(CS_THREADS) void cs_codes_kernel(const uint64_t* __restrict__ keys,
                                                              const uint32_t* __restrict__ rows, long total, long n,
                                                              int j0, const long* __restrict__ tcnt,
                                                              long gid_base, int* __restrict__ codes,
                                                              double* __restrict__ uval, int* __restrict__ ucol,
                                                              long* __restrict__ colfirst) {
  __shared__ long sh[CS_WAVES];
  // the thread's CS_PER consecutive entries
  const long e0 = (long)blockIdx.x * CS_TILE + (long)threadIdx.x * CS_PER;
  int hc = 0;
  bool hd[CS_PER];
#pragma unroll
  for (int q = 0; q < CS_PER; ++q) {
    const long e = e0 + q;
    hd[q] = e < total && cs_head(keys, e, n);
    hc += hd[q];
  }
  // block exclusive scan of hc
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  long inc = hc;
  for (int off = 1; off < 64; off <<= 1) {
    const long o = __shfl_up(inc, off, 64);
    if (lane >= off) inc += o;
  }
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  long pre = 0;
  for (int q = 0; q < w; ++q) pre += sh[q];
  long g = gid_base + tcnt[blockIdx.x] + pre + inc - hc - 1;  // gid of the entry before my first
#pragma unroll
  for (int q = 0; q < CS_PER; ++q) {
    const long e = e0 + q;
    if (e < total) {
      if (hd[q]) {
        ++g;
        uval[g] = key_val(keys[e]);
        const int c = (int)(e / n);
        ucol[g] = j0 + c;
        if (e % n == 0) colfirst[c] = g;
      }
    }
  }
  // second sweep (colfirst of my column is written by the block holding the column's first
  // entry, possibly another block): codes are written as global ids here and made column-
  // relative by cs_relcodes_kernel
  g = gid_base + tcnt[blockIdx.x] + pre + inc - hc - 1;
#pragma unroll
  for (int q = 0; q < CS_PER; ++q) {
    const long e = e0 + q;
    if (e < total) {
      if (hd[q]) ++g;
      const long c = e / n;
      codes[c * n + rows[e]] = (int)g;
    }
  }
}

__global__ __launch_bounds__(CS_THREADS) void cs_relcodes_kernel(int* __restrict__ codes, long n, int nc,
                                                                 const long* __restrict__ colfirst) {
  const long total = n * (long)nc;
  for (long e = (long)blockIdx.x * CS_THREADS + threadIdx.x; e < total; e += (long)gridDim.x * CS_THREADS)
    codes[e] -= (int)colfirst[e / n];
}

// counts[(off[j] + code[j][i])·L + li[i]] += 1 for every row i, column j of the chunk
__global__ __launch_bounds__(CS_THREADS) void cs_chist_kernel(const int* __restrict__ codes, long n, int nc,
                                                              const long* __restrict__ coloff,
                                                              const int* __restrict__ li, int L,
                                                              int* __restrict__ counts) {
  const long total = n * (long)nc;
  for (long e = (long)blockIdx.x * CS_THREADS + threadIdx.x; e < total; e += (long)gridDim.x * CS_THREADS) {
    const long c = e / n, i = e - c * n;
    const int l = li[i];
    if (l >= 0 && l < L) atomicAdd(&counts[(coloff[c] + codes[e]) * (long)L + l], 1);
  }
}

inline unsigned grid_for(long work, long per_block, long cap) {
  long b = (work + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (unsigned)b;
}

}  // namespace

FMLX_API int fmlx_cs_tile() { return CS_TILE; }
FMLX_API int fmlx_cs_lds_ints() { return CS_LDS_INTS; }

// out[3] = {min, max, any non-integer (1.0) / 0.0} of X[:n, :d]; part: double[3 · 1024]
FMLX_API int fmlx_cs_flags(int dtype, const void* X, long ld, long n, int d, double* part, double* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const unsigned nb = grid_for(n * (long)d, CS_THREADS * 16L, 1024);
  if (dtype == DT_F64)
    hipLaunchKernelGGL(cs_flags_kernel<double>, dim3(nb), dim3(CS_THREADS), 0, s, (const double*)X, ld, n, d, part);
  else if (dtype == DT_F32)
    hipLaunchKernelGGL(cs_flags_kernel<float>, dim3(nb), dim3(CS_THREADS), 0, s, (const float*)X, ld, n, d, part);
  else
    return -1;
  hipLaunchKernelGGL(cs_flags_final, dim3(1), dim3(64), 0, s, part, (int)nb, out);
  return (int)hipGetLastError();
}

// counts[R] (zeroed by the caller) of the integer values of X[:, col] in [lo, lo + R)
FMLX_API int fmlx_cs_ihist(int dtype, const void* X, long ld, long n, int col, long lo, int R, int* counts,
                           void* stream) {
  if (R < 1) return -2;
  hipStream_t s = (hipStream_t)stream;
  const unsigned nb = grid_for(n, CS_THREADS * 64L, 512);
  const size_t lds = R <= CS_LDS_INTS ? (size_t)R * sizeof(int) : 0;
  if (dtype == DT_F64)
    hipLaunchKernelGGL(cs_ihist_kernel<double>, dim3(nb), dim3(CS_THREADS), lds, s, (const double*)X, ld, n, col, lo,
                       R, counts);
  else if (dtype == DT_F32)
    hipLaunchKernelGGL(cs_ihist_kernel<float>, dim3(nb), dim3(CS_THREADS), lds, s, (const float*)X, ld, n, col, lo, R,
                       counts);
  else if (dtype == DT_I32)
    hipLaunchKernelGGL(cs_ihist_kernel<int>, dim3(nb), dim3(CS_THREADS), lds, s, (const int*)X, ld, n, col, lo, R,
                       counts);
  else
    return -1;
  return (int)hipGetLastError();
}

// counts[d][L][V] (zeroed by the caller): X integer values in [vmin, vmin + V), label indices li
FMLX_API int fmlx_cs_hist(int dtype, const void* X, long ld, long n, int d, const int* li, int L, long vmin, int V,
                          int* counts, void* stream) {
  if (L < 1 || V < 1 || d < 1) return -2;
  hipStream_t s = (hipStream_t)stream;
  const long LV = (long)L * V;
  const int FS = (int)(LV | 1);  // odd feature stride in LDS
  const long tsize = (long)d * FS;
  const bool priv = tsize <= CS_LDS_INTS;
  const size_t lds = priv ? (size_t)tsize * sizeof(int) : 0;
  // ceil(2^64 / d): row = umulhi(e, magic) for e < 2^32 (d = 1 handled in the kernel)
  const uint64_t magic = d > 1 ? (uint64_t)((((unsigned __int128)1) << 64) / (unsigned)d) + 1 : 0;
  // privatised: enough blocks to fill the chip, each amortising its table over many elements
  const unsigned nb = grid_for(n * (long)d, CS_THREADS * 64L, priv ? 512 : 4096);
#define FMLX_CS_HIST(T, P)                                                                                    \
  hipLaunchKernelGGL((cs_hist_kernel<T, P>), dim3(nb), dim3(CS_THREADS), lds, s, (const T*)X, ld, n, d, li, L, \
                     vmin, V, counts, magic, FS)
  if (dtype == DT_F64) {
    if (priv) FMLX_CS_HIST(double, true); else FMLX_CS_HIST(double, false);
  } else if (dtype == DT_F32) {
    if (priv) FMLX_CS_HIST(float, true); else FMLX_CS_HIST(float, false);
  } else {
    return -1;
  }
#undef FMLX_CS_HIST
  return (int)hipGetLastError();
}

// keys / rows of columns [j0, j0 + nc) in column-major order (segment c = [c·n, (c+1)·n)) and the
// keys' {OR, AND} (orand: device, the caller fills {0, ~0})
FMLX_API int fmlx_cs_col_keys(int dtype, const void* X, long ld, long n, int j0, int nc, uint64_t* keys,
                              uint32_t* rows, unsigned long long* orand, void* stream) {
  if (n >= (1L << 32)) return -2;
  hipStream_t s = (hipStream_t)stream;
  const unsigned nb = grid_for(n * (long)nc, CS_THREADS * 8L, 4096);
  if (dtype == DT_F64)
    hipLaunchKernelGGL(cs_col_keys_kernel<double>, dim3(nb), dim3(CS_THREADS), 0, s, (const double*)X, ld, n, j0, nc,
                       keys, rows, orand);
  else if (dtype == DT_F32)
    hipLaunchKernelGGL(cs_col_keys_kernel<float>, dim3(nb), dim3(CS_THREADS), 0, s, (const float*)X, ld, n, j0, nc,
                       keys, rows, orand);
  else
    return -1;
  return (int)hipGetLastError();
}

// Distinct values of the sorted columns (keys / rows as sorted by fmlx_sort_u64, nc segments of n):
// tcnt int64[ntiles + 1] scratch (tiles of fmlx_cs_tile()); after the call tcnt[ntiles] = number of
// distinct (column, value) pairs U (read it before sizing uval / ucol for the NEXT step: this call
// writes uval[gid_base + g] / ucol[...] for g < U, so the caller sizes them for n·nc).
FMLX_API int fmlx_cs_distinct(const uint64_t* keys, const uint32_t* rows, long n, int nc, int j0, long* tcnt,
                              long gid_base, int* codes, double* uval, int* ucol, long* colfirst, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const long total = n * (long)nc;
  if (total <= 0) return 0;
  const long nt = (total + CS_TILE - 1) / CS_TILE;
  hipLaunchKernelGGL(cs_heads_kernel, dim3((unsigned)nt), dim3(CS_THREADS), 0, s, keys, total, n, tcnt);
  hipLaunchKernelGGL(cs_scan_kernel, dim3(1), dim3(1024), 0, s, tcnt, nt);
  hipLaunchKernelGGL(cs_codes_kernel, dim3((unsigned)nt), dim3(CS_THREADS), 0, s, keys, rows, total, n, j0, tcnt,
                     gid_base, codes, uval, ucol, colfirst);
  hipLaunchKernelGGL(cs_relcodes_kernel, dim3(grid_for(total, CS_THREADS * 8L, 4096)), dim3(CS_THREADS), 0, s, codes,
                     n, nc, colfirst);
  return (int)hipGetLastError();
}

// counts[(coloff[c] + codes[c][i])·L + li[i]] += 1 (counts zeroed by the caller)
FMLX_API int fmlx_cs_chist(const int* codes, long n, int nc, const long* coloff, const int* li, int L, int* counts,
                           void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const long total = n * (long)nc;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(cs_chist_kernel, dim3(grid_for(total, CS_THREADS * 8L, 4096)), dim3(CS_THREADS), 0, s, codes, n,
                     nc, coloff, li, L, counts);
  return (int)hipGetLastError();
}

// ---- bounded distinct counts per column (VectorIndexer.java:96-106: a column is categorical when
// it holds at most maxCategories distinct values). Only "how many, up to cap" is needed: per
// (row chunk, column) block an LDS hash set of 64-bit keys (NaN canonical, −0 folded into +0 — the
// keys of the later keyed distinct), merged into one global set per column; a column whose count
// passes cap raises its flag and every block drops it at the next check, so a continuous column
// costs a few hundred rows instead of a full sort. Probing is bounded by the table size.
namespace {
constexpr unsigned long long SD_EMPTY = ~0ull;  // a NaN payload the key canonicalisation never yields
constexpr int SD_MAXCAP = 1024;
__device__ __forceinline__ unsigned long long sd_key(double v) {
  if (v != v) return 0x7ff8000000000000ull;
  return (unsigned long long)__double_as_longlong(v + 0.0);
}
__device__ __forceinline__ unsigned sd_hash(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (unsigned)k;
}
// 0 = present already, 1 = inserted, 2 = table full
__device__ __forceinline__ int sd_insert(unsigned long long* tab, int S, unsigned long long k) {
  unsigned h = sd_hash(k) & (unsigned)(S - 1);
  for (int t = 0; t < S; ++t) {
    const unsigned long long old = atomicCAS(&tab[h], SD_EMPTY, k);
    if (old == SD_EMPTY) return 1;
    if (old == k) return 0;
    h = (h + 1) & (unsigned)(S - 1);
  }
  return 2;
}
__global__ __launch_bounds__(256) void small_distinct_kernel(const double* __restrict__ X, long ld, long n, int d,
                                                             long rows_per_block, int cap, int S,
                                                             unsigned long long* __restrict__ gtab,
                                                             int* __restrict__ gcnt, int* __restrict__ over) {
  __shared__ unsigned long long tab[2 * SD_MAXCAP + 512];
  __shared__ int cnt, stop;
  const int c = blockIdx.y;
  for (int i = threadIdx.x; i < S; i += blockDim.x) tab[i] = SD_EMPTY;
  if (threadIdx.x == 0) {
    cnt = 0;
    stop = 0;
  }
  __syncthreads();
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = r0 + rows_per_block < n ? r0 + rows_per_block : n;
  volatile int* vover = over;
  volatile int* vstop = &stop;
  for (long base = r0; base < r1; base += 256 * 16) {
    if (threadIdx.x == 0 && vover[c]) stop = 1;
    __syncthreads();
    if (stop) break;
    for (int u = 0; u < 16; ++u) {
      if (*vstop) break;  // (no inserts past the overflow: a full table would cost S probes each)
      const long r = base + (long)u * 256 + threadIdx.x;
      if (r < r1) {
        const int res = sd_insert(tab, S, sd_key(X[r * ld + c]));
        if (res == 2 || (res == 1 && atomicAdd(&cnt, 1) + 1 > cap)) {
          stop = 1;
          atomicOr(&over[c], 1);
        }
      }
    }
    __syncthreads();
  }
  __syncthreads();
  if (stop || vover[c]) return;
  // merge into the column's global set
  unsigned long long* gt = gtab + (long)c * S;
  for (int i = threadIdx.x; i < S; i += blockDim.x) {
    const unsigned long long k = tab[i];
    if (k == SD_EMPTY) continue;
    const int res = sd_insert(gt, S, k);
    if (res == 2 || (res == 1 && atomicAdd(&gcnt[c], 1) + 1 > cap)) atomicOr(&over[c], 1);
  }
}
}  // namespace

FMLX_API int fmlx_cs_small_distinct_maxcap() { return SD_MAXCAP; }

// X f64 [n, d] (row stride ld); cap <= 1024. gtab u64 [d][S] filled with ~0, gcnt / over int [d]
// zeroed by the caller, S = the power of two >= 2·cap + 256 (passed in, checked). Afterwards a
// column holds gcnt distinct values, or more than cap if over != 0.
FMLX_API int fmlx_cs_small_distinct(const double* X, long ld, long n, int d, int cap, int S, unsigned long long* gtab,
                                    int* gcnt, int* over, void* stream) {
  if (n <= 0 || d <= 0) return 0;
  if (X == nullptr || cap < 1 || cap > SD_MAXCAP || S < 2 * cap + 256 || S > 2 * SD_MAXCAP + 512 || (S & (S - 1)) ||
      d > 65535 || gtab == nullptr || gcnt == nullptr || over == nullptr)
    return -1;
  long want = 2048 / d + 1;
  long chunks = (n + 4095) / 4096;
  if (chunks > want) chunks = want;
  const long rpb = (n + chunks - 1) / chunks;
  chunks = (n + rpb - 1) / rpb;
  hipLaunchKernelGGL(small_distinct_kernel, dim3((unsigned)chunks, (unsigned)d), dim3(256), 0, (hipStream_t)stream, X,
                     ld, n, d, rpb, cap, S, gtab, gcnt, over);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
