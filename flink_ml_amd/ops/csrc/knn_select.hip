// KNN predict for any k and fp64 (K13, the paths knn.hip does not cover: k > 64 on the fused
// kernel / k > 32 on the product scan, and the fp64 parity mode).
//
// Reference: KnnModel.predictLabel (flink-ml-lib/.../classification/knn/KnnModel.java:154-194) —
// per query, dist_i = sqrt(|‖q‖² + ‖t_i‖² − 2·q·t_i|), the k smallest kept in a priority queue
// whose strict '>' replacement keeps the earlier training point among equal distances; no limit
// on k. Here G = Q·Tᵀ is one library GEMM (fp32 or fp64) over a block of queries and this kernel
// selects each row's k nearest from it by radix selection, not by a k-long sorted list per lane:
//   * one 1024-thread block per query row; the ranking key |‖q‖²+‖t‖²−2q·t| is formed on the fly
//     (sqrt is monotone: never applied) and read as its IEEE bits (non-negative: the unsigned
//     order is the numeric order, NaN last);
//   * radix passes of 11 bits over the row (LDS histogram with integer atomics, a block scan)
//     narrow down the bin of the k-th smallest key; as soon as the keys of that bin and below fit
//     the LDS (after one or two passes for continuous data: the top bits are mostly exponent) one
//     more pass collects them and a bitonic sort by (key, index) ends it. Otherwise the passes run
//     to the last digit: the k-th smallest key T and how many keys equal to T belong to the result;
//   * one pass appends every key < T; a second takes the keys equal to T in INDEX order (each
//     wave owns a contiguous segment, ranks by ballot + mbcnt after a scan of the waves' counts) —
//     the reference's tie rule;
//   * the k (key, index) pairs are bitonic-sorted in LDS by (key, index) and written out.
// The row is re-read once per pass (at most 3 + 2 for fp32 / 6 + 2 for fp64); it stays in L2 /
// the Infinity Cache for the usual query blocks.
#include "common.h"

#include <math.h>
#include <stdint.h>

namespace {

constexpr int SEL_NT = 1024;
constexpr int SEL_BITS = 11;
constexpr int SEL_NB = 1 << SEL_BITS;
constexpr int SEL_KMAX = 8192;

template <typename A>
struct SelKey;
template <>
struct SelKey<float> {
  typedef uint32_t U;
  __device__ static U bits(float v) { return __float_as_uint(fabsf(v)); }
};
template <>
struct SelKey<double> {
  typedef unsigned long long U;
  __device__ static U bits(double v) { return (U)__double_as_longlong(fabs(v)); }
};

// exclusive scan of one int per thread over the block; *total = the sum
__device__ __forceinline__ int sel_exscan(int v, int* tmp, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  if (lane == 63) tmp[w] = x;
  __syncthreads();
  if (w == 0) {
    int s = lane < SEL_NT / 64 ? tmp[lane] : 0;
#pragma unroll
    for (int o = 1; o < SEL_NT / 64; o <<= 1) {
      const int t = __shfl_up(s, o, 64);
      if (lane >= o) s += t;
    }
    if (lane < SEL_NT / 64) tmp[lane] = s;
  }
  __syncthreads();
  const int pre = w ? tmp[w - 1] : 0;
  *total = tmp[SEL_NT / 64 - 1];
  __syncthreads();
  return pre + x - v;
}

template <typename A>
__global__ __launch_bounds__(SEL_NT) void knn_select_kernel(const A* __restrict__ G, long ldg, long n,
                                                            const A* __restrict__ qn, const A* __restrict__ tn,
                                                            int k, int kp, int cap, int* __restrict__ out, long ldo) {
  typedef typename SelKey<A>::U U;
  constexpr int TOTAL = (int)sizeof(U) * 8;
  extern __shared__ __align__(16) unsigned char sel_smem[];
  int* hist = reinterpret_cast<int*>(sel_smem);              // [SEL_NB]
  U* sk = reinterpret_cast<U*>(hist + SEL_NB);               // [cap] selected keys
  int* si = reinterpret_cast<int*>(sk + cap);                // [cap] selected indices
  __shared__ int tmp[SEL_NT / 64];
  __shared__ int wcnt[SEL_NT / 64];
  __shared__ int s_digit, s_rem, s_lt, s_hbin;
  const long row = blockIdx.x;
  const A* __restrict__ g = G + row * ldg;
  const A q = qn[row];
  const int tid = threadIdx.x;
  auto key = [&](long j) -> U { return SelKey<A>::bits(q + tn[j] - (A)2 * g[j]); };

  // bitonic sort of sk/si[0, S) by (key, index), S a power of two; the first k indices out
  auto sort_and_write = [&](int S) {
    for (int size = 2; size <= S; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = tid; i < S / 2; i += SEL_NT) {
          const int a = 2 * i - (i & (stride - 1));
          const int b = a + stride;
          const bool up = (a & size) == 0;
          const U ka = sk[a], kb = sk[b];
          const int ia = si[a], ib = si[b];
          const bool gt = ka > kb || (ka == kb && ia > ib);
          if (gt == up) {
            sk[a] = kb;
            sk[b] = ka;
            si[a] = ib;
            si[b] = ia;
          }
        }
        __syncthreads();
      }
    }
    for (int i = tid; i < k; i += SEL_NT) out[row * ldo + i] = si[i];
  };
  // ---- radix select: T = the k-th smallest key, rem = how many keys equal to T are taken
  U prefix = 0;
  int rem = k;
  int hi = TOTAL;  // bits above `hi` are fixed in prefix
  while (hi > 0) {
    const int lo = hi > SEL_BITS ? hi - SEL_BITS : 0;
    const U dmask = (U)((1u << (hi - lo)) - 1u);
    for (int i = tid; i < SEL_NB; i += SEL_NT) hist[i] = 0;
    __syncthreads();
    for (long j = tid; j < n; j += SEL_NT) {
      const U u = key(j);
      if (hi == TOTAL || (u >> hi) == (prefix >> hi)) atomicAdd(&hist[(int)((u >> lo) & dmask)], 1);
    }
    __syncthreads();
    // the bin holding the rem-th smallest of the keys still in play (two bins per thread)
    const int h0 = hist[2 * tid], h1 = hist[2 * tid + 1];
    int tot;
    const int before = sel_exscan(h0 + h1, tmp, &tot);
    if (before < rem && rem <= before + h0) {
      s_digit = 2 * tid;
      s_rem = rem - before;
      s_hbin = h0;
    } else if (before + h0 < rem && rem <= before + h0 + h1) {
      s_digit = 2 * tid + 1;
      s_rem = rem - before - h0;
      s_hbin = h1;
    }
    __syncthreads();
    if ((k - s_rem) + s_hbin <= cap) {
      // the keys whose bits above `lo` are at most the k-th one's — every key below its bin plus
      // the bin itself — fit the LDS: collect them in one more pass and sort them by (key, index);
      // the first k are the answer, ties included (the usual case after one or two radix passes)
      const U top = (prefix >> lo) | (U)s_digit;
      if (tid == 0) s_lt = 0;
      __syncthreads();
      for (long j = tid; j < n; j += SEL_NT) {
        const U u = key(j);
        if ((u >> lo) <= top) {
          const int p = atomicAdd(&s_lt, 1);
          if (p < cap) {
            sk[p] = u;
            si[p] = (int)j;
          }
        }
      }
      __syncthreads();
      const int cnt = s_lt < cap ? s_lt : cap;
      int S = 2;
      while (S < cnt) S <<= 1;
      for (int i = cnt + tid; i < S; i += SEL_NT) {
        sk[i] = ~(U)0;
        si[i] = 0x7fffffff;
      }
      __syncthreads();
      sort_and_write(S);
      return;
    }
    prefix |= (U)s_digit << lo;
    rem = s_rem;
    hi = lo;
    __syncthreads();
  }
  const U T = prefix;
  const int need = rem;  // keys equal to T in the result; k − need keys are below T
  // ---- keys below T (any order), and each wave's count of keys equal to T over its segment
  if (tid == 0) s_lt = 0;
  const int lane = tid & 63, w = tid >> 6;
  const long seg = ((n + SEL_NT / 64 - 1) / (SEL_NT / 64) + 63) / 64 * 64;
  const long j0 = (long)w * seg, j1 = j0 + seg < n ? j0 + seg : n;
  __syncthreads();
  int eq = 0;
  for (long jb = j0; jb < j1; jb += 64) {
    const long j = jb + lane;
    const U u = j < j1 ? key(j) : ~(U)0;
    if (j < j1 && u < T) {
      const int p = atomicAdd(&s_lt, 1);
      if (p < kp) {
        sk[p] = u;
        si[p] = (int)j;
      }
    }
    eq += __popcll(__ballot(j < j1 && u == T));
  }
  if (lane == 0) wcnt[w] = eq;
  __syncthreads();
  // ---- the first `need` keys equal to T in index order (waves own consecutive segments)
  if (need > 0) {
    int base = 0;
    for (int i = 0; i < w; ++i) base += wcnt[i];
    const int lt = k - need;
    for (long jb = j0; jb < j1 && base < need; jb += 64) {
      const long j = jb + lane;
      const bool e = j < j1 && key(j) == T;
      const unsigned long long m = __ballot(e);
      const int r = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
      if (e && r < need) {
        sk[lt + r] = T;
        si[lt + r] = (int)j;
      }
      base += __popcll(m);
    }
  }
  // ---- pad to kp and bitonic-sort by (key, index)
  for (int i = k + tid; i < kp; i += SEL_NT) {
    sk[i] = ~(U)0;
    si[i] = 0x7fffffff;
  }
  __syncthreads();
  sort_and_write(kp);
}

}  // namespace

FMLX_API int fmlx_knn_select_max_k() { return SEL_KMAX; }

// idx[nq][k] (int32, nearest first, ties to the lower index) from the product block G[nq][n]
// (row stride ldg), the queries' and the training points' squared norms. acc_f64 selects the
// element type of G / qn / tn.
FMLX_API int fmlx_knn_select(int acc_f64, const void* G, long ldg, long nq, long n, const void* qn, const void* tn,
                             int k, int* idx, long ldo, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (k < 1 || k > SEL_KMAX || k > n || n >= (long)INT32_MAX || ldg < n || ldo < k) return -1;
  if (nq == 0) return 0;
  int kp = 1;
  while (kp < k) kp <<= 1;
  if (kp < 2) kp = 2;
  const size_t es = acc_f64 ? 8 : 4;
  const int cap = kp > 2048 ? kp : 2048;  // LDS entries: the k winners, or the two-pass candidates
  const size_t lds = (size_t)SEL_NB * 4 + (size_t)cap * (es + 4);
  if (acc_f64)
    hipLaunchKernelGGL(knn_select_kernel<double>, dim3((unsigned)nq), dim3(SEL_NT), lds, s, (const double*)G, ldg, n,
                       (const double*)qn, (const double*)tn, k, kp, cap, idx, ldo);
  else
    hipLaunchKernelGGL(knn_select_kernel<float>, dim3((unsigned)nq), dim3(SEL_NT), lds, s, (const float*)G, ldg, n,
                       (const float*)qn, (const float*)tn, k, kp, cap, idx, ldo);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
