// KNN predict (K13): distance epilogue + per-query top-k over the query×train product.
//
// Reference: KnnModel.predictLabel (flink-ml-lib/.../classification/knn/KnnModel.java:154-194)
// computes, per query, gemv(T, q) → dist_i = sqrt(|‖q‖² + ‖t_i‖² − 2·q·t_i|) and keeps the k
// smallest in a priority queue (strict '>' replacement ⇒ among equal distances the earlier
// training point stays).
//
// Here the product G = Q·Tᵀ is one library GEMM (hipBLASLt, fp32) over a block of queries, and
// this kernel is everything after it, reading G exactly once:
//   * one wave64 per query row; lane l streams columns l·4 + 256·it (+0..3) with 16-B loads, so
//     each lane sees its columns in increasing index order;
//   * the ranking key |‖q‖²+‖t‖²−2q·t| is formed in registers (no broadcast matrix, no abs or
//     sqrt passes; sqrt is monotone, so it is applied to the k winners only);
//   * every lane keeps a sorted (dist, index) list of length K in VGPRs (fully unrolled
//     compare-exchange insertion, no scratch); with strict '<' and increasing indices the list
//     is ordered lexicographically by (dist, index) — the reference's tie rule;
//   * the 64 lane lists are merged by k rounds of a butterfly (dist, index) arg-min; the lane
//     that owns the winner pops its head.
//   * each row's columns are split over S waves (stage 1) whose k-best candidates a second
//     wave per row merges (stage 2); elements are admitted only below a wave-wide bound (see
//     wave_bound) so the insertion sort rarely runs.
#include "common.h"

#include <math.h>

namespace {

__device__ __forceinline__ bool lex_less(float da, int ia, float db, int ib) {
  return da < db || (da == db && ia < ib);
}

template <int K>
__device__ __forceinline__ void topk_insert(float (&bd)[K], int (&bi)[K], float d, int j) {
  // (d, j) < tail already checked; drop the tail, bubble the new element up in (dist, index)
  // order (an equal distance seen later keeps its place behind the earlier one)
  bd[K - 1] = d;
  bi[K - 1] = j;
#pragma unroll
  for (int i = K - 1; i > 0; --i) {
    if (lex_less(bd[i], bi[i], bd[i - 1], bi[i - 1])) {
      float td = bd[i]; bd[i] = bd[i - 1]; bd[i - 1] = td;
      int ti = bi[i]; bi[i] = bi[i - 1]; bi[i - 1] = ti;
    }
  }
}

// Merge the 64 lane lists of one wave into the k best (dist, index) pairs, written with
// stride 1 at od/oi (lane 0 writes).
template <int K, bool SQRT>
__device__ __forceinline__ void wave_merge_out(float (&bd)[K], int (&bi)[K], int lane, int k, float* od, int* oi) {
  for (int t = 0; t < k; ++t) {
    float wd = bd[0];
    int wi = bi[0];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float xd = __shfl_xor(wd, off, 64);
      const int xi = __shfl_xor(wi, off, 64);
      if (lex_less(xd, xi, wd, wi)) { wd = xd; wi = xi; }
    }
    if (lane == 0) {
      oi[t] = wi;
      if (od) od[t] = SQRT ? __builtin_sqrtf(wd) : wd;
    }
    if (bi[0] == wi && wi != INT32_MAX) {  // (dist, index) pairs are unique: one lane pops
#pragma unroll
      for (int i = 0; i < K - 1; ++i) { bd[i] = bd[i + 1]; bi[i] = bi[i + 1]; }
      bd[K - 1] = INFINITY;
      bi[K - 1] = INT32_MAX;
    }
  }
}

// Ranking key |‖q‖² + ‖t‖² − 2·q·t|: sqrt is monotone, so the k nearest by key are the k nearest by
// distance (ties → lower index either way); the sqrt is only taken for the k outputs.
__device__ __forceinline__ float knn_key(float q, float t, float g) {
  const float d = fabsf((q + t) - 2.0f * g);
  return __builtin_isnan(d) ? INFINITY : d;
}

// Wave-wide admission bound: the lexicographic min over lanes of each lane's k-th best. Any
// lane's k-th best bounds the wave's k-th best from above (that lane alone holds k entries at or
// below it), so an element that is not below the min can never reach the wave's top-k. This cuts
// insertions from ~64·k/j per element (a per-lane bound over 1/64 of the stream) to ~k/j, which
// is what keeps the scan memory-bound for k up to 32. The bound goes stale between refreshes
// (it only ever loosens relative to the lane's own list), so admission also checks the lane tail.
template <int K>
__device__ __forceinline__ void wave_bound(const float (&bd)[K], const int (&bi)[K], int k, float& td, int& ti) {
  td = bd[0];
  ti = bi[0];
#pragma unroll
  for (int i = 1; i < K; ++i)
    if (i == k - 1) { td = bd[i]; ti = bi[i]; }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float xd = __shfl_xor(td, off, 64);
    const int xi = __shfl_xor(ti, off, 64);
    if (lex_less(xd, xi, td, ti)) { td = xd; ti = xi; }
  }
}

// Stage 1: wave (row, segment) scans columns [seg·L, (seg+1)·L) of its row and emits that
// segment's k best. With S == 1 it writes the final answer; otherwise a candidate block that
// stage 2 merges. Several waves per row keep ≫ 1 load in flight per CU even for small query
// blocks (one wave per row left the kernel latency-bound).
template <int K, bool VEC>
__global__ __launch_bounds__(256) void knn_topk_scan_kernel(const float* __restrict__ G, long ldg, long nq, long n,
                                                            int S, const float* __restrict__ qn,
                                                            const float* __restrict__ tn, int k,
                                                            int* __restrict__ out_i, float* __restrict__ out_d) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int seg = blockIdx.y;
  if (row >= nq) return;  // whole wave leaves together; no block barriers below

  float bd[K];
  int bi[K];
#pragma unroll
  for (int i = 0; i < K; ++i) { bd[i] = INFINITY; bi[i] = INT32_MAX; }
  // empty slots are (inf, INT32_MAX): every real (dist, index) sorts before them, infinite
  // distances included; a NaN distance is ranked as +inf (torch.topk also ranks NaN last).
  // All comparisons are lexicographic on (dist, index), so ties go to the lower index no
  // matter in which order a lane meets them.

  const float* g = G + row * ldg;
  const float q = qn[row];
  if constexpr (VEC) {
    typedef float f32x4_t __attribute__((ext_vector_type(4)));
    const long n4 = n >> 2;
    const long L = (n4 + S - 1) / S;
    const long c0 = seg * L, c1 = c0 + L < n4 ? c0 + L : n4;
    const f32x4_t* g4 = reinterpret_cast<const f32x4_t*>(g);
    const f32x4_t* t4 = reinterpret_cast<const f32x4_t*>(tn);
    long c = c0 + lane;
    float td = INFINITY;
    int ti = INT32_MAX;
    // U chunks (4·U keys) in flight per lane; one wave-uniform branch per block of 4·U keys
    // skips the insertion code unless some lane has a key at or below the bound. The trip
    // count is wave-uniform so the shuffles in wave_bound see every lane.
    constexpr int U = K >= 16 ? 2 : 4;  // long lists: fewer keys in flight, fewer VGPRs
    const long iters = (c1 - c0) / (64 * U);
    for (long it = 0; it < iters; ++it, c += 64 * U) {
      f32x4_t gv[U], tv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) gv[u] = __builtin_nontemporal_load(g4 + c + 64 * u);
#pragma unroll
      for (int u = 0; u < U; ++u) tv[u] = t4[c + 64 * u];
      float key[4 * U];
      float m = INFINITY;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          key[4 * u + e] = knn_key(q, tv[u][e], gv[u][e]);
          m = fminf(m, key[4 * u + e]);
        }
      if (m <= td) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = key[4 * u + e];
            const int j = (int)((c + 64 * u) * 4 + e);
            if (lex_less(d, j, td, ti) && lex_less(d, j, bd[K - 1], bi[K - 1])) topk_insert<K>(bd, bi, d, j);
          }
      }
      wave_bound<K>(bd, bi, k, td, ti);
    }
    for (; c < c1; c += 64) {
      const f32x4_t ga = __builtin_nontemporal_load(g4 + c);
      const f32x4_t ta = t4[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = knn_key(q, ta[e], ga[e]);
        const int j = (int)(c * 4 + e);
        if (lex_less(d, j, td, ti) && lex_less(d, j, bd[K - 1], bi[K - 1])) topk_insert<K>(bd, bi, d, j);
      }
    }
  } else {
    const long L = (n + S - 1) / S;
    const long j0 = seg * L, j1 = j0 + L < n ? j0 + L : n;
    for (long j = j0 + lane; j < j1; j += 64) {
      const float d = knn_key(q, tn[j], g[j]);
      if (lex_less(d, (int)j, bd[K - 1], bi[K - 1])) topk_insert<K>(bd, bi, d, (int)j);
    }
  }
  const long o = (row * S + seg) * k;
  if (S == 1)
    wave_merge_out<K, true>(bd, bi, lane, k, out_d ? out_d + o : nullptr, out_i + o);
  else  // candidates keep the raw key for stage 2
    wave_merge_out<K, false>(bd, bi, lane, k, out_d + o, out_i + o);
}

// Stage 2: wave per row merges the S·k segment candidates (lexicographic (dist, index), so the
// reference's tie rule survives the split).
template <int K>
__global__ __launch_bounds__(256) void knn_topk_merge_kernel(const float* __restrict__ cd, const int* __restrict__ ci,
                                                             long nq, int S, int k, int* __restrict__ out_i,
                                                             float* __restrict__ out_d) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nq) return;
  float bd[K];
  int bi[K];
#pragma unroll
  for (int i = 0; i < K; ++i) { bd[i] = INFINITY; bi[i] = INT32_MAX; }
  const long m = (long)S * k;
  for (long c = lane; c < m; c += 64) {
    const float d = cd[row * m + c];
    const int j = ci[row * m + c];
    if (lex_less(d, j, bd[K - 1], bi[K - 1])) topk_insert<K>(bd, bi, d, j);
  }
  wave_merge_out<K, true>(bd, bi, lane, k, out_d ? out_d + row * k : nullptr, out_i + row * k);
}

template <int K>
int launch_topk(const float* G, long ldg, long nq, long n, int S, const float* qn, const float* tn, int k, int* idx,
                float* dist, float* ws_d, int* ws_i, hipStream_t s) {
  const int blocks = fmlx_ceil_div(nq, 4);
  const bool vec = (n % 4 == 0) && (ldg % 4 == 0) && ((uintptr_t)G % 16 == 0) && ((uintptr_t)tn % 16 == 0);
  int* si = S > 1 ? ws_i : idx;
  float* sd = S > 1 ? ws_d : dist;
  if (vec)
    hipLaunchKernelGGL((knn_topk_scan_kernel<K, true>), dim3(blocks, S), dim3(256), 0, s, G, ldg, nq, n, S, qn, tn,
                       k, si, sd);
  else
    hipLaunchKernelGGL((knn_topk_scan_kernel<K, false>), dim3(blocks, S), dim3(256), 0, s, G, ldg, nq, n, S, qn, tn,
                       k, si, sd);
  if (S > 1)
    hipLaunchKernelGGL((knn_topk_merge_kernel<K>), dim3(blocks), dim3(256), 0, s, ws_d, ws_i, nq, S, k, idx, dist);
  FMLX_CHECK_LAUNCH();
}

}  // namespace

// Largest k the kernel handles (callers fall back to a sort above it).
FMLX_API int fmlx_knn_topk_max_k() { return 32; }

// G: [nq, n] fp32 row-major (leading dim ldg) = Q·Tᵀ; qn [nq], tn [n] squared norms (fp32).
// Writes the k nearest training indices per query (nearest first, ties → lower index) into
// idx [nq, k] int32 and, if dist is non-null, their distances into dist [nq, k].
// S column segments per row (1..256); S > 1 needs workspaces ws_d/ws_i of nq·S·k entries.
// Requires 1 <= k <= min(32, n) and n < 2^31.
FMLX_API int fmlx_knn_topk(const float* G, long ldg, long nq, long n, int S, const float* qn, const float* tn, int k,
                           int* idx, float* dist, float* ws_d, int* ws_i, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (k < 1 || k > 32 || k > n || n >= (long)INT32_MAX || ldg < n || S < 1 || S > 256) return -1;
  if (S > 1 && (ws_d == nullptr || ws_i == nullptr)) return -1;
  if (nq == 0) return 0;
  if (k <= 1) return launch_topk<1>(G, ldg, nq, n, S, qn, tn, k, idx, dist, ws_d, ws_i, s);
  if (k <= 2) return launch_topk<2>(G, ldg, nq, n, S, qn, tn, k, idx, dist, ws_d, ws_i, s);
  if (k <= 4) return launch_topk<4>(G, ldg, nq, n, S, qn, tn, k, idx, dist, ws_d, ws_i, s);
  if (k <= 8) return launch_topk<8>(G, ldg, nq, n, S, qn, tn, k, idx, dist, ws_d, ws_i, s);
  if (k <= 16) return launch_topk<16>(G, ldg, nq, n, S, qn, tn, k, idx, dist, ws_d, ws_i, s);
  return launch_topk<32>(G, ldg, nq, n, S, qn, tn, k, idx, dist, ws_d, ws_i, s);
}
