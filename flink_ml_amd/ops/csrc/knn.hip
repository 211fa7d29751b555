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


// ------------------------------------------------------------------------------------------
// Fused distance GEMM + top-k (no nq×n block in HBM)
// ------------------------------------------------------------------------------------------
// MFMA v_mfma_f32_32x32x2_f32 (exact fp32: a k-ordered fmaf chain, the same numerics class as
// the library fp32 GEMM of the split path). Roles are chosen so a query owns a LANE: the
// training tile is the A operand (rows) and the wave's 32 queries are the B operand (columns),
// so the C layout (col = lane&31, row = (r&3) + 8(r>>2) + 4·(lane>>5)) hands lane l the 16
// distances of query l&31 against 16 training rows of each 32-row subtile. Every lane therefore
// keeps one sorted (dist, index) list for ONE query (the two half-waves l, l+32 each see half
// the training rows and merge at the end), exactly like the scan kernel's per-lane lists.
//
//  * queries: the wave's 32 rows × D live in registers for the whole kernel (B fragment of
//    k-step s is Q[q][2s + h]); ‖q‖² is summed from them.
//  * training points: pre-arranged once per model into the exact LDS image of a tile
//    ([sub][h][row][DP+4], element T[row][2s+h] at s, pad for conflict-free ds_read_b128, then
//    the tile's norms), so staging is LDS-DMA (global_load_lds_dwordx4) into a double buffer
//    shared by the block's 4 waves (128 queries per block): no staging VGPRs or ds_writes, and
//    every training byte is read once per block, from L2/MALL.
//  * accumulators start at −‖t‖²/2, so key = |‖q‖² − 2·acc| = |‖q‖² + ‖t‖² − 2·q·t| is one fma
//    per element (sqrt only for the k outputs); the 32 keys of a tile
//    are min-reduced per lane and compared against the admission bound (the lexicographic min of
//    the two half-lanes' k-th best), so the insertion code only runs for tiles that can change
//    the answer (~k·ln(n/k) insertions per query over the whole scan); a tile's admitted slots
//    are a bit mask drained one insertion per trip, so a wave pays max-over-lanes insertions.
//  * S training segments per query block (grid.y) keep ≫256 blocks in flight for small query
//    counts; their k-best candidates go through knn_topk_merge_kernel.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

// k-th entry (0-based k-1) of a sorted lane list, as a wave-uniform-index select
template <int K>
__device__ __forceinline__ void kth_entry(const float (&bd)[K], const int (&bi)[K], int k, float& td, int& ti) {
  td = bd[0];
  ti = bi[0];
#pragma unroll
  for (int i = 1; i < K; ++i)
    if (i == k - 1) { td = bd[i]; ti = bi[i]; }
}

// v[b] for a per-lane b in [0, 32) as a linear select chain on register values. (A select TREE
// gets folded into an indexed load of the array — select(load a, load b) → load(select) — which
// demotes the whole key array to scratch.)
__device__ __forceinline__ float select32(const float (&v)[32], int b) {
  float r = INFINITY;
#pragma unroll
  for (int i = 0; i < 32; ++i) r = b == i ? v[i] : r;
  return r;
}

template <int K>
__device__ __forceinline__ void topk_pop(float (&bd)[K], int (&bi)[K]) {
#pragma unroll
  for (int i = 0; i < K - 1; ++i) { bd[i] = bd[i + 1]; bi[i] = bi[i + 1]; }
  bd[K - 1] = INFINITY;
  bi[K - 1] = INT32_MAX;
}

// floats per staged training tile: 128 (sub, h, row) rows of dp + 4 (the +4 pad keeps the b128
// fragment reads conflict-free), then a 1-KiB block holding the 64 squared norms
__host__ __device__ constexpr int fused_tile_floats(int dp) { return 128 * (dp + 4) + 256; }

template <int K, int DPMAX>
__global__ __launch_bounds__(256, K >= 32 ? 1 : 2) void knn_fused_kernel(
    const float* __restrict__ Q, long ldq, long nq, int D, const float* Tt, long n, int dp, int k, int S,
    int* __restrict__ out_i, float* __restrict__ out_d) {
  __shared__ __align__(16) float lds[2 * fused_tile_floats(DPMAX)];
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef __attribute__((address_space(1))) void* glb_ptr_t;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int stride = dp + 4;
  const int tf = fused_tile_floats(dp);
  const int npieces = tf / 256;  // 1-KiB LDS-DMA pieces per tile, dealt round-robin to the 4 waves
  const long qrow = (long)blockIdx.x * 128 + wave * 32 + r32;
  const bool qok = qrow < nq;

  // ---- B fragments (this lane's query, k-steps of parity h) and ‖q‖²
  float qb[DPMAX];
  float qp = 0.f;
#pragma unroll
  for (int s = 0; s < DPMAX; ++s) {
    const int c = 2 * s + h;
    float v = 0.f;
    if (qok && s < dp && c < D) v = Q[qrow * ldq + c];
    qb[s] = v;
    qp = __builtin_fmaf(v, v, qp);
  }
  const float qn = qp + __shfl_xor(qp, 32, 64);

  const long ntiles = (n + 63) / 64;
  const long L = (ntiles + S - 1) / S;
  const long t0 = (long)blockIdx.y * L;
  const long t1 = t0 + L < ntiles ? t0 + L : ntiles;

  // tile staging by LDS-DMA (global_load_lds_dwordx4): the host already laid the tile out exactly
  // as the LDS image, padding included, so each 1-KiB piece is a lane-linear copy — no staging
  // VGPRs, no ds_write. The block barrier at the end of a tile (vmcnt(0) + s_barrier) publishes it.
  auto stage = [&](long t, int buf) {
    const float* src = Tt + t * (long)tf;
    float* dst = lds + buf * fused_tile_floats(DPMAX);
    for (int p = wave; p < npieces; p += 4)
      __builtin_amdgcn_global_load_lds((glb_ptr_t)(src + p * 256 + lane * 4), (lds_ptr_t)(dst + p * 256), 16, 0, 0);
  };

  float bd[K];
  int bi[K];
#pragma unroll
  for (int i = 0; i < K; ++i) { bd[i] = INFINITY; bi[i] = INT32_MAX; }
  float td = INFINITY;
  int ti = INT32_MAX;

  if (t0 < t1) stage(t0, 0);
  __syncthreads();
  for (long t = t0; t < t1; ++t) {
    const int cur = (int)((t - t0) & 1);
    if (t + 1 < t1) stage(t + 1, cur ^ 1);
    const float* tb = lds + cur * fused_tile_floats(DPMAX);
    const float* a0 = tb + (0 * 2 + h) * 32 * stride + r32 * stride;
    const float* a1 = tb + (1 * 2 + h) * 32 * stride + r32 * stride;
    const float* tnl = tb + 128 * stride;
    // accumulators start at −‖t‖²/2 of their rows, so the MFMA chain yields q·t − ‖t‖²/2 and the
    // key |‖q‖² + ‖t‖² − 2q·t| is one fma (+ abs modifier) per element
    f32x16_t acc0, acc1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4_t v0 = *reinterpret_cast<const f32x4_t*>(tnl + 8 * g + 4 * h);
      const f32x4_t v1 = *reinterpret_cast<const f32x4_t*>(tnl + 32 + 8 * g + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc0[4 * g + e] = -0.5f * v0[e];
        acc1[4 * g + e] = -0.5f * v1[e];
      }
    }
    // A fragments one 4-step group ahead: group s4+1 is read (unconditionally — beyond dp it is
    // in-bounds padding of the DPMAX-sized buffer) before group s4's MFMAs
    f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(a0);
    f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(a1);
#pragma unroll
    for (int s4 = 0; s4 < DPMAX / 4; ++s4) {
      if (4 * s4 < dp) {
        f32x4_t y0 = x0, y1 = x1;
        if (s4 + 1 < DPMAX / 4) {
          y0 = *reinterpret_cast<const f32x4_t*>(a0 + 4 * s4 + 4);
          y1 = *reinterpret_cast<const f32x4_t*>(a1 + 4 * s4 + 4);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x0[e], qb[4 * s4 + e], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(x1[e], qb[4 * s4 + e], acc1, 0, 0, 0);
        }
        x0 = y0;
        x1 = y1;
      }
    }
    // ---- epilogue: 32 keys per lane, admission-bound filter, rare insertions. A NaN key fails
    // every '>' test, so it is admitted only while the list still has room and then ranks as +inf
    // (torch.topk also ranks NaN last).
    float key[32];
    float m = INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      key[i] = fabsf(__builtin_fmaf(-2.0f, acc0[i], qn));
      key[16 + i] = fabsf(__builtin_fmaf(-2.0f, acc1[i], qn));
      m = fminf(m, fminf(key[i], key[16 + i]));
    }
    const long jb = t * 64;
    if (!(m > td)) {
      // Admitted slots of this tile as a bit mask, then one insertion per loop trip: the wave
      // runs max-over-lanes(admissions) trips, not one per slot that ANY lane admits (with 64
      // lanes nearly every slot has some admitting lane while the bounds settle).
      unsigned mask = 0u;
#pragma unroll
      for (int i = 0; i < 32; ++i) mask |= (key[i] > td ? 0u : 1u) << i;
      if (jb + 64 > n) {  // last tile: drop the padded rows
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          const long jl = jb + (i >> 4) * 32 + (i & 3) + 8 * ((i & 15) >> 2) + 4 * h;
          if (jl >= n) mask &= ~(1u << i);
        }
      }
      while (mask) {
        const int b = __builtin_ctz(mask);
        mask &= mask - 1u;
        float d = select32(key, b);
        d = __builtin_isnan(d) ? INFINITY : d;
        const int j = (int)(jb + (b >> 4) * 32 + (b & 3) + 8 * ((b & 15) >> 2) + 4 * h);
        if (lex_less(d, j, td, ti) && lex_less(d, j, bd[K - 1], bi[K - 1])) topk_insert<K>(bd, bi, d, j);
      }
    }
    // refresh the admission bound: this lane's k-th best vs the partner half-lane's
    kth_entry<K>(bd, bi, k, td, ti);
    {
      const float xd = __shfl_xor(td, 32, 64);
      const int xi = __shfl_xor(ti, 32, 64);
      if (lex_less(xd, xi, td, ti)) { td = xd; ti = xi; }
    }
    __syncthreads();  // next tile landed (vmcnt(0)) and everyone is done with this one
  }

  // ---- merge the two half-lane lists of each query; lane h == 0 writes
  const long o = (qrow * S + blockIdx.y) * k;
  for (int t = 0; t < k; ++t) {
    const float wd = bd[0];
    const int wi = bi[0];
    const float xd = __shfl_xor(wd, 32, 64);
    const int xi = __shfl_xor(wi, 32, 64);
    const bool mine = lex_less(wd, wi, xd, xi);
    if (h == 0 && qok) {
      const float od = mine ? wd : xd;
      out_i[o + t] = mine ? wi : xi;
      if (out_d) out_d[o + t] = S == 1 ? __builtin_sqrtf(od) : od;
    }
    if (mine) topk_pop<K>(bd, bi);
  }
}

template <int K, int DPMAX>
int launch_fused(const float* Q, long ldq, long nq, int D, const float* Tt, long n, int dp, int k, int S, int* idx,
                 float* dist, float* ws_d, int* ws_i, hipStream_t s) {
  const int bq = fmlx_ceil_div(nq, 128);
  int* si = S > 1 ? ws_i : idx;
  float* sd = S > 1 ? ws_d : dist;
  hipLaunchKernelGGL((knn_fused_kernel<K, DPMAX>), dim3(bq, S), dim3(256), 0, s, Q, ldq, nq, D, Tt, n, dp, k, S, si,
                     sd);
  if (S > 1)
    hipLaunchKernelGGL((knn_topk_merge_kernel<K>), dim3(fmlx_ceil_div(nq, 4)), dim3(256), 0, s, ws_d, ws_i, nq, S, k,
                       idx, dist);
  FMLX_CHECK_LAUNCH();
}

template <int K>
int launch_fused_k(const float* Q, long ldq, long nq, int D, const float* Tt, long n, int dp, int k, int S, int* idx,
                   float* dist, float* ws_d, int* ws_i, hipStream_t s) {
  if (dp <= 16) return launch_fused<K, 16>(Q, ldq, nq, D, Tt, n, dp, k, S, idx, dist, ws_d, ws_i, s);
  if (dp <= 32) return launch_fused<K, 32>(Q, ldq, nq, D, Tt, n, dp, k, S, idx, dist, ws_d, ws_i, s);
  return launch_fused<K, 64>(Q, ldq, nq, D, Tt, n, dp, k, S, idx, dist, ws_d, ws_i, s);
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

// Fused KNN: Q [nq, D] fp32 (leading dim ldq); training points pre-arranged as ceil(n/64) tiles
// of fused_tile_floats(dp) floats: [sub 2][h 2][r 32][dp + 4] with element T[64·t + 32·sub + r][2s + h]
// at s (zero padded), then the tile's 64 squared norms and 192 zeros. dp = ceil(D/2) rounded up
// to 4, ≤ 64 (D ≤ 128). k nearest per query (nearest first, ties → lower index) into idx [nq, k] and,
// if non-null, dist [nq, k]. S training segments (1..256); S > 1 needs ws_d/ws_i of nq·S·k.
FMLX_API int fmlx_knn_fused_max_k() { return 64; }

namespace {
template <int K, int DPMAX>
int fused_blocks_per_cu() {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, knn_fused_kernel<K, DPMAX>, 256, 0) != hipSuccess) return 1;
  return b > 0 ? b : 1;
}
template <int K>
int fused_blocks_per_cu_k(int dp) {
  if (dp <= 16) return fused_blocks_per_cu<K, 16>();
  if (dp <= 32) return fused_blocks_per_cu<K, 32>();
  return fused_blocks_per_cu<K, 64>();
}
}  // namespace

// Resident fused-kernel blocks per CU for (k, dp) — the host sizes the segment split with it.
FMLX_API int fmlx_knn_fused_blocks_per_cu(int k, int dp) {
  if (k <= 4) return fused_blocks_per_cu_k<4>(dp);
  if (k <= 8) return fused_blocks_per_cu_k<8>(dp);
  if (k <= 16) return fused_blocks_per_cu_k<16>(dp);
  if (k <= 32) return fused_blocks_per_cu_k<32>(dp);
  return fused_blocks_per_cu_k<64>(dp);
}

FMLX_API int fmlx_knn_fused(const float* Q, long ldq, long nq, int D, const float* Tt, long n, int dp, int k, int S,
                            int* idx, float* dist, float* ws_d, int* ws_i, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (k < 1 || k > 64 || k > n || n >= (long)INT32_MAX - 64 || D < 1 || ldq < D) return -1;
  if (dp % 4 != 0 || dp > 64 || 2 * dp < D || S < 1 || S > 256) return -1;
  if (S > 1 && (ws_d == nullptr || ws_i == nullptr)) return -1;
  if (nq == 0) return 0;
  if (k <= 4) return launch_fused_k<4>(Q, ldq, nq, D, Tt, n, dp, k, S, idx, dist, ws_d, ws_i, s);
  if (k <= 8) return launch_fused_k<8>(Q, ldq, nq, D, Tt, n, dp, k, S, idx, dist, ws_d, ws_i, s);
  if (k <= 16) return launch_fused_k<16>(Q, ldq, nq, D, Tt, n, dp, k, S, idx, dist, ws_d, ws_i, s);
  if (k <= 32) return launch_fused_k<32>(Q, ldq, nq, D, Tt, n, dp, k, S, idx, dist, ws_d, ws_i, s);
  return launch_fused_k<64>(Q, ldq, nq, D, Tt, n, dp, k, S, idx, dist, ws_d, ws_i, s);
}

FMLX_DEFINE_PRELOAD()
