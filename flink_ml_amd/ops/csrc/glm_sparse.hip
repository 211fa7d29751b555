// Sparse (CSR) SGD rounds (LinearSVC / LR on 1M-wide sparse features).
//
// Reference hot loop: LIB/common/optimizer/SGD.java:263-285 over SparseVector rows with
// LIB/common/lossfunc/HingeLoss.java:39-57 (dot, hinge loss, axpy of the multiplier into the
// gradient), the update of SGD.java:231-243 and RegularizationUtils.java:47-91.
//
// Three round forms, picked per fit by ops/glm.py (DeviceGlmTrainer):
//  * single-visit bucket round (glm_bkt_*): the reference's regime (each batch visited once or a
//    few times): nothing is precomputed per batch;
//  * transposed rounds (glm_csr_fwd / glm_csr_cell_fwd + glm_csc_bwd / glm_csc_tile_bwd): batches
//    visited many times (or FMLX_DETERMINISTIC=1) amortise a per-batch column-major copy
//    (csc_build.hip) and run atomic-free, deterministic backward passes;
//  * glm_grad_csr_kernel: the scattered-atomic fallback when neither fits.
#include "common.h"
#include "glm_core.h"

namespace {

// ------------------------------------------------------------------------------------------
// CSR (sparse features) gradient — a wave per row, gather dot, atomic scatter of mult·x into
// a dense gradient (K5 sparse path, for the 1M-feature LinearSVC config).
// ------------------------------------------------------------------------------------------
template <typename A>
__global__ __launch_bounds__(256) void glm_grad_csr_kernel(const long* __restrict__ indptr, const int* __restrict__ idx,
                                                           const A* __restrict__ val, const A* __restrict__ y,
                                                           const A* __restrict__ wt, const A* __restrict__ coef, long n,
                                                           int d, long B, int loss, const int* __restrict__ state,
                                                           A* __restrict__ grad /* d+2, zeroed */) {
  int e;
  if (!round_running(state, e)) return;
  const long P = (n + B - 1) / B;
  const long start = (long)(e % P) * B;
  const long end = start + B < n ? start + B : n;
  const int lane = threadIdx.x & 63;
  const long gw = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long W = ((long)gridDim.x * blockDim.x) >> 6;
  A wsum = 0, lsum = 0;
  for (long r = start + gw; r < end; r += W) {
    const long s0 = indptr[r], s1 = indptr[r + 1];
    A s = 0;
    for (long j = s0 + lane; j < s1; j += 64) s += val[j] * coef[idx[j]];
    s = wave_sum(s);
    const A yy = y[r];
    const A ww = wt ? wt[r] : (A)1;
    A l, m;
    loss_and_mult(loss, s, yy, ww, l, m);
    wsum += ww;
    lsum += l;
    if (m != (A)0)
      for (long j = s0 + lane; j < s1; j += 64) atomicAdd(&grad[idx[j]], m * val[j]);
  }
  if (lane == 0) {
    atomicAdd(&grad[d], wsum);
    atomicAdd(&grad[d + 1], lsum);
  }
}

template <typename A>
__global__ void glm_csr_predict_kernel(const long* __restrict__ indptr, const int* __restrict__ idx,
                                       const A* __restrict__ val, const A* __restrict__ coef, long n,
                                       double* __restrict__ dots) {
  const int lane = threadIdx.x & 63;
  const long gw = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long W = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = gw; r < n; r += W) {
    A s = 0;
    for (long j = indptr[r] + lane; j < indptr[r + 1]; j += 64) s += val[j] * coef[idx[j]];
    s = wave_sum(s);
    if (lane == 0) dots[r] = (double)s;
  }
}

// ------------------------------------------------------------------------------------------
// Sparse (CSR) SGD round without atomics on the gradient
// ------------------------------------------------------------------------------------------
// Batches are the fixed row ranges [b·B, min((b+1)·B, n)) (SGD.java:192-206 slicing), so the
// transpose of every batch can be built once when the trainer starts (ops/glm.py
// build_batch_csc): per batch, its non-zeros re-sorted by column with the batch-relative row id,
// at the SAME offsets as the CSR (batch b's non-zeros are CSR positions [indptr[bB], indptr[bB+B])),
// plus a dense int32 column pointer [P][d+1]. A round is then two launches:
//   forward  — a G-lane group per row: gathered dot, loss + multiplier m_r (stored, B floats,
//              L2-resident), Σweight/Σloss into a parity slot of `wl`;
//   backward — a thread per column: g_c = Σ m_row·val over the column's batch entries (a
//              segmented gather, no atomics), then either the SGD update + termination check in
//              place (1 GPU) or the feedback row for the all-reduce (N GPUs).
// The 1M-wide scatter of atomicAdds it replaces (glm_grad_csr_kernel) was 472 µs per round on the
// 100k × 64-nnz batch of the sparse LinearSVC config; the reads here are the batch once in each
// layout plus one column-pointer row.
template <int G, typename A>
__device__ __forceinline__ A group_sum(A v) {
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Forward: K independent (index, value) slots per lane are loaded before any coefficient gather,
// so a row costs one dependent step (indptr → entries → coef) instead of a chain per element;
// entries are streamed non-temporally, which keeps the gathered coefficient vector in L2.
constexpr int WL_SLOTS = 256;  // Σweight/Σloss accumulator: [2 parities][WL_SLOTS][WL_STRIDE]
constexpr int WL_STRIDE = 32;  // 128 B apart

template <typename A, int G>
__global__ __launch_bounds__(256) void glm_csr_fwd_kernel(const long* __restrict__ indptr, const int* __restrict__ idx,
                                                          const A* __restrict__ val, const A* __restrict__ y,
                                                          const A* __restrict__ wt, const A* __restrict__ coef, long n,
                                                          long B, int loss, const int* __restrict__ state,
                                                          A* __restrict__ mult, A* __restrict__ wl) {
  constexpr int K = G >= 32 ? 2 : 4;
  int e;
  if (!round_running(state, e)) return;
  const long P = (n + B - 1) / B;
  const long start = (long)(e % P) * B;
  const long end = start + B < n ? start + B : n;
  const int lane = threadIdx.x & (G - 1);
  const long grp = ((long)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const long NG = ((long)gridDim.x * blockDim.x) / G;
  A wsum = 0, lsum = 0;
  for (long r = start + grp; r < end; r += NG) {
    const long s0 = indptr[r], s1 = indptr[r + 1];
    A s = 0;
    for (long jb = s0; jb < s1; jb += K * G) {
      int ii[K];
      A vv[K];
#pragma unroll
      for (int t = 0; t < K; ++t) {
        const long j = jb + lane + t * G;
        const bool ok = j < s1;
        const long jj = ok ? j : s0;
        ii[t] = __builtin_nontemporal_load(idx + jj);
        const A v = __builtin_nontemporal_load(val + jj);
        vv[t] = ok ? v : (A)0;
      }
#pragma unroll
      for (int t = 0; t < K; ++t) s += vv[t] * coef[ii[t]];
    }
    s = group_sum<G>(s);
    if (lane == 0) {
      const A ww = wt ? wt[r] : (A)1;
      A l, m;
      loss_and_mult(loss, s, y[r], ww, l, m);
      mult[r - start] = m;
      wsum += ww;
      lsum += l;
    }
  }
  __shared__ A red[2][4];
  wsum = wave_sum(wsum);
  lsum = wave_sum(lsum);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = wsum; red[1][w] = lsum; }
  __syncthreads();
  if (threadIdx.x == 0) {
    A a0 = 0, a1 = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { a0 += red[0][i]; a1 += red[1][i]; }
    // one of WL_SLOTS cache lines per block: same-address float atomics from thousands of
    // blocks serialise at the coherence point (measured: the single-address version cost more
    // than the row math); the backward sums the slots in a fixed order
    A* slot = wl + ((long)(e & 1) * WL_SLOTS + (blockIdx.x & (WL_SLOTS - 1))) * WL_STRIDE;
    if (a0 != (A)0) atomicAdd(&slot[0], a0);
    if (a1 != (A)0) atomicAdd(&slot[1], a1);
  }
}

// Forward over row-block × column-split cells (BatchCsc cells, csc_build.hip cell_keys … cell_store):
// cell (rb, s) holds the batch's entries of rows [rb·2^CELL_RBB, …) with columns in [s·CS, (s+1)·CS),
// stored column-sorted and packed (column − s·CS) | pos << cb, pos = the entry's rank in the cell's
// row-major order; roff[cell·2^CELL_RBB + r] = first entry of row r of the cell. A block takes a
// cell: its lanes gather coefficients in column order from one slice (consecutive lanes share
// cache lines — the one-row-per-lane-group kernel gathers a random line per lane, ~40 µs per 6.4M,
// profiles/r5/micro_gather_*), write each product into LDS slot pos (plain stores: LDS float
// atomics cost ~27 µs more per round, profiles/r5/svc_cell_forward_ab.jsonl), then every row sums
// its slots in order and the cell stores its row partials. The last of a row block's S cells to
// arrive sums the S partials of every row in split order (deterministic), evaluates loss and
// multiplier, and adds Σweight / Σloss into the slots.
constexpr int CELL_THREADS = 1024;
constexpr int CELL_RBB_MAX = 11;  // rows per row block: 2^rbb ≤ 2^11 (two rows per thread)
constexpr int CELL_U = 8;

template <typename A>
__global__ __launch_bounds__(CELL_THREADS) void glm_csr_cell_fwd_kernel(
    const long* __restrict__ indptr, const uint32_t* __restrict__ cent, const A* __restrict__ cval,
    const int* __restrict__ roff, long rstride, int rbb, int S, int CS, int cb, const A* __restrict__ y,
    const A* __restrict__ wt, const A* __restrict__ coef, long n, long B, int loss, const int* __restrict__ state,
    A* __restrict__ mult, A* __restrict__ wl, A* __restrict__ partial, int* __restrict__ cnt, int xcd) {
  const int RB = 1 << rbb;
  extern __shared__ __align__(16) unsigned char cell_lds[];
  A* prod = reinterpret_cast<A*>(cell_lds);  // [the largest cell's entries]
  __shared__ A red[2][CELL_THREADS / 64];
  __shared__ int sflag;
  int e;
  if (!round_running(state, e)) return;
  const long P = (n + B - 1) / B;
  const long b = (long)(e % P);
  const long start = b * B;
  const long blen = (start + B < n ? start + B : n) - start;
  const int nrb = (int)((blen + RB - 1) >> rbb);
  const int ncell = nrb * S;
  int rb, sp;
  if (xcd) {
    // XCD-aware order: block b runs on XCD b mod 8 (round-robin dispatch); give XCD x the cells
    // of a contiguous split-major range, so its L2 holds the coefficient slices of ≤ 2 splits
    // (a bijection of [0, grid): XCD x holds the n_x = ⌈(grid − x) / 8⌉ blocks b ≡ x mod 8, so it
    // starts at Σ_{y<x} n_y = x·⌊grid/8⌋ + min(x, grid mod 8))
    const int x = (int)(blockIdx.x & 7), q = (int)(gridDim.x >> 3), r = (int)(gridDim.x & 7);
    const int g = x * q + (x < r ? x : r) + (int)(blockIdx.x >> 3);
    if (g >= ncell) return;
    sp = g / nrb;
    rb = g - sp * nrb;
  } else {
    if ((int)blockIdx.x >= ncell) return;  // (the grid covers the largest batch)
    rb = blockIdx.x / S;
    sp = blockIdx.x - rb * S;
  }
  const int c = rb * S + sp;
  const int tid = threadIdx.x;
  const long base = indptr[start];
  const int* __restrict__ ro = roff + b * rstride + ((long)c << rbb);
  const int k0 = ro[0], k1 = ro[RB];
  const uint32_t* __restrict__ en = cent + base;
  const A* __restrict__ ev = cval + base;
  const A* __restrict__ cs = coef + (long)sp * CS;
  const uint32_t cmask = (1u << cb) - 1;
  uint32_t xx[CELL_U];
  A vv[CELL_U];
  if (k0 < k1) {  // (an empty cell may sit at the end of the array: nothing to load)
#pragma unroll
    for (int u = 0; u < CELL_U; ++u) {
      const int k = k0 + tid + u * CELL_THREADS;
      const int kk = k < k1 ? k : k0;
      xx[u] = __builtin_nontemporal_load(en + kk);
      vv[u] = __builtin_nontemporal_load(ev + kk);
    }
  }
  for (int kb = k0 + tid; kb < k1; kb += CELL_U * CELL_THREADS) {
    uint32_t nx[CELL_U];
    A nv[CELL_U];
    const int kn = kb + CELL_U * CELL_THREADS;
    if (kn < k1) {
#pragma unroll
      for (int u = 0; u < CELL_U; ++u) {
        const int k = kn + u * CELL_THREADS;
        const int kk = k < k1 ? k : kn;
        nx[u] = __builtin_nontemporal_load(en + kk);
        nv[u] = __builtin_nontemporal_load(ev + kk);
      }
    }
    // every gather first (lanes past the cell hold its first entry: valid addresses), then the
    // slot stores — a gather per store would serialise CELL_U memory latencies per step
    A pp[CELL_U];
#pragma unroll
    for (int u = 0; u < CELL_U; ++u) pp[u] = vv[u] * cs[xx[u] & cmask];
#pragma unroll
    for (int u = 0; u < CELL_U; ++u)
      if (kb + u * CELL_THREADS < k1) prod[xx[u] >> cb] = pp[u];
#pragma unroll
    for (int u = 0; u < CELL_U; ++u) {
      xx[u] = nx[u];
      vv[u] = nv[u];
    }
  }
  const long rb0 = (long)rb << rbb;
  const int nr = blen - rb0 < RB ? (int)(blen - rb0) : RB;
  constexpr int RQ = (1 << CELL_RBB_MAX) / CELL_THREADS;
  int r0s[RQ], r1s[RQ];
#pragma unroll
  for (int q = 0; q < RQ; ++q) {  // (row offsets loaded before the barrier)
    const int r = tid + q * CELL_THREADS;
    r0s[q] = r < nr ? ro[r] - k0 : 0;
    r1s[q] = r < nr ? ro[r + 1] - k0 : 0;
  }
  __syncthreads();
  A* __restrict__ mine = partial + (long)c * RB;
#pragma unroll
  for (int q = 0; q < RQ; ++q) {
    const int r = tid + q * CELL_THREADS;
    A t = 0;
    for (int j = r0s[q]; j < r1s[q]; ++j) t += prod[j];
    if (r < nr) st_agent(mine + r, t);
  }
  if (!arrive_last(&cnt[rb], S, &sflag)) return;
  if (tid == 0) st_agent(&cnt[rb], 0);  // every arrival of this launch is in: re-arm for the next
  A ws = 0, ls = 0;
  for (int r = tid; r < nr; r += CELL_THREADS) {
    A dot = 0;
    for (int q = 0; q < S; ++q) dot += ld_agent(partial + ((long)rb * S + q) * RB + r);
    const long gr = start + rb0 + r;
    const A ww = wt ? wt[gr] : (A)1;
    A l, m;
    loss_and_mult(loss, dot, y[gr], ww, l, m);
    mult[rb0 + r] = m;
    ws += ww;
    ls += l;
  }
  ws = wave_sum(ws);
  ls = wave_sum(ls);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = ws;
    red[1][tid >> 6] = ls;
  }
  __syncthreads();
  if (tid == 0) {
    A a0 = 0, a1 = 0;
    for (int i = 0; i < CELL_THREADS / 64; ++i) {
      a0 += red[0][i];
      a1 += red[1][i];
    }
    A* slot = wl + ((long)(e & 1) * WL_SLOTS + (rb & (WL_SLOTS - 1))) * WL_STRIDE;
    if (a0 != (A)0) atomicAdd(&slot[0], a0);
    if (a1 != (A)0) atomicAdd(&slot[1], a1);
  }
}

// Backward: a block owns 256 consecutive columns, whose batch entries are one contiguous CSC
// range. The block walks that range coalesced (every thread loads independent entries: row id →
// multiplier gather → product into LDS), then each thread adds its column's slice of the LDS
// products in entry order — deterministic, no atomics, no per-column dependent load chains.
constexpr int CSC_CAP = 4096;  // entries staged per pass (16 KB fp32 / 32 KB fp64)

// Σweight / Σloss of round e: fixed-order sum of the forward's WL_SLOTS slots (all 256 threads)
template <typename A>
__device__ __forceinline__ void slot_sums(const A* __restrict__ wl, int e, A& W, A& L) {
  __shared__ A red[2][4];
  const bool own = threadIdx.x < WL_SLOTS;  // (blocks of ≥ 256 threads)
  const A* sl = wl + ((long)(e & 1) * WL_SLOTS + (own ? threadIdx.x : 0)) * WL_STRIDE;
  const A w0 = wave_sum(own ? sl[0] : (A)0), l0 = wave_sum(own ? sl[1] : (A)0);
  if ((threadIdx.x & 63) == 0 && own) { red[0][threadIdx.x >> 6] = w0; red[1][threadIdx.x >> 6] = l0; }
  __syncthreads();
  W = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  L = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
}

template <typename A, bool FUSE>
__global__ __launch_bounds__(256) void glm_csc_bwd_kernel(const long* __restrict__ indptr,
                                                          const int* __restrict__ colptr, const int* __restrict__ erow,
                                                          const A* __restrict__ eval, const A* __restrict__ mult,
                                                          long n, int d, long B, int* __restrict__ state,
                                                          A* __restrict__ wl, A* __restrict__ fb, A* __restrict__ coef,
                                                          int max_iter, A tol, A lr, A reg, A en, int weighted) {
  __shared__ A prod[CSC_CAP];
  int e;
  const bool run = round_running(state, e);
  // re-arm the other parity's slots (they held the previous round's sums, consumed by now)
  if (blockIdx.x == 0) {
    A* o = wl + ((long)((e + 1) & 1) * WL_SLOTS + threadIdx.x) * WL_STRIDE;
    o[0] = 0;
    o[1] = 0;
  }
  if (!run) {
    if (FUSE) arrive_and_advance(state, e, false, 0);
    return;
  }
  const long P = (n + B - 1) / B;
  const long b = (long)(e % P);
  const long base = indptr[b * B];
  const int* __restrict__ cp = colptr + b * (long)(d + 1);
  const int* __restrict__ er = erow + base;
  const A* __restrict__ ev = eval + base;
  // Σweight of the round: the batch's row count when unweighted, else the fixed-order sum of the
  // forward's slots (identical in every block). Σloss only feeds the termination test, which the
  // last arriving block makes (and block 0 of the feedback path, which exports it).
  A W, L = 0;
  if (weighted || (!FUSE && blockIdx.x == 0)) {
    slot_sums(wl, e, W, L);
  }
  if (!weighted) {
    const long end = (b + 1) * B < n ? (b + 1) * B : n;
    W = (A)(end - b * B);
  }
  for (int cb = blockIdx.x * 256; cb < d; cb += gridDim.x * 256) {
    const int c = cb + (int)threadIdx.x;
    const int ce = cb + 256 < d ? cb + 256 : d;
    const int lo = cp[cb], hi = cp[ce];
    const int j0 = c < d ? cp[c] : hi, j1 = c < d ? cp[c + 1] : hi;
    A g = 0;
    for (int pb = lo; pb < hi; pb += CSC_CAP) {
      const int top = pb + CSC_CAP < hi ? pb + CSC_CAP : hi;
      for (int k0 = pb + (int)threadIdx.x; k0 < top; k0 += 4 * 256) {
        int rr[4];
        A vv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = k0 + t * 256;
          const int kk = k < top ? k : k0;
          rr[t] = __builtin_nontemporal_load(er + kk);
          vv[t] = __builtin_nontemporal_load(ev + kk);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = k0 + t * 256;
          const A p = mult[rr[t]] * vv[t];
          if (k < top) prod[k - pb] = p;
        }
      }
      __syncthreads();
      const int a = j0 > pb ? j0 : pb, z = j1 < top ? j1 : top;
      for (int j = a; j < z; ++j) g += prod[j - pb];
      __syncthreads();
    }
    if (c < d) {
      if (FUSE)
        coef[c] = sgd_apply<A>(coef[c], g, W, lr, reg, en);
      else
        fb[c] = g;
    }
  }
  if (!FUSE && blockIdx.x == 0 && threadIdx.x == 0) {
    fb[d] = W;
    fb[d + 1] = L;
  }
  if (FUSE) {
    __shared__ int last;
    __syncthreads();
    if (threadIdx.x == 0)
      last = __hip_atomic_fetch_add(&state[ST_ARRIVE], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (int)gridDim.x - 1;
    __syncthreads();
    if (last) {  // every other block has finished its reads of the state words (see arrive_and_advance)
      A w2;
      slot_sums(wl, e, w2, L);
      if (threadIdx.x == 0) {
        const bool cont = (e + 1 < max_iter) && (L / W > tol);
        state[ST_RUN0 + ((e + 1) & 1)] = cont ? 1 : 0;
        state[ST_EXECUTED] += 1;
        state[ST_ROUND] = e + 1;
        state[ST_ARRIVE] = 0;
      }
    }
  }
}

// Tiled backward (BatchCsc tiles, csc_build.hip csc_tiles / csc_tile_keys / csc_tile_store): the
// batch's columns are cut into tiles of ≤ ET entries (or one heavy column of > EL), and inside a light
// tile the entries are sorted by ROW, each carrying its slot in the tile's column-ordered range
// (erow = row | slot << rb). A block takes a tile: the multiplier gathers of consecutive lanes
// then fall on the same or nearby cache lines (the one-column-block form gathers a random row per
// lane: measured ~40 µs for 6.4M such 4-byte gathers, the cost scaling with distinct lines per
// wave instruction), each product goes to its column-ordered LDS slot, and a thread per column
// sums its slots in entry order — the same per-column order as the untiled kernel, so results
// are deterministic. A heavy column is a block-strided sum with a fixed-order block reduction.
constexpr int TILE_THREADS = 1024;
constexpr int TILE_U = 8;     // entries per thread per gather step
constexpr int TILE_COLS = 8;  // columns per thread whose pointers are prefetched

template <typename A, bool FUSE>
__global__ __launch_bounds__(TILE_THREADS) void glm_csc_tile_bwd_kernel(
    const long* __restrict__ indptr, const int* __restrict__ colptr, const int2* __restrict__ tiles,
    const int* __restrict__ ntiles, int tstride, const int* __restrict__ erow, const A* __restrict__ eval,
    const A* __restrict__ mult, long n, int d, long B, int rb, int EL, int* __restrict__ state, A* __restrict__ wl,
    A* __restrict__ fb, A* __restrict__ coef, int max_iter, A tol, A lr, A reg, A en, int weighted,
    long long* __restrict__ trace) {
  extern __shared__ unsigned char tile_smem[];
  if (trace && threadIdx.x == 0) trace[(long)blockIdx.x * 4] = (long long)__builtin_amdgcn_s_memrealtime();
  A* prod = reinterpret_cast<A*>(tile_smem);
  __shared__ A hred[TILE_THREADS / 64];
  int e;
  const bool run = round_running(state, e);
  if (blockIdx.x == 0 && threadIdx.x < WL_SLOTS) {
    A* o = wl + ((long)((e + 1) & 1) * WL_SLOTS + threadIdx.x) * WL_STRIDE;
    o[0] = 0;
    o[1] = 0;
  }
  if (!run) {
    if (FUSE) arrive_and_advance(state, e, false, 0);
    return;
  }
  const long P = (n + B - 1) / B;
  const long b = (long)(e % P);
  const long base = indptr[b * B];
  const int* __restrict__ cp = colptr + b * (long)(d + 1);
  const int2* __restrict__ tl = tiles + b * (long)tstride;
  const int nt = ntiles[b];
  const int* __restrict__ er = erow + base;
  const A* __restrict__ ev = eval + base;
  const uint32_t rmask = (1u << rb) - 1;
  A W, L = 0;
  if (weighted || (!FUSE && blockIdx.x == 0)) slot_sums(wl, e, W, L);
  if (!weighted) {
    const long end = (b + 1) * B < n ? (b + 1) * B : n;
    W = (A)(end - b * B);
  }
  const int tid = threadIdx.x;
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const int2 ta = tl[t], tz = tl[t + 1];  // (start column, first entry) of this and the next tile
    const int c0 = ta.x, c1 = tz.x, k0 = ta.y, k1 = tz.y;
    if (c1 - c0 == 1 && k1 - k0 > EL) {  // heavy column (block-uniform branch)
      A g = 0;
      for (int k = k0 + tid; k < k1; k += TILE_THREADS) {
        const uint32_t x = (uint32_t)__builtin_nontemporal_load(er + k);
        g += mult[x & rmask] * __builtin_nontemporal_load(ev + k);
      }
      g = wave_sum(g);
      if ((tid & 63) == 0) hred[tid >> 6] = g;
      __syncthreads();
      if (tid == 0) {
        A s = 0;
        for (int i = 0; i < TILE_THREADS / 64; ++i) s += hred[i];
        if (FUSE)
          coef[c0] = sgd_apply<A>(coef[c0], s, W, lr, reg, en);
        else
          fb[c0] = s;
      }
      __syncthreads();
      continue;
    }
    // the thread's columns of the tile (c0 + tid + i·TILE_THREADS, i < TILE_COLS): pointers and
    // coefficients loaded before the gathers, so the column pass after the barrier reads only LDS
    const bool few = c1 - c0 <= TILE_COLS * TILE_THREADS;  // (block-uniform)
    int ca[TILE_COLS], cz[TILE_COLS];
    A cw[TILE_COLS];
    if (few) {
#pragma unroll
      for (int i = 0; i < TILE_COLS; ++i) {
        const int c = c0 + tid + i * TILE_THREADS;
        const int cc = c < c1 ? c : c0;
        ca[i] = cp[cc];
        cz[i] = c < c1 ? cp[cc + 1] : ca[i];
        cw[i] = FUSE ? coef[cc] : (A)0;
      }
    }
    constexpr int TU = sizeof(A) == 8 ? TILE_U / 2 : TILE_U;
    // products into their column-ordered slots: TU entries per thread per step (8; 4 for fp64,
    // which spilled at 8 under the 1024-thread register budget), the next
    // step's entries loaded before this step's multiplier gathers (measured against one step of
    // 32 per thread: 71.0 vs 72.3 µs per round; 8 without the overlap: 71.8)
    uint32_t xx[TU];
    A vv[TU];
    if (k0 < k1) {  // (an empty tile may sit at the end of the array: nothing to load)
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int k = k0 + tid + u * TILE_THREADS;
        const int kk = k < k1 ? k : k0;
        xx[u] = (uint32_t)__builtin_nontemporal_load(er + kk);
        vv[u] = __builtin_nontemporal_load(ev + kk);
      }
    }
    for (int kb = k0 + tid; kb < k1; kb += TU * TILE_THREADS) {
      uint32_t nx[TU];
      A nv[TU];
      const int kn = kb + TU * TILE_THREADS;
      if (kn < k1) {
#pragma unroll
        for (int u = 0; u < TU; ++u) {
          const int k = kn + u * TILE_THREADS;
          const int kk = k < k1 ? k : kn;
          nx[u] = (uint32_t)__builtin_nontemporal_load(er + kk);
          nv[u] = __builtin_nontemporal_load(ev + kk);
        }
      }
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const A p = mult[xx[u] & rmask] * vv[u];
        if (kb + u * TILE_THREADS < k1) prod[xx[u] >> rb] = p;
      }
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        xx[u] = nx[u];
        vv[u] = nv[u];
      }
    }
    if (trace && tid == 0) trace[(long)blockIdx.x * 4 + 1] = (long long)__builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (trace && tid == 0) trace[(long)blockIdx.x * 4 + 2] = (long long)__builtin_amdgcn_s_memrealtime();
    if (few) {
#pragma unroll
      for (int i = 0; i < TILE_COLS; ++i) {
        const int c = c0 + tid + i * TILE_THREADS;
        A g = 0;
        for (int j = ca[i] - k0; j < cz[i] - k0; ++j) g += prod[j];
        if (c < c1) {
          if (FUSE)
            coef[c] = sgd_apply<A>(cw[i], g, W, lr, reg, en);
          else
            fb[c] = g;
        }
      }
    } else {
      for (int c = c0 + tid; c < c1; c += TILE_THREADS) {
        const int a = cp[c] - k0, z = cp[c + 1] - k0;
        A g = 0;
        for (int j = a; j < z; ++j) g += prod[j];
        if (FUSE)
          coef[c] = sgd_apply<A>(coef[c], g, W, lr, reg, en);
        else
          fb[c] = g;
      }
    }
    __syncthreads();
  }
  if (!FUSE && blockIdx.x == 0 && tid == 0) {
    fb[d] = W;
    fb[d + 1] = L;
  }
  if (trace && tid == 0) trace[(long)blockIdx.x * 4 + 3] = (long long)__builtin_amdgcn_s_memrealtime();
  if (FUSE) {
    __shared__ int last;
    __syncthreads();
    if (tid == 0)
      last = __hip_atomic_fetch_add(&state[ST_ARRIVE], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (int)gridDim.x - 1;
    __syncthreads();
    if (last) {
      A w2;
      slot_sums(wl, e, w2, L);
      if (tid == 0) {
        const bool cont = (e + 1 < max_iter) && (L / W > tol);
        state[ST_RUN0 + ((e + 1) & 1)] = cont ? 1 : 0;
        state[ST_EXECUTED] += 1;
        state[ST_ROUND] = e + 1;
        state[ST_ARRIVE] = 0;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Single-visit sparse round: column-slice buckets built inside the round (no per-batch transpose)
// ------------------------------------------------------------------------------------------
// The reference's LinearSVC benchmark visits every 100k-row batch once (maxIter 20 over 10M rows:
// SGD.java:263-268), so a column-major copy built per batch (radix passes, ~0.25 ms per 6.4M-entry
// batch) never pays back. Here a round is three launches over the CSR batch as it stands:
//   count    — per column slice of 2^csb columns (a "bucket"), the batch's entries: LDS histograms,
//              one device atomic per (block, bucket); the last block scans them into bucket starts
//              and reservation cursors;
//   forward  — a block takes RB rows: a G-lane group per row gathers its dot (as glm_csr_fwd_kernel),
//              loss + multiplier into LDS, then reserves each bucket's run for the block (ONE
//              device atomic per (block, bucket)) and writes every entry's (column in slice,
//              m_row·x) into its bucket, staged through LDS in pieces so that each piece's stores
//              are bucket-sorted runs (coalesced), not 64 random lines per wave instruction;
//   backward — a block takes a chunk of one bucket (contiguous reads), adds it into an LDS slab of
//              the slice's gradient (ds_add: no device atomics), then applies the SGD update +
//              regularisation to the slice (1 GPU) or writes its feedback slice (N GPUs); a bucket
//              of several chunks sums them through float atomics on whole 256-B rows and the last
//              chunk (arrival ticket) finishes the slice.
// A device atomic per ENTRY would run at the scattered-atomic rate (~0.08 TB/s: the 472 µs of
// glm_grad_csr_kernel); per (block, bucket) there are ~100k of them per round. Float LDS atomics
// make the last bits depend on arrival order: FMLX_DETERMINISTIC=1 keeps the transposed path.
constexpr int BK_NT = 1024;     // threads of the three kernels
constexpr int BK_ECAP = 4096;   // forward: entries staged per piece
constexpr int BK_EPT = BK_ECAP / BK_NT;
constexpr int BK_NB_MAX = 1024; // buckets
constexpr int BK_UNROLL = 8;    // backward: entries in flight per thread

struct BktArgs {
  int csb, nb;     // slice bits, buckets = ceil(d / 2^csb)
  int rb;          // forward rows per block
  int chunk;       // backward entries per work item
  int* cnt;        // [nb] zero between rounds (the count finisher re-zeroes it)
  int* off;        // [nb + 1] bucket starts of the round's batch
  int* cur;        // [nb] reservation cursors
  int* tick;       // [2] arrival tickets (zero between rounds)
  int* done;       // [nb] chunk arrivals of multi-chunk buckets (zero between rounds)
  uint16_t* key;   // [largest batch nnz] column within the slice
  void* val;       // [largest batch nnz] m_row · x
  void* acc;       // [d] zero between rounds: partial slices of multi-chunk buckets
  int dbg;         // (A/B timing: 1 skip reservation, 2 skip pieces, 4 skip histogram)
};

// exclusive scan of one int per thread over the block (BK_NT threads); *total = the sum
__device__ __forceinline__ int bk_exscan(int v, int* tmp, int* total) {
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
    int s = lane < BK_NT / 64 ? tmp[lane] : 0;
#pragma unroll
    for (int o = 1; o < BK_NT / 64; o <<= 1) {
      const int t = __shfl_up(s, o, 64);
      if (lane >= o) s += t;
    }
    if (lane < BK_NT / 64) tmp[lane] = s;
  }
  __syncthreads();
  const int pre = w ? tmp[w - 1] : 0;
  *total = tmp[BK_NT / 64 - 1];
  __syncthreads();  // (tmp is reused by the next scan)
  return pre + x - v;
}

template <typename A>
__global__ __launch_bounds__(BK_NT) void glm_bkt_count_kernel(const long* __restrict__ indptr,
                                                              const int* __restrict__ idx, long n, long B,
                                                              const int* __restrict__ state, BktArgs k) {
  extern __shared__ int bk_hist[];  // [nb]
  __shared__ int tmp[BK_NT / 64];
  __shared__ int sflag;
  int e;
  if (!round_running(state, e)) return;
  const long P = (n + B - 1) / B;
  const long start = (long)(e % P) * B;
  const long end = start + B < n ? start + B : n;
  const long j0 = indptr[start], j1 = indptr[end];
  for (int i = threadIdx.x; i < k.nb; i += BK_NT) bk_hist[i] = 0;
  __syncthreads();
  const long stride = (long)gridDim.x * BK_NT;
  long j = j0 + (long)blockIdx.x * BK_NT + threadIdx.x;
  for (; j + 3 * stride < j1; j += 4 * stride) {
    int c[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) c[t] = __builtin_nontemporal_load(idx + j + t * stride);
#pragma unroll
    for (int t = 0; t < 4; ++t) atomicAdd(&bk_hist[c[t] >> k.csb], 1);
  }
  for (; j < j1; j += stride) atomicAdd(&bk_hist[__builtin_nontemporal_load(idx + j) >> k.csb], 1);
  __syncthreads();
  for (int i = threadIdx.x; i < k.nb; i += BK_NT)
    if (bk_hist[i]) atomicAdd(&k.cnt[i], bk_hist[i]);
  if (!arrive_last(&k.tick[0], gridDim.x, &sflag)) return;
  // the last block: bucket starts (each thread a run of consecutive buckets), counts re-zeroed
  const int per = (k.nb + BK_NT - 1) / BK_NT;
  const int b0 = threadIdx.x * per;
  int mine = 0;
  for (int i = 0; i < per; ++i)
    if (b0 + i < k.nb) {
      const int c = __hip_atomic_exchange(&k.cnt[b0 + i], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bk_hist[b0 + i] = c;
      mine += c;
    }
  int total;
  int run = bk_exscan(mine, tmp, &total);
  for (int i = 0; i < per; ++i)
    if (b0 + i < k.nb) {
      st_agent(&k.off[b0 + i], run);
      st_agent(&k.cur[b0 + i], run);
      run += bk_hist[b0 + i];
    }
  if (threadIdx.x == 0) {
    st_agent(&k.off[k.nb], total);
    st_agent(&k.tick[0], 0);
  }
}

template <typename A, int G>
__global__ __launch_bounds__(BK_NT) void glm_bkt_fwd_kernel(const long* __restrict__ indptr,
                                                            const int* __restrict__ idx, const A* __restrict__ val,
                                                            const A* __restrict__ y, const A* __restrict__ wt,
                                                            const A* __restrict__ coef, long n, long B, int loss,
                                                            const int* __restrict__ state, A* __restrict__ wl,
                                                            BktArgs k) {
  constexpr int K = G >= 32 ? 2 : 4;
  constexpr int NG = BK_NT / G;
  extern __shared__ __align__(16) unsigned char bk_smem[];
  // [nb] hist | base | lcum | ph | pofs, then rp[rb + 1], mrow[rb], scol[ECAP], sval[ECAP]
  int* hist = reinterpret_cast<int*>(bk_smem);
  int* base = hist + k.nb;
  int* lcum = base + k.nb;
  int* ph = lcum + k.nb;
  int* pofs = ph + k.nb;
  int* rp = pofs + k.nb;
  A* mrow = reinterpret_cast<A*>(bk_smem + (((5 * (long)k.nb + k.rb + 1) * 4 + 15) & ~15L));
  int* scol = reinterpret_cast<int*>(mrow + k.rb);
  A* sval = reinterpret_cast<A*>(scol + BK_ECAP);
  __shared__ int tmp[BK_NT / 64];
  __shared__ A red[2][BK_NT / 64];
  int e;
  if (!round_running(state, e)) return;
  const long P = (n + B - 1) / B;
  const long start = (long)(e % P) * B;
  const long end = start + B < n ? start + B : n;
  const long r0 = start + (long)blockIdx.x * k.rb;
  if (r0 >= end) return;  // (the grid covers the largest batch)
  const int nr = end - r0 < k.rb ? (int)(end - r0) : k.rb;
  const long jb = indptr[r0];
  const int tid = threadIdx.x;
  for (int i = tid; i < k.nb; i += BK_NT) {
    hist[i] = 0;
    lcum[i] = 0;
  }
  for (int i = tid; i <= nr; i += BK_NT) rp[i] = (int)(indptr[r0 + i] - jb);
  __syncthreads();
  // ---- forward: a G-lane group per row (dot, loss, multiplier) + the block's bucket histogram
  const int lane = tid & (G - 1), grp = tid / G;
  const int csb = k.csb;
  A wsum = 0, lsum = 0;
  for (int q = grp; q < nr; q += NG) {
    const int s0 = rp[q], s1 = rp[q + 1];
    A s = 0;
    for (int jq = s0; jq < s1; jq += K * G) {
      int ii[K];
      A vv[K];
#pragma unroll
      for (int t = 0; t < K; ++t) {
        const int j = jq + lane + t * G;
        const bool ok = j < s1;
        const long jj = jb + (ok ? j : s0);
        ii[t] = idx[jj];
        const A v = val[jj];
        vv[t] = ok ? v : (A)0;
      }
#pragma unroll
      for (int t = 0; t < K; ++t) s += vv[t] * coef[ii[t]];
#pragma unroll
      for (int t = 0; t < K; ++t)
        if (!(k.dbg & 4) && jq + lane + t * G < s1) atomicAdd(&hist[ii[t] >> csb], 1);
    }
    s = group_sum<G>(s);
    if (lane == 0) {
      const long r = r0 + q;
      const A ww = wt ? wt[r] : (A)1;
      A l, m;
      loss_and_mult(loss, s, y[r], ww, l, m);
      mrow[q] = m;
      wsum += ww;
      lsum += l;
    }
  }
  wsum = wave_sum(wsum);
  lsum = wave_sum(lsum);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = wsum;
    red[1][tid >> 6] = lsum;
  }
  __syncthreads();
  // ---- reserve the block's run in every bucket it touches (one device atomic each)
  for (int i = tid; i < k.nb; i += BK_NT) {
    const int c = hist[i];
    base[i] = c && !(k.dbg & 1) ? atomicAdd(&k.cur[i], c) : 0;
  }
  if (tid == 0) {
    A a0 = 0, a1 = 0;
    for (int i = 0; i < BK_NT / 64; ++i) {
      a0 += red[0][i];
      a1 += red[1][i];
    }
    A* slot = wl + ((long)(e & 1) * WL_SLOTS + (blockIdx.x & (WL_SLOTS - 1))) * WL_STRIDE;
    if (a0 != (A)0) atomicAdd(&slot[0], a0);
    if (a1 != (A)0) atomicAdd(&slot[1], a1);
  }
  __syncthreads();
  // ---- the block's entries in pieces of ECAP: bucket-sorted in LDS, then stored run by run
  const int E = rp[nr];
  const uint32_t mask = (1u << csb) - 1;
  A* bval = reinterpret_cast<A*>(k.val);
  const int per = (k.nb + BK_NT - 1) / BK_NT;
  for (int p0 = 0; p0 < ((k.dbg & 2) ? 0 : E); p0 += BK_ECAP) {
    const int pe = E - p0 < BK_ECAP ? E - p0 : BK_ECAP;
    for (int i = tid; i < k.nb; i += BK_NT) ph[i] = 0;
    __syncthreads();
    int col[BK_EPT], rk[BK_EPT];
    A pv[BK_EPT];
#pragma unroll
    for (int u = 0; u < BK_EPT; ++u) {
      const int t = tid + u * BK_NT;
      col[u] = 0;
      pv[u] = 0;
      rk[u] = 0;
      if (t < pe) {
        const int j = p0 + t;
        col[u] = idx[jb + j];
        pv[u] = val[jb + j];
      }
    }
#pragma unroll
    for (int u = 0; u < BK_EPT; ++u) {
      const int t = tid + u * BK_NT;
      if (t < pe) {
        const int j = p0 + t;
        int lo = 0, hi = nr;  // the entry's row: rp[lo] <= j < rp[hi]
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (rp[mid] <= j) lo = mid; else hi = mid;
        }
        pv[u] *= mrow[lo];
        rk[u] = atomicAdd(&ph[col[u] >> csb], 1);
      }
    }
    __syncthreads();
    {  // piece offsets per bucket
      const int q0 = tid * per;
      int mine = 0;
      for (int i = 0; i < per; ++i) mine += q0 + i < k.nb ? ph[q0 + i] : 0;
      int total;
      int run = bk_exscan(mine, tmp, &total);
      for (int i = 0; i < per; ++i)
        if (q0 + i < k.nb) {
          pofs[q0 + i] = run;
          run += ph[q0 + i];
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < BK_EPT; ++u) {
      const int t = tid + u * BK_NT;
      if (t < pe) {
        const int slot = pofs[col[u] >> csb] + rk[u];
        scol[slot] = col[u];
        sval[slot] = pv[u];
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < BK_EPT; ++u) {
      const int t = tid + u * BK_NT;
      if (t < pe) {
        const int c = scol[t];
        const int bk = c >> csb;
        const long dst = (long)base[bk] + lcum[bk] + (t - pofs[bk]);
        k.key[dst] = (uint16_t)(c & mask);
        bval[dst] = sval[t];
      }
    }
    __syncthreads();
    for (int i = tid; i < k.nb; i += BK_NT) lcum[i] += ph[i];
    // (the next piece's first barrier orders these updates before their reads)
  }
}

template <typename A, bool FUSE>
__global__ __launch_bounds__(BK_NT) void glm_bkt_bwd_kernel(const long* __restrict__ indptr, long n, int d, long B,
                                                            int* __restrict__ state, A* __restrict__ wl,
                                                            A* __restrict__ fb, A* __restrict__ coef, int max_iter,
                                                            A tol, A lr, A reg, A en, int weighted, BktArgs k) {
  extern __shared__ __align__(16) unsigned char bk_smem[];
  A* slab = reinterpret_cast<A*>(bk_smem);                     // [2^csb]
  int* iofs = reinterpret_cast<int*>(slab + (1 << k.csb));      // [nb + 1] first item of each bucket
  __shared__ int tmp[BK_NT / 64];
  __shared__ int sflag;
  int e;
  const bool run = round_running(state, e);
  if (blockIdx.x == 0 && threadIdx.x < WL_SLOTS) {  // re-arm the other parity's Σw/Σloss slots
    A* o = wl + ((long)((e + 1) & 1) * WL_SLOTS + threadIdx.x) * WL_STRIDE;
    o[0] = 0;
    o[1] = 0;
  }
  if (!run) {
    if (FUSE) arrive_and_advance(state, e, false, 0);
    return;
  }
  const long P = (n + B - 1) / B;
  const long b = (long)(e % P);
  A W, L = 0;
  if (weighted || (!FUSE && blockIdx.x == 0)) slot_sums(wl, e, W, L);
  if (!weighted) {
    const long end = (b + 1) * B < n ? (b + 1) * B : n;
    W = (A)(end - b * B);
  }
  // work items: chunks of `chunk` entries of each bucket (at least one per bucket: every column is
  // updated, regularisation included)
  const int per = (k.nb + BK_NT - 1) / BK_NT;
  {
    const int q0 = threadIdx.x * per;
    int mine = 0;
    for (int i = 0; i < per; ++i)
      if (q0 + i < k.nb) {
        const int len = k.off[q0 + i + 1] - k.off[q0 + i];
        mine += len > k.chunk ? (len + k.chunk - 1) / k.chunk : 1;
      }
    int total;
    int r = bk_exscan(mine, tmp, &total);
    for (int i = 0; i < per; ++i)
      if (q0 + i < k.nb) {
        iofs[q0 + i] = r;
        const int len = k.off[q0 + i + 1] - k.off[q0 + i];
        r += len > k.chunk ? (len + k.chunk - 1) / k.chunk : 1;
      }
    if (threadIdx.x == 0) iofs[k.nb] = total;
  }
  __syncthreads();
  const int T = iofs[k.nb];
  const int CS = 1 << k.csb;
  const A* __restrict__ bval = reinterpret_cast<const A*>(k.val);
  A* acc = reinterpret_cast<A*>(k.acc);
  for (int it = blockIdx.x; it < T; it += gridDim.x) {
    int lo = 0, hi = k.nb;  // iofs[lo] <= it < iofs[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (iofs[mid] <= it) lo = mid; else hi = mid;
    }
    const int bk = lo, nch = iofs[bk + 1] - iofs[bk], ch = it - iofs[bk];
    for (int c = threadIdx.x; c < CS; c += BK_NT) slab[c] = (A)0;
    __syncthreads();
    const int bo = k.off[bk], be = k.off[bk + 1];
    const int k0 = bo + ch * k.chunk;
    const int k1 = k0 + k.chunk < be ? k0 + k.chunk : be;
    int q = k0 + threadIdx.x;
    for (; q + (BK_UNROLL - 1) * BK_NT < k1; q += BK_UNROLL * BK_NT) {
      uint16_t kk[BK_UNROLL];
      A vv[BK_UNROLL];
#pragma unroll
      for (int u = 0; u < BK_UNROLL; ++u) {
        kk[u] = __builtin_nontemporal_load(k.key + q + u * BK_NT);
        vv[u] = __builtin_nontemporal_load(bval + q + u * BK_NT);
      }
#pragma unroll
      for (int u = 0; u < BK_UNROLL; ++u) atomicAdd(&slab[kk[u]], vv[u]);
    }
    for (; q < k1; q += BK_NT) atomicAdd(&slab[k.key[q]], bval[q]);
    __syncthreads();
    const long c0 = (long)bk << k.csb;
    const int cols = d - c0 < CS ? (int)(d - c0) : CS;
    if (nch == 1) {
      for (int c = threadIdx.x; c < cols; c += BK_NT) {
        if (FUSE)
          coef[c0 + c] = sgd_apply<A>(coef[c0 + c], slab[c], W, lr, reg, en);
        else
          fb[c0 + c] = slab[c];
      }
    } else {
      for (int c = threadIdx.x; c < cols; c += BK_NT) atomicAdd(&acc[c0 + c], slab[c]);
      if (arrive_last(&k.done[bk], nch, &sflag)) {
        for (int c = threadIdx.x; c < cols; c += BK_NT) {
          const A g = __hip_atomic_exchange(&acc[c0 + c], (A)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (FUSE)
            coef[c0 + c] = sgd_apply<A>(coef[c0 + c], g, W, lr, reg, en);
          else
            fb[c0 + c] = g;
        }
        if (threadIdx.x == 0) st_agent(&k.done[bk], 0);
      }
    }
    __syncthreads();
  }
  if (!FUSE && blockIdx.x == 0 && threadIdx.x == 0) {
    fb[d] = W;
    fb[d + 1] = L;
  }
  if (FUSE) {
    __shared__ int last;
    __syncthreads();
    if (threadIdx.x == 0)
      last = __hip_atomic_fetch_add(&state[ST_ARRIVE], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (int)gridDim.x - 1;
    __syncthreads();
    if (last) {  // every other block has finished its reads of the state words
      A w2;
      slot_sums(wl, e, w2, L);
      if (threadIdx.x == 0) {
        const bool cont = (e + 1 < max_iter) && (L / W > tol);
        state[ST_RUN0 + ((e + 1) & 1)] = cont ? 1 : 0;
        state[ST_EXECUTED] += 1;
        state[ST_ROUND] = e + 1;
        state[ST_ARRIVE] = 0;
      }
    }
  }
}

}  // namespace

static long long* g_sparse_trace = nullptr;  // per-block timestamps of the tiled backward (diagnostics)
FMLX_API void fmlx_glm_sparse_set_trace(void* trace) { g_sparse_trace = (long long*)trace; }

FMLX_API int fmlx_glm_grad_csr(int acc_f64, const long* indptr, const int* idx, const void* val, const void* y,
                               const void* wt, const void* coef, long n, int d, long B, int loss, const int* state,
                               void* grad, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  long waves = B < n ? B : n;
  int blocks = (int)((waves + 3) / 4);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  if (acc_f64)
    hipLaunchKernelGGL(glm_grad_csr_kernel<double>, dim3(blocks), dim3(256), 0, s, indptr, idx, (const double*)val,
                       (const double*)y, (const double*)wt, (const double*)coef, n, d, B, loss, state, (double*)grad);
  else
    hipLaunchKernelGGL(glm_grad_csr_kernel<float>, dim3(blocks), dim3(256), 0, s, indptr, idx, (const float*)val,
                       (const float*)y, (const float*)wt, (const float*)coef, n, d, B, loss, state, (float*)grad);
  return (int)hipGetLastError();
}

static int g_csc_fwd_cap = 65535, g_csc_bwd_cap = 1024, g_csc_tile_cap = 0;  // 0: CUs × tile blocks per CU

FMLX_API void fmlx_glm_set_csc_tuning(int fwd_cap, int bwd_cap) {
  g_csc_fwd_cap = fwd_cap > 0 ? fwd_cap : 65535;
  g_csc_bwd_cap = bwd_cap > 0 ? bwd_cap : 1024;
  g_csc_tile_cap = bwd_cap > 0 ? bwd_cap : 0;
}

// tiled backward: the column tiles of the batches (BatchCsc.tiles) and the packing of erow
// forward cells in XCD-aware order (default; fmlx_glm_set_cell_xcd(0): launch order) — 63.5 → 61.4 µs
// per SVC round, profiles/r5/svc_cell_forward_ab.jsonl
static int g_cell_xcd = 1;
struct CscTiles {
  const int2* tiles;  // [P][tstride] (start column, first entry) per tile (nullptr: untiled layout)
  const int* ntiles;  // int32 [P]
  int tstride, rb, EL, ET;  // EL: heavy-column threshold (entries)
  // row-block × column-split cells of the forward (cent == nullptr: the one-row-per-group forward)
  const uint32_t* cent;
  const void* cval;
  const int* roff;  // [P][rstride] first entry of every (cell, row): cell·2^CELL_RBB + row
  int rstride, rbb, S, CS, cb, cells;  // cells: grid (cells of the largest batch); rows per block 2^rbb
  int cmax;         // entries of the largest cell (its LDS slots)
  void* partial;    // [cells][2^CELL_RBB] row partials
  int* cnt;         // [row blocks] arrival tickets (zeroed once, re-armed by the finishers)
};
FMLX_API int fmlx_glm_wl_elems() { return 2 * WL_SLOTS * WL_STRIDE; }

template <typename A, int G>
static void launch_csc_round(const long* indptr, const int* idx, const A* val, const A* y, const A* wt, A* coef,
                             long n, int d, long B, int loss, int* state, A* mult, A* wl, const int* colptr,
                             const int* erow, const A* eval, A* fb, int fuse, int max_iter, A tol, A lr, A reg, A en,
                             const CscTiles& ti, hipStream_t s) {
  if (ti.cent != nullptr) {
    hipLaunchKernelGGL(glm_csr_cell_fwd_kernel<A>, dim3(ti.cells), dim3(CELL_THREADS), (size_t)ti.cmax * sizeof(A),
                       s, indptr, ti.cent, (const A*)ti.cval, ti.roff, (long)ti.rstride, ti.rbb, ti.S, ti.CS, ti.cb, y, wt,
                       (const A*)coef, n, B, loss, state, mult, wl, (A*)ti.partial, ti.cnt, g_cell_xcd);
  } else {
    const long groups = B < n ? B : n;
    long fb_blocks = (groups * G + 255) / 256;  // one row per lane group: the batch in one pass
    if (fb_blocks > g_csc_fwd_cap) fb_blocks = g_csc_fwd_cap;
    if (fb_blocks < 1) fb_blocks = 1;
    hipLaunchKernelGGL((glm_csr_fwd_kernel<A, G>), dim3((int)fb_blocks), dim3(256), 0, s, indptr, idx, val, y, wt,
                       (const A*)coef, n, B, loss, state, mult, wl);
  }
  const int weighted = wt != nullptr;
  if (ti.tiles != nullptr) {
    const size_t lds = (size_t)ti.ET * sizeof(A);
    int per_cu = (int)(LDS_PER_CU / (lds + 2048));
    per_cu = per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu);  // ≤ 32 waves per CU at 1024 threads
    int tb = g_csc_tile_cap > 0 ? g_csc_tile_cap : NUM_CU * per_cu;
    if (tb > ti.tstride) tb = ti.tstride;
#define FMLX_TILE_BWD(F)                                                                                             \
  hipLaunchKernelGGL((glm_csc_tile_bwd_kernel<A, F>), dim3(tb), dim3(TILE_THREADS), lds, s, indptr, colptr, ti.tiles, \
                     ti.ntiles, ti.tstride, erow, eval, (const A*)mult, n, d, B, ti.rb, ti.EL, state, wl, fb, coef,    \
                     max_iter, tol, lr, reg, en, weighted, g_sparse_trace)
    if (fuse)
      FMLX_TILE_BWD(true);
    else
      FMLX_TILE_BWD(false);
#undef FMLX_TILE_BWD
    return;
  }
  int bb = (d + 255) / 256;  // grid-strided: each block takes the arrival ticket once
  if (bb > g_csc_bwd_cap) bb = g_csc_bwd_cap;
  if (fuse)
    hipLaunchKernelGGL((glm_csc_bwd_kernel<A, true>), dim3(bb), dim3(256), 0, s, indptr, colptr, erow, eval,
                       (const A*)mult, n, d, B, state, wl, fb, coef, max_iter, tol, lr, reg, en, weighted);
  else
    hipLaunchKernelGGL((glm_csc_bwd_kernel<A, false>), dim3(bb), dim3(256), 0, s, indptr, colptr, erow, eval,
                       (const A*)mult, n, d, B, state, wl, fb, coef, max_iter, tol, lr, reg, en, weighted);
}

template <typename A>
static int dispatch_csc_round(int G, const long* indptr, const int* idx, const void* val, const void* y,
                              const void* wt, void* coef, long n, int d, long B, int loss, int* state, void* mult,
                              void* wl, const int* colptr, const int* erow, const void* eval, void* fb, int fuse,
                              int max_iter, double tol, double lr, double reg, double en, const CscTiles& ti,
                              hipStream_t s) {
#define FMLX_CSC(GG)                                                                                                 \
  launch_csc_round<A, GG>(indptr, idx, (const A*)val, (const A*)y, (const A*)wt, (A*)coef, n, d, B, loss, state,     \
                          (A*)mult, (A*)wl, colptr, erow, (const A*)eval, (A*)fb, fuse, max_iter, (A)tol, (A)lr,     \
                          (A)reg, (A)en, ti, s)
  switch (G) {
    case 4: FMLX_CSC(4); break;
    case 8: FMLX_CSC(8); break;
    case 16: FMLX_CSC(16); break;
    case 32: FMLX_CSC(32); break;
    case 64: FMLX_CSC(64); break;
    default: return -1;
  }
#undef FMLX_CSC
  return (int)hipGetLastError();
}

// One sparse SGD round through the per-batch transpose (see glm_csc_bwd_kernel). fuse=1: the
// backward applies the update + termination (1 GPU); fuse=0: it writes fb[d+2] for the
// all-reduce and fmlx_glm_update follows.
FMLX_API void fmlx_glm_set_cell_xcd(int on) { g_cell_xcd = on != 0; }

FMLX_API int fmlx_glm_csc_round(int acc_f64, int G, const long* indptr, const int* idx, const void* val,
                                const void* y, const void* wt, void* coef, long n, int d, long B, int loss, int* state,
                                void* mult, void* wl, const int* colptr, const int* erow, const void* eval, void* fb,
                                int fuse, int max_iter, double tol, double lr, double reg, double en,
                                const int* tiles, const int* ntiles, int tstride, int rb, int EL, int ET,
                                const uint32_t* cent, const void* cval, const int* roff, int rstride, int rbb, int S,
                                int CS, int cb, int cells, int cmax, void* partial, int* ccnt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n <= 0 || B <= 0) return -2;
  const CscTiles ti{reinterpret_cast<const int2*>(tiles), ntiles, tstride, rb, EL, ET, cent, cval, roff, rstride,
                    rbb, S, CS, cb, cells, cmax, partial, ccnt};
  if (cent != nullptr) {
    // (cell ids, packed entries and the row blocks of the largest batch: host-checked sizes)
    const long lds = (long)cmax * (acc_f64 ? 8 : 4);
    if (cval == nullptr || roff == nullptr || partial == nullptr || ccnt == nullptr || S < 1 || CS < 1 || cb < 1 ||
        cb >= 32 || rbb < 1 || rbb > CELL_RBB_MAX || cells < 1 || (long)rstride < ((long)cells << rbb) + 1 ||
        (long)CS * S < d || cmax < 0 ||
        cmax > (int)(1u << (32 - cb)) || lds > 150 * 1024)
      return -5;
  }
  if (tiles != nullptr) {
    const size_t esz = acc_f64 ? 8 : 4;
    // the packed erow (row | slot << rb) and the LDS slot array of a light tile (< ET entries)
    if (rb < 1 || ET < 2 || EL < 1 || EL >= ET || tstride < 2 || (size_t)ET * esz > (size_t)LDS_PER_CU - 1024) return -3;
    if (((long)ET - 1) >> (32 - rb) != 0 || (B - 1) >> rb != 0) return -4;
  }
  if (acc_f64)
    return dispatch_csc_round<double>(G, indptr, idx, val, y, wt, coef, n, d, B, loss, state, mult, wl, colptr, erow,
                                      eval, fb, fuse, max_iter, tol, lr, reg, en, ti, s);
  return dispatch_csc_round<float>(G, indptr, idx, val, y, wt, coef, n, d, B, loss, state, mult, wl, colptr, erow,
                                   eval, fb, fuse, max_iter, tol, lr, reg, en, ti, s);
}

FMLX_API int fmlx_glm_csr_predict(int acc_f64, const long* indptr, const int* idx, const void* val, const void* coef,
                                  long n, double* dots, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return 0;
  int blocks = (int)((n + 3) / 4);
  if (blocks > 4096) blocks = 4096;
  if (acc_f64)
    hipLaunchKernelGGL(glm_csr_predict_kernel<double>, dim3(blocks), dim3(256), 0, s, indptr, idx, (const double*)val,
                       (const double*)coef, n, dots);
  else
    hipLaunchKernelGGL(glm_csr_predict_kernel<float>, dim3(blocks), dim3(256), 0, s, indptr, idx, (const float*)val,
                       (const float*)coef, n, dots);
  return (int)hipGetLastError();
}

// ---- single-visit bucket round (glm_bkt_*) ----
static int g_bkt_dbg = 0;
FMLX_API void fmlx_glm_bkt_set_debug(int v) { g_bkt_dbg = v; }
FMLX_API int fmlx_glm_bkt_limits(int* out) {
  out[0] = BK_NT;
  out[1] = BK_ECAP;
  out[2] = BK_NB_MAX;
  return 0;
}

static size_t bkt_fwd_lds(const BktArgs& k, size_t es) {
  return (((5 * (size_t)k.nb + k.rb + 1) * 4 + 15) & ~(size_t)15) + (size_t)k.rb * es + BK_ECAP * (4 + es);
}

template <typename A, int G>
static void launch_bkt_round(const long* indptr, const int* idx, const A* val, const A* y, const A* wt, A* coef,
                             long n, int d, long B, int loss, int* state, A* wl, A* fb, int fuse, int max_iter, A tol,
                             A lr, A reg, A en, const BktArgs& k, int bwd_blocks, hipStream_t s) {
  hipLaunchKernelGGL(glm_bkt_count_kernel<A>, dim3(NUM_CU), dim3(BK_NT), (size_t)k.nb * 4, s, indptr, idx, n, B,
                     state, k);
  const long rows = B < n ? B : n;
  const int fblocks = (int)((rows + k.rb - 1) / k.rb);
  hipLaunchKernelGGL((glm_bkt_fwd_kernel<A, G>), dim3(fblocks), dim3(BK_NT), bkt_fwd_lds(k, sizeof(A)), s, indptr, idx,
                     val, y, wt, (const A*)coef, n, B, loss, state, wl, k);
  const size_t blds = ((size_t)1 << k.csb) * sizeof(A) + ((size_t)k.nb + 1) * 4;
  const int weighted = wt != nullptr;
  if (fuse)
    hipLaunchKernelGGL((glm_bkt_bwd_kernel<A, true>), dim3(bwd_blocks), dim3(BK_NT), blds, s, indptr, n, d, B, state,
                       wl, fb, coef, max_iter, tol, lr, reg, en, weighted, k);
  else
    hipLaunchKernelGGL((glm_bkt_bwd_kernel<A, false>), dim3(bwd_blocks), dim3(BK_NT), blds, s, indptr, n, d, B, state,
                       wl, fb, coef, max_iter, tol, lr, reg, en, weighted, k);
}

// One sparse SGD round through column-slice buckets (see glm_bkt_count_kernel …). fuse=1: the
// backward applies the update + termination (1 GPU); fuse=0: it writes fb[d+2] for the
// all-reduce and fmlx_glm_update follows. Host-checked: key/val hold the largest batch's entries,
// acc[d], cnt/done[nb] and tick[2] are zero, off[nb + 1] and cur[nb] exist.
FMLX_API int fmlx_glm_bkt_round(int acc_f64, int G, const long* indptr, const int* idx, const void* val,
                                const void* y, const void* wt, void* coef, long n, int d, long B, int loss, int* state,
                                void* wl, void* fb, int fuse, int max_iter, double tol, double lr, double reg,
                                double en, int csb, int rb, int chunk, int* cnt, int* off, int* cur, int* tick,
                                int* done, void* key, void* bval, void* acc, int bwd_blocks, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n <= 0 || B <= 0 || d <= 0) return -2;
  const size_t es = acc_f64 ? 8 : 4;
  if (csb < 1 || csb > 16 || ((size_t)es << csb) > 64 * 1024) return -3;
  const long nb = ((long)d + (1L << csb) - 1) >> csb;
  if (nb > BK_NB_MAX || rb < BK_NT / G || rb > 4096 || chunk < BK_NT || bwd_blocks < 1) return -4;
  const BktArgs k{csb, (int)nb, rb, chunk, cnt, off, cur, tick, done, (uint16_t*)key, bval, acc, g_bkt_dbg};
  if (bkt_fwd_lds(k, es) > (size_t)LDS_PER_CU / 2) return -5;
#define FMLX_BKT(GG)                                                                                                  \
  if (acc_f64)                                                                                                        \
    launch_bkt_round<double, GG>(indptr, idx, (const double*)val, (const double*)y, (const double*)wt, (double*)coef,  \
                                 n, d, B, loss, state, (double*)wl, (double*)fb, fuse, max_iter, tol, lr, reg, en, k, \
                                 bwd_blocks, s);                                                                      \
  else                                                                                                                \
    launch_bkt_round<float, GG>(indptr, idx, (const float*)val, (const float*)y, (const float*)wt, (float*)coef, n, d, \
                                B, loss, state, (float*)wl, (float*)fb, fuse, max_iter, (float)tol, (float)lr,        \
                                (float)reg, (float)en, k, bwd_blocks, s);
  switch (G) {
    case 4: FMLX_BKT(4); break;
    case 8: FMLX_BKT(8); break;
    case 16: FMLX_BKT(16); break;
    case 32: FMLX_BKT(32); break;
    case 64: FMLX_BKT(64); break;
    default: return -1;
  }
#undef FMLX_BKT
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
