// Per-batch column-major copies for the sparse SGD trainer (ops/glm.py BatchCsc; consumed by
// glm.hip glm_csc_bwd_kernel). A run of consecutive batches b0 … b1−1 (rows r0 … r1−1, CSR
// entries j0 … j1−1) is transposed by
//
//   csc_keys    one wave per row: key = slot·d + column (slot = batch within the run), the
//               entry's batch-relative row, and the identity payload for the sort
//   (stable segmented radix sort of the keys by column, one segment per batch: radix.hip)
//   csc_fill    erow / evals of the run in sorted order, written straight into the partition-wide
//               arrays (one gather of the row id and of the value per entry; fp64 values)
//   csc_keys64  fp32 values: (value bits, row) ride through the sort as one 64-bit payload that
//               the sort's last pass splits straight into erow / evals (radix.hip split output)
//   csc_colptr  every batch's dense column pointer straight from the sorted keys: thread i writes
//               the bins (key[i−1], key[i]] (each bin exactly once), relative to its batch's first
//               entry, which is indptr[batch·B] − j0 (a batch's entries are its own CSR range)
//
// and, for the tiled backward (glm.hip glm_csc_tile_bwd_kernel), a post-pass over each built batch:
//
//   csc_tiles      the batch's columns cut into tiles: runs of consecutive columns holding at most
//                  ET = EB + EL entries, or one "heavy" column of more than EL entries (start flags
//                  from the column pointer: per-chunk counts, their scan, the starts written)
//   csc_tile_keys  per entry: key = tile · 2^(rb+pb) | row · 2^pb | position in the tile's
//                  column-ordered range (pb bits), payload = the fp32 value bits / the entry index
//   (stable radix sort of the keys' tile and row bits: entries row-sorted inside their tile)
//   csc_tile_store erow := row | position << rb (the backward's packed LDS slot), evals in the
//                  new order
//
// replacing ~10 torch ops and their run-sized temporaries (repeat_interleave of the row ids and
// slots, int64 sort indices, gather copies, the bucket-start array and its two slicing copies):
// a whole fit that transposes its batches lazily pays for those allocations inside the fit.
#include <algorithm>

#include "common.h"

namespace {

__global__ __launch_bounds__(256) void csc_keys_kernel(const long* __restrict__ indptr, const int* __restrict__ idx,
                                                       long r0, long r1, long B, int d, long j0,
                                                       int* __restrict__ key, int* __restrict__ rel,
                                                       int* __restrict__ iota) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = r0 + wave; r < r1; r += nw) {
    const long s0 = indptr[r], s1 = indptr[r + 1];
    const long slot = (r - r0) / B;
    const int kb = (int)(slot * d);
    const int rr = (int)(r - r0 - slot * B);
    for (long j = s0 + lane; j < s1; j += 64) {
      const long o = j - j0;
      key[o] = kb + idx[j];
      rel[o] = rr;
      iota[o] = (int)o;
    }
  }
}

// fp32 values: the payload is (value bits << 32) | batch-relative row, so the sort moves both and
// the copy out is sequential (no random gathers; csc_fill's two gathers per entry cost ~4× more).
// A wave takes KR_ROWS consecutive rows per step: one load brings their KR_ROWS + 1 row starts (a
// lane each), their entries are one contiguous range whose loads all go out together (a lane finds
// its entry's row among the KR_ROWS starts), and the slot division is done once per row. (A wave
// per row — indptr, then entries, then the next row — measured 233 µs over 64M entries: 89 % of
// wave cycles waiting on memory.)
constexpr int KR_ROWS = 8;
constexpr int KR_K = 4;  // 64-entry chunks per lane in flight

__global__ __launch_bounds__(256) void csc_keys64_kernel(const long* __restrict__ indptr, const int* __restrict__ idx,
                                                         const float* __restrict__ values, long r0, long r1, long B,
                                                         int d, long j0, int* __restrict__ key,
                                                         uint64_t* __restrict__ payload, int pack) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long rg = r0 + wave * KR_ROWS; rg < r1; rg += nw * KR_ROWS) {
    const int nr = r1 - rg < KR_ROWS ? (int)(r1 - rg) : KR_ROWS;
    // lane q <= nr: start of row rg + q; lane q < nr: that row's slot key base and batch row
    const long ip = lane <= nr ? indptr[rg + lane] : 0;
    int kbl = 0;
    uint32_t rrl = 0;
    if (lane < nr) {
      const long rel = rg + lane - r0;
      const long slot = rel / B;
      kbl = (int)(slot * d);
      rrl = (uint32_t)(rel - slot * B);
    }
    long st[KR_ROWS + 1];
#pragma unroll
    for (int q = 0; q <= KR_ROWS; ++q) st[q] = __shfl(ip, q < nr ? q : nr, 64);  // uniform
    const long e0 = st[0], e1 = st[KR_ROWS];
    for (long jb = e0; jb < e1; jb += 64 * KR_K) {
      int iv[KR_K];
      float vv[KR_K];
#pragma unroll
      for (int k = 0; k < KR_K; ++k) {
        const long j = jb + k * 64 + lane;
        const long jj = j < e1 ? j : e0;
        iv[k] = __builtin_nontemporal_load(idx + jj);
        vv[k] = __builtin_nontemporal_load(values + jj);
      }
#pragma unroll
      for (int k = 0; k < KR_K; ++k) {
        const long j = jb + k * 64 + lane;
        int q = 0;
#pragma unroll
        for (int t = 1; t < KR_ROWS; ++t) q += j >= st[t] ? 1 : 0;  // row of entry j (st ascends)
        const int kb = __shfl(kbl, q, 64);
        const uint32_t rr = (uint32_t)__shfl((int)rrl, q, 64);
        if (j < e1) {
          const long o = j - j0;
          if (key != nullptr) key[o] = kb + iv[k];  // (the bucket path sorts the CSR columns instead)
          // pack: the column's low 10 bits ride at bits 22..31 above the 22-bit batch row
          const uint32_t lo = pack ? (rr | ((uint32_t)iv[k] & 1023u) << 22) : rr;
          payload[o] = ((uint64_t)__float_as_uint(vv[k]) << 32) | lo;
        }
      }
    }
  }
}

template <typename V>
__global__ __launch_bounds__(256) void csc_fill_kernel(const int* __restrict__ order, long m, long j0,
                                                       const int* __restrict__ rel, const V* __restrict__ values,
                                                       int* __restrict__ erow, V* __restrict__ evals) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const int o = order[i];
    erow[j0 + i] = rel[o];
    evals[j0 + i] = values[j0 + o];
  }
}

constexpr int CP_MAXS = 32;  // batches per run (radix.hip RS_MAXS)

// every batch's first entry relative to the run's (a kernel argument: no dependent indptr loads)
struct RunStarts {
  int start[CP_MAXS + 1];
};

// thread t owns boundaries i = 4t … 4t + 3 (one 16-B load of keys[4t … 4t+3] plus key[4t − 1]);
// int32 index math (slots·d < 2^31, m < 2^31: host-checked), one division per boundary with
// bins, the batch starts from the argument table — the one-boundary-per-thread int64 form with an
// indptr load per bin measured 241 µs over 64M keys (1 TB/s)
__global__ __launch_bounds__(256) void csc_colptr_kernel(const int* __restrict__ keys, int m, int slots, int d,
                                                         RunStarts rs, long b0, int* __restrict__ colptr) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int i0 = t * 4;
  if (i0 > m) return;
  const int nb = slots * d;
  int k[5];
  k[0] = i0 > 0 ? keys[i0 - 1] : -1;
  if (i0 + 4 <= m) {
    const int4 v = *reinterpret_cast<const int4*>(keys + i0);
    k[1] = v.x; k[2] = v.y; k[3] = v.z; k[4] = v.w;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) k[q + 1] = i0 + q < m ? keys[i0 + q] : nb;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = i0 + q;
    if (i > m) break;
    const int lo = k[q], hi = i < m ? k[q + 1] : nb;
    if (hi <= lo) continue;
    // bins (lo, hi]: c = s·d + cc walked with a carried (s, cc)
    int c = lo + 1;
    int s = c / d, cc = c - s * d;
    for (; c <= hi; ++c, ++cc) {
      if (cc == d) {
        cc = 0;
        ++s;
      }
      if (cc == 0 && s > 0)  // the previous batch ends here: its entry count
        colptr[(b0 + s - 1) * (d + 1) + d] = i - rs.start[s - 1];
      if (s < slots) colptr[(b0 + s) * (d + 1) + cc] = i - rs.start[s];
    }
  }
}

// ---------------------------- row-sorted column tiles ----------------------------------------
constexpr int TL_THREADS = 1024;

// column c starts a tile: the first column, a heavy column (> EL entries) or the one after it, or
// the column whose first entry falls in a later EB-entry bucket than its predecessor's. A light
// tile's columns then start inside one bucket, so it holds < EB + (its last column's ≤ EL)
// entries; tiles average about EB entries.
__device__ __forceinline__ bool tile_start(const int* __restrict__ cp, int c, int EB, int EL) {
  if (c == 0) return true;
  const int a = cp[c - 1], b = cp[c], z = cp[c + 1];
  return z - b > EL || b - a > EL || b / EB != a / EB;
}

// three passes over a batch's columns, TL_CHUNK per block: count the tile starts of every chunk,
// scan the chunk counts (one block per batch), write the starts at the scanned offsets. (One block
// walking the 1M column pointers of a batch serially took ~0.4 ms per batch.)
constexpr int TL_CHUNK = 256;

__device__ __forceinline__ int chunk_rank(bool f, int& total) {  // exclusive rank of f in the block
  __shared__ int wc[TL_CHUNK / 64];
  const unsigned long long m = __ballot(f);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) wc[w] = __popcll(m);
  __syncthreads();
  int off = 0;
  total = 0;
#pragma unroll
  for (int i = 0; i < TL_CHUNK / 64; ++i) {
    off += i < w ? wc[i] : 0;
    total += wc[i];
  }
  return off + __popcll(m & ((1ull << lane) - 1));
}

__global__ __launch_bounds__(TL_CHUNK) void csc_tiles_count_kernel(const int* __restrict__ colptr, long b0, int d,
                                                                   int EB, int EL, int nchunks, int* __restrict__ cnt) {
  const long b = b0 + blockIdx.y;
  const int c = blockIdx.x * TL_CHUNK + threadIdx.x;
  const bool f = c < d && tile_start(colptr + b * (long)(d + 1), c, EB, EL);
  int total;
  chunk_rank(f, total);
  if (threadIdx.x == 0) cnt[(long)blockIdx.y * nchunks + blockIdx.x] = total;
}

__global__ __launch_bounds__(TL_THREADS) void csc_tiles_scan_kernel(int* __restrict__ cnt, int nchunks,
                                                                    const int* __restrict__ colptr, long b0, int d,
                                                                    int2* __restrict__ tiles, int tstride,
                                                                    int* __restrict__ ntiles) {
  int* __restrict__ cc = cnt + (long)blockIdx.x * nchunks;
  const int per = (nchunks + TL_THREADS - 1) / TL_THREADS;
  const int i0 = (int)threadIdx.x * per;
  int loc = 0;
  for (int i = i0; i < i0 + per && i < nchunks; ++i) loc += cc[i];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  __shared__ int wtot[TL_THREADS / 64];
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  int off = inc - loc;
  for (int i = 0; i < w; ++i) off += wtot[i];
  for (int i = i0; i < i0 + per && i < nchunks; ++i) {  // counts → exclusive offsets, in place
    const int v = cc[i];
    cc[i] = off;
    off += v;
  }
  if (threadIdx.x == TL_THREADS - 1) {
    const long b = b0 + blockIdx.x;
    const int nt = off < tstride - 1 ? off : tstride - 1;  // (bounded by construction)
    tiles[b * (long)tstride + nt] = make_int2(d, colptr[b * (long)(d + 1) + d]);  // sentinel
    ntiles[b] = nt;
  }
}

__global__ __launch_bounds__(TL_CHUNK) void csc_tiles_write_kernel(const int* __restrict__ colptr, long b0, int d,
                                                                   int EB, int EL, int nchunks,
                                                                   const int* __restrict__ offs,
                                                                   int2* __restrict__ tiles, int tstride) {
  const long b = b0 + blockIdx.y;
  const int c = blockIdx.x * TL_CHUNK + threadIdx.x;
  const int* __restrict__ cp = colptr + b * (long)(d + 1);
  const bool f = c < d && tile_start(cp, c, EB, EL);
  int total;
  const int r = chunk_rank(f, total) + offs[(long)blockIdx.y * nchunks + blockIdx.x];
  if (f && r < tstride - 1) tiles[b * (long)tstride + r] = make_int2(c, cp[c]);
}

// one block per tile (grid-strided over the run's batches' tiles, batch by blockIdx.y)
template <typename V>
__global__ __launch_bounds__(256) void csc_tile_keys_kernel(const int* __restrict__ colptr, long b0, int d,
                                                            const int2* __restrict__ tiles, int tstride,
                                                            const int* __restrict__ ntiles, const long* __restrict__ bstart,
                                                            const int* __restrict__ erow, const V* __restrict__ evals,
                                                            long j0, int rb, int pb, int EL, uint64_t* __restrict__ keys,
                                                            uint32_t* __restrict__ pay) {
  const long b = b0 + blockIdx.y;
  const int* __restrict__ cp = colptr + b * (long)(d + 1);
  const int2* __restrict__ tl = tiles + b * (long)tstride;
  const long base = bstart[blockIdx.y];  // the batch's first entry (absolute)
  const int nt = ntiles[b];
  for (int t = blockIdx.x; t < nt; t += gridDim.x) {
    const int2 ta = tl[t], tz = tl[t + 1];
    const int k0 = ta.y, k1 = tz.y;
    const bool heavy = tz.x - ta.x == 1 && k1 - k0 > EL;
    for (int k = k0 + (int)threadIdx.x; k < k1; k += 256) {
      const long a = base + k;
      const uint64_t pos = heavy ? 0 : (uint64_t)(k - k0);
      keys[a - j0] = ((uint64_t)t << (rb + pb)) | ((uint64_t)(uint32_t)erow[a] << pb) | pos;
      if constexpr (sizeof(V) == 4)
        pay[a - j0] = __float_as_uint(evals[a]);
      else
        pay[a - j0] = (uint32_t)(a - j0);
    }
  }
}

// sorted order → erow (row | pos << rb) and evals (fp32: from the payload; fp64: gathered from a
// copy of the run's values, `src`)
template <typename V>
__global__ __launch_bounds__(256) void csc_tile_store_kernel(const uint64_t* __restrict__ keys,
                                                             const uint32_t* __restrict__ pay, long m, long j0, int rb,
                                                             int pb, const V* __restrict__ src, int* __restrict__ erow,
                                                             V* __restrict__ evals) {
  const uint64_t rmask = (1ull << rb) - 1, pmask = (1ull << pb) - 1;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const uint64_t k = keys[i];
    const uint32_t row = (uint32_t)((k >> pb) & rmask), pos = (uint32_t)(k & pmask);
    erow[j0 + i] = (int)(row | (pos << rb));
    if constexpr (sizeof(V) == 4)
      evals[j0 + i] = __uint_as_float(pay[i]);
    else
      evals[j0 + i] = src[pay[i]];
  }
}

// ---------------------------- row-block × column-split cells (sparse forward) ----------------
// glm.hip glm_csr_cell_fwd_kernel reads each batch as cells: rows [rb·RB, (rb+1)·RB) of the batch ×
// columns [s·CS, (s+1)·CS), cell id rb·S + s. A cell's entries are stored column-sorted (its
// coefficient gathers walk one column slice in order: lanes of a wave instruction share cache
// lines), each packed as (column − s·CS) | pos << cb, pos = the entry's rank in the cell's
// row-major order: the kernel writes each product into LDS slot pos and sums every row's slots
// from the row offsets of the cell (no float atomics).
//   cell_keys    wave per row: key = (cell << (RBB + cb)) | row-in-block << cb | (col − s·CS),
//                payload = fp32 value bits / the entry's run index (fp64)
//   sort A       stable on the (cell, row) bits: row-major cells (CSR order within a row)
//   cell_bounds  first entry of every (cell, row) id = cell·RB + row: the row offsets
//   cell_rekey   key = (cell << cb | col) << 32 | row-major position
//   sort B       stable on the (cell, column) bits
//   cell_store   entries (column, pos) and values in column order
__global__ __launch_bounds__(256) void cell_keys_kernel(const long* __restrict__ indptr, const int* __restrict__ idx,
                                                        const float* __restrict__ values, long r0, long r1, long B,
                                                        long j0, int RBB, int S, int CS, int cb,
                                                        uint64_t* __restrict__ keys, uint32_t* __restrict__ pay,
                                                        int f64) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = r0 + wave; r < r1; r += nw) {
    const long rel = r - r0;
    const long rl = rel - (rel / B) * B;  // row within its batch
    const uint64_t rb = (uint64_t)(rl >> RBB), rin = (uint64_t)(rl & ((1L << RBB) - 1));
    const long s0 = indptr[r], s1 = indptr[r + 1];
    for (long j = s0 + lane; j < s1; j += 64) {
      const int c = idx[j];
      const int sp = c / CS;
      const uint64_t cell = rb * (uint64_t)S + (uint64_t)sp;
      keys[j - j0] = (((cell << RBB) | rin) << cb) | (uint64_t)(c - sp * CS);
      pay[j - j0] = f64 ? (uint32_t)(j - j0) : __float_as_uint(values[j]);
    }
  }
}

__global__ __launch_bounds__(256) void cell_rekey_kernel(const uint64_t* __restrict__ ka, long m, int RBB, int cb,
                                                         uint64_t* __restrict__ kb) {
  const uint64_t cm = (1ull << cb) - 1;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const uint64_t k = ka[i];
    const uint64_t cell = k >> (RBB + cb);
    kb[i] = (((cell << cb) | (k & cm)) << 32) | (uint64_t)i;
  }
}

// sorted B keys → ent = column | pos << cb (pos: row-major rank inside the cell, from the row
// offsets roff of the entry's batch), values from the payload
template <typename V>
__global__ __launch_bounds__(256) void cell_store_kernel(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ pay, long m, long j0, RunStarts rs,
                                                         int slots, long b0, const int* __restrict__ roff, int rstride,
                                                         int RBB, int cb, const V* __restrict__ src,
                                                         uint32_t* __restrict__ ent, V* __restrict__ val) {
  const uint64_t cm = (1ull << cb) - 1;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const uint64_t k = keys[i];
    const long pa = (long)(uint32_t)k;  // run-relative row-major position
    int s = 0;
    while (s + 1 < slots && rs.start[s + 1] <= pa) ++s;
    const long cell = (long)(k >> (32 + cb));
    const int first = roff[(b0 + s) * (long)rstride + (cell << RBB)];
    const uint32_t pos = (uint32_t)(pa - rs.start[s] - first);
    ent[j0 + i] = (uint32_t)((k >> 32) & cm) | (pos << cb);
    if constexpr (sizeof(V) == 4)
      val[j0 + i] = __uint_as_float(pay[i]);
    else
      val[j0 + i] = src[pay[i]];
  }
}

// sorted keys of a run → off[(b0 + s)·cstride + c] = first entry of id c (key >> shift) of batch
// b0 + s, relative to the batch's first entry; off[..+ ncell] = the batch's entry count. Position i
// writes the ids (id(key[i−1]), id(key[i])] of the batch holding it; cell_tails_kernel writes the
// ids after every batch's last key (empty batches: all of them) — each slot exactly once.
__global__ __launch_bounds__(256) void cell_bounds_kernel(const uint64_t* __restrict__ keys, long m, int shift,
                                                          RunStarts rs, int slots, long b0, int cstride,
                                                          int* __restrict__ off) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  int s = 0;
  while (s < slots && !(rs.start[s] <= i && i < rs.start[s + 1])) ++s;
  if (s == slots) return;
  const long bs = rs.start[s];
  const int lo = i > bs ? (int)(keys[i - 1] >> shift) : -1;
  const int hi = (int)(keys[i] >> shift);
  int* o = off + (b0 + s) * (long)cstride;
  for (int c = lo + 1; c <= hi; ++c) o[c] = (int)(i - bs);
}

__global__ __launch_bounds__(256) void cell_tails_kernel(const uint64_t* __restrict__ keys, int shift, RunStarts rs,
                                                         int slots, int ncell, long b0, int cstride,
                                                         int* __restrict__ off) {
  const int p = blockIdx.y;
  if (p >= slots) return;
  const long bs = rs.start[p], be = rs.start[p + 1];
  const int last = be > bs ? (int)(keys[be - 1] >> shift) : -1;
  int* o = off + (b0 + p) * (long)cstride;
  for (long c = (long)blockIdx.x * blockDim.x + threadIdx.x; c <= ncell; c += (long)gridDim.x * blockDim.x)
    if (c > last) o[c] = (int)(be - bs);
}

inline unsigned grid_for(long work, long per_block, unsigned cap) {
  long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (unsigned)(g < cap ? g : cap);
}

}  // namespace

// keys/rel/iota: int32[j1 − j0] with j0 = indptr[r0], j1 = indptr[r1]; slots·d < 2^31 (caller)
FMLX_API int fmlx_csc_keys(const long* indptr, const int* idx, long r0, long r1, long B, int d, long j0, int* key,
                           int* rel, int* iota, void* stream) {
  if (r1 <= r0) return 0;
  if (B <= 0 || d <= 0) return -1;
  hipLaunchKernelGGL(csc_keys_kernel, dim3(grid_for(r1 - r0, 4, 1u << 16)), dim3(256), 0, (hipStream_t)stream,
                     indptr, idx, r0, r1, B, d, j0, key, rel, iota);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_csc_keys64(const long* indptr, const int* idx, const float* values, long r0, long r1, long B, int d,
                             long j0, int* key, uint64_t* payload, int pack, void* stream) {
  if (r1 <= r0) return 0;
  if (B <= 0 || d <= 0 || (pack && B > (1L << 22))) return -1;
  hipLaunchKernelGGL(csc_keys64_kernel, dim3(grid_for(r1 - r0, 4 * KR_ROWS, 1u << 16)), dim3(256), 0, (hipStream_t)stream,
                     indptr, idx, values, r0, r1, B, d, j0, key, payload, pack);
  return (int)hipGetLastError();
}


FMLX_API int fmlx_csc_fill(int f64, const int* order, long m, long j0, const int* rel, const void* values, int* erow,
                           void* evals, void* stream) {
  if (m <= 0) return 0;
  const dim3 g(grid_for(m, 256, 1u << 16));
  if (f64)
    hipLaunchKernelGGL(csc_fill_kernel<double>, g, dim3(256), 0, (hipStream_t)stream, order, m, j0, rel,
                       (const double*)values, erow, (double*)evals);
  else
    hipLaunchKernelGGL(csc_fill_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, order, m, j0, rel,
                       (const float*)values, erow, (float*)evals);
  return (int)hipGetLastError();
}

// colptr: int32 [P, d + 1] of the whole partition; rows b0 … b0 + slots − 1 are written.
// starts: HOST array, starts[s] = first entry of batch b0 + s relative to the run (s ≤ slots)
FMLX_API int fmlx_csc_colptr(const int* sorted_keys, long m, int slots, int d, const long* starts, long b0,
                             int* colptr, void* stream) {
  if (slots <= 0 || slots > CP_MAXS || d <= 0 || m < 0 || m >= (1L << 31) || (long)slots * d >= (1L << 31)) return -1;
  if ((reinterpret_cast<uintptr_t>(sorted_keys) & 15) != 0) return -2;  // the 16-B key loads
  RunStarts rs{};
  for (int s = 0; s <= slots; ++s) rs.start[s] = (int)starts[s];
  const long threads = m / 4 + 1;  // boundaries 0 … m
  hipLaunchKernelGGL(csc_colptr_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     sorted_keys, (int)m, slots, d, rs, b0, colptr);
  return (int)hipGetLastError();
}

// Tiles of batches b0 … b0 + slots − 1 (colptr rows already built): tiles int32 [P][tstride][2]
// = (start column, its batch-relative first entry), the entry after the last tile = (d, nnz_b)
// (tstride ≥ min(d, nnz_b / EB + 2·(nnz_b / EL) + 1) + 1 bounds every batch's tile count: the
// bucket changes plus two starts per heavy column), ntiles int32 [P].
FMLX_API int fmlx_csc_tiles(const int* colptr, long b0, int slots, int d, int EB, int EL, int* tiles, int tstride,
                            int* ntiles, int* scratch, long scratch_ints, void* stream) {
  if (slots <= 0 || d <= 0 || EB <= 0 || EL <= 0 || tstride < 2) return -1;
  const int nchunks = (d + TL_CHUNK - 1) / TL_CHUNK;
  if (scratch_ints < (long)slots * nchunks) return -2;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(csc_tiles_count_kernel, dim3(nchunks, slots), dim3(TL_CHUNK), 0, s, colptr, b0, d, EB, EL, nchunks,
                     scratch);
  hipLaunchKernelGGL(csc_tiles_scan_kernel, dim3(slots), dim3(TL_THREADS), 0, s, scratch, nchunks, colptr, b0, d,
                     (int2*)tiles, tstride, ntiles);
  hipLaunchKernelGGL(csc_tiles_write_kernel, dim3(nchunks, slots), dim3(TL_CHUNK), 0, s, colptr, b0, d, EB, EL, nchunks,
                     scratch, (int2*)tiles, tstride);
  return (int)hipGetLastError();
}

FMLX_API long fmlx_csc_tiles_scratch(int slots, int d) { return (long)slots * ((d + TL_CHUNK - 1) / TL_CHUNK); }

// Keys of a run's entries j0 … j0 + m − 1 (batch s starts at bstart[s], DEVICE array, absolute).
// keys: uint64 [m]; pay: uint32 [m]. rb + pb ≤ 32 (the packed erow), pb ≥ bits(ET − 1).
FMLX_API int fmlx_csc_tile_keys(int f64, const int* colptr, long b0, int slots, int d, const int* tiles, int tstride,
                                const int* ntiles, const long* bstart, const int* erow, const void* evals, long j0,
                                int rb, int pb, int EL, uint64_t* keys, uint32_t* pay, void* stream) {
  if (slots <= 0 || rb < 1 || pb < 1 || rb + pb > 32) return -1;
  const dim3 g(tstride < 1024 ? tstride : 1024, slots);
  if (f64)
    hipLaunchKernelGGL(csc_tile_keys_kernel<double>, g, dim3(256), 0, (hipStream_t)stream, colptr, b0, d, (const int2*)tiles,
                       tstride, ntiles, bstart, erow, (const double*)evals, j0, rb, pb, EL, keys, pay);
  else
    hipLaunchKernelGGL(csc_tile_keys_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, colptr, b0, d, (const int2*)tiles,
                       tstride, ntiles, bstart, erow, (const float*)evals, j0, rb, pb, EL, keys, pay);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_csc_tile_store(int f64, const uint64_t* keys, const uint32_t* pay, long m, long j0, int rb, int pb,
                                 const void* src, int* erow, void* evals, void* stream) {
  if (m <= 0) return 0;
  if (rb < 1 || pb < 1 || rb + pb > 32 || (f64 && src == nullptr)) return -1;
  const dim3 g(grid_for(m, 256, 1u << 16));
  if (f64)
    hipLaunchKernelGGL(csc_tile_store_kernel<double>, g, dim3(256), 0, (hipStream_t)stream, keys, pay, m, j0, rb, pb,
                       (const double*)src, erow, (double*)evals);
  else
    hipLaunchKernelGGL(csc_tile_store_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, keys, pay, m, j0, rb, pb,
                       (const float*)nullptr, erow, (float*)evals);
  return (int)hipGetLastError();
}

// Cells of the run's batches (see cell_keys_kernel): keys uint64 [m], pay uint32 [m] (m = j1 − j0).
FMLX_API int fmlx_cell_keys(int f64, const long* indptr, const int* idx, const float* values, long r0, long r1, long B,
                            long j0, int RBB, int S, int CS, int cb, uint64_t* keys, uint32_t* pay, void* stream) {
  if (r1 <= r0) return 0;
  if (B <= 0 || RBB < 1 || S < 1 || CS < 1 || cb < 1 || cb + RBB > 32) return -1;
  hipLaunchKernelGGL(cell_keys_kernel, dim3(grid_for(r1 - r0, 4, 1u << 16)), dim3(256), 0, (hipStream_t)stream,
                     indptr, idx, values, r0, r1, B, j0, RBB, S, CS, cb, keys, pay, f64);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_cell_rekey(const uint64_t* ka, long m, int RBB, int cb, uint64_t* kb, void* stream) {
  if (m <= 0) return 0;
  if (m >= (1L << 32) || cb < 1 || cb + RBB > 32) return -1;
  hipLaunchKernelGGL(cell_rekey_kernel, dim3(grid_for(m, 256, 1u << 16)), dim3(256), 0, (hipStream_t)stream, ka, m,
                     RBB, cb, kb);
  return (int)hipGetLastError();
}

// starts: HOST array of the run's batch starts relative to j0 (slots + 1 values)
FMLX_API int fmlx_cell_store(int f64, const uint64_t* keys, const uint32_t* pay, long m, long j0, const long* starts,
                             int slots, long b0, const int* roff, int rstride, int RBB, int cb, const void* src,
                             uint32_t* ent, void* val, void* stream) {
  if (m <= 0) return 0;
  if ((f64 && src == nullptr) || slots <= 0 || slots > CP_MAXS || m >= (1L << 31)) return -1;
  RunStarts rs{};
  for (int s = 0; s <= slots; ++s) rs.start[s] = (int)starts[s];
  const dim3 g(grid_for(m, 256, 1u << 16));
  if (f64)
    hipLaunchKernelGGL(cell_store_kernel<double>, g, dim3(256), 0, (hipStream_t)stream, keys, pay, m, j0, rs, slots,
                       b0, roff, rstride, RBB, cb, (const double*)src, ent, (double*)val);
  else
    hipLaunchKernelGGL(cell_store_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, keys, pay, m, j0, rs, slots, b0,
                       roff, rstride, RBB, cb, (const float*)nullptr, ent, (float*)val);
  return (int)hipGetLastError();
}

// starts: HOST array of the run's batch starts relative to j0 (slots + 1 values)
FMLX_API int fmlx_cell_bounds(const uint64_t* keys, long m, int shift, const long* starts, int slots, int ncell,
                              long b0, int cstride, int* off, void* stream) {
  if (slots <= 0 || slots > CP_MAXS || m < 0 || m >= (1L << 31) || ncell + 1 > cstride) return -1;
  RunStarts rs{};
  for (int s = 0; s <= slots; ++s) rs.start[s] = (int)starts[s];
  if (m > 0)
    hipLaunchKernelGGL(cell_bounds_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, keys,
                       m, shift, rs, slots, b0, cstride, off);
  const unsigned gx = (unsigned)std::min<long>(((long)ncell + 1 + 255) / 256, 1024);
  hipLaunchKernelGGL(cell_tails_kernel, dim3(gx, slots), dim3(256), 0, (hipStream_t)stream, keys, shift, rs, slots,
                     ncell, b0, cstride, off);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
