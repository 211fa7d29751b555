// Segmented stable LSD radix sort of (int32 key, payload) pairs — no library sort (SURVEY §2.1 K5:
// the sparse hinge / logistic trainer's per-batch column-major copies, HingeLoss.java:39-57 over
// SGD.java:263-283's minibatch slices).
//
// The input is a run of S contiguous segments (the batches of a run of CSR rows). Inside segment s
// the pairs are sorted by the digit value of (key − kbase[s]) over key_bits bits, stably (equal
// keys keep their input order, i.e. the CSR row order); segments never mix. For the column-major
// copies key = slot·d + column and kbase[slot] = slot·d, so a 1M-column batch needs 20 key bits =
// two 10-bit passes instead of the three 8-bit passes hipCUB's onesweep makes over the 24-bit
// run-wide keys.
//
// One pass (digit width DB ≤ 10 bits, the groupsort.hip stable counting-sort machinery extended to
// segments and payloads):
//   rs_hist     per tile (RS_TILE pairs, never across a segment boundary): per-wave LDS digit
//               histograms, summed → T[tile][digit];
//   rs_colscan  per group of RS_TG tiles of one segment and digit: T ← exclusive in-group prefix,
//               G[group][digit] = the group's total;
//   rs_base     one block per segment: per digit the exclusive prefix over the segment's groups,
//               then over the digits (+ the segment's first position) → G[group][digit] = where
//               the group's pairs of that digit start;
//   rs_scatter  per tile: per-wave histograms again → cursors; each wave walks its 1024-pair
//               segment 64 pairs at a time in input order; one ballot per digit bit gives every
//               pair the set of lanes holding its digit, and its rank among them (lanes below);
//               the pairs are placed in LDS in tile-local sorted order, then written out digit
//               run by digit run.
// Every step is order-deterministic; no global atomics.
#include "common.h"

namespace {

constexpr int RS_WAVES = 8;
constexpr int RS_THREADS = RS_WAVES * 64;
constexpr int RS_SEG = 1024;                 // pairs per wave segment
constexpr int RS_TILE = RS_WAVES * RS_SEG;   // 8192 pairs per tile
constexpr int RS_TG = 64;                    // tiles per column-scan group
constexpr int RS_MAXS = 32;                  // segments per sort
constexpr int RS_MAX_DIGIT_BITS = 10;        // scatter LDS: (8 + 2)·1024 ints + 8192 × (4 + 8) B = 136 KiB

struct SegTable {
  int S, ntile, ngrp, pad;
  long bound[RS_MAXS + 1];  // segment s = pairs [bound[s], bound[s+1])
  int tile0[RS_MAXS + 1];   // first tile of segment s (tile0[S] = ntile)
  int grp0[RS_MAXS + 1];    // first group of segment s (grp0[S] = ngrp)
  int kbase[RS_MAXS];       // the segment's key offset, subtracted before the digit is taken
};

__device__ __forceinline__ int seg_of(const int* first, int S, int x) {
  int s = 0;
  while (s + 1 < S && first[s + 1] <= x) ++s;
  return s;
}

// the tile's pair range and its segment's key offset
__device__ __forceinline__ void tile_range(const SegTable& tb, int t, long& a, long& b, int& kb) {
  const int s = seg_of(tb.tile0, tb.S, t);
  a = tb.bound[s] + (long)(t - tb.tile0[s]) * RS_TILE;
  b = a + RS_TILE < tb.bound[s + 1] ? a + RS_TILE : tb.bound[s + 1];
  kb = tb.kbase[s];
}

__device__ __forceinline__ void rs_wave_hist(const int* __restrict__ keys, long a, long b, int kb, int shift, int mask,
                                             int* h) {
  const int lane = threadIdx.x & 63;
  for (long i = a + lane; i < b; i += 64) atomicAdd(&h[((keys[i] - kb) >> shift) & mask], 1);  // LDS
}

__global__ __launch_bounds__(RS_THREADS) void rs_hist_kernel(const int* __restrict__ keys, SegTable tb, int shift,
                                                             int mask, int* __restrict__ T) {
  extern __shared__ int sh[];
  const int nd = mask + 1, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < RS_WAVES * nd; i += RS_THREADS) sh[i] = 0;
  __syncthreads();
  long a, b;
  int kb;
  tile_range(tb, blockIdx.x, a, b, kb);
  const long wa = a + (long)w * RS_SEG;
  rs_wave_hist(keys, wa, wa + RS_SEG < b ? wa + RS_SEG : b, kb, shift, mask, sh + (long)w * nd);
  __syncthreads();
  int* out = T + (long)blockIdx.x * nd;
  for (int c = threadIdx.x; c < nd; c += RS_THREADS) {
    int s = 0;
#pragma unroll
    for (int q = 0; q < RS_WAVES; ++q) s += sh[q * nd + c];
    out[c] = s;
  }
}

// grid (ceil(nd / 256), ngrp): thread = digit; walks the group's tiles in order
__global__ __launch_bounds__(256) void rs_colscan_kernel(int* __restrict__ T, SegTable tb, int nd,
                                                         int* __restrict__ G) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= nd) return;
  const int g = blockIdx.y;
  const int s = seg_of(tb.grp0, tb.S, g);
  const int t0 = tb.tile0[s] + (g - tb.grp0[s]) * RS_TG;
  const int t1 = t0 + RS_TG < tb.tile0[s + 1] ? t0 + RS_TG : tb.tile0[s + 1];
  int run = 0;
  for (int t = t0; t < t1; t += 16) {
    int v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = t + q < t1 ? T[(long)(t + q) * nd + c] : 0;  // 16 loads in flight
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (t + q < t1) T[(long)(t + q) * nd + c] = run;
      run += v[q];
    }
  }
  G[(long)g * nd + c] = run;
}

// one block per segment: G[g][c] ← segment start + digit prefix + group prefix
__global__ __launch_bounds__(1024) void rs_base_kernel(int* __restrict__ G, SegTable tb, int nd) {
  __shared__ long wtot[16];
  __shared__ long carry;
  const int s = blockIdx.x;
  const int g0 = tb.grp0[s], g1 = tb.grp0[s + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = tb.bound[s];
  __syncthreads();
  for (int base = 0; base < nd; base += 1024) {
    const int c = base + threadIdx.x;
    long cnt = 0;
    if (c < nd)
      for (int g = g0; g < g1; ++g) {  // per digit: exclusive prefix over the segment's groups
        const int v = G[(long)g * nd + c];
        G[(long)g * nd + c] = (int)cnt;
        cnt += v;
      }
    long inc = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const long o = __shfl_up(inc, off, 64);
      if (lane >= off) inc += o;
    }
    if (lane == 63) wtot[wv] = inc;
    __syncthreads();
    long p = 0;
    for (int i = 0; i < wv; ++i) p += wtot[i];
    const long ex = carry + p + inc - cnt;  // first position of digit c in the segment
    if (c < nd)
      for (int g = g0; g < g1; ++g) G[(long)g * nd + c] += (int)ex;
    __syncthreads();
    if (threadIdx.x == 1023) carry = ex + cnt;
    __syncthreads();
  }
}

// The tile is ranked into LDS first and written out in digit order: consecutive threads store
// consecutive positions of one digit's run, instead of 64 lanes each storing 12 bytes into 64
// different buckets (the direct form measured 1.95 ms per pass over 64M pairs: 0.8 TB/s).
// SPLIT (64-bit payloads, last pass): the payload's low / high words go straight to two arrays
// (the column-major copy's row ids and values) at split_off + position, so no separate unpack pass.
template <typename V, bool SPLIT>
__global__ __launch_bounds__(RS_THREADS) void rs_scatter_kernel(const int* __restrict__ kin, const V* __restrict__ vin,
                                                                int* __restrict__ kout, V* __restrict__ vout,
                                                                const int* __restrict__ T, const int* __restrict__ G,
                                                                SegTable tb, int shift, int mask,
                                                                int* __restrict__ split_lo,
                                                                unsigned* __restrict__ split_hi, long split_off) {
  extern __shared__ __align__(16) int shs[];
  const int nd = mask + 1;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = blockIdx.x;
  int* hw = shs;                                 // [RS_WAVES][nd] per-wave counts → wave cursors
  int* loc = hw + RS_WAVES * nd;                 // [nd] tile-local start of each digit
  int* gbase = loc + nd;                         // [nd] global start of the tile's digit run
  int* lk = gbase + nd;                          // [RS_TILE] keys in tile-local sorted order
  V* lv = reinterpret_cast<V*>(lk + RS_TILE);    // [RS_TILE] payloads (8-B aligned: nd even)
  int* wsum = reinterpret_cast<int*>(lv + RS_TILE);  // [RS_WAVES] wave totals of the digit scan
  for (int i = threadIdx.x; i < RS_WAVES * nd; i += RS_THREADS) hw[i] = 0;
  __syncthreads();
  long a, b;
  int kb;
  tile_range(tb, t, a, b, kb);
  const long wa = a + (long)w * RS_SEG;
  const long wb = wa + RS_SEG < b ? wa + RS_SEG : b;
  rs_wave_hist(kin, wa, wb, kb, shift, mask, hw + (long)w * nd);
  __syncthreads();
  // tile totals per digit → exclusive scan over the digits (block-wide) → loc; wave cursors;
  // global bases (group base + in-group prefix of this tile)
  const int s = seg_of(tb.tile0, tb.S, t);
  const int g = tb.grp0[s] + (t - tb.tile0[s]) / RS_TG;
  const int* Tt = T + (long)t * nd;
  const int* Gg = G + (long)g * nd;
  constexpr int DPT = 4;  // digits per thread (nd <= RS_THREADS·DPT = 2048)
  int tot[DPT];
  int run = 0;
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const int c = threadIdx.x * DPT + j;
    int v = 0;
    if (c < nd)
#pragma unroll
      for (int q = 0; q < RS_WAVES; ++q) v += hw[q * nd + c];
    tot[j] = v;
    run += v;
  }
  int inc = run;  // inclusive scan of the per-thread sums over the block
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(inc, off, 64);
    if (lane >= off) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int base = inc - run;
  for (int q = 0; q < w; ++q) base += wsum[q];
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const int c = threadIdx.x * DPT + j;
    if (c < nd) {
      loc[c] = base;
      gbase[c] = Gg[c] + Tt[c];
      int r = base;
#pragma unroll
      for (int q = 0; q < RS_WAVES; ++q) {
        const int v = hw[q * nd + c];
        hw[q * nd + c] = r;
        r += v;
      }
    }
    base += tot[j];
  }
  __syncthreads();
  int* cur = hw + (long)w * nd;
  const int db = 31 - __builtin_clz(nd);  // digit bits
  const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes below this one
  for (long i0 = wa; i0 < wb; i0 += 64) {
    const long i = i0 + lane;
    const bool valid = i < wb;
    int key = 0, dg = 0;
    V val = 0;
    if (valid) {
      key = kin[i];
      val = vin[i];
      dg = ((key - kb) >> shift) & mask;
    }
    // stable rank among equal digits of the 64: the lanes holding my digit (one ballot per digit
    // bit, no cross-lane data movement), then the count of those below me
    unsigned long long peers = __ballot(valid);
    for (int bit = 0; bit < db; ++bit) {
      const bool mine = (dg >> bit) & 1;
      const unsigned long long bb = __ballot(mine);
      peers &= mine ? bb : ~bb;
    }
    const int rank = __popcll(peers & lt);
    const bool leader = valid && (peers >> lane) == 1ull;  // the highest lane of my digit's run
    int pos = 0;
    if (valid) pos = cur[dg] + rank;  // tile-local
    // every lane read its cursor above before a leader advances it (one wave: its LDS accesses
    // complete in program order)
    __builtin_amdgcn_wave_barrier();
    if (leader) cur[dg] = pos + 1;
    if (valid) {
      lk[pos] = key;
      lv[pos] = val;
    }
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // out in tile-local sorted order: a digit's run of the tile is one contiguous global range
  const int len = (int)(b - a);
  for (int i = threadIdx.x; i < len; i += RS_THREADS) {
    const int key = lk[i];
    const int dg = ((key - kb) >> shift) & mask;
    const int gp = gbase[dg] + (i - loc[dg]);
    kout[gp] = key;
    if constexpr (SPLIT) {
      const uint64_t u = (uint64_t)lv[i];
      split_lo[split_off + gp] = (int)(unsigned)u;
      split_hi[split_off + gp] = (unsigned)(u >> 32);
    } else {
      vout[gp] = lv[i];
    }
  }
}

// host table from the flat description: bound[0..S], kbase[0..S-1]
static int make_table(const long* bound, const int* kbase, int S, SegTable& tb) {
  if (S < 1 || S > RS_MAXS) return -2;
  tb.S = S;
  int nt = 0, ng = 0;
  for (int s = 0; s < S; ++s) {
    const long len = bound[s + 1] - bound[s];
    if (len < 0) return -3;
    tb.bound[s] = bound[s];
    tb.tile0[s] = nt;
    tb.grp0[s] = ng;
    tb.kbase[s] = kbase[s];
    const long tiles = (len + RS_TILE - 1) / RS_TILE;
    if (nt + tiles >= (1L << 30)) return -4;
    nt += (int)tiles;
    ng += (int)((tiles + RS_TG - 1) / RS_TG);
  }
  tb.bound[S] = bound[S];
  tb.tile0[S] = nt;
  tb.grp0[S] = ng;
  tb.ntile = nt;
  tb.ngrp = ng;
  return 0;
}

template <typename V>
int seg_sort(int* keys, V* vals, int* keys_alt, V* vals_alt, const long* bound, const int* kbase, int S, int key_bits,
             int digit_bits, int* scratch, long scratch_ints, hipStream_t st, int* split_lo = nullptr,
             unsigned* split_hi = nullptr, long split_off = 0) {
  SegTable tb{};
  int rc = make_table(bound, kbase, S, tb);
  if (rc) return rc;
  if (digit_bits < 1 || digit_bits > RS_MAX_DIGIT_BITS || key_bits < 1 || key_bits > 31) return -5;
  const int passes = (key_bits + digit_bits - 1) / digit_bits;
  const int db = (key_bits + passes - 1) / passes;  // balanced digits: 20 bits → 10 + 10
  const int nd = 1 << db;
  if (scratch_ints < (long)(tb.ntile + tb.ngrp) * nd) return -6;
  if (tb.ntile == 0) return 0;
  int* T = scratch;
  int* G = scratch + (long)tb.ntile * nd;
  const size_t lds = (size_t)RS_WAVES * nd * sizeof(int);
  // scatter: per-wave cursors + loc + gbase + the tile's keys and payloads
  const size_t lds_sc = (size_t)(RS_WAVES + 2) * nd * sizeof(int) + (size_t)RS_TILE * (sizeof(int) + sizeof(V)) +
                        RS_WAVES * sizeof(int);
  int* kin = keys;
  V* vin = vals;
  int* kout = keys_alt;
  V* vout = vals_alt;
  for (int p = 0; p < passes; ++p) {
    const int shift = p * db;
    const int mask = nd - 1;
    hipLaunchKernelGGL(rs_hist_kernel, dim3(tb.ntile), dim3(RS_THREADS), lds, st, kin, tb, shift, mask, T);
    hipLaunchKernelGGL(rs_colscan_kernel, dim3((nd + 255) / 256, tb.ngrp), dim3(256), 0, st, T, tb, nd, G);
    hipLaunchKernelGGL(rs_base_kernel, dim3(tb.S), dim3(1024), 0, st, G, tb, nd);
    if (sizeof(V) == 8 && split_lo != nullptr && p == passes - 1)
      hipLaunchKernelGGL((rs_scatter_kernel<V, true>), dim3(tb.ntile), dim3(RS_THREADS), lds_sc, st, kin, vin, kout,
                         vout, T, G, tb, shift, mask, split_lo, split_hi, split_off);
    else
      hipLaunchKernelGGL((rs_scatter_kernel<V, false>), dim3(tb.ntile), dim3(RS_THREADS), lds_sc, st, kin, vin, kout,
                         vout, T, G, tb, shift, mask, (int*)nullptr, (unsigned*)nullptr, 0L);
    int* tk = kin;
    kin = kout;
    kout = tk;
    V* tv = vin;
    vin = vout;
    vout = tv;
  }
  rc = (int)hipGetLastError();
  if (rc) return rc;
  return (passes & 1) ? 1 : 0;  // 1: the sorted pairs are in the _alt buffers
}

}  // namespace

// ints of scratch a sort of S segments with these bounds needs (digits of <= digit_bits bits)
FMLX_API long fmlx_seg_sort_scratch(const long* bound, int S, int key_bits, int digit_bits) {
  if (S < 1 || S > RS_MAXS || digit_bits < 1 || digit_bits > RS_MAX_DIGIT_BITS || key_bits < 1 || key_bits > 31)
    return -1;
  long nt = 0, ng = 0;
  for (int s = 0; s < S; ++s) {
    const long tiles = (bound[s + 1] - bound[s] + RS_TILE - 1) / RS_TILE;
    nt += tiles;
    ng += (tiles + RS_TG - 1) / RS_TG;
  }
  const int passes = (key_bits + digit_bits - 1) / digit_bits;
  const int db = (key_bits + passes - 1) / passes;
  return (nt + ng) * (1L << db);
}

// Sorts pairs [bound[0], bound[S]) (positions relative to the arrays' starts) segment by segment
// by the low key_bits bits of (key − kbase[s]); `bound` / `kbase` are HOST arrays. Returns 0 when
// the result is in keys / vals, 1 when it is in keys_alt / vals_alt, < 0 on a bad argument.
// split_lo / split_hi (may be null): the last pass writes the payloads' low / high 32-bit words to
// split_lo[split_off + i] / split_hi[split_off + i] instead of vals (the keys still go to the
// returned key buffer).
FMLX_API int fmlx_seg_sort64(int* keys, uint64_t* vals, int* keys_alt, uint64_t* vals_alt, const long* bound,
                             const int* kbase, int S, int key_bits, int digit_bits, int* scratch, long scratch_ints,
                             int* split_lo, unsigned* split_hi, long split_off, void* stream) {
  return seg_sort<uint64_t>(keys, vals, keys_alt, vals_alt, bound, kbase, S, key_bits, digit_bits, scratch,
                            scratch_ints, (hipStream_t)stream, split_lo, split_hi, split_off);
}

FMLX_API int fmlx_seg_sort32(int* keys, uint32_t* vals, int* keys_alt, uint32_t* vals_alt, const long* bound,
                             const int* kbase, int S, int key_bits, int digit_bits, int* scratch, long scratch_ints,
                             void* stream) {
  return seg_sort<uint32_t>(keys, vals, keys_alt, vals_alt, bound, kbase, S, key_bits, digit_bits, scratch,
                            scratch_ints, (hipStream_t)stream);
}
