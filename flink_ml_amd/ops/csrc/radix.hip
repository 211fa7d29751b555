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

constexpr int RS_PER_LANE = RS_SEG / 64;  // pairs per lane of a wave segment

// digit of a key: int32 keys are offset by the segment's kbase (the column-major copies' slot·d);
// 64-bit keys (fmlx_sort_u64: ordered fp64 scores / value bits) carry no offset
__device__ __forceinline__ int rs_digit(int key, int kb, int shift, int mask) { return ((key - kb) >> shift) & mask; }
__device__ __forceinline__ int rs_digit(uint64_t key, int, int shift, int mask) {
  return (int)(key >> shift) & mask;
}

// the wave's segment [wa, wb) into registers, all loads in flight at once (one memory latency
// per segment, not one per 64 pairs: at one 136 KiB-LDS block per CU the scatter has 2 waves per
// SIMD and a load-then-use loop waited out each load)
template <typename V, typename K = int>
__device__ __forceinline__ void rs_load_seg(const K* __restrict__ kin, const V* __restrict__ vin, long wa, long wb,
                                            K (&k)[RS_PER_LANE], V (&v)[RS_PER_LANE]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < RS_PER_LANE; ++j) {
    const long i = wa + j * 64 + lane;
    if (kin != nullptr) k[j] = i < wb ? kin[i] : K(0);
    if (vin != nullptr) v[j] = i < wb ? vin[i] : V(0);
  }
}

template <typename K>
__device__ __forceinline__ void rs_wave_hist(const K (&k)[RS_PER_LANE], long wa, long wb, int kb, int shift,
                                             int mask, int* h) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < RS_PER_LANE; ++j)
    if (wa + j * 64 + lane < wb) atomicAdd(&h[rs_digit(k[j], kb, shift, mask)], 1);  // LDS
}

template <typename K>
__global__ __launch_bounds__(RS_THREADS) void rs_hist_kernel(const K* __restrict__ keys, SegTable tb, int shift,
                                                             int mask, int* __restrict__ T) {
  extern __shared__ int sh[];
  const int nd = mask + 1, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < RS_WAVES * nd; i += RS_THREADS) sh[i] = 0;
  __syncthreads();
  long a, b;
  int kb;
  tile_range(tb, blockIdx.x, a, b, kb);
  const long wa = a + (long)w * RS_SEG;
  const long wb = wa + RS_SEG < b ? wa + RS_SEG : b;
  K k[RS_PER_LANE];
  int dummy[RS_PER_LANE];
  rs_load_seg<int, K>(keys, nullptr, wa, wb, k, dummy);
  rs_wave_hist(k, wa, wb, kb, shift, mask, sh + (long)w * nd);
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

// Per-wave digit counts hw[q][c] of one tile → loc[c] = the tile-local start of digit c (an
// exclusive scan over the digits, block-wide) and hw[q][c] = wave q's cursor for digit c (loc[c]
// plus the counts of the waves before q). Block-wide; ends with a barrier.
__device__ __forceinline__ void rs_tile_cursors(int* hw, int nd, int* loc, int* wsum) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
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
}

// The wave's segment (registers kr / vr, positions wa … wb) placed in tile-local stable digit order:
// place(pos, key, val, digit) for every valid pair, pos = the wave's cursor for the digit + the
// pair's rank among the equal digits of its 64. The rank: the lanes holding my digit (one ballot
// per digit bit, no cross-lane data movement), then the count of those below me.
template <typename V, typename Place, typename K = int>
__device__ __forceinline__ void rs_rank_place(const K (&kr)[RS_PER_LANE], const V (&vr)[RS_PER_LANE], long wa,
                                              long wb, int kb, int shift, int mask, int* cur, Place place) {
  const int lane = threadIdx.x & 63;
  const int db = 31 - __builtin_clz(mask + 1);  // digit bits
  const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes below this one
#pragma unroll
  for (int j = 0; j < RS_PER_LANE; ++j) {
    const bool valid = wa + j * 64 + lane < wb;
    const K key = kr[j];
    const int dg = valid ? rs_digit(key, kb, shift, mask) : 0;
    unsigned long long peers = __ballot(valid);
    for (int bit = 0; bit < db; ++bit) {
      // M = all ones where my digit has this bit, else 0; the lanes agreeing with me on it are
      // ballot XNOR M (one bfe, one compare, two xnor, two and per bit)
      const int M = (int)((unsigned)dg << (31 - bit)) >> 31;
      const unsigned long long bb = __ballot(M != 0);
      const unsigned lo = ~((unsigned)bb ^ (unsigned)M), hi = ~((unsigned)(bb >> 32) ^ (unsigned)M);
      peers &= ((unsigned long long)hi << 32) | lo;
    }
    const int rank = __popcll(peers & lt);
    const bool leader = valid && (peers >> lane) == 1ull;  // the highest lane of my digit's run
    int pos = 0;
    if (valid) pos = cur[dg] + rank;  // tile-local
    // every lane read its cursor above before a leader advances it (one wave: its LDS accesses
    // complete in program order)
    __builtin_amdgcn_wave_barrier();
    if (leader) cur[dg] = pos + 1;
    if (valid) place(pos, key, vr[j], dg);
    __builtin_amdgcn_wave_barrier();
  }
}

// The tile is ranked into LDS first and written out in digit order: consecutive threads store
// consecutive positions of one digit's run, instead of 64 lanes each storing 12 bytes into 64
// different buckets (the direct form measured 1.95 ms per pass over 64M pairs: 0.8 TB/s).
// SPLIT (64-bit payloads, last pass): the payload's low / high words go straight to two arrays
// (the column-major copy's row ids and values) at split_off + position, so no separate unpack pass.
template <typename V, bool SPLIT, typename K = int>
__global__ __launch_bounds__(RS_THREADS) void rs_scatter_kernel(const K* __restrict__ kin, const V* __restrict__ vin,
                                                                K* __restrict__ kout, V* __restrict__ vout,
                                                                const int* __restrict__ T, const int* __restrict__ G,
                                                                SegTable tb, int shift, int mask,
                                                                int* __restrict__ split_lo,
                                                                unsigned* __restrict__ split_hi, long split_off) {
  extern __shared__ __align__(16) int shs[];
  const int nd = mask + 1;
  const int w = threadIdx.x >> 6;
  const int t = blockIdx.x;
  int* hw = shs;                                 // [RS_WAVES][nd] per-wave counts → wave cursors
  int* loc = hw + RS_WAVES * nd;                 // [nd] tile-local start of each digit
  int* gbase = loc + nd;                         // [nd] global start of the tile's digit run
  K* lk = reinterpret_cast<K*>(gbase + nd);      // [RS_TILE] keys in tile-local sorted order (8-B aligned: nd even)
  V* lv = reinterpret_cast<V*>(lk + RS_TILE);    // [RS_TILE] payloads
  int* wsum = reinterpret_cast<int*>(lv + RS_TILE);  // [RS_WAVES] wave totals of the digit scan
  for (int i = threadIdx.x; i < RS_WAVES * nd; i += RS_THREADS) hw[i] = 0;
  __syncthreads();
  long a, b;
  int kb;
  tile_range(tb, t, a, b, kb);
  const long wa = a + (long)w * RS_SEG;
  const long wb = wa + RS_SEG < b ? wa + RS_SEG : b;
  K kr[RS_PER_LANE];
  V vr[RS_PER_LANE];
  rs_load_seg<V, K>(kin, vin, wa, wb, kr, vr);
  rs_wave_hist(kr, wa, wb, kb, shift, mask, hw + (long)w * nd);
  __syncthreads();
  rs_tile_cursors(hw, nd, loc, wsum);
  // global bases: group base + in-group prefix of this tile
  const int s = seg_of(tb.tile0, tb.S, t);
  const int g = tb.grp0[s] + (t - tb.tile0[s]) / RS_TG;
  const int* Tt = T + (long)t * nd;
  const int* Gg = G + (long)g * nd;
  for (int c = threadIdx.x; c < nd; c += RS_THREADS) gbase[c] = Gg[c] + Tt[c];
  rs_rank_place(kr, vr, wa, wb, kb, shift, mask, hw + (long)w * nd, [&](int pos, K key, V val, int) {
    lk[pos] = key;
    lv[pos] = val;
  });
  __syncthreads();
  // out in tile-local sorted order: a digit's run of the tile is one contiguous global range
  const int len = (int)(b - a);
  for (int i = threadIdx.x; i < len; i += RS_THREADS) {
    const K key = lk[i];
    const int dg = rs_digit(key, kb, shift, mask);
    const int gp = gbase[dg] + (i - loc[dg]);
    if (kout != nullptr) kout[gp] = key;  // (the packed column-major copy carries no keys out)
    if constexpr (SPLIT) {
      const uint64_t u = (uint64_t)lv[i];
      split_lo[split_off + gp] = (int)(unsigned)u;
      split_hi[split_off + gp] = (unsigned)(u >> 32);
    } else {
      vout[gp] = lv[i];
    }
  }
}

// The column-major copy's second (last) pass, bucket-local: after a stable pass on the HIGH
// column digit (key bits 10 …), segment s's pairs of high digit h — the columns h·1024 … h·1024 +
// 1023 of batch s — are one contiguous run ("bucket") of the array. One block per bucket sorts it
// by the low 10 bits, stably, in chunks of RS_TILE pairs (one chunk for a bucket of ≤ 8192 pairs:
// the 64M-pair, 1M-column SVC run averages 6,250), and writes
//   * the payload halves (row id, value bits) to erow / evals, each pair straight from registers
//     to its final position: the stores of a block stay inside its bucket's ~25 KB of each array,
//     so L2 assembles whole lines (no LDS staging: 40 KB of LDS, 3 blocks per CU);
//   * the bucket's columns' entries of the column pointer, from its column histogram — no sorted
//     keys are written and no separate column-pointer pass reads them back.
// Replaces an LSD second pass (global digit scatter + its histogram / scans) plus the column-
// pointer kernel (155–241 µs over the 256 MB of sorted keys).
constexpr int CB_ND = 1024;  // columns per bucket (low digit)

// PACKED: the payload carries the column's low 10 bits at bits 22..31 above a 22-bit batch row
// (fmlx_csc_keys64 packing), so this pass reads no keys at all. (122 VGPRs: two 8-wave blocks per
// CU. Forcing three — ≤ 80 VGPRs — spills 144 bytes per lane: 2.26 vs 1.65 ms per 10-batch run.)
template <bool PACKED>
__global__ __launch_bounds__(RS_THREADS) void rs_csc_bucket_kernel(const int* __restrict__ kin,
                                                                   const uint64_t* __restrict__ vin,
                                                                   const int* __restrict__ G, SegTable tb, int ndA,
                                                                   int d, long b0, int* __restrict__ colptr,
                                                                   int* __restrict__ erow,
                                                                   unsigned* __restrict__ evals, long split_off) {
  extern __shared__ __align__(16) int shs[];
  int* hw = shs;                     // [RS_WAVES][CB_ND] per-wave counts → wave cursors
  int* loc = hw + RS_WAVES * CB_ND;  // [CB_ND] chunk-local start of each column
  int* cb = loc + CB_ND;             // [CB_ND] bucket-local start of each column's next entries
  int* wsum = cb + CB_ND;            // [RS_WAVES]
  const int w = threadIdx.x >> 6;
  const int s = blockIdx.x / ndA, h = blockIdx.x - s * ndA;
  const long seg0 = tb.bound[s], seg1 = tb.bound[s + 1];
  long start = seg0, end = seg0;
  if (seg1 > seg0) {  // an empty segment has no group rows in G
    const int* Gs = G + (long)tb.grp0[s] * ndA;
    start = Gs[h];
    end = h + 1 < ndA ? Gs[h + 1] : seg1;
  }
  const int kb = tb.kbase[s];
  const int c0 = h * CB_ND;
  const int ncol = d - c0 < CB_ND ? d - c0 : CB_ND;
  int* cp = colptr + (b0 + s) * (long)(d + 1);
  const int rel = (int)(start - seg0);
  if (h == 0 && threadIdx.x == 0) cp[d] = (int)(seg1 - seg0);
  const bool one = end - start <= RS_TILE;
  if (!one) {  // the whole bucket's column histogram first → bucket-local column starts
    for (int i = threadIdx.x; i < RS_WAVES * CB_ND; i += RS_THREADS) hw[i] = 0;
    __syncthreads();
    for (long i = start + threadIdx.x; i < end; i += RS_THREADS) {
      const int c = PACKED ? (int)(vin[i] >> 22) : kin[i] - kb;
      atomicAdd(&hw[c & (CB_ND - 1)], 1);
    }
    __syncthreads();
    rs_tile_cursors(hw, CB_ND, cb, wsum);  // (one row of counts: the others are zero)
    for (int c = threadIdx.x; c < ncol; c += RS_THREADS) cp[c0 + c] = rel + cb[c];
  }
  const int* base = one ? loc : cb;  // a one-chunk bucket: the chunk's column starts are the bucket's
  for (long a = start; a < end || (one && a == start); a += RS_TILE) {
    const long b = a + RS_TILE < end ? a + RS_TILE : end;
    for (int i = threadIdx.x; i < RS_WAVES * CB_ND; i += RS_THREADS) hw[i] = 0;
    __syncthreads();
    const long wa = a + (long)w * RS_SEG;
    const long wb = wa + RS_SEG < b ? wa + RS_SEG : b;
    int kr[RS_PER_LANE];
    uint64_t vr[RS_PER_LANE];
    rs_load_seg<uint64_t, int>(PACKED ? nullptr : kin, vin, wa, wb, kr, vr);
    if constexpr (PACKED) {
#pragma unroll
      for (int j = 0; j < RS_PER_LANE; ++j) kr[j] = (int)(vr[j] >> 22) & (CB_ND - 1);  // (kb = 0 below)
    }
    const int kbk = PACKED ? 0 : kb;
    rs_wave_hist(kr, wa, wb, kbk, 0, CB_ND - 1, hw + (long)w * CB_ND);
    __syncthreads();
    rs_tile_cursors(hw, CB_ND, loc, wsum);
    if (one)
      for (int c = threadIdx.x; c < ncol; c += RS_THREADS) cp[c0 + c] = rel + loc[c];
    rs_rank_place(kr, vr, wa, wb, kbk, 0, CB_ND - 1, hw + (long)w * CB_ND, [&](int pos, int, uint64_t val, int dg) {
      const long gp = split_off + start + base[dg] + (pos - loc[dg]);  // = start + pos for one chunk
      erow[gp] = PACKED ? (int)((unsigned)val & 0x3FFFFFu) : (int)(unsigned)val;
      evals[gp] = (unsigned)(val >> 32);
    });
    if (one) break;
    __syncthreads();
    const int len = (int)(b - a);
    for (int c = threadIdx.x; c < CB_ND; c += RS_THREADS) cb[c] += (c + 1 < CB_ND ? loc[c + 1] : len) - loc[c];
    __syncthreads();
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
  if (bound[S] - bound[0] >= (1L << 31) || bound[S] >= (1L << 31)) return -7;  // int32 output positions
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
    hipLaunchKernelGGL((rs_hist_kernel<int>), dim3(tb.ntile), dim3(RS_THREADS), lds, st, kin, tb, shift, mask, T);
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

// Stable LSD sort of every segment by key bits [bit_lo, bit_hi) (kbase 0): balanced digits of at
// most RS_MAX_DIGIT_BITS bits. 64-bit keys: the ordered bit images of fp64 scores / values, with
// the constant bits (equal in every key) left out of the range by the caller. Returns 0 / 1 as
// seg_sort (1: result in the _alt buffers).
template <typename K, typename V>
int sort_bits(K* keys, V* vals, K* keys_alt, V* vals_alt, const long* bound, int S, int bit_lo, int bit_hi,
              int* scratch, long scratch_ints, hipStream_t st) {
  SegTable tb{};
  int kb0[RS_MAXS] = {0};
  int rc = make_table(bound, kb0, S, tb);
  if (rc) return rc;
  const int nbits = bit_hi - bit_lo;
  if (bit_lo < 0 || nbits < 1 || bit_hi > (int)(8 * sizeof(K))) return -5;
  if (keys == nullptr || vals == nullptr || keys_alt == nullptr || vals_alt == nullptr) return -1;
  const int passes = (nbits + RS_MAX_DIGIT_BITS - 1) / RS_MAX_DIGIT_BITS;
  const int db = (nbits + passes - 1) / passes;
  const int nd = 1 << db;
  if (scratch_ints < (long)(tb.ntile + tb.ngrp) * nd) return -6;
  if (tb.ntile == 0) return 0;
  int* T = scratch;
  int* G = scratch + (long)tb.ntile * nd;
  const size_t lds = (size_t)RS_WAVES * nd * sizeof(int);
  const size_t lds_sc = (size_t)(RS_WAVES + 2) * nd * sizeof(int) + (size_t)RS_TILE * (sizeof(K) + sizeof(V)) +
                        RS_WAVES * sizeof(int);
  K* kin = keys;
  V* vin = vals;
  K* kout = keys_alt;
  V* vout = vals_alt;
  for (int p = 0; p < passes; ++p) {
    const int shift = bit_lo + p * db;
    const int mask = nd - 1;
    hipLaunchKernelGGL((rs_hist_kernel<K>), dim3(tb.ntile), dim3(RS_THREADS), lds, st, kin, tb, shift, mask, T);
    hipLaunchKernelGGL(rs_colscan_kernel, dim3((nd + 255) / 256, tb.ngrp), dim3(256), 0, st, T, tb, nd, G);
    hipLaunchKernelGGL(rs_base_kernel, dim3(tb.S), dim3(1024), 0, st, G, tb, nd);
    hipLaunchKernelGGL((rs_scatter_kernel<V, false, K>), dim3(tb.ntile), dim3(RS_THREADS), lds_sc, st, kin, vin, kout,
                       vout, T, G, tb, shift, mask, (int*)nullptr, (unsigned*)nullptr, 0L);
    K* tk = kin;
    kin = kout;
    kout = tk;
    V* tv = vin;
    vin = vout;
    vout = tv;
  }
  rc = (int)hipGetLastError();
  if (rc) return rc;
  return (passes & 1) ? 1 : 0;
}

}  // namespace

// ints of scratch fmlx_sort_u64 needs for these segments and an nbits-wide key range
FMLX_API long fmlx_sort_bits_scratch(const long* bound, int S, int nbits) {
  if (S < 1 || S > RS_MAXS || nbits < 1 || nbits > 64) return -1;
  long nt = 0, ng = 0;
  for (int s = 0; s < S; ++s) {
    const long tiles = (bound[s + 1] - bound[s] + RS_TILE - 1) / RS_TILE;
    nt += tiles;
    ng += (tiles + RS_TG - 1) / RS_TG;
  }
  const int passes = (nbits + RS_MAX_DIGIT_BITS - 1) / RS_MAX_DIGIT_BITS;
  const int db = (nbits + passes - 1) / passes;
  return (nt + ng) * (1L << db);
}

// Stable sort of (uint64 key, uint32 payload) pairs, segment by segment (`bound`: HOST array of
// S + 1 positions), by key bits [bit_lo, bit_hi). 0: result in keys / vals; 1: in the _alt buffers.
FMLX_API int fmlx_sort_u64(uint64_t* keys, uint32_t* vals, uint64_t* keys_alt, uint32_t* vals_alt, const long* bound,
                           int S, int bit_lo, int bit_hi, int* scratch, long scratch_ints, void* stream) {
  return sort_bits<uint64_t, uint32_t>(keys, vals, keys_alt, vals_alt, bound, S, bit_lo, bit_hi, scratch, scratch_ints,
                                       (hipStream_t)stream);
}

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

// The fp32 column-major copy of a run of batches in two passes (see rs_csc_bucket_kernel):
// keys = slot·d + column over 11 … 20 key bits, 64-bit (value bits << 32 | row) payloads. Pass 1
// sorts every segment stably by the key's high bits (keys / vals → keys_alt / vals_alt), pass 2
// writes erow / evals at split_off + position and the column pointer rows b0 … b0 + S − 1
// (int32 [*, d + 1]). `bound` / `kbase` are HOST arrays; scratch as fmlx_seg_sort_scratch.
FMLX_API int fmlx_csc_sort_split(int* keys, uint64_t* vals, int* keys_alt, uint64_t* vals_alt, const long* bound,
                                 const int* kbase, int S, int key_bits, int d, int* scratch, long scratch_ints,
                                 int* erow, unsigned* evals, long split_off, int* colptr, long b0, int packed,
                                 void* stream) {
  SegTable tb{};
  int rc = make_table(bound, kbase, S, tb);
  if (rc) return rc;
  if (key_bits < 11 || key_bits > 20 || d < 1 || d > (1 << key_bits)) return -5;
  const int dbA = key_bits - 10;
  const int ndA = 1 << dbA;
  if (scratch_ints < (long)(tb.ntile + tb.ngrp) * ndA) return -6;
  hipStream_t st = (hipStream_t)stream;
  int* T = scratch;
  int* G = scratch + (long)tb.ntile * ndA;
  if (tb.ntile > 0) {
    const size_t lds = (size_t)RS_WAVES * ndA * sizeof(int);
    const size_t lds_sc = (size_t)(RS_WAVES + 2) * ndA * sizeof(int) + (size_t)RS_TILE * (sizeof(int) + 8) +
                          RS_WAVES * sizeof(int);
    hipLaunchKernelGGL((rs_hist_kernel<int>), dim3(tb.ntile), dim3(RS_THREADS), lds, st, keys, tb, 10, ndA - 1, T);
    hipLaunchKernelGGL(rs_colscan_kernel, dim3((ndA + 255) / 256, tb.ngrp), dim3(256), 0, st, T, tb, ndA, G);
    hipLaunchKernelGGL(rs_base_kernel, dim3(tb.S), dim3(1024), 0, st, G, tb, ndA);
    hipLaunchKernelGGL((rs_scatter_kernel<uint64_t, false>), dim3(tb.ntile), dim3(RS_THREADS), lds_sc, st, keys, vals,
                       packed ? nullptr : keys_alt, vals_alt, T, G, tb, 10, ndA - 1, (int*)nullptr,
                       (unsigned*)nullptr, 0L);
  }
  const size_t lds_b = (size_t)(RS_WAVES + 2) * CB_ND * sizeof(int) + RS_WAVES * sizeof(int);
  if (packed)
    hipLaunchKernelGGL(rs_csc_bucket_kernel<true>, dim3((unsigned)(S * ndA)), dim3(RS_THREADS), lds_b, st, keys_alt,
                       vals_alt, G, tb, ndA, d, b0, colptr, erow, evals, split_off);
  else
    hipLaunchKernelGGL(rs_csc_bucket_kernel<false>, dim3((unsigned)(S * ndA)), dim3(RS_THREADS), lds_b, st, keys_alt,
                       vals_alt, G, tb, ndA, d, b0, colptr, erow, evals, split_off);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
