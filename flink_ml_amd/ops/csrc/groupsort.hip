// Group rows by a small integer key (KMeans labels, hash-shuffle partitions): a counting sort in
// three launches, no library sort. SURVEY §2.1 K9 (KMeans.java:287-295 accumulates per-cluster
// sums; here the rows are first grouped by cluster so the sums are contiguous segment reductions).
//
//  1. group_hist     every block builds an LDS histogram of a GS_TILE-row tile of keys (LDS
//                    atomics) and adds its non-zero bins to the global counts (one atomic per
//                    (tile, key) present);
//  2. group_scan     one block: exclusive scan of the counts → offsets[k + 1], the chunk offsets of
//                    the segment-sum kernels (ceil(count / chunk) per key, optional), the per-key
//                    write cursors; the counts are re-zeroed for the next round (hipGraph replays
//                    need no memset);
//  3. group_scatter  every block rebuilds its tile histogram, reserves one contiguous range per
//                    key with one global atomic, then writes its row indices through LDS cursors.
//
// Rows of one key end up contiguous but in an order that depends on atomic arrival (tiles and
// lanes), so a float reduction over a group is reproducible only to rounding; the KMeans
// deterministic mode (FMLX_DETERMINISTIC=1) keeps the stable radix sort (sort.hip).
// Keys outside [0, k) are dropped from the grouping (counted nowhere).
#include "common.h"

namespace {
constexpr int GS_TILE = 8192;
constexpr int GS_THREADS = 1024;

__global__ __launch_bounds__(GS_THREADS) void group_hist_kernel(const int* __restrict__ keys, long n, int k,
                                                                int* __restrict__ counts) {
  extern __shared__ int h[];
  for (int c = threadIdx.x; c < k; c += GS_THREADS) h[c] = 0;
  __syncthreads();
  const long r0 = (long)blockIdx.x * GS_TILE;
  const long r1 = r0 + GS_TILE < n ? r0 + GS_TILE : n;
  for (long r = r0 + threadIdx.x; r < r1; r += GS_THREADS) {
    const int c = keys[r];
    if ((unsigned)c < (unsigned)k) atomicAdd(&h[c], 1);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < k; c += GS_THREADS) {
    const int v = h[c];
    if (v) atomicAdd(&counts[c], v);
  }
}

__global__ __launch_bounds__(GS_THREADS) void group_scan_kernel(int* __restrict__ counts, int k, int chunk,
                                                                long* __restrict__ offsets, long* __restrict__ chunk_off,
                                                                int* __restrict__ cursor) {
  __shared__ long wtot[2][GS_THREADS / 64];
  __shared__ long carry[2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x < 2) carry[threadIdx.x] = 0;
  __syncthreads();
  for (int base = 0; base <= k; base += GS_THREADS) {
    const int c = base + threadIdx.x;
    const long cnt = c < k ? counts[c] : 0;
    const long chk = chunk > 0 ? (cnt + chunk - 1) / chunk : 0;
    long i0 = cnt, i1 = chk;  // inclusive wave scans of both sequences
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const long o0 = __shfl_up(i0, off, 64), o1 = __shfl_up(i1, off, 64);
      if (lane >= off) {
        i0 += o0;
        i1 += o1;
      }
    }
    if (lane == 63) {
      wtot[0][wv] = i0;
      wtot[1][wv] = i1;
    }
    __syncthreads();
    long p0 = 0, p1 = 0;
    for (int i = 0; i < wv; ++i) {
      p0 += wtot[0][i];
      p1 += wtot[1][i];
    }
    const long e0 = carry[0] + p0 + i0 - cnt, e1 = carry[1] + p1 + i1 - chk;
    if (c <= k) {
      offsets[c] = e0;
      if (chunk_off) chunk_off[c] = e1;
    }
    if (c < k) {
      cursor[c] = (int)e0;
      counts[c] = 0;  // ready for the next round's histogram
    }
    __syncthreads();
    if (threadIdx.x == GS_THREADS - 1) {
      carry[0] = e0 + cnt;
      carry[1] = e1 + chk;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(GS_THREADS) void group_scatter_kernel(const int* __restrict__ keys, long n, int k,
                                                                   int* __restrict__ cursor, int* __restrict__ order) {
  extern __shared__ int h[];
  for (int c = threadIdx.x; c < k; c += GS_THREADS) h[c] = 0;
  __syncthreads();
  const long r0 = (long)blockIdx.x * GS_TILE;
  const long r1 = r0 + GS_TILE < n ? r0 + GS_TILE : n;
  for (long r = r0 + threadIdx.x; r < r1; r += GS_THREADS) {
    const int c = keys[r];
    if ((unsigned)c < (unsigned)k) atomicAdd(&h[c], 1);
  }
  __syncthreads();
  // one reservation per key present in the tile; h[c] becomes the tile's write cursor
  for (int c = threadIdx.x; c < k; c += GS_THREADS) {
    const int v = h[c];
    if (v) h[c] = atomicAdd(&cursor[c], v);
  }
  __syncthreads();
  for (long r = r0 + threadIdx.x; r < r1; r += GS_THREADS) {
    const int c = keys[r];
    if ((unsigned)c < (unsigned)k) order[atomicAdd(&h[c], 1)] = (int)r;
  }
}
// ---------------------------------------------------------------------------------------------
// Stable variant (KMeans default): rows of one key keep their row order, so segment sums over a
// group are bit-reproducible and the result equals a stable sort by key. Tiles of ST_TILE rows;
// inside a tile, wave w owns the contiguous segment [w·ST_SEG, (w+1)·ST_SEG).
//  1. st_hist      per-tile key counts T[t][c] (per-wave LDS histograms, summed);
//  2. st_colscan   per group of ST_TG tiles and key: T[t][c] ← exclusive prefix inside the group,
//                  S[g][c] = the group's total;
//  3. st_base      one block: per key the exclusive prefix over groups (+ the key offset), the key
//                  offsets / chunk offsets (same outputs as group_scan);
//  4. st_scatter   per tile: per-wave histograms again, cursors = group base + in-group prefix +
//                  earlier waves; each wave walks its segment 64 rows at a time in row order:
//                  one ballot per key bit gives every row the set of lanes holding its key and
//                  its rank among them (lane order = row order); the highest lane of each key's
//                  run advances the cursor (was a 21-step bitonic sort of packed (key, lane)).
// Every step is order-deterministic; no global atomics.
constexpr int ST_WAVES = 8;
constexpr int ST_THREADS = ST_WAVES * 64;
constexpr int ST_SEG = 1024;                  // rows per wave segment
constexpr int ST_TILE = ST_WAVES * ST_SEG;    // 8192 rows per tile
constexpr int ST_TG = 64;                     // tiles per column-scan group
constexpr int ST_MAX_KEYS = 2048;             // [ST_WAVES][k] int32 LDS histograms: 64 KiB

__device__ __forceinline__ void st_wave_hist(const int* __restrict__ keys, long n, int k, long seg0, int* h) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < ST_SEG; i += 64) {
    const long r = seg0 + i;
    if (r < n) {
      const int c = keys[r];
      if ((unsigned)c < (unsigned)k) atomicAdd(&h[c], 1);  // LDS, the wave's own row
    }
  }
}

__global__ __launch_bounds__(ST_THREADS) void st_hist_kernel(const int* __restrict__ keys, long n, int k,
                                                             int* __restrict__ T) {
  extern __shared__ int sh[];
  const int w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < ST_WAVES * k; i += ST_THREADS) sh[i] = 0;
  __syncthreads();
  st_wave_hist(keys, n, k, (long)blockIdx.x * ST_TILE + (long)w * ST_SEG, sh + (long)w * k);
  __syncthreads();
  int* out = T + (long)blockIdx.x * k;
  for (int c = threadIdx.x; c < k; c += ST_THREADS) {
    int s = 0;
#pragma unroll
    for (int q = 0; q < ST_WAVES; ++q) s += sh[q * k + c];
    out[c] = s;
  }
}

// grid (ceil(k / 256), groups): thread = key; walks the group's tiles in order
__global__ __launch_bounds__(256) void st_colscan_kernel(int* __restrict__ T, int tiles, int k, int* __restrict__ S) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= k) return;
  const int t0 = blockIdx.y * ST_TG;
  const int t1 = t0 + ST_TG < tiles ? t0 + ST_TG : tiles;
  int run = 0;
  for (int tb = t0; tb < t1; tb += 16) {
    int v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = tb + q < t1 ? T[(long)(tb + q) * k + c] : 0;  // 16 loads in flight
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (tb + q < t1) T[(long)(tb + q) * k + c] = run;
      run += v[q];
    }
  }
  S[(long)blockIdx.y * k + c] = run;
}

// one block: S[g][c] ← key offset + exclusive prefix over groups; offsets / chunk offsets
__global__ __launch_bounds__(1024) void st_base_kernel(int* __restrict__ S, int groups, int k, int chunk,
                                                      long* __restrict__ offsets, long* __restrict__ chunk_off) {
  __shared__ long wtot[2][16];
  __shared__ long carry[2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x < 2) carry[threadIdx.x] = 0;
  __syncthreads();
  for (int base = 0; base <= k; base += 1024) {
    const int c = base + threadIdx.x;
    long cnt = 0;
    if (c < k) {
      for (int g = 0; g < groups; ++g) {  // per key: exclusive prefix over groups (in place)
        const int v = S[(long)g * k + c];
        S[(long)g * k + c] = (int)cnt;
        cnt += v;
      }
    }
    const long chk = chunk > 0 ? (cnt + chunk - 1) / chunk : 0;
    long i0 = cnt, i1 = chk;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const long o0 = __shfl_up(i0, off, 64), o1 = __shfl_up(i1, off, 64);
      if (lane >= off) {
        i0 += o0;
        i1 += o1;
      }
    }
    if (lane == 63) {
      wtot[0][wv] = i0;
      wtot[1][wv] = i1;
    }
    __syncthreads();
    long p0 = 0, p1 = 0;
    for (int i = 0; i < wv; ++i) {
      p0 += wtot[0][i];
      p1 += wtot[1][i];
    }
    const long e0 = carry[0] + p0 + i0 - cnt, e1 = carry[1] + p1 + i1 - chk;
    if (c <= k) {
      offsets[c] = e0;
      if (chunk_off) chunk_off[c] = e1;
    }
    if (c < k)
      for (int g = 0; g < groups; ++g) S[(long)g * k + c] += (int)e0;
    __syncthreads();
    if (threadIdx.x == 1023) {
      carry[0] = e0 + cnt;
      carry[1] = e1 + chk;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(ST_THREADS) void st_scatter_kernel(const int* __restrict__ keys, long n, int k,
                                                                const int* __restrict__ T, const int* __restrict__ S,
                                                                int* __restrict__ order) {
  extern __shared__ int sh[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = blockIdx.x;
  for (int i = threadIdx.x; i < ST_WAVES * k; i += ST_THREADS) sh[i] = 0;
  __syncthreads();
  const long seg0 = (long)t * ST_TILE + (long)w * ST_SEG;
  st_wave_hist(keys, n, k, seg0, sh + (long)w * k);
  __syncthreads();
  // cursors: the tile's base of key c (group base + in-group prefix) + earlier waves' counts
  const int* Tt = T + (long)t * k;
  const int* Sg = S + (long)(t / ST_TG) * k;
  for (int c = threadIdx.x; c < k; c += ST_THREADS) {
    int run = Sg[c] + Tt[c];
#pragma unroll
    for (int q = 0; q < ST_WAVES; ++q) {
      const int v = sh[q * k + c];
      sh[q * k + c] = run;
      run += v;
    }
  }
  __syncthreads();
  int* cur = sh + (long)w * k;
  int kb = 0;  // key bits
  while ((1 << kb) < k) ++kb;
  const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;  // lanes below this one
  for (int i0 = 0; i0 < ST_SEG; i0 += 64) {
    const long r = seg0 + i0 + lane;
    int key = -1;
    if (r < n) {
      key = keys[r];
      if ((unsigned)key >= (unsigned)k) key = -1;
    }
    const bool valid = key >= 0;
    // stable rank among equal keys of the 64 rows (lane order = row order): the lanes holding
    // my key (one ballot per key bit, no cross-lane data movement), then those below me
    unsigned long long peers = __ballot(valid);
    for (int bit = 0; bit < kb; ++bit) {
      // M = all ones where my key has this bit: the lanes agreeing with me are ballot XNOR M
      const int M = (int)((unsigned)key << (31 - bit)) >> 31;
      const unsigned long long bb = __ballot(M != 0);
      const unsigned lo = ~((unsigned)bb ^ (unsigned)M), hi = ~((unsigned)(bb >> 32) ^ (unsigned)M);
      peers &= ((unsigned long long)hi << 32) | lo;
    }
    const int rank = __popcll(peers & lt);
    const bool leader = valid && (peers >> lane) == 1ull;  // the highest lane of my key's run
    int pos = 0;
    if (valid) pos = cur[key] + rank;
    // every lane read its cursor above before a leader advances it (one wave: its LDS accesses
    // complete in program order)
    __builtin_amdgcn_wave_barrier();
    if (leader) cur[key] = pos + 1;
    if (valid) order[pos] = (int)r;
    __builtin_amdgcn_wave_barrier();
  }
}

}  // namespace

FMLX_API int fmlx_group_max_keys() { return 16384; }  // LDS histogram: 64 KiB
FMLX_API int fmlx_group_stable_max_keys() { return ST_MAX_KEYS; }

// Scratch ints of the stable grouping for n rows and k keys: T [tiles][k] + S [groups][k].
FMLX_API long fmlx_group_stable_scratch(long n, int k) {
  const long tiles = (n + ST_TILE - 1) / ST_TILE;
  const long groups = (tiles + ST_TG - 1) / ST_TG;
  return (tiles + (groups > 0 ? groups : 1)) * (long)k;
}

// Stable grouping: order[offsets[c] .. offsets[c+1]) = the rows with key c in row order.
// scratch: int32[fmlx_group_stable_scratch(n, k)]; offsets int64[k + 1]; chunk_off int64[k + 1]
// or null (chunk <= 0). Keys outside [0, k) are dropped.
FMLX_API int fmlx_group_by_key_stable(const int* keys, long n, int k, int chunk, int* scratch, long* offsets,
                                      long* chunk_off, int* order, void* stream) {
  if (k <= 0 || k > ST_MAX_KEYS) return -2;
  hipStream_t s = (hipStream_t)stream;
  const long tiles = (n + ST_TILE - 1) / ST_TILE;
  if (tiles >= (1L << 31)) return -3;
  const int groups = (int)((tiles + ST_TG - 1) / ST_TG);
  int* T = scratch;
  int* S = scratch + tiles * (long)k;
  const size_t lds = (size_t)ST_WAVES * k * sizeof(int);
  if (tiles > 0) {
    hipLaunchKernelGGL(st_hist_kernel, dim3((unsigned)tiles), dim3(ST_THREADS), lds, s, keys, n, k, T);
    hipLaunchKernelGGL(st_colscan_kernel, dim3((unsigned)((k + 255) / 256), (unsigned)groups), dim3(256), 0, s, T,
                       (int)tiles, k, S);
  }
  hipLaunchKernelGGL(st_base_kernel, dim3(1), dim3(1024), 0, s, S, groups, k, chunk, offsets, chunk_off);
  if (tiles > 0)
    hipLaunchKernelGGL(st_scatter_kernel, dim3((unsigned)tiles), dim3(ST_THREADS), lds, s, keys, n, k, T, S, order);
  return (int)hipGetLastError();
}

// counts: int32[k], zero before the first call (group_scan re-zeroes it); cursor: int32[k];
// offsets: int64[k + 1]; chunk_off: int64[k + 1] or null (chunk <= 0).
FMLX_API int fmlx_group_by_key(const int* keys, long n, int k, int chunk, int* counts, int* cursor, long* offsets,
                               long* chunk_off, int* order, void* stream) {
  if (k <= 0 || k > 16384) return -2;
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = (size_t)k * sizeof(int);
  const unsigned tiles = (unsigned)((n + GS_TILE - 1) / GS_TILE);
  if (n > 0) hipLaunchKernelGGL(group_hist_kernel, dim3(tiles), dim3(GS_THREADS), lds, s, keys, n, k, counts);
  hipLaunchKernelGGL(group_scan_kernel, dim3(1), dim3(GS_THREADS), 0, s, counts, k, chunk, offsets, chunk_off,
                     cursor);
  if (n > 0) hipLaunchKernelGGL(group_scatter_kernel, dim3(tiles), dim3(GS_THREADS), lds, s, keys, n, k, cursor, order);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
