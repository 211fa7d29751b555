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
}  // namespace

FMLX_API int fmlx_group_max_keys() { return 16384; }  // LDS histogram: 64 KiB

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
