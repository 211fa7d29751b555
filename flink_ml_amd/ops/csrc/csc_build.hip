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
// replacing ~10 torch ops and their run-sized temporaries (repeat_interleave of the row ids and
// slots, int64 sort indices, gather copies, the bucket-start array and its two slicing copies):
// a whole fit that transposes its batches lazily pays for those allocations inside the fit.
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
// the copy out is sequential (no random gathers; csc_fill's two gathers per entry cost ~4× more)
__global__ __launch_bounds__(256) void csc_keys64_kernel(const long* __restrict__ indptr, const int* __restrict__ idx,
                                                         const float* __restrict__ values, long r0, long r1, long B,
                                                         int d, long j0, int* __restrict__ key,
                                                         uint64_t* __restrict__ payload) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = r0 + wave; r < r1; r += nw) {
    const long s0 = indptr[r], s1 = indptr[r + 1];
    const long slot = (r - r0) / B;
    const int kb = (int)(slot * d);
    const uint32_t rr = (uint32_t)(r - r0 - slot * B);
    for (long j = s0 + lane; j < s1; j += 64) {
      const long o = j - j0;
      key[o] = kb + idx[j];
      payload[o] = ((uint64_t)__float_as_uint(values[j]) << 32) | rr;
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

__global__ __launch_bounds__(256) void csc_colptr_kernel(const int* __restrict__ keys, long m, int slots, int d,
                                                         const long* __restrict__ indptr, long b0, long B, long n,
                                                         long j0, int* __restrict__ colptr) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i > m) return;
  const long nb = (long)slots * d;
  const long lo = i > 0 ? keys[i - 1] : -1;
  const long hi = i < m ? keys[i] : nb;
  for (long c = lo + 1; c <= hi; ++c) {
    const long s = c / d;
    const long cc = c - s * d;
    if (cc == 0 && s > 0) {  // the previous batch ends here: its entry count
      const long rb = (b0 + s - 1) * B;
      colptr[(b0 + s - 1) * (d + 1) + d] = (int)(i - (indptr[rb < n ? rb : n] - j0));
    }
    if (s < slots) {
      const long rb = (b0 + s) * B;
      colptr[(b0 + s) * (d + 1) + cc] = (int)(i - (indptr[rb < n ? rb : n] - j0));
    }
  }
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
                             long j0, int* key, uint64_t* payload, void* stream) {
  if (r1 <= r0) return 0;
  if (B <= 0 || d <= 0) return -1;
  hipLaunchKernelGGL(csc_keys64_kernel, dim3(grid_for(r1 - r0, 4, 1u << 16)), dim3(256), 0, (hipStream_t)stream,
                     indptr, idx, values, r0, r1, B, d, j0, key, payload);
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

// colptr: int32 [P, d + 1] of the whole partition; rows b0 … b0 + slots − 1 are written
FMLX_API int fmlx_csc_colptr(const int* sorted_keys, long m, int slots, int d, const long* indptr, long b0, long B,
                             long n, long j0, int* colptr, void* stream) {
  if (slots <= 0 || d <= 0 || m < 0 || m >= (1L << 31) || (long)slots * d >= (1L << 31)) return -1;
  hipLaunchKernelGGL(csc_colptr_kernel, dim3((unsigned)((m + 1 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     sorted_keys, m, slots, d, indptr, b0, B, n, j0, colptr);
  return (int)hipGetLastError();
}
