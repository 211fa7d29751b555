// Stable key/index radix sort over the low `bits` bits of int32 keys (hipCUB/rocPRIM onesweep),
// used to group KMeans rows by cluster (K9): labels < k need only ceil(log2 k) bits — 2 passes for
// k = 1024 instead of the 8 passes of a full 64-bit argsort. Radix sort is stable, so the row
// order inside a cluster — and with it the fp summation order — is the same every run.
#include <hipcub/hipcub.hpp>

#include "common.h"

FMLX_API long fmlx_sort_pairs_temp_bytes(long n, int bits) {
  size_t bytes = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int*)nullptr, (int*)nullptr,
                                                     (const int*)nullptr, (int*)nullptr, (int)n, 0, bits);
  return e == hipSuccess ? (long)bytes : -1;
}

FMLX_API int fmlx_sort_pairs(const int* keys_in, int* keys_out, const int* vals_in, int* vals_out, long n, int bits,
                             void* temp, long temp_bytes, void* stream) {
  if (n <= 0) return 0;
  size_t tb = (size_t)temp_bytes;
  return (int)hipcub::DeviceRadixSort::SortPairs(temp, tb, keys_in, keys_out, vals_in, vals_out, (int)n, 0, bits,
                                                  (hipStream_t)stream);
}

// Same with 64-bit payloads (the sparse trainer's column-major copies carry (value bits, row) in
// one payload through the sort instead of gathering both afterwards, csc_build.hip)
FMLX_API long fmlx_sort_pairs64_temp_bytes(long n, int bits) {
  size_t bytes = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int*)nullptr, (int*)nullptr,
                                                     (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)n, 0, bits);
  return e == hipSuccess ? (long)bytes : -1;
}

FMLX_API int fmlx_sort_pairs64(const int* keys_in, int* keys_out, const uint64_t* vals_in, uint64_t* vals_out, long n,
                               int bits, void* temp, long temp_bytes, void* stream) {
  if (n <= 0) return 0;
  size_t tb = (size_t)temp_bytes;
  return (int)hipcub::DeviceRadixSort::SortPairs(temp, tb, keys_in, keys_out, vals_in, vals_out, (int)n, 0, bits,
                                                  (hipStream_t)stream);
}

// Bucket starts of SORTED int32 keys in [0, nbins): out[c] = first position holding a key >= c,
// out[nbins] = n — the column pointers of the sparse trainer's per-batch column-major copies
// straight from the sorted keys (a histogram + scan over 16M bins took 5.5 ms per 16-batch run).
// Thread i fills the bins (key[i-1], key[i]] with i, so every bin is written exactly once.
namespace {
__global__ __launch_bounds__(256) void sorted_bounds_kernel(const int* __restrict__ keys, long n, int nbins,
                                                            int* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i > n) return;
  const int lo = i > 0 ? keys[i - 1] : -1;
  const int hi = i < n ? keys[i] : nbins;
  for (int c = lo + 1; c <= hi; ++c) out[c] = (int)i;
}
}  // namespace

FMLX_API int fmlx_sorted_bounds(const int* keys, long n, int nbins, int* out, void* stream) {
  if (n < 0 || nbins < 0 || n >= (1L << 31)) return -1;
  const long threads = n + 1;
  hipLaunchKernelGGL(sorted_bounds_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, keys, n, nbins, out);
  return (int)hipGetLastError();
}
