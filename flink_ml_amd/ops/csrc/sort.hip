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
