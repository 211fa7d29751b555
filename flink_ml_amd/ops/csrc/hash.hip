// Device murmur3_32 (Guava semantics, seed 0) over pre-encoded UTF-16 strings + the HashingTF /
// FeatureHasher bucket index. One thread per string; the host encodes a batch
// of strings once into a flat code-unit buffer with offsets.
#include "common.h"

namespace {
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t mixk(uint32_t k1) { return rotl32(k1 * 0xcc9e2d51u, 15) * 0x1b873593u; }
__device__ __forceinline__ uint32_t mixh(uint32_t h1, uint32_t k1) {
  h1 ^= k1;
  return rotl32(h1, 13) * 5u + 0xe6546b64u;
}
__device__ __forceinline__ uint32_t fmix32(uint32_t h1, uint32_t len) {
  h1 ^= len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  return h1 ^ (h1 >> 16);
}

// mode 0: HashingTF nonNegativeMod(h, m); mode 1: FeatureHasher floorMod(|h|, m)
__global__ __launch_bounds__(256) void murmur3_chars_kernel(const uint16_t* __restrict__ units,
                                                            const long* __restrict__ offsets, long n, int mod,
                                                            int mode, int* __restrict__ hash_out,
                                                            int* __restrict__ index_out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const uint16_t* cs = units + offsets[i];
    const long len = offsets[i + 1] - offsets[i];
    uint32_t h1 = 0;
    for (long j = 1; j < len; j += 2) h1 = mixh(h1, mixk((uint32_t)cs[j - 1] | ((uint32_t)cs[j] << 16)));
    if (len & 1) h1 ^= mixk((uint32_t)cs[len - 1]);
    const int h = (int)fmix32(h1, (uint32_t)(2 * len));
    if (hash_out) hash_out[i] = h;
    if (index_out && mod > 0) {
      if (mode == 0) {
        int r = h % mod;
        index_out[i] = r < 0 ? r + mod : r;
      } else {
        int a = h == (int)0x80000000 ? h : (h < 0 ? -h : h);  // Math.abs(Integer.MIN_VALUE) stays negative
        int r = a % mod;
        index_out[i] = r < 0 ? r + mod : r;
      }
    }
  }
}
}  // namespace

FMLX_API int fmlx_murmur3_chars_device(const void* units, const long* offsets, long n, int mod, int mode,
                                       int* hash_out, int* index_out, void* stream) {
  if (n <= 0) return 0;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(murmur3_chars_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint16_t*)units,
                     offsets, n, mod, mode, hash_out, index_out);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
