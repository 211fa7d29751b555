// MinHash signatures for MinHashLSH (reference MinHashLSHModelData.hashFunction,
// flink-ml-lib/.../feature/lsh/MinHashLSHModelData.java:95-112): for every row of a CSR set matrix
// and every hash function k,  h_k = min over nonzero indices i of ((1 + i) * a_k + b_k) mod P,
// P = 2038074743, written as fp64 (the reference stores the values in DenseVectors).
//
// MI355X design: one thread per (row, k) pair — lanes of a wave share a row, so the row's index
// list is read once from L2/L1 and broadcast; the 62-bit product is reduced with a Barrett step
// (one 64-bit mul-hi + mul + 2 conditional subtracts) instead of a 64-bit integer division, which
// CDNA has no hardware for.
#include "common.h"

namespace {
constexpr unsigned long long kPrime = 2038074743ull;
// floor((2^64 - 1) / P)
constexpr unsigned long long kBarrett = 0xFFFFFFFFFFFFFFFFull / kPrime;

__device__ __forceinline__ unsigned long long mod_p(unsigned long long x) {
  const unsigned long long q = __umul64hi(x, kBarrett);
  unsigned long long r = x - q * kPrime;
  r = r >= kPrime ? r - kPrime : r;
  return r >= kPrime ? r - kPrime : r;
}

__global__ __launch_bounds__(256) void minhash_csr_kernel(const long* __restrict__ indptr,
                                                          const int* __restrict__ indices, long n, int K,
                                                          const int* __restrict__ coef_a,
                                                          const int* __restrict__ coef_b,
                                                          double* __restrict__ out) {
  const long total = n * (long)K;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const long row = t / K;
    const int k = (int)(t - row * K);
    const unsigned long long a = (unsigned int)coef_a[k];
    const unsigned long long b = (unsigned int)coef_b[k];
    const long s = indptr[row], e = indptr[row + 1];
    unsigned long long m = kPrime;
    long j = s;
    for (; j + 4 <= e; j += 4) {
      const unsigned long long v0 = mod_p((1ull + (unsigned int)indices[j]) * a + b);
      const unsigned long long v1 = mod_p((1ull + (unsigned int)indices[j + 1]) * a + b);
      const unsigned long long v2 = mod_p((1ull + (unsigned int)indices[j + 2]) * a + b);
      const unsigned long long v3 = mod_p((1ull + (unsigned int)indices[j + 3]) * a + b);
      const unsigned long long m01 = v0 < v1 ? v0 : v1;
      const unsigned long long m23 = v2 < v3 ? v2 : v3;
      const unsigned long long mm = m01 < m23 ? m01 : m23;
      m = mm < m ? mm : m;
    }
    for (; j < e; ++j) {
      const unsigned long long v = mod_p((1ull + (unsigned int)indices[j]) * a + b);
      m = v < m ? v : m;
    }
    out[t] = (double)m;
  }
}
}  // namespace

// indptr: int64 [n+1]; indices: int32; coef_a/coef_b: int32 [K]; out: fp64 [n, K] row-major.
FMLX_API int fmlx_minhash_csr(const long* indptr, const int* indices, long n, int K, const int* coef_a,
                              const int* coef_b, double* out, void* stream) {
  if (n <= 0 || K <= 0) return 0;
  const long total = n * (long)K;
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(minhash_csr_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, indptr, indices,
                     n, K, coef_a, coef_b, out);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
