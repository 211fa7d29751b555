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

// ---- FeatureHasher row assembly: W (index, value) pairs per row -> the row's sparse vector
// (reference FeatureHasher.HashFunction.map, FeatureHasher.java:118-141 + updateMap :184-194: a
// TreeMap<Integer, Double> that stores the first value of an index as it is and adds the later
// ones in column order). One thread per row: the W pairs are sorted by index in registers with an
// odd-even transposition network (adjacent swaps on strictly greater keys: stable, so equal
// indices keep their column order) and merged by a left-to-right sum. Phase 0 writes the row's
// distinct count to cnt[r]; phase 1 (after the host's scan into indptr) writes the entries.
// Group g of desc[W][4] = {index ptr, value ptr (0: 1.0), mode, const}; mode 0 = int32 final
// indices, 1 = raw int32 Java hashes (floorMod(Math.abs(h), const)), 2 = the constant index
// `const`, 3 = int64 final indices.
template <int WP>
__global__ __launch_bounds__(256) void fh_rows_kernel(const long long* __restrict__ desc, int W, long n, int phase,
                                                      long long* __restrict__ cnt, const long long* __restrict__ indptr,
                                                      int* __restrict__ oi, double* __restrict__ ov) {
  constexpr int PAD = 0x7fffffff;
  for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (long)gridDim.x * blockDim.x) {
    int key[WP];
    double val[WP];
#pragma unroll
    for (int g = 0; g < WP; ++g) {
      key[g] = PAD;
      val[g] = 0.0;
      if (g < W) {
        const long long* d = desc + 4 * g;
        const int mode = (int)d[2];
        if (mode == 2) {
          key[g] = (int)d[3];
        } else if (mode == 3) {
          key[g] = (int)reinterpret_cast<const long long*>(d[0])[r];
        } else {
          const int h = reinterpret_cast<const int*>(d[0])[r];
          if (mode == 1) {
            const int m = (int)d[3];
            const int a = h == (int)0x80000000 ? h : (h < 0 ? -h : h);  // Math.abs(Integer.MIN_VALUE) < 0
            const int q = a % m;
            key[g] = q < 0 ? q + m : q;
          } else {
            key[g] = h;
          }
        }
        val[g] = d[1] ? reinterpret_cast<const double*>(d[1])[r] : 1.0;
      }
    }
#pragma unroll
    for (int pass = 0; pass < WP; ++pass) {
#pragma unroll
      for (int i = pass & 1; i + 1 < WP; i += 2) {
        if (key[i] > key[i + 1]) {
          const int tk = key[i];
          key[i] = key[i + 1];
          key[i + 1] = tk;
          const double tv = val[i];
          val[i] = val[i + 1];
          val[i + 1] = tv;
        }
      }
    }
    if (phase == 0) {
      long long c = 0;
#pragma unroll
      for (int i = 0; i < WP; ++i) c += (i < W && (i == 0 || key[i] != key[i - 1])) ? 1 : 0;
      cnt[r] = c;
    } else {
      long long p = indptr[r];
      int prev = key[0];
      double acc = val[0];
#pragma unroll
      for (int i = 1; i < WP; ++i) {
        if (i < W) {
          if (key[i] != prev) {
            oi[p] = prev;
            ov[p] = acc;
            ++p;
            prev = key[i];
            acc = val[i];
          } else {
            acc += val[i];
          }
        }
      }
      oi[p] = prev;
      ov[p] = acc;
    }
  }
}

// ---- HashingTF per-document term counts: CSR rows of bucket indices (int64 or int32) -> each
// row's ascending distinct indices with their counts (HashingTF.java:101-125's per-row map).
// One thread per row, the row sorted in registers as above; a row longer than WP raises *flag
// (phase 0) and the host takes the general path.
template <int WP>
__global__ __launch_bounds__(256) void tf_rows_kernel(const long long* __restrict__ off, const void* __restrict__ keys,
                                                      int key64, long n, int phase, long long* __restrict__ cnt,
                                                      int* __restrict__ flag, const long long* __restrict__ indptr,
                                                      int* __restrict__ oi, double* __restrict__ ov, int binary) {
  constexpr int PAD = 0x7fffffff;
  for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (long)gridDim.x * blockDim.x) {
    const long long b = off[r];
    const int L = (int)(off[r + 1] - b);
    if (L > WP) {
      if (phase == 0) {
        *flag = 1;
        cnt[r] = 0;
      }
      continue;
    }
    int key[WP];
#pragma unroll
    for (int i = 0; i < WP; ++i)
      key[i] = i < L ? (key64 ? (int)reinterpret_cast<const long long*>(keys)[b + i]
                               : reinterpret_cast<const int*>(keys)[b + i])
                     : PAD;
#pragma unroll
    for (int pass = 0; pass < WP; ++pass) {
#pragma unroll
      for (int i = pass & 1; i + 1 < WP; i += 2) {
        const int lo = min(key[i], key[i + 1]), hi = max(key[i], key[i + 1]);
        key[i] = lo;
        key[i + 1] = hi;
      }
    }
    if (phase == 0) {
      long long c = 0;
#pragma unroll
      for (int i = 0; i < WP; ++i) c += (i < L && (i == 0 || key[i] != key[i - 1])) ? 1 : 0;
      cnt[r] = c;
    } else if (L > 0) {
      long long p = indptr[r];
      int prev = key[0];
      double c = 1.0;
#pragma unroll
      for (int i = 1; i < WP; ++i) {
        if (i < L) {
          if (key[i] != prev) {
            oi[p] = prev;
            ov[p] = binary ? 1.0 : c;
            ++p;
            prev = key[i];
            c = 1.0;
          } else {
            c += 1.0;
          }
        }
      }
      oi[p] = prev;
      ov[p] = binary ? 1.0 : c;
    }
  }
}

// ---- CountVectorizer term / document frequencies and first occurrences in one pass over the
// dictionary codes (CountVectorizer.java:151-204: per document a term counts once toward df and
// every time toward tf; the first-seen order decides the vocabulary order). A wave per document,
// per-block LDS histograms (integer atomics), a per-wave presence bitmap of V bits: the lane whose
// atomicOr first sets a term's bit in this document counts its df; the wave clears its bitmap
// after the document. Block results go out with one global atomic per non-zero term.
constexpr int CV_VMAX = 4096;
__global__ __launch_bounds__(256) void cv_tfdf_kernel(const int* __restrict__ codes, const long long* __restrict__ off,
                                                      long nd, int V, long docs_per_block,
                                                      unsigned long long* __restrict__ tf,
                                                      unsigned long long* __restrict__ df,
                                                      unsigned long long* __restrict__ first) {
  __shared__ unsigned tfl[CV_VMAX];
  __shared__ unsigned dfl[CV_VMAX];
  __shared__ unsigned fl[CV_VMAX];
  __shared__ unsigned bm[4][CV_VMAX / 32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int words = (V + 31) >> 5;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    tfl[i] = 0u;
    dfl[i] = 0u;
    fl[i] = 0xffffffffu;
  }
  for (int i = lane; i < words; i += 64) bm[w][i] = 0u;
  __syncthreads();
  const long d0 = (long)blockIdx.x * docs_per_block;
  const long d1 = d0 + docs_per_block < nd ? d0 + docs_per_block : nd;
  const long long base = d0 < nd ? off[d0] : 0;
  for (long d = d0 + w; d < d1; d += 4) {
    const long long b = off[d], e = off[d + 1];
    for (long long j = b + lane; j < e; j += 64) {
      const int c = codes[j];
      atomicAdd(&tfl[c], 1u);
      atomicMin(&fl[c], (unsigned)(j - base));
      const unsigned bit = 1u << (c & 31);
      if ((atomicOr(&bm[w][c >> 5], bit) & bit) == 0u) atomicAdd(&dfl[c], 1u);
    }
    for (int i = lane; i < words; i += 64) bm[w][i] = 0u;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    if (tfl[i]) {
      atomicAdd(&tf[i], (unsigned long long)tfl[i]);
      atomicAdd(&df[i], (unsigned long long)dfl[i]);
      atomicMin(&first[i], (unsigned long long)base + fl[i]);
    }
  }
}

// ---- NGram over dictionary codes (NGram.java:81-100): a row of L codes yields max(0, L − n + 1)
// grams, each the base-V number of n consecutive codes. Mark pass: one thread per row writes its
// gram count and sets present[g] (a byte per possible gram, V^n small; racing writers store the
// same 1). After the host's scans (row offsets, inclusive gram ranks) the emit pass writes every
// gram's rank — its index in the sorted distinct grams — at its final place.
__global__ __launch_bounds__(256) void ngram_mark_kernel(const int* __restrict__ codes, const long long* __restrict__ off,
                                                         long nd, int n, long long V, unsigned char* __restrict__ present,
                                                         long long* __restrict__ cnt) {
  for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < nd; r += (long)gridDim.x * blockDim.x) {
    const long long b = off[r];
    const long long c = off[r + 1] - b - n + 1;
    cnt[r] = c > 0 ? c : 0;
    for (long long t = 0; t < c; ++t) {
      long long g = 0;
      for (int j = 0; j < n; ++j) g = g * V + codes[b + t + j];
      present[g] = 1;
    }
  }
}
__global__ __launch_bounds__(256) void ngram_emit_kernel(const int* __restrict__ codes, const long long* __restrict__ off,
                                                         long nd, int n, long long V, const int* __restrict__ rank,
                                                         const long long* __restrict__ noff, int* __restrict__ out) {
  for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < nd; r += (long)gridDim.x * blockDim.x) {
    const long long b = off[r];
    const long long c = off[r + 1] - b - n + 1;
    const long long o = noff[r];
    for (long long t = 0; t < c; ++t) {
      long long g = 0;
      for (int j = 0; j < n; ++j) g = g * V + codes[b + t + j];
      out[o + t] = rank[g] - 1;
    }
  }
}
}  // namespace

// phase 0: present (u8 [V^n], zeroed by the caller) and cnt (int64 [nd]); phase 1: out at noff
// from the inclusive ranks (int32 [V^n])
FMLX_API int fmlx_ngram_codes(const int* codes, const long long* off, long nd, int n, long long V, int phase,
                              unsigned char* present, long long* cnt, const int* rank, const long long* noff, int* out,
                              void* stream) {
  if (nd <= 0) return 0;
  if (off == nullptr || n < 1 || V < 1 || (phase == 0 && (present == nullptr || cnt == nullptr)) ||
      (phase != 0 && (rank == nullptr || noff == nullptr || out == nullptr)))
    return -1;
  const long want = (nd + 255) / 256;
  const int blocks = (int)(want < 16384 ? want : 16384);
  hipStream_t s = (hipStream_t)stream;
  if (phase == 0)
    hipLaunchKernelGGL(ngram_mark_kernel, dim3(blocks), dim3(256), 0, s, codes, off, nd, n, V, present, cnt);
  else
    hipLaunchKernelGGL(ngram_emit_kernel, dim3(blocks), dim3(256), 0, s, codes, off, nd, n, V, rank, noff, out);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_cv_vmax() { return CV_VMAX; }

// codes int32 [N] in [0, V), off int64 [nd+1]; tf / df zeroed and first filled with N by the
// caller (u64 [V] each). A block's codes must span < 2^32 positions.
FMLX_API int fmlx_cv_tfdf(const int* codes, const long long* off, long nd, int V, unsigned long long* tf,
                          unsigned long long* df, unsigned long long* first, void* stream) {
  if (nd <= 0) return 0;
  if (V < 1 || V > CV_VMAX || off == nullptr || tf == nullptr || df == nullptr || first == nullptr) return -1;
  long blocks = 2048;
  if (blocks > (nd + 3) / 4) blocks = (nd + 3) / 4;
  const long per = (nd + blocks - 1) / blocks;
  blocks = (nd + per - 1) / per;
  hipLaunchKernelGGL(cv_tfdf_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, codes, off, nd, V, per,
                     tf, df, first);
  return (int)hipGetLastError();
}

// off: int64 [n+1] row offsets; keys int64 (key64) or int32 bucket indices in [0, 2^31 − 1).
// Phase 0: cnt[n] = distinct per row, *flag = 1 if a row exceeds 32 entries; phase 1: entries.
FMLX_API int fmlx_tf_rows(const long long* off, const void* keys, int key64, long n, int maxlen, int phase,
                          long long* cnt, int* flag, const long long* indptr, int* oi, double* ov, int binary,
                          void* stream) {
  if (n <= 0) return 0;
  if (off == nullptr || (phase == 0 && (cnt == nullptr || flag == nullptr)) ||
      (phase != 0 && (indptr == nullptr || oi == nullptr || ov == nullptr)))
    return -1;
  long want = (n + 255) / 256;
  const int blocks = (int)(want < 16384 ? want : 16384);
  hipStream_t s = (hipStream_t)stream;
  if (maxlen <= 8)
    hipLaunchKernelGGL(tf_rows_kernel<8>, dim3(blocks), dim3(256), 0, s, off, keys, key64, n, phase, cnt, flag, indptr,
                       oi, ov, binary);
  else if (maxlen <= 16)
    hipLaunchKernelGGL(tf_rows_kernel<16>, dim3(blocks), dim3(256), 0, s, off, keys, key64, n, phase, cnt, flag,
                       indptr, oi, ov, binary);
  else
    hipLaunchKernelGGL(tf_rows_kernel<32>, dim3(blocks), dim3(256), 0, s, off, keys, key64, n, phase, cnt, flag,
                       indptr, oi, ov, binary);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_fh_rows_wmax() { return 16; }

// desc: device int64 [W][4] (see fh_rows_kernel); phase 0 -> cnt[n], phase 1 -> oi / ov at indptr
FMLX_API int fmlx_fh_rows(const long long* desc, int W, long n, int phase, long long* cnt, const long long* indptr,
                          int* oi, double* ov, void* stream) {
  if (n <= 0) return 0;
  if (W < 1 || W > 16 || desc == nullptr || (phase == 0 && cnt == nullptr) ||
      (phase != 0 && (indptr == nullptr || oi == nullptr || ov == nullptr)))
    return -1;
  long want = (n + 255) / 256;
  const int blocks = (int)(want < 16384 ? want : 16384);
  hipStream_t s = (hipStream_t)stream;
  if (W <= 4)
    hipLaunchKernelGGL(fh_rows_kernel<4>, dim3(blocks), dim3(256), 0, s, desc, W, n, phase, cnt, indptr, oi, ov);
  else if (W <= 8)
    hipLaunchKernelGGL(fh_rows_kernel<8>, dim3(blocks), dim3(256), 0, s, desc, W, n, phase, cnt, indptr, oi, ov);
  else
    hipLaunchKernelGGL(fh_rows_kernel<16>, dim3(blocks), dim3(256), 0, s, desc, W, n, phase, cnt, indptr, oi, ov);
  return (int)hipGetLastError();
}

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
