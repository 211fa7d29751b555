// Bit-exact java.util.Random streams on the GPU for the benchmark data generators
// (reference flink-ml-benchmark/.../datagenerator/common/*Generator.java; RowGenerator seeds each
// task with new Random(Tuple2.of(seed, taskIdx).hashCode()) and draws row after row).
//
// java.util.Random is a 48-bit LCG, so the state after k draws is an affine map of the seed:
// x_k = A_k x + C_k (mod 2^48). Every thread jumps straight to its row's first draw with
// (A_k, C_k) computed by binary powering (the low 48 bits of 64-bit products are exact), then
// runs the row's "program" sequentially: nextDouble (2 draws) or nextInt(bound) (1 draw;
// power-of-two bounds never reject). For other bounds Java's nextInt rejects u with
// u - u % bound + bound - 1 >= 2^31 and draws again (probability ~ bound / 2^31 per draw);
// the kernel reports the first row that would reject and the host replays that row
// sequentially and relaunches for the remaining rows at the shifted offset, so the output is
// exactly the reference stream.
//
// Outputs: the first `nvec` program slots go to a dense [n, nvec] buffer in the requested dtype
// (the features column, written coalesced); the remaining slots go to an fp64 [n, nscalar] buffer
// (label / weight / scalar columns).
#include "common.h"

namespace {
constexpr unsigned long long kMult = 0x5DEECE66DULL;
constexpr unsigned long long kAdd = 0xBULL;
constexpr unsigned long long kMask = (1ULL << 48) - 1;

__device__ __forceinline__ unsigned long long jump(unsigned long long x, unsigned long long k) {
  unsigned long long A = 1, C = 0;  // accumulated map
  unsigned long long a = kMult, c = kAdd;  // map for 2^i steps
  while (k) {
    if (k & 1) {
      A = (A * a) & kMask;
      C = (C * a + c) & kMask;
    }
    c = (c * a + c) & kMask;
    a = (a * a) & kMask;
    k >>= 1;
  }
  return (A * x + C) & kMask;
}

__device__ __forceinline__ int next_bits(unsigned long long& s, int bits) {
  s = (s * kMult + kAdd) & kMask;
  return (int)(long long)(s >> (48 - bits));
}

template <typename T>
__device__ __forceinline__ void store(T* p, double v) {
  *p = (T)v;
}
template <>
__device__ __forceinline__ void store<bf16_t>(bf16_t* p, double v) {
  *p = f32_to_bf16((float)v);
}

// ops: per slot, 0 = nextDouble, >0 = nextInt(bound).
constexpr int CHUNK = 16;
constexpr int kRowsPerBlock = 256;

// One thread per row, generating the row's program sequentially (the jump-ahead is paid once per
// row: a wave-uniform jump to the block's first row plus a short per-lane jump of at most
// 256·draws_per_row). Vector slots are staged through an LDS tile [256][CHUNK+1] and stored
// cooperatively so each store instruction writes whole 16-element row segments.
template <typename T>
__global__ __launch_bounds__(256) void java_rows_kernel(unsigned long long seed, unsigned long long start_draw,
                                                        long row0, long nrows, const int* __restrict__ ops,
                                                        int nslots, int nvec, int draws_per_row,
                                                        T* __restrict__ vec, double* __restrict__ scal,
                                                        unsigned long long* first_reject) {
  __shared__ T tile[kRowsPerBlock][CHUNK + 1];
  const int tid = threadIdx.x;
  const long rbase = (long)blockIdx.x * kRowsPerBlock;
  const long r = rbase + tid;
  const bool live = r < nrows;
  const unsigned long long base = jump(seed, start_draw + (unsigned long long)rbase * draws_per_row);
  unsigned long long s = jump(base, (unsigned long long)tid * draws_per_row);
  const int nsc = nslots - nvec;
  for (int j0 = 0; j0 < nslots; j0 += CHUNK) {
    const int j1 = j0 + CHUNK < nslots ? j0 + CHUNK : nslots;
    if (live) {
      for (int j = j0; j < j1; ++j) {
        const int op = ops[j];
        double v;
        if (op == 0) {
          const long long hi = next_bits(s, 26);
          const long long lo = next_bits(s, 27);
          v = (double)((hi << 27) + lo) * (1.0 / (double)(1ULL << 53));
        } else {
          const int u = next_bits(s, 31);
          if ((op & (op - 1)) == 0) {
            v = (double)(int)(((long long)op * (long long)u) >> 31);
          } else {
            const int rr = u % op;
            if ((long long)u - rr + (op - 1) >= (1LL << 31)) {
              atomicMin(first_reject, (unsigned long long)r);
              v = 0.0;
            } else {
              v = (double)rr;
            }
          }
        }
        if (j < nvec)
          store(&tile[tid][j - j0], v);
        else
          scal[(row0 + r) * (long)nsc + (j - nvec)] = v;
      }
    }
    if (j0 < nvec) {
      const int w = (nvec < j1 ? nvec : j1) - j0;
      __syncthreads();
      for (int idx = tid; idx < kRowsPerBlock * w; idx += kRowsPerBlock) {
        const int rr = idx / w, jj = idx - rr * w;
        if (rbase + rr < nrows) vec[(row0 + rbase + rr) * (long)nvec + j0 + jj] = tile[rr][jj];
      }
      __syncthreads();
    }
  }
}

template <typename T>
int launch(unsigned long long seed, unsigned long long start_draw, long row0, long nrows, const int* ops,
           const int* slot_off, int nslots, int nvec, int draws_per_row, void* vec, double* scal,
           unsigned long long* first_reject, hipStream_t st) {
  if (nrows <= 0) return 0;
  (void)slot_off;
  const long blocks = (nrows + kRowsPerBlock - 1) / kRowsPerBlock;
  hipLaunchKernelGGL((java_rows_kernel<T>), dim3((unsigned)blocks), dim3(kRowsPerBlock), 0, st, seed, start_draw,
                     row0, nrows, ops, nslots, nvec, draws_per_row, (T*)vec, scal, first_reject);
  return (int)hipGetLastError();
}
}  // namespace

// seed: the already scrambled LCG state ((seed ^ 0x5DEECE66D) & mask); start_draw: draws consumed
// before row0. first_reject must be preset to ULLONG_MAX; it receives the smallest local row index
// (relative to row0) whose nextInt would have rejected.
namespace {
// Raw nextInt(bound) draws at consecutive sequence positions [start, start + count): r = u % bound
// and whether Java's rejection loop accepts u (u − r + bound − 1 < 2^31). 16 positions per thread
// after one jump-ahead. The host compacts the accepted draws with a prefix sum, which reproduces
// Random.nextInt's sequential rejection loop for rows whose draws all use the same bound.
__global__ __launch_bounds__(256) void java_int_draws_kernel(unsigned long long x0, unsigned long long start,
                                                             long count, int bound, int* __restrict__ r_out,
                                                             unsigned char* __restrict__ ok_out) {
  const long base = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (base >= count) return;
  unsigned long long s = jump(x0, start + (unsigned long long)base);
  const long end = base + 16 < count ? base + 16 : count;
  for (long p = base; p < end; ++p) {
    const int u = next_bits(s, 31);
    const int r = u % bound;
    r_out[p] = r;
    ok_out[p] = ((long long)u - r + bound - 1) < (1LL << 31) ? 1 : 0;
  }
}
}  // namespace

namespace {
// Raw next(31) values at consecutive sequence positions [start, start + count), 16 per thread
// after one jump-ahead (the device reservoir sampler's draw stream, ops/datagen.py).
__global__ __launch_bounds__(256) void java_next31_kernel(unsigned long long x0, unsigned long long start, long count,
                                                          int* __restrict__ u_out) {
  const long base = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (base >= count) return;
  unsigned long long s = jump(x0, start + (unsigned long long)base);
  const long end = base + 16 < count ? base + 16 : count;
  for (long p = base; p < end; ++p) u_out[p] = next_bits(s, 31);
}
}  // namespace

namespace {
// Final pass of the device reservoir sampler: position p of the draw stream (not rejected) is the
// accepted draw of element i = p + k − R(p), R(p) = rejected positions before p (rej: ascending);
// it writes slot nextInt-result if that is < k. The last writer of a slot wins: atomicMax over i.
// The stream is regenerated by jump-ahead (16 positions per thread), not read back.
__global__ __launch_bounds__(256) void reservoir_final_kernel(unsigned long long x0, long end, int k,
                                                              const long* __restrict__ rej, long nrej,
                                                              int* __restrict__ out) {
  const long base = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 16;
  if (base >= end) return;
  long lo = 0, hi = nrej;  // R(base) = lower_bound(rej, base)
  while (lo < hi) {
    const long mid = (lo + hi) >> 1;
    if (rej[mid] < base) lo = mid + 1; else hi = mid;
  }
  long R = lo;
  unsigned long long s = jump(x0, (unsigned long long)base);
  const long stop = base + 16 < end ? base + 16 : end;
  for (long p = base; p < stop; ++p) {
    const long long u = next_bits(s, 31);
    if (R < nrej && rej[R] == p) {  // a rejected draw: the same element draws again at p + 1
      ++R;
      continue;
    }
    const long i = p + k - R;
    const long b = i + 1;
    const long slot = (b & (b - 1)) == 0 ? (long)((b * u) >> 31) : (long)(u % b);
    if (slot < k) atomicMax(&out[slot], (int)i);
  }
}

// the stream positions that can hold a rejected draw (u_p + p >= 2^31 − k − 1, see
// reservoir_sample_device), compacted in ANY order through one counter: they are a tiny fraction
// of the stream (≈ npos² / 2^32) and the host orders them before its sequential scan
__global__ __launch_bounds__(256) void reservoir_cand_kernel(const int* __restrict__ u, long npos, long thr, long cap,
                                                             int* __restrict__ cp, int* __restrict__ cu,
                                                             unsigned long long* __restrict__ cnt) {
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < npos; p += (long)gridDim.x * blockDim.x) {
    const int v = u[p];
    if ((long)v + p >= thr) {
      const unsigned long long at = atomicAdd(cnt, 1ull);
      if ((long)at < cap) {
        cp[at] = (int)p;
        cu[at] = v;
      }
    }
  }
}
}  // namespace

// cnt: one u64, zeroed by the caller; entries past cap are counted but not stored
FMLX_API int fmlx_reservoir_candidates(const int* u, long npos, int k, long cap, int* cp, int* cu,
                                       unsigned long long* cnt, void* stream) {
  if (npos <= 0) return 0;
  if (u == nullptr || cnt == nullptr || cap < 0 || (cap > 0 && (cp == nullptr || cu == nullptr))) return -1;
  const long want = (npos + 255) / 256;
  const int blocks = (int)(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(reservoir_cand_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, u, npos,
                     (1L << 31) - (long)k - 1, cap, cp, cu, cnt);
  return (int)hipGetLastError();
}

// out: int32[k], preset to 0 .. k − 1 (the reservoir's initial fill)
FMLX_API int fmlx_reservoir_final(unsigned long long seed, long end, int k, const long* rej, long nrej, int* out,
                                  void* stream) {
  if (end <= 0) return 0;
  const long threads = (end + 15) / 16;
  hipLaunchKernelGGL(reservoir_final_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     seed, end, k, rej, nrej, out);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_java_next31(unsigned long long seed, unsigned long long start, long count, int* u_out,
                              void* stream) {
  if (count <= 0) return 0;
  const long threads = (count + 15) / 16;
  hipLaunchKernelGGL(java_next31_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     seed, start, count, u_out);
  return (int)hipGetLastError();
}

// seed: the scrambled Random state; see java_int_draws_kernel.
FMLX_API int fmlx_java_int_draws(unsigned long long seed, unsigned long long start, long count, int bound, int* r_out,
                                 unsigned char* ok_out, void* stream) {
  if (count <= 0) return 0;
  if (bound <= 0) return -1;
  const long threads = (count + 15) / 16;
  hipLaunchKernelGGL(java_int_draws_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, seed, start, count, bound, r_out, ok_out);
  return (int)hipGetLastError();
}

// ---- rare-rejection compaction of the int draws: the rejected positions (ok == 0) compacted in
// any order through one counter (the host sorts the few of them), then every accepted draw copied
// to its final place: output i reads source i + #{j : q_j <= i} with q_j = p_j − j for the sorted
// rejected positions p_j (a binary search) — one read and one write per draw instead of a boolean
// mask index (a prefix sum over the whole stream).
namespace {
__global__ __launch_bounds__(256) void zero_positions_kernel(const unsigned char* __restrict__ ok, long n, long cap,
                                                             long long* __restrict__ pos,
                                                             unsigned long long* __restrict__ cnt) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    if (ok[i] == 0) {
      const unsigned long long at = atomicAdd(cnt, 1ull);
      if ((long)at < cap) pos[at] = i;
    }
  }
}
__global__ __launch_bounds__(256) void remove_positions_kernel(const int* __restrict__ src, const long long* __restrict__ q,
                                                               int nq, int* __restrict__ dst, long nout) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nout; i += (long)gridDim.x * blockDim.x) {
    int lo = 0, hi = nq;  // #{j : q_j <= i}
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (q[mid] <= i)
        lo = mid + 1;
      else
        hi = mid;
    }
    dst[i] = src[i + lo];
  }
}
}  // namespace

// pos: int64 [cap]; cnt: one u64 zeroed by the caller (counts past cap too)
FMLX_API int fmlx_u8_zero_positions(const unsigned char* ok, long n, long cap, long long* pos, unsigned long long* cnt,
                                    void* stream) {
  if (n <= 0) return 0;
  if (ok == nullptr || cnt == nullptr || (cap > 0 && pos == nullptr)) return -1;
  const long want = (n + 255) / 256;
  const int blocks = (int)(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(zero_positions_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, ok, n, cap, pos, cnt);
  return (int)hipGetLastError();
}

// q: int64 [nq] non-decreasing (sorted rejected positions minus their rank); src holds at least
// nout + nq entries
FMLX_API int fmlx_remove_positions_i32(const int* src, const long long* q, int nq, int* dst, long nout, void* stream) {
  if (nout <= 0) return 0;
  if (src == nullptr || dst == nullptr || nq < 0 || (nq > 0 && q == nullptr)) return -1;
  const long want = (nout + 255) / 256;
  const int blocks = (int)(want < 16384 ? want : 16384);
  hipLaunchKernelGGL(remove_positions_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src, q, nq, dst, nout);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_java_rows(int vec_dtype, unsigned long long seed, unsigned long long start_draw, long row0,
                            long nrows, const int* ops, const int* slot_off, int nslots, int nvec, int draws_per_row,
                            void* vec, double* scal, unsigned long long* first_reject, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (vec_dtype == DT_F64)
    return launch<double>(seed, start_draw, row0, nrows, ops, slot_off, nslots, nvec, draws_per_row, vec, scal,
                          first_reject, st);
  if (vec_dtype == DT_F32)
    return launch<float>(seed, start_draw, row0, nrows, ops, slot_off, nslots, nvec, draws_per_row, vec, scal,
                         first_reject, st);
  if (vec_dtype == DT_BF16)
    return launch<bf16_t>(seed, start_draw, row0, nrows, ops, slot_off, nslots, nvec, draws_per_row, vec, scal,
                          first_reject, st);
  return -1;
}

FMLX_DEFINE_PRELOAD()
