// BinaryClassificationEvaluator on the device (reference
// LIB/evaluation/binaryclassification/BinaryClassificationEvaluator.java:79-724).
//
// The reference sorts every range partition by descending score (:131), gives every tie group its
// average ascending rank for the AUC rank sum (AccumulateMultiScoreOperator :221-267, closed at
// :162-181), and walks the sorted partition once more for the trapezoid sums of the PR and Lorenz
// curves and the KS maximum (updateBinaryMetrics). Here, per rank:
//
//   bc_keys      scores → 64-bit keys whose ascending order is Double.compare's order of −score
//                (descending scores, NaN last), row ids as payloads, and the OR / AND of all keys
//                (the host sorts only the bit range that differs between keys);
//   radix.hip    stable LSD sort of the (key, row) pairs over that range (fmlx_sort_u64);
//   bc_agg       per 4096-row tile of the sorted order: #positives, #negatives, last tie-group
//                head and first tie-group tail;
//   bc_carry     one block: exclusive prefix counts over the tiles, prefix max of the heads and
//                suffix min of the tails (the tie groups that cross tile boundaries);
//   bc_metrics   per tile, with the carries: cumulative TP / FP counts, every row's tie group
//                [gs, ge] (block max-/min-scans), and the partial sums Σ w·(gs + ge) over the
//                positives (→ Σ_g avg_rank_g · Σ_{g, pos} w), Σ w of positives / negatives, the PR
//                and Lorenz trapezoids and the KS max — written per tile;
//   bc_final     one block sums the tile partials in a fixed order (bit-reproducible).
//
// Ties are rows with equal scores (+0 and −0 equal, every NaN its own group), as the reference's
// `score != t.f0` test; rows of a tie keep their input order (the sort is stable).
#include "common.h"

namespace {

constexpr int BC_THREADS = 256;
constexpr int BC_PER = 16;                       // consecutive sorted rows per thread
constexpr int BC_TILE = BC_THREADS * BC_PER;     // rows per block
constexpr int BC_WAVES = BC_THREADS / 64;
constexpr uint64_t NAN_KEY = 0xFFF8000000000000ull;  // key of the canonical NaN
constexpr int NPART = 6;  // Σ w(gs+ge) | Σ w pos | Σ w neg | lorenz | pr | ks

__device__ __forceinline__ uint64_t desc_key(double s) {
  double v = -s;
  if (v == 0.0) v = 0.0;  // −0 ties with +0
  uint64_t b = (uint64_t)__double_as_longlong(v);
  if (v != v) b = 0x7ff8000000000000ull;  // every NaN: after +inf (Double.compare)
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ bool new_group(uint64_t prev, uint64_t cur) { return cur != prev || cur == NAN_KEY; }

// payload of a row: its id in bits 0..30, its label (1 = positive) in bit 31 — the scans then read
// the label from the sorted payload instead of gathering it by row id
constexpr uint32_t POS_BIT = 0x80000000u;

__global__ __launch_bounds__(BC_THREADS) void bc_keys_kernel(const double* __restrict__ score,
                                                             const uint8_t* __restrict__ pos, long n,
                                                             uint64_t* __restrict__ keys, uint32_t* __restrict__ idx,
                                                             unsigned long long* __restrict__ orand) {
  __shared__ unsigned long long s_or[BC_WAVES], s_and[BC_WAVES];
  unsigned long long o = 0, a = ~0ull;
  for (long i = (long)blockIdx.x * BC_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * BC_THREADS) {
    const uint64_t k = desc_key(score[i]);
    keys[i] = k;
    idx[i] = (uint32_t)i | (pos[i] ? POS_BIT : 0u);
    o |= k;
    a &= k;
  }
  for (int off = 32; off > 0; off >>= 1) {
    o |= __shfl_xor(o, off, 64);
    a &= __shfl_xor(a, off, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_or[w] = o;
    s_and[w] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < BC_WAVES; ++q) {
      o |= s_or[q];
      a &= s_and[q];
    }
    atomicOr(orand, o);
    atomicAnd(orand + 1, a);
  }
}

// --- block scans over one value per thread (BC_THREADS threads) ---------------------------------
template <typename T, typename Op>
__device__ __forceinline__ T block_excl_scan(T v, T ident, Op op, T* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T o = __shfl_up(inc, off, 64);
    if (lane >= off) inc = op(inc, o);
  }
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  T pre = ident;
  for (int q = 0; q < w; ++q) pre = op(pre, sh[q]);
  T ex = __shfl_up(inc, 1, 64);
  if (lane == 0) ex = ident;
  __syncthreads();
  return op(pre, ex);
}

template <typename T, typename Op>
__device__ __forceinline__ T block_excl_suffix_scan(T v, T ident, Op op, T* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T o = __shfl_down(inc, off, 64);
    if (lane + off < 64) inc = op(inc, o);
  }
  if (lane == 0) sh[w] = inc;
  __syncthreads();
  T suf = ident;
  for (int q = BC_WAVES - 1; q > w; --q) suf = op(suf, sh[q]);
  T ex = __shfl_down(inc, 1, 64);
  if (lane == 63) ex = ident;
  __syncthreads();
  return op(suf, ex);
}

struct Lmax {
  __device__ long operator()(long a, long b) const { return a > b ? a : b; }
};
struct Lmin {
  __device__ long operator()(long a, long b) const { return a < b ? a : b; }
};
struct Iadd {
  __device__ int operator()(int a, int b) const { return a + b; }
};

// the thread's rows of tile t: sorted positions r0 … r0 + cnt − 1
__device__ __forceinline__ void thread_rows(long n, long& r0, int& cnt) {
  r0 = (long)blockIdx.x * BC_TILE + (long)threadIdx.x * BC_PER;
  const long rem = n - r0;
  cnt = rem <= 0 ? 0 : (rem < BC_PER ? (int)rem : BC_PER);
}

// the thread's (up to) BC_PER consecutive sorted keys and payloads: 16-byte loads (the 64 lanes'
// 128-byte runs are whole lines, reused from L1 by the following loads)
__device__ __forceinline__ void load_rows(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ idx,
                                          long r0, int cnt, uint64_t (&k)[BC_PER], uint32_t (&p)[BC_PER]) {
  if (cnt == BC_PER) {
#pragma unroll
    for (int j = 0; j < BC_PER; j += 2) {
      const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(keys + r0 + j);
      k[j] = v.x;
      k[j + 1] = v.y;
    }
#pragma unroll
    for (int j = 0; j < BC_PER; j += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(idx + r0 + j);
      p[j] = v.x;
      p[j + 1] = v.y;
      p[j + 2] = v.z;
      p[j + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < BC_PER; ++j) {
      k[j] = j < cnt ? keys[r0 + j] : 0;
      p[j] = j < cnt ? idx[r0 + j] : 0;
    }
  }
}

// agg[t] = {#pos, #neg, last head, first tail} of tile t (head/tail: −1 / n when none)
__global__ __launch_bounds__(BC_THREADS) void bc_agg_kernel(const uint64_t* __restrict__ keys,
                                                            const uint32_t* __restrict__ idx, long n,
                                                            long* __restrict__ agg) {
  __shared__ long sh[2 * BC_WAVES];
  __shared__ long sh2[2 * BC_WAVES];
  long r0;
  int cnt;
  thread_rows(n, r0, cnt);
  uint64_t k[BC_PER];
  uint32_t pl[BC_PER];
  load_rows(keys, idx, r0, cnt, k, pl);
  const uint64_t kprev = (cnt > 0 && r0 > 0) ? keys[r0 - 1] : 0;
  const uint64_t knext = (cnt > 0 && r0 + cnt < n) ? keys[r0 + cnt] : 0;
  int np = 0, nn = 0;
  long head = -1, tail = n;
#pragma unroll
  for (int j = 0; j < BC_PER; ++j) {
    if (j < cnt) {
      const long r = r0 + j;
      const bool p = (pl[j] & POS_BIT) != 0;
      np += p;
      nn += !p;
      const uint64_t pk = j == 0 ? kprev : k[j - 1];
      if (r == 0 || new_group(pk, k[j])) head = r;
    }
  }
#pragma unroll
  for (int j = BC_PER - 1; j >= 0; --j) {
    if (j < cnt) {
      const long r = r0 + j;
      const uint64_t nk = j + 1 < cnt ? k[j + 1] : knext;
      if (r == n - 1 || new_group(k[j], nk)) tail = r;
    }
  }
  // block reductions: sums (ints), max head, min tail
  long a = np, b = nn;
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off, 64);
    b += __shfl_xor(b, off, 64);
    const long h = __shfl_xor(head, off, 64), t = __shfl_xor(tail, off, 64);
    head = h > head ? h : head;
    tail = t < tail ? t : tail;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[w] = a;
    sh[BC_WAVES + w] = b;
    sh2[w] = head;
    sh2[BC_WAVES + w] = tail;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < BC_WAVES; ++q) {
      a += sh[q];
      b += sh[BC_WAVES + q];
      head = sh2[q] > head ? sh2[q] : head;
      tail = sh2[BC_WAVES + q] < tail ? sh2[BC_WAVES + q] : tail;
    }
    long* o = agg + (long)blockIdx.x * 4;
    o[0] = a;
    o[1] = b;
    o[2] = head;
    o[3] = tail;
  }
}

// one block of 1024: carry[t] = {#pos before t, #neg before t, max head before t, min tail after t},
// chunks of 1024 tiles with block scans (forward for the first three, backward for the tails)
__global__ __launch_bounds__(1024) void bc_carry_kernel(const long* __restrict__ agg, long nt,
                                                        long* __restrict__ carry) {
  __shared__ long wsum[3][16];
  __shared__ long run[3];
  __shared__ long runmin;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    run[0] = 0;
    run[1] = 0;
    run[2] = -1;
    runmin = 0x7fffffffffffffffL;
  }
  __syncthreads();
  for (long base = 0; base < nt; base += 1024) {
    const long t = base + threadIdx.x;
    const bool ok = t < nt;
    long a = ok ? agg[t * 4 + 0] : 0, b = ok ? agg[t * 4 + 1] : 0, h = ok ? agg[t * 4 + 2] : -1;
    long ia = a, ib = b, ih = h;  // inclusive wave scans
    for (int off = 1; off < 64; off <<= 1) {
      const long oa = __shfl_up(ia, off, 64), ob = __shfl_up(ib, off, 64), oh = __shfl_up(ih, off, 64);
      if (lane >= off) {
        ia += oa;
        ib += ob;
        ih = oh > ih ? oh : ih;
      }
    }
    if (lane == 63) {
      wsum[0][w] = ia;
      wsum[1][w] = ib;
      wsum[2][w] = ih;
    }
    __syncthreads();
    long pa = run[0], pb = run[1], ph = run[2];
    for (int q = 0; q < w; ++q) {
      pa += wsum[0][q];
      pb += wsum[1][q];
      ph = wsum[2][q] > ph ? wsum[2][q] : ph;
    }
    const long ea = pa + ia - a, eb = pb + ib - b;  // exclusive
    long eh = __shfl_up(ih, 1, 64);
    if (lane == 0) eh = -1;
    eh = eh > ph ? eh : ph;
    if (ok) {
      carry[t * 4 + 0] = ea;
      carry[t * 4 + 1] = eb;
      carry[t * 4 + 2] = eh;
    }
    __syncthreads();
    if (threadIdx.x == 1023) {
      run[0] = ea + a;
      run[1] = eb + b;
      run[2] = (h > eh ? h : eh);
    }
    __syncthreads();
  }
  for (long top = nt; top > 0; top -= 1024) {
    const long base = top > 1024 ? top - 1024 : 0;
    const long t = base + threadIdx.x;
    const bool ok = t < top;
    const long v = ok ? agg[t * 4 + 3] : 0x7fffffffffffffffL;
    long iv = v;  // inclusive suffix min within the wave
    for (int off = 1; off < 64; off <<= 1) {
      const long o = __shfl_down(iv, off, 64);
      if (lane + off < 64) iv = o < iv ? o : iv;
    }
    if (lane == 0) wsum[0][w] = iv;
    __syncthreads();
    long sm = runmin;
    for (int q = 15; q > w; --q) sm = wsum[0][q] < sm ? wsum[0][q] : sm;
    long ev = __shfl_down(iv, 1, 64);
    if (lane == 63) ev = 0x7fffffffffffffffL;
    ev = ev < sm ? ev : sm;
    if (ok) carry[t * 4 + 3] = ev;
    __syncthreads();
    if (threadIdx.x == 0) runmin = v < ev ? v : ev;
    __syncthreads();
  }
}

struct Totals {
  double before_t, before_f, tot_t, tot_f;
};

__device__ __forceinline__ void rates(double a, double b, const Totals& T, double& tpr, double& fpr, double& prec,
                                      double& prate) {
  tpr = T.tot_t != 0.0 ? a / T.tot_t : 1.0;
  fpr = T.tot_f != 0.0 ? b / T.tot_f : 1.0;
  prec = (a + b == 0.0) ? 1.0 : a / (a + b);
  prate = (a + b) / (T.tot_t + T.tot_f);
}

__global__ __launch_bounds__(BC_THREADS) void bc_metrics_kernel(const uint64_t* __restrict__ keys,
                                                                const uint32_t* __restrict__ idx,
                                                                const double* __restrict__ wt, long n,
                                                                const long* __restrict__ carry, Totals T,
                                                                double* __restrict__ part) {
  __shared__ long shl[BC_WAVES];
  __shared__ int shi[BC_WAVES];
  __shared__ double shd[NPART][BC_WAVES];
  long r0;
  int cnt;
  thread_rows(n, r0, cnt);
  const long* cy = carry + (long)blockIdx.x * 4;
  // pass 1 over the thread's rows: local counts, last head, first tail
  int np = 0, nn = 0;
  long head = -1, tail = 0x7fffffffffffffffL;
  uint64_t k[BC_PER];
  uint32_t pl[BC_PER];
  bool p[BC_PER];
  double w[BC_PER];
  load_rows(keys, idx, r0, cnt, k, pl);
#pragma unroll
  for (int j = 0; j < BC_PER; ++j) {
    p[j] = j < cnt && (pl[j] & POS_BIT) != 0;
    w[j] = j >= cnt ? 0.0 : (wt != nullptr ? wt[pl[j] & ~POS_BIT] : 1.0);
  }
  const uint64_t kprev = (cnt > 0 && r0 > 0) ? keys[r0 - 1] : 0;
  const uint64_t knext = (cnt > 0 && r0 + cnt < n) ? keys[r0 + cnt] : 0;
#pragma unroll
  for (int j = 0; j < BC_PER; ++j) {
    if (j < cnt) {
      const long r = r0 + j;
      np += p[j];
      nn += !p[j];
      const uint64_t pk = j == 0 ? kprev : k[j - 1];
      if (r == 0 || new_group(pk, k[j])) head = r;
    }
  }
#pragma unroll
  for (int j = BC_PER - 1; j >= 0; --j) {
    if (j < cnt) {
      const long r = r0 + j;
      const uint64_t nk = j + 1 < cnt ? k[j + 1] : knext;
      if (r == n - 1 || new_group(k[j], nk)) tail = r;
    }
  }
  // carries into this thread: counts before it, last head before it, first tail after it
  const int cp_in = block_excl_scan<int>(np, 0, Iadd(), shi);
  const int cn_in = block_excl_scan<int>(nn, 0, Iadd(), shi);
  long hin = block_excl_scan<long>(head, -1, Lmax(), shl);
  long tin = block_excl_suffix_scan<long>(tail, 0x7fffffffffffffffL, Lmin(), shl);
  hin = hin > cy[2] ? hin : cy[2];
  tin = tin < cy[3] ? tin : cy[3];
  // ge of row j: the first tail at or after j (scan right to left), gs: the last head at or before j
  long ge[BC_PER];
  {
    long t = tin;
#pragma unroll
    for (int j = BC_PER - 1; j >= 0; --j) {
      if (j < cnt) {
        const long r = r0 + j;
        const uint64_t nk = j + 1 < cnt ? k[j + 1] : knext;
        if (r == n - 1 || new_group(k[j], nk)) t = r;
      }
      ge[j] = t;
    }
  }
  double acc[NPART] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  double cpt = T.before_t + (double)(cy[0] + cp_in), cnf = T.before_f + (double)(cy[1] + cn_in);
  long gs = hin;
#pragma unroll
  for (int j = 0; j < BC_PER; ++j) {
    if (j < cnt) {
      const long r = r0 + j;
      const uint64_t pk = j == 0 ? kprev : k[j - 1];
      if (r == 0 || new_group(pk, k[j])) gs = r;
      const double a0 = cpt, b0 = cnf;
      if (p[j]) {
        acc[0] += w[j] * (double)(gs + ge[j]);
        acc[1] += w[j];
        cpt += 1.0;
      } else {
        acc[2] += w[j];
        cnf += 1.0;
      }
      double tpr, fpr, prec, prate, tpr0, fpr0, prec0, prate0;
      rates(cpt, cnf, T, tpr, fpr, prec, prate);
      rates(a0, b0, T, tpr0, fpr0, prec0, prate0);
      acc[3] += (prate - prate0) * (tpr + tpr0) / 2.0;
      acc[4] += (tpr - tpr0) * (prec + prec0) / 2.0;
      const double ks = fabs(fpr - tpr);
      acc[5] = ks > acc[5] ? ks : acc[5];
    }
  }
  // block reduction in a fixed order (wave butterflies, then waves 0..3)
#pragma unroll
  for (int q = 0; q < NPART; ++q) {
    double v = acc[q];
    for (int off = 32; off > 0; off >>= 1) {
      const double o = __shfl_xor(v, off, 64);
      v = q == 5 ? (o > v ? o : v) : v + o;
    }
    acc[q] = v;
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < NPART; ++q) shd[q][wv] = acc[q];
  __syncthreads();
  if (threadIdx.x < NPART) {
    const int q = threadIdx.x;
    double v = shd[q][0];
    for (int i = 1; i < BC_WAVES; ++i) v = q == 5 ? (shd[q][i] > v ? shd[q][i] : v) : v + shd[q][i];
    part[(long)blockIdx.x * NPART + q] = v;
  }
}

__global__ __launch_bounds__(64) void bc_final_kernel(const double* __restrict__ part, long nt,
                                                      double* __restrict__ out) {
  // one wave: lane l sums tiles l, l + 64, … ; then a fixed butterfly
  for (int q = 0; q < NPART; ++q) {
    double v = 0.0;
    for (long t = threadIdx.x; t < nt; t += 64) {
      const double x = part[t * NPART + q];
      v = q == 5 ? (x > v ? x : v) : v + x;
    }
    for (int off = 32; off > 0; off >>= 1) {
      const double o = __shfl_xor(v, off, 64);
      v = q == 5 ? (o > v ? o : v) : v + o;
    }
    if (threadIdx.x == 0) out[q] = v;
  }
}

}  // namespace

FMLX_API int fmlx_bc_tile() { return BC_TILE; }

// keys[i] / payloads (row | label << 31) for the sort; orand = {OR, AND} of all keys (device; the
// caller fills {0, ~0}); n < 2^31
FMLX_API int fmlx_bc_keys(const double* score, const uint8_t* pos, long n, uint64_t* keys, uint32_t* idx,
                          unsigned long long* orand, void* stream) {
  if (n <= 0) return 0;
  if (n >= (1L << 31)) return -2;
  long blocks = (n + BC_THREADS * 8 - 1) / (BC_THREADS * 8);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(bc_keys_kernel, dim3((unsigned)blocks), dim3(BC_THREADS), 0, (hipStream_t)stream, score, pos, n,
                     keys, idx, orand);
  return (int)hipGetLastError();
}

// Metrics of the sorted rows (keys / payloads in sorted order, the payload carrying row id and
// label; wt by original row, may be null). scratch: int64[8 · tiles], part: double[6 · tiles] with tiles = ceil(n / fmlx_bc_tile()).
// out[6] = {Σ_pos w·(gs + ge), Σ_pos w, Σ_neg w, lorenz, pr, ks} (gs / ge: local sorted positions).
FMLX_API int fmlx_bc_metrics(const uint64_t* keys, const uint32_t* idx, const double* wt, long n,
                             double before_t, double before_f, double tot_t, double tot_f, long* scratch,
                             double* part, double* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const long nt = (n + BC_TILE - 1) / BC_TILE;
  if (n <= 0) {
    (void)hipMemsetAsync(out, 0, NPART * sizeof(double), s);
    return (int)hipGetLastError();
  }
  long* agg = scratch;
  long* carry = scratch + nt * 4;
  hipLaunchKernelGGL(bc_agg_kernel, dim3((unsigned)nt), dim3(BC_THREADS), 0, s, keys, idx, n, agg);
  hipLaunchKernelGGL(bc_carry_kernel, dim3(1), dim3(1024), 0, s, agg, nt, carry);
  Totals T{before_t, before_f, tot_t, tot_f};
  hipLaunchKernelGGL(bc_metrics_kernel, dim3((unsigned)nt), dim3(BC_THREADS), 0, s, keys, idx, wt, n, carry, T,
                     part);
  hipLaunchKernelGGL(bc_final_kernel, dim3(1), dim3(64), 0, s, part, nt, out);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
