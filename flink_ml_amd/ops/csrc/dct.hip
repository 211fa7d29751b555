// DCT-II / DCT-III of every row (reference LIB/feature/dct/DCT.java:103-123,
// JTransforms DoubleDCT_1D scaled): the orthonormal transform Y = X·Mᵀ (forward) or X = Y·M
// (inverse) of rows of n ≤ 128 f32 values, on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32); fp64
// rows (parity mode) on v_mfma_f64_16x16x4_f64 (dct_rows_f64_kernel).
//
// Even/odd butterfly: the basis rows satisfy M[k][n−1−i] = (−1)^k M[k][i], so with h = ⌈n/2⌉
//   forward   Y[2k']   = Σ_{i<h} u_i M[2k'][i],     u_i = x_i + x_{n−1−i}  (u_mid = x_mid, n odd)
//             Y[2k'+1] = Σ_{i<h} v_i M[2k'+1][i],   v_i = x_i − x_{n−1−i}  (v_mid = 0)
//   inverse   E_i = Σ_{k'} y_{2k'} M[2k'][i],  O_i = Σ_{k'} y_{2k'+1} M[2k'+1][i]  (i < h)
//             x_i = E_i + O_i,  x_{n−1−i} = E_i − O_i
// — two GEMMs of K, N ≤ h instead of one of n × n: at n = 100, 104 MFMAs per 16 rows instead of
// 175, which puts the f32 MFMA time (≈ 0.9 ms for 10M rows) under the HBM time of one read and
// one write of the rows. The butterflies ride on the fragment reads (forward) and on the
// accumulator read-out (inverse): the lane holding E_i also holds O_i.
//
// Persistent blocks of 4 waves; the block keeps both half bases in LDS for its whole life, laid
// out as the MFMA B fragments are consumed ([k step][h][r][tile]), and walks 64-row tiles:
//   * a tile (64 contiguous rows = one contiguous 256·n-byte range) streams in with 16-byte loads
//     into LDS rows of stride S (S/4 odd: the strided fragment reads hit distinct banks); the
//     loads of the NEXT tile are issued before this tile's MFMAs, so they fly under the math;
//   * each wave owns 16 rows: its A fragments of both GEMMs go to registers first (butterflied);
//     per k step the lane's B fragments of every output tile are one 16-byte LDS read, issued a
//     step ahead, then one MFMA per 16-column output tile;
//   * the wave's 16 × n result goes back through its own LDS rows and out as contiguous 16-byte
//     stores (its 16 rows are one contiguous range of Y).
#include "common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int DCT_THREADS = 256;
constexpr int DCT_ROWS = 64;    // rows per block tile (16 per wave)
constexpr int DCT_MAXN = 128;
constexpr int DCT_PF = 8;       // 16-byte prefetch loads per thread per tile (64 rows × 128 cols / 256 thr / 4)

struct DctGeom {
  int n, h, ho, KP, S, NT, NT8;
};

// h = ⌈n/2⌉ (even-half size), ho = ⌊n/2⌋; KP = h rounded up to the k step (4); NT = ⌈h/16⌉ output
// tiles per half GEMM, NT8 = NT rounded up to even (fragment reads of 8 / 16 bytes);
// S: LDS row stride of the X tile with S/4 odd
__host__ __device__ inline DctGeom dct_geom(int n) {
  DctGeom g;
  g.n = n;
  g.h = (n + 1) / 2;
  g.ho = n / 2;
  g.KP = (g.h + 3) / 4 * 4;
  const int np = (n + 3) / 4 * 4;
  g.S = ((np / 4) & 1) ? np : np + 4;
  g.NT = (g.h + 15) / 16;
  g.NT8 = (g.NT + 1) / 2 * 2;
  return g;
}

// KS = KP/4 k steps of each half GEMM (NT = ⌈KS/4⌉ follows), INV: DCT-III, VEC: n % 4 == 0.
// The k loop is fully unrolled with the A fragments in registers and no per-step branches.
template <int KS, bool INV, bool VEC>
__global__ __launch_bounds__(DCT_THREADS) void dct_rows_kernel(const float* __restrict__ X, long rows, int n,
                                                               const float* __restrict__ basis,
                                                               float* __restrict__ Y, int diag) {
  constexpr int NT = (KS + 3) / 4;
  constexpr int NT8 = (NT + 1) / 2 * 2;
  constexpr int BHALF = KS * 64 * NT8;  // floats of one half basis
  extern __shared__ __align__(16) float sm[];
  const DctGeom g = dct_geom(n);
  float* sb = sm;                  // half bases [2][KS][4][16][NT8]
  float* sx = sm + 2 * BHALF;      // tile [64][S]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < 2 * BHALF; i += DCT_THREADS) sb[i] = basis[i];
  const long ntiles = (rows + DCT_ROWS - 1) / DCT_ROWS;
  float4 pf[DCT_PF];
  // prefetch: thread tid loads float4 number tid + q·256 of the tile's contiguous 64·n floats
  auto load_tile = [&](long t) {
    const long base = t * DCT_ROWS * (long)n;
    const long lim = (rows - t * DCT_ROWS < DCT_ROWS ? rows - t * DCT_ROWS : DCT_ROWS) * (long)n;
#pragma unroll
    for (int q = 0; q < DCT_PF; ++q) {
      const long e = (long)(tid + q * DCT_THREADS) * 4;
      if (VEC) {
        pf[q] = e < lim ? *reinterpret_cast<const float4*>(X + base + e) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        pf[q].x = e < lim ? X[base + e] : 0.f;
        pf[q].y = e + 1 < lim ? X[base + e + 1] : 0.f;
        pf[q].z = e + 2 < lim ? X[base + e + 2] : 0.f;
        pf[q].w = e + 3 < lim ? X[base + e + 3] : 0.f;
      }
    }
  };
  // row / column of a flat tile offset e < 64·n without an integer divide: (e + ½)/n in f32 is
  // at least ½/n ≥ 1/256 away from an integer and e < 2^13 keeps the f32 error below 1e-3
  const float invn = 1.0f / (float)n;
  auto rowof = [&](int e) { return (int)(((float)e + 0.5f) * invn); };
  auto store_tile = [&]() {
#pragma unroll
    for (int q = 0; q < DCT_PF; ++q) {
      const int e = (tid + q * DCT_THREADS) * 4;
      if (e < DCT_ROWS * n) {
        if (VEC) {  // a float4 never straddles a row: one 16-byte LDS store
          const int rr = rowof(e);
          *reinterpret_cast<float4*>(sx + rr * g.S + (e - rr * n)) = pf[q];
        } else {
          const float v[4] = {pf[q].x, pf[q].y, pf[q].z, pf[q].w};
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int ee = e + c;
            const int rr = rowof(ee);
            if (ee < DCT_ROWS * n) sx[rr * g.S + (ee - rr * n)] = v[c];
          }
        }
      }
    }
  };
  long t = blockIdx.x;
  if (t < ntiles) load_tile(t);
  __syncthreads();  // bases visible
  const int r = lane & 15, hh = lane >> 4;
  float* wx = sx + (long)(w * 16) * g.S;  // this wave's 16 rows
  const float* b1p = sb + (long)(hh * 16 + r) * NT8;  // + q · 64 · NT8 for k step q
  const float* b2p = b1p + BHALF;
  for (; t < ntiles; t += gridDim.x) {
    store_tile();
    __syncthreads();
    const long tn = t + gridDim.x;
    if (tn < ntiles && !(diag & 2)) load_tile(tn);  // in flight under the MFMAs below
    // A fragments of both half GEMMs, k index kk = 4q + hh of the half
    float a1[KS], a2[KS];
    const float* xr = wx + r * g.S;
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      const int kk = 4 * q + hh;
      if (!INV) {  // u / v butterflies of the row
        const float lo = kk < g.h ? xr[kk] : 0.f;
        const float hi = kk < g.ho ? xr[n - 1 - kk] : 0.f;
        a1[q] = lo + hi;  // (mid of an odd row: hi = 0)
        a2[q] = kk < g.ho ? lo - hi : 0.f;
      } else {  // even / odd coefficients of the row
        a1[q] = kk < g.h ? xr[2 * kk] : 0.f;
        a2[q] = kk < g.ho ? xr[2 * kk + 1] : 0.f;
      }
    }
    f32x4 c1[NT], c2[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      c1[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      c2[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    auto ldb = [&](const float* p, float (&b)[NT8]) {
#pragma unroll
      for (int c = 0; c + 4 <= NT8; c += 4) {
        const float4 v = *reinterpret_cast<const float4*>(p + c);
        b[c] = v.x;
        b[c + 1] = v.y;
        b[c + 2] = v.z;
        b[c + 3] = v.w;
      }
      if constexpr (NT8 % 4 == 2) {
        const float2 v = *reinterpret_cast<const float2*>(p + NT8 - 2);
        b[NT8 - 2] = v.x;
        b[NT8 - 1] = v.y;
      }
    };
    float bq1[2][NT8], bq2[2][NT8];
    ldb(b1p, bq1[0]);
    ldb(b2p, bq2[0]);
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      if (diag & 1) {  // diagnostics: no MFMAs (memory pipeline alone)
        c1[0][0] += a1[q];
        c2[0][0] += a2[q];
        continue;
      }
      if (q + 1 < KS) {
        ldb(b1p + (long)(q + 1) * 64 * NT8, bq1[(q + 1) & 1]);
        ldb(b2p + (long)(q + 1) * 64 * NT8, bq2[(q + 1) & 1]);
      }
#pragma unroll
      for (int c = 0; c < NT; ++c) c1[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[q], bq1[q & 1][c], c1[c], 0, 0, 0);
#pragma unroll
      for (int c = 0; c < NT; ++c) c2[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[q], bq2[q & 1][c], c2[c], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * ((NT8 + 3) / 4), 0);  // next step's DS reads
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * NT, 0);               // this step's MFMAs
    }
    // C: col = lane & 15 (output index within the tile), row = 4·(lane >> 4) + reg → the wave's
    // LDS rows (interleaved / butterflied into natural order), then contiguous out
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      const int o = 16 * c + r;  // k' (forward) or i (inverse)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float* yr = wx + (4 * hh + q) * g.S;
        if (!INV) {
          if (o < g.h) yr[2 * o] = c1[c][q];
          if (o < g.ho) yr[2 * o + 1] = c2[c][q];
        } else {
          if (o < g.h) yr[o] = c1[c][q] + c2[c][q];
          if (o < g.ho) yr[n - 1 - o] = c1[c][q] - c2[c][q];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    const long row0 = t * DCT_ROWS + w * 16;
    const long nr = rows - row0 < 16 ? rows - row0 : 16;
    if (nr > 0 && !(diag & 4)) {
      const int m = (int)nr * n;  // this wave's rows: one contiguous range of Y
      float* yo = Y + row0 * (long)n;
      for (int e = lane * 4; e < m; e += 256) {
        if (VEC) {
          const int rr = rowof(e);
          *reinterpret_cast<float4*>(yo + e) = *reinterpret_cast<const float4*>(wx + rr * g.S + (e - rr * n));
        } else {
          for (int c = 0; c < 4; ++c) {
            const int ee = e + c;
            const int rr = rowof(ee);
            if (ee < m) yo[ee] = wx[rr * g.S + (ee - rr * n)];
          }
        }
      }
    }
    __syncthreads();  // every wave done with the tile before the next one lands
  }
}

// fp64 (parity mode: the reference computes in double, DCT.java:103-123): the same even/odd
// butterfly and basis layout on v_mfma_f64_16x16x4_f64 — one double per lane per A / B fragment,
// four per lane of each 16 × 16 accumulator (row 4·q + (lane >> 4), column lane & 15: unlike the
// f32 16x16x4 form, measured by tests/test_dct_gpu.py). Simpler
// than the f32 kernel (no tile prefetch under the MFMAs): fp64 rows are the exact-parity path.
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int KS, bool INV>
__global__ __launch_bounds__(DCT_THREADS) void dct_rows_f64_kernel(const double* __restrict__ X, long rows, int n,
                                                                   const double* __restrict__ basis,
                                                                   double* __restrict__ Y) {
  constexpr int NT = (KS + 3) / 4;
  constexpr int NT8 = (NT + 1) / 2 * 2;
  constexpr int BHALF = KS * 64 * NT8;  // doubles of one half basis
  extern __shared__ __align__(16) double smd[];
  const DctGeom g = dct_geom(n);
  double* sb = smd;              // half bases [2][KS][4][16][NT8]
  double* sx = smd + 2 * BHALF;  // tile [64][S]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < 2 * BHALF; i += DCT_THREADS) sb[i] = basis[i];
  const long ntiles = (rows + DCT_ROWS - 1) / DCT_ROWS;
  const int r = lane & 15, hh = lane >> 4;
  double* wx = sx + (long)(w * 16) * g.S;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long row0 = t * DCT_ROWS;
    const int nrows = rows - row0 < DCT_ROWS ? (int)(rows - row0) : DCT_ROWS;
    __syncthreads();  // (bases in; the previous tile's rows written out)
    for (int e = tid; e < DCT_ROWS * n; e += DCT_THREADS) {
      const int rr = e / n, cc = e - rr * n;
      sx[rr * g.S + cc] = rr < nrows ? X[(row0 + rr) * n + cc] : 0.0;
    }
    __syncthreads();
    double a1[KS], a2[KS];
    const double* xr = wx + r * g.S;
#pragma unroll
    for (int q = 0; q < KS; ++q) {
      const int kk = 4 * q + hh;
      if (!INV) {
        const double lo = kk < g.h ? xr[kk] : 0.0;
        const double hi = kk < g.ho ? xr[n - 1 - kk] : 0.0;
        a1[q] = lo + hi;
        a2[q] = kk < g.ho ? lo - hi : 0.0;
      } else {
        a1[q] = kk < g.h ? xr[2 * kk] : 0.0;
        a2[q] = kk < g.ho ? xr[2 * kk + 1] : 0.0;
      }
    }
    f64x4 c1[NT], c2[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      c1[c] = f64x4{0.0, 0.0, 0.0, 0.0};
      c2[c] = f64x4{0.0, 0.0, 0.0, 0.0};
    }
    const double* b1p = sb + (long)(hh * 16 + r) * NT8;
#pragma unroll
    for (int q = 0; q < KS; ++q) {
#pragma unroll
      for (int c = 0; c < NT; ++c) {
        c1[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[q], b1p[(long)q * 64 * NT8 + c], c1[c], 0, 0, 0);
        c2[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[q], b1p[BHALF + (long)q * 64 * NT8 + c], c2[c], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < NT; ++c) {
      const int o = 16 * c + r;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double* yr = wx + (4 * q + hh) * g.S;  // (the f64 accumulator: row 4·q + (lane >> 4))
        if (!INV) {
          if (o < g.h) yr[2 * o] = c1[c][q];
          if (o < g.ho) yr[2 * o + 1] = c2[c][q];
        } else {
          if (o < g.h) yr[o] = c1[c][q] + c2[c][q];
          if (o < g.ho) yr[n - 1 - o] = c1[c][q] - c2[c][q];
        }
      }
    }
    __syncthreads();
    for (int e = tid; e < nrows * n; e += DCT_THREADS) {
      const int rr = e / n, cc = e - rr * n;
      Y[(row0 + rr) * n + cc] = sx[rr * g.S + cc];
    }
  }
}

int g_dct_diag = 0;  // diagnostics (fmlx_dct_set_diag): 1 no MFMAs, 2 no tile loads, 4 no stores
int g_dct_per_cu = 0;  // blocks per CU (0: as many as the LDS allows, at most 4)

}  // namespace

FMLX_API void fmlx_dct_set_diag(int diag, int per_cu) {
  g_dct_diag = diag;
  g_dct_per_cu = per_cu;
}

// Basis layout the kernel expects: float [2][KP/4][4][16][nt8] — half p (0: even rows of M, 1:
// odd rows), element [p][q][hh][r][c] = B_p[4q + hh][16c + r] with B_p[kk][o] = M[2o + p][kk]
// (forward) or M[2kk + p][o] (inverse), zero outside the half's range; KP and nt8 out.
FMLX_API int fmlx_dct_basis_shape(int n, int* kp, int* nt8) {
  if (n < 1 || n > DCT_MAXN) return -1;
  const DctGeom g = dct_geom(n);
  *kp = g.KP;
  *nt8 = g.NT8;
  return 0;
}

// Y[rows][n] = DCT-II (inverse = 0) or DCT-III (inverse = 1) of X[rows][n] (f32, contiguous
// rows, 16-byte aligned); basis as fmlx_dct_basis_shape for the same direction.
FMLX_API int fmlx_dct_rows(const float* X, long rows, int n, const float* basis, float* Y, int inverse, int num_cu,
                           void* stream) {
  if (n < 1 || n > DCT_MAXN) return -1;
  if (rows <= 0) return 0;
  if (((uintptr_t)X | (uintptr_t)Y) & 15) return -2;
  const DctGeom g = dct_geom(n);
  const size_t lds = ((size_t)2 * g.KP * 16 * g.NT8 + (size_t)DCT_ROWS * g.S) * sizeof(float);
  const long ntiles = (rows + DCT_ROWS - 1) / DCT_ROWS;
  // two blocks per CU: measured at 10M × 100, 1.77 ms vs 2.33 with the three the LDS allows and
  // 2.49 with one (the extra block's loads and stores contend more than they hide;
  // profiles/r5/dct_pipeline_ab.jsonl)
  int per_cu = (int)((160 * 1024) / lds);
  if (per_cu > 2) per_cu = 2;
  if (g_dct_per_cu > 0 && g_dct_per_cu < per_cu) per_cu = g_dct_per_cu;
  if (per_cu < 1) per_cu = 1;
  long grid = (long)(num_cu > 0 ? num_cu : 256) * per_cu;
  if (grid > ntiles) grid = ntiles;
  const bool vec = (n % 4) == 0;
  hipStream_t s = (hipStream_t)stream;
#define FMLX_DCT_LAUNCH(KSV, IV, VV)                                                                           \
  hipLaunchKernelGGL((dct_rows_kernel<KSV, IV, VV>), dim3((unsigned)grid), dim3(DCT_THREADS), lds, s, X, rows, n, \
                     basis, Y, g_dct_diag)
#define FMLX_DCT_CASE(KSV)                              \
  case KSV:                                             \
    if (inverse) {                                      \
      if (vec) FMLX_DCT_LAUNCH(KSV, true, true);        \
      else FMLX_DCT_LAUNCH(KSV, true, false);           \
    } else {                                            \
      if (vec) FMLX_DCT_LAUNCH(KSV, false, true);       \
      else FMLX_DCT_LAUNCH(KSV, false, false);          \
    }                                                   \
    break;
  switch (g.KP / 4) {
    FMLX_DCT_CASE(1)
    FMLX_DCT_CASE(2)
    FMLX_DCT_CASE(3)
    FMLX_DCT_CASE(4)
    FMLX_DCT_CASE(5)
    FMLX_DCT_CASE(6)
    FMLX_DCT_CASE(7)
    FMLX_DCT_CASE(8)
    FMLX_DCT_CASE(9)
    FMLX_DCT_CASE(10)
    FMLX_DCT_CASE(11)
    FMLX_DCT_CASE(12)
    FMLX_DCT_CASE(13)
    FMLX_DCT_CASE(14)
    FMLX_DCT_CASE(15)
    FMLX_DCT_CASE(16)
    default:
      return -3;
  }
#undef FMLX_DCT_CASE
#undef FMLX_DCT_LAUNCH
  return (int)hipGetLastError();
}

// fp64 rows (parity mode): Y = DCT-II / DCT-III of X, both double, basis as fmlx_dct_basis_shape
// (in double)
FMLX_API int fmlx_dct_rows_f64(const double* X, long rows, int n, const double* basis, double* Y, int inverse,
                               int num_cu, void* stream) {
  if (n < 1 || n > DCT_MAXN) return -1;
  if (rows <= 0) return 0;
  const DctGeom g = dct_geom(n);
  const size_t lds = ((size_t)2 * g.KP * 16 * g.NT8 + (size_t)DCT_ROWS * g.S) * sizeof(double);
  if (lds > 160 * 1024) return -4;
  const long ntiles = (rows + DCT_ROWS - 1) / DCT_ROWS;
  long grid = (long)(num_cu > 0 ? num_cu : 256) * ((160 * 1024) / lds >= 2 ? 2 : 1);
  if (grid > ntiles) grid = ntiles;
  hipStream_t s = (hipStream_t)stream;
#define FMLX_DCT64(KSV)                                                                                        \
  case KSV:                                                                                                    \
    if (inverse)                                                                                               \
      hipLaunchKernelGGL((dct_rows_f64_kernel<KSV, true>), dim3((unsigned)grid), dim3(DCT_THREADS), lds, s, X, \
                         rows, n, basis, Y);                                                                   \
    else                                                                                                       \
      hipLaunchKernelGGL((dct_rows_f64_kernel<KSV, false>), dim3((unsigned)grid), dim3(DCT_THREADS), lds, s, X, \
                         rows, n, basis, Y);                                                                   \
    break;
  switch (g.KP / 4) {
    FMLX_DCT64(1)
    FMLX_DCT64(2)
    FMLX_DCT64(3)
    FMLX_DCT64(4)
    FMLX_DCT64(5)
    FMLX_DCT64(6)
    FMLX_DCT64(7)
    FMLX_DCT64(8)
    FMLX_DCT64(9)
    FMLX_DCT64(10)
    FMLX_DCT64(11)
    FMLX_DCT64(12)
    FMLX_DCT64(13)
    FMLX_DCT64(14)
    FMLX_DCT64(15)
    FMLX_DCT64(16)
    default:
      return -3;
  }
#undef FMLX_DCT64
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
