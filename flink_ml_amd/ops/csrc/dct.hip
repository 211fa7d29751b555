// DCT-II / DCT-III of every row (reference LIB/feature/dct/DCT.java:103-123,
// JTransforms DoubleDCT_1D scaled): Y = X · Bm with the orthonormal basis Bm (n ≤ 128; forward
// Bm = Mᵀ, inverse Bm = M), on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32: f32 in, f32 accumulate).
//
// Persistent blocks of 4 waves; the block keeps the zero-padded basis [KP][NPS] in LDS for its
// whole life and walks 64-row tiles of X:
//   * the tile (64 contiguous rows = one contiguous 256·n-byte range) streams in with 16-byte
//     loads into LDS rows of stride S ≡ 4 (mod 64) — the A-fragment reads below hit 64 distinct banks;
//     the loads of the NEXT tile are issued before this tile's MFMAs, so they fly under the math;
//   * each wave owns 16 rows: per 4-wide k step one A fragment (X[r][4s + h]) and, per 16-column
//     output tile, one B fragment (basis stride NPS ≡ 16 or 48 mod 64: conflict-free), one MFMA;
//   * the wave's 16 × n result goes back through its own LDS rows and out as contiguous 16-byte
//     stores (its 16 rows are one contiguous range of Y).
// Memory: one read and one write of the rows; at n = 100 the f32 MFMA work (2·n² flops per row)
// is of the same order as the HBM time, so both are kept busy by two blocks per CU.
#include "common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int DCT_THREADS = 256;
constexpr int DCT_ROWS = 64;    // rows per block tile (16 per wave)
constexpr int DCT_MAXN = 128;
constexpr int DCT_MAXT = DCT_MAXN / 16;  // 16-column output tiles
constexpr int DCT_PF = 8;       // 16-byte prefetch loads per thread per tile (64 rows × 128 cols / 256 thr / 4)

struct DctGeom {
  int n, KP, S, NT, NPS;
};

__host__ __device__ inline DctGeom dct_geom(int n) {
  DctGeom g;
  g.n = n;
  g.KP = (n + 3) / 4 * 4;
  g.S = g.KP + ((4 - g.KP % 64) % 64 + 64) % 64;  // S ≡ 4 (mod 64)
  g.NT = (n + 15) / 16;
  const int np = g.NT * 16;
  g.NPS = (np % 64 == 0 || np % 64 == 32) ? np + 16 : np;
  return g;
}

__global__ __launch_bounds__(DCT_THREADS) void dct_rows_kernel(const float* __restrict__ X, long rows, int n,
                                                               const float* __restrict__ basis,
                                                               float* __restrict__ Y) {
  extern __shared__ __align__(16) float sm[];
  const DctGeom g = dct_geom(n);
  float* sb = sm;                            // basis [KP][NPS]
  float* sx = sm + (long)g.KP * g.NPS;       // tile [64][S]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < g.KP * g.NPS; i += DCT_THREADS) sb[i] = basis[i];
  // padded k columns n … KP − 1 of the tile are zero for good (tile loads never touch them)
  for (int i = tid; i < DCT_ROWS * (g.KP - n); i += DCT_THREADS) {
    const int r = i / (g.KP - n), c = n + i % (g.KP - n);
    sx[r * g.S + c] = 0.f;
  }
  const long ntiles = (rows + DCT_ROWS - 1) / DCT_ROWS;
  const bool vec = (n % 4) == 0;
  float4 pf[DCT_PF];
  // prefetch: thread tid loads float4 number tid + q·256 of the tile's contiguous 64·n floats
  auto load_tile = [&](long t) {
    const long base = t * DCT_ROWS * (long)n;
    const long lim = (rows - t * DCT_ROWS < DCT_ROWS ? rows - t * DCT_ROWS : DCT_ROWS) * (long)n;
#pragma unroll
    for (int q = 0; q < DCT_PF; ++q) {
      const long e = (long)(tid + q * DCT_THREADS) * 4;
      if (vec) {
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
        if (vec) {  // a float4 never straddles a row: one 16-byte LDS store
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
  __syncthreads();  // basis + padding visible
  const int r = lane & 15, h = lane >> 4;
  float* wx = sx + (long)(w * 16) * g.S;  // this wave's 16 rows
  for (; t < ntiles; t += gridDim.x) {
    store_tile();
    __syncthreads();
    const long tn = t + gridDim.x;
    if (tn < ntiles) load_tile(tn);  // in flight under the MFMAs below
    f32x4 acc[DCT_MAXT];
#pragma unroll
    for (int c = 0; c < DCT_MAXT; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int ksteps = g.KP / 4;
    for (int s = 0; s < ksteps; ++s) {
      const float a = wx[r * g.S + 4 * s + h];
      const float* brow = sb + (long)(4 * s + h) * g.NPS + r;
#pragma unroll
      for (int c = 0; c < DCT_MAXT; ++c)
        if (c < g.NT) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, brow[16 * c], acc[c], 0, 0, 0);
    }
    // C: col = lane & 15, row = 4·(lane >> 4) + reg → the wave's LDS rows, then contiguous out
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < DCT_MAXT; ++c) {
      if (c < g.NT) {
        const int col = 16 * c + r;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (col < n) wx[(4 * h + q) * g.S + col] = acc[c][q];
      }
    }
    __builtin_amdgcn_wave_barrier();
    const long row0 = t * DCT_ROWS + w * 16;
    const long nr = rows - row0 < 16 ? rows - row0 : 16;
    if (nr > 0) {
      const long m = nr * n;  // this wave's rows: one contiguous range of Y
      float* yo = Y + row0 * (long)n;
      for (int e = lane * 4; e < (int)m; e += 256) {
        if (vec) {
          const int rr = rowof(e);
          *reinterpret_cast<float4*>(yo + e) = *reinterpret_cast<const float4*>(wx + rr * g.S + (e - rr * n));
        } else {
          for (int c = 0; c < 4; ++c) {
            const int ee = e + c;
            const int rr = rowof(ee);
            if (ee < (int)m) yo[ee] = wx[rr * g.S + (ee - rr * n)];
          }
        }
      }
    }
    __syncthreads();  // every wave done with the tile before the next one lands
  }
}

}  // namespace

// Padded basis layout the kernel expects: float [KP][NPS] (zeros outside [n][n]); both sizes out.
FMLX_API int fmlx_dct_basis_shape(int n, int* kp, int* nps) {
  if (n < 1 || n > DCT_MAXN) return -1;
  const DctGeom g = dct_geom(n);
  *kp = g.KP;
  *nps = g.NPS;
  return 0;
}

// Y[rows][n] = X[rows][n] · basis (f32, contiguous rows); basis as fmlx_dct_basis_shape.
FMLX_API int fmlx_dct_rows(const float* X, long rows, int n, const float* basis, float* Y, int num_cu, void* stream) {
  if (n < 1 || n > DCT_MAXN) return -1;
  if (rows <= 0) return 0;
  if (((uintptr_t)X | (uintptr_t)Y) & 15) return -2;
  const DctGeom g = dct_geom(n);
  const size_t lds = ((size_t)g.KP * g.NPS + (size_t)DCT_ROWS * g.S) * sizeof(float);
  const long ntiles = (rows + DCT_ROWS - 1) / DCT_ROWS;
  long grid = (long)(num_cu > 0 ? num_cu : 256) * 2;  // two blocks per CU
  if (grid > ntiles) grid = ntiles;
  hipLaunchKernelGGL(dct_rows_kernel, dim3((unsigned)grid), dim3(DCT_THREADS), lds, (hipStream_t)stream, X, rows, n,
                     basis, Y);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
