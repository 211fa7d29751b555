// Micro-benchmark: streaming 51 MB (6.4M int32 + 6.4M fp32, the SVC batch's column-major
// entries) the way glm.hip glm_csc_tile_bwd_kernel does — each block a contiguous tile, every
// thread UU strided loads of each array in one step — against other block / tile shapes.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/bin/micro_tile_stream scripts/micro_tile_stream.hip
// One JSON line per (threads per block, entries per tile, UU, mode) with the median µs of 20 launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

// MODE 0: non-temporal loads; 1: plain loads; 2: non-temporal + every value stored to a 128 KB
// LDS slot array (one block per CU); 3: as 2 behind a two-load dependent header (the kernel's
// state word → batch offset chain)
template <int T, int UU, int MODE>
__global__ __launch_bounds__(T) void tile_stream(const int* __restrict__ er, const float* __restrict__ ev, long n,
                                                 int tile, float* __restrict__ out) {
  extern __shared__ float lds[];
  float s = 0;
  long ntiles = (n + tile - 1) / tile;
  if (MODE == 3) {  // out[1] = 0 and out[2 + 0] = ntiles written by the host: two dependent loads
    const int i = (int)out[1];
    ntiles = (long)out[2 + i];
  }
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long k0 = t * tile, k1 = k0 + tile < n ? k0 + tile : n;
    for (long kb = k0 + threadIdx.x; kb < k1; kb += (long)UU * T) {
      int xx[UU];
      float vv[UU];
#pragma unroll
      for (int u = 0; u < UU; ++u) {
        const long k = kb + (long)u * T;
        const long kk = k < k1 ? k : kb;
        if (MODE != 1) {
          xx[u] = __builtin_nontemporal_load(er + kk);
          vv[u] = __builtin_nontemporal_load(ev + kk);
        } else {
          xx[u] = er[kk];
          vv[u] = ev[kk];
        }
      }
#pragma unroll
      for (int u = 0; u < UU; ++u) {
        if (MODE >= 2) {
          const long k = kb + (long)u * T;
          if (k < k1) lds[(xx[u] + (int)(k - k0)) & 32767] = vv[u];
        } else {
          s += vv[u] * (float)xx[u];
        }
      }
    }
  }
  if (MODE >= 2) {
    __syncthreads();
    s = lds[threadIdx.x];
  }
  if (s == 12345.678f) out[0] = s;
}

template <int T, int UU, int MODE>
static float run(const int* er, const float* ev, long n, int tile, float* out) {
  const long ntiles = (n + tile - 1) / tile;
  const int blocks = (int)ntiles;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ts;
  for (int r = 0; r < 23; ++r) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((tile_stream<T, UU, MODE>), dim3(blocks), dim3(T), MODE >= 2 ? 131072 : 0, 0, er, ev, n, tile,
                       out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 3) ts.push_back(ms * 1000.f);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

#define CASE(T, UU, MODE, TILE)                                                                                \
  printf("{\"threads\": %d, \"uu\": %d, \"mode\": %d, \"tile\": %d, \"blocks\": %ld, \"us\": %.2f}\n", T, UU, \
         MODE, TILE, (n + TILE - 1) / TILE, run<T, UU, MODE>(d_er, d_ev, n, TILE, d_out));                      \
  fflush(stdout)

int main() {
  const long n = 6400000;
  int* d_er;
  float *d_ev, *d_out;
  CK(hipMalloc(&d_er, n * 4));
  CK(hipMalloc(&d_ev, n * 4));
  CK(hipMemset(d_er, 0, n * 4));
  CK(hipMemset(d_ev, 0, n * 4));
  {
    const float h[3] = {0.f, 0.f, (float)((n + 28671) / 28672)};
    CK(hipMalloc(&d_out, 16));
    CK(hipMemcpy(d_out, h, 12, hipMemcpyHostToDevice));
  }
  CASE(1024, 28, 2, 28672);
  CASE(1024, 28, 3, 28672);
  CASE(1024, 8, 2, 28672);
  CASE(1024, 28, 0, 28672);  // the tiled backward today: 224 blocks, one step
  CASE(1024, 28, 1, 28672);
  CASE(1024, 8, 0, 28672);
  CASE(1024, 4, 0, 28672);
  CASE(512, 28, 0, 14336);   // half tiles, two blocks per CU
  CASE(512, 8, 0, 14336);
  CASE(256, 28, 0, 7168);
  CASE(256, 8, 0, 7168);
  CASE(256, 4, 0, 4096);
  CASE(256, 4, 0, 1024);
  CK(hipFree(d_er));
  CK(hipFree(d_ev));
  CK(hipFree(d_out));
  return 0;
}
