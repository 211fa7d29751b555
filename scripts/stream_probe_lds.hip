// Does streaming the SGD round's rows through LDS-DMA (global_load_lds_dwordx4 into a per-wave
// LDS ring, counted vmcnt waits, ds_read_b128 back) read HBM faster than 16-B non-temporal
// register loads? A/B in one process, hipEvent timing: 100k-row × 2000-B bf16 batches (200 MB)
// rotating through a 4 GB buffer, one wave per row, rows interleaved over the grid's waves, a
// trivial consumer. Prints µs per 200 MB batch and GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/sp_lds scripts/stream_probe_lds.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// register path: U rows per step, two steps in flight (the round kernel's shape)
template <int U, int WPB>
__global__ __launch_bounds__(WPB * 64) void rows_reg(const u32x4* __restrict__ x, long rows, float* out) {
  const int lane = threadIdx.x & 63;
  const long W = (long)gridDim.x * WPB;
  const long gw = (long)blockIdx.x * WPB + (threadIdx.x >> 6);
  const int c0 = lane, c1 = lane + 64 < 125 ? lane + 64 : 124;
  float s = 0.f;
  u32x4 a[U][2], b[U][2];
  auto load = [&](long r0, u32x4 (&d)[U][2]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long r = r0 + u * W;
      r = r < rows ? r : rows - 1;
      d[u][0] = __builtin_nontemporal_load(x + r * 125 + c0);
      d[u][1] = __builtin_nontemporal_load(x + r * 125 + c1);
    }
  };
  auto use = [&](u32x4 (&d)[U][2]) {
#pragma unroll
    for (int u = 0; u < U; ++u) s += __uint_as_float(d[u][0].x) + __uint_as_float(d[u][1].w);
  };
  const long step = (long)U * W;
  long r = gw;
  load(r, a);
  while (true) {
    load(r + step, b);
    use(a);
    r += step;
    if (r >= rows) break;
    load(r + step, a);
    use(b);
    r += step;
    if (r >= rows) break;
  }
  if (s == 1234.5f) out[0] = s;
}

// LDS-DMA path: each wave owns S slots of 2 KiB; a row = two 1-KiB global_load_lds_dwordx4
// (lanes of the second past the row's 125 chunks re-read its last chunk), S − 1 rows in flight
template <int S, int WPB, bool NT>
__global__ __launch_bounds__(WPB * 64) void rows_glds(const u32x4* __restrict__ x, long rows, float* out) {
  __shared__ __align__(16) u32x4 ring[WPB][S][128];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long W = (long)gridDim.x * WPB;
  const long gw = (long)blockIdx.x * WPB + wave;
  const int c0 = lane, c1 = lane + 64 < 125 ? lane + 64 : 124;
  auto issue = [&](long r, int slot) {
    r = r < rows ? r : rows - 1;
    const u32x4* p0 = x + r * 125 + c0;
    const u32x4* p1 = x + r * 125 + c1;
    const unsigned d0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)&ring[wave][slot][0]);
    const unsigned d1 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)&ring[wave][slot][64]);
    if constexpr (NT) {
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(p0), "s"(d0) : "memory");
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(p1), "s"(d1) : "memory");
    } else {
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(p0), "s"(d0) : "memory");
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(p1), "s"(d1) : "memory");
    }
  };
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < S - 1; ++k) issue(gw + k * W, k);
  int slot = 0;
  for (long r = gw; r < rows; r += W) {
    int nxt = slot + S - 1;
    nxt = nxt >= S ? nxt - S : nxt;
    issue(r + (long)(S - 1) * W, nxt);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (S - 1)) : "memory");  // row r's two loads landed
    const u32x4 v0 = ring[wave][slot][lane];
    const u32x4 v1 = ring[wave][slot][64 + lane];
    s += __uint_as_float(v0.x) + __uint_as_float(v1.w);
    slot = slot + 1 == S ? 0 : slot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (s == 1234.5f) out[0] = s;
}

int main() {
  const long rows_total = 2000000, batch = 100000;
  const size_t bytes = (size_t)rows_total * 2000;
  u32x4* x;
  float* out;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(x, 0x3c, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int P = (int)(rows_total / batch);
  const double gb = batch * 2000.0 / 1e9;
  auto run = [&](const char* name, auto launch) -> int {
    for (int i = 0; i < 20; ++i) launch(x + (size_t)(i % P) * batch * 125);
    CK(hipEventRecord(e0));
    const int iters = 200;
    for (int i = 0; i < iters; ++i) launch(x + (size_t)(i % P) * batch * 125);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    printf("%-34s %8.2f us/batch %8.0f GB/s\n", name, us, gb / (us * 1e-6));
    fflush(stdout);
    return 0;
  };
  for (int rep = 0; rep < 2; ++rep) {
    run("reg U2 512x512", [&](const u32x4* p) { rows_reg<2, 8><<<512, 512>>>(p, batch, out); });
    run("reg U4 512x512", [&](const u32x4* p) { rows_reg<4, 8><<<512, 512>>>(p, batch, out); });
    run("glds S4 512x512", [&](const u32x4* p) { rows_glds<4, 8, false><<<512, 512>>>(p, batch, out); });
    run("glds S4 512x512 nt", [&](const u32x4* p) { rows_glds<4, 8, true><<<512, 512>>>(p, batch, out); });
    run("glds S8 256x512 nt", [&](const u32x4* p) { rows_glds<8, 8, true><<<256, 512>>>(p, batch, out); });
    run("glds S4 1024x256 nt", [&](const u32x4* p) { rows_glds<4, 4, true><<<1024, 256>>>(p, batch, out); });
    run("glds S3 512x512 nt", [&](const u32x4* p) { rows_glds<3, 8, true><<<512, 512>>>(p, batch, out); });
    run("glds S5 512x512 nt", [&](const u32x4* p) { rows_glds<5, 8, true><<<512, 512>>>(p, batch, out); });
  }
  return 0;
}
