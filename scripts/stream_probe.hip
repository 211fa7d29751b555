// Streaming-read ceiling probe for the SGD round body (A/B, one process, hipEvent timing).
// Reads 100k-row × 2000-B batches (the flagship bf16 batch, 200 MB) rotating through a 4 GB
// buffer, with: (a) a flat grid-stride 16-B/lane stream, (b) the round kernel's access
// pattern (one wave per 2000-B row, rows interleaved over waves, 2·U rows in flight), with a
// trivial consumer. Prints GB/s per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <bool NT>
__global__ __launch_bounds__(256) void flat_stream(const u32x4* __restrict__ x, long n16, float* out) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) {
    u32x4 v = ld16<NT>(x + i);
    s += __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) + __uint_as_float(v.w);
  }
  if (s == 1234.5f) out[0] = s;
}

// rows of 125 16-B chunks; wave per row; U rows per batch, 2 batches in flight
template <int U, bool NT, int WPB>
__global__ __launch_bounds__(WPB * 64) void row_stream(const u32x4* __restrict__ x, long rows, float* out) {
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
      d[u][0] = ld16<NT>(x + r * 125 + c0);
      d[u][1] = ld16<NT>(x + r * 125 + c1);
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

// row stream + the round's per-row math, stage by stage (LEVEL 1: dot, 2: + wave sum,
// 3: + logistic loss/multiplier, 4: + gradient axpy)
__device__ __forceinline__ float wsum_dpp(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

template <int U, int LEVEL, int WPB, int DACC = 1>
__global__ __launch_bounds__(WPB * 64) void row_math(const u32x4* x, long rows, const float* coef, float* out) {
  const int lane = threadIdx.x & 63;
  const long W = (long)gridDim.x * WPB;
  const long gw = (long)blockIdx.x * WPB + (threadIdx.x >> 6);
  const int c0 = lane, c1 = lane + 64 < 125 ? lane + 64 : 124;
  float w[16], acc[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    w[i] = coef[c0 * 8 + i];
    w[8 + i] = c1 == lane + 64 ? coef[c1 * 8 + i] : 0.f;
    acc[i] = acc[8 + i] = 0.f;
  }
  float ls = 0.f;
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
    float f[U][16];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const unsigned int v = d[u][h][q];
          f[u][h * 8 + 2 * q] = __uint_as_float(v << 16);
          f[u][h * 8 + 2 * q + 1] = __uint_as_float(v & 0xffff0000u);
        }
    float dot[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float s[DACC];
#pragma unroll
      for (int q = 0; q < DACC; ++q) s[q] = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i % DACC] += f[u][i] * w[i];
#pragma unroll
      for (int q = 1; q < DACC; ++q) s[0] += s[q];
      dot[u] = s[0];
    }
    if constexpr (LEVEL >= 2) {
#pragma unroll
      for (int u = 0; u < U; ++u) dot[u] = wsum_dpp(dot[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float m = dot[u];
      if constexpr (LEVEL >= 3) {
        const float ys = (u & 1) ? 1.f : -1.f;
        const float z = -dot[u] * ys;
        ls += z > 0.f ? z + log1pf(expf(-z)) : log1pf(expf(z));
        m = -ys / (expf(dot[u] * ys) + 1.f);
      }
      if constexpr (LEVEL >= 4) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] += m * f[u][i];
      } else {
        ls += m;
      }
    }
  };
  const long step = (long)U * W;
  long r = gw;
  load(r, a);
  while (true) {
    load(r + step, b);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    use(a);
    r += step;
    if (r >= rows) break;
    load(r + step, a);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    use(b);
    r += step;
    if (r >= rows) break;
  }
  float t = ls;
#pragma unroll
  for (int i = 0; i < 16; ++i) t += acc[i];
  if (t == 1234.5f) out[0] = t;
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
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    printf("%-34s %8.2f us/batch %8.0f GB/s\n", name, us, gb / (us * 1e-6));
    return 0;
  };
  float* coef;
  CK(hipMalloc(&coef, 4096 * 4));
  CK(hipMemset(coef, 0, 4096 * 4));
  for (int rep = 0; rep < 2; ++rep) {
    run("math L1 dot", [&](const u32x4* p) { row_math<2, 1, 8><<<512, 512>>>(p, batch, coef, out); });
    run("math L2 +dpp", [&](const u32x4* p) { row_math<2, 2, 8><<<512, 512>>>(p, batch, coef, out); });
    run("math L3 +loss", [&](const u32x4* p) { row_math<2, 3, 8><<<512, 512>>>(p, batch, coef, out); });
    run("math L4 +axpy", [&](const u32x4* p) { row_math<2, 4, 8><<<512, 512>>>(p, batch, coef, out); });
    run("math L4 U4", [&](const u32x4* p) { row_math<4, 4, 8><<<512, 512>>>(p, batch, coef, out); });
    run("math L4 1024 blocks", [&](const u32x4* p) { row_math<2, 4, 8><<<1024, 512>>>(p, batch, coef, out); });
    run("math L4 256 blocks", [&](const u32x4* p) { row_math<2, 4, 8><<<256, 512>>>(p, batch, coef, out); });
    run("math L4 256x1024", [&](const u32x4* p) { row_math<2, 4, 16><<<256, 1024>>>(p, batch, coef, out); });
    run("math L4 dacc4 512", [&](const u32x4* p) { row_math<2, 4, 8, 4><<<512, 512>>>(p, batch, coef, out); });
    run("math L4 dacc4 256", [&](const u32x4* p) { row_math<2, 4, 8, 4><<<256, 512>>>(p, batch, coef, out); });
    run("math L4 U1 512", [&](const u32x4* p) { row_math<1, 4, 8><<<512, 512>>>(p, batch, coef, out); });
    run("math L4 U1 1024", [&](const u32x4* p) { row_math<1, 4, 8><<<1024, 512>>>(p, batch, coef, out); });
  }
  for (int rep = 0; rep < 0; ++rep) {
    run("flat 2048x256", [&](const u32x4* p) { flat_stream<false><<<2048, 256>>>(p, batch * 125, out); });
    run("flat 2048x256 nt", [&](const u32x4* p) { flat_stream<true><<<2048, 256>>>(p, batch * 125, out); });
    run("flat 4096x256 nt", [&](const u32x4* p) { flat_stream<true><<<4096, 256>>>(p, batch * 125, out); });
    run("rows U2 512x512", [&](const u32x4* p) { row_stream<2, false, 8><<<512, 512>>>(p, batch, out); });
    run("rows U2 512x512 nt", [&](const u32x4* p) { row_stream<2, true, 8><<<512, 512>>>(p, batch, out); });
    run("rows U4 512x512 nt", [&](const u32x4* p) { row_stream<4, true, 8><<<512, 512>>>(p, batch, out); });
    run("rows U2 1024x512 nt", [&](const u32x4* p) { row_stream<2, true, 8><<<1024, 512>>>(p, batch, out); });
    run("rows U2 256x1024 nt", [&](const u32x4* p) { row_stream<2, true, 16><<<256, 1024>>>(p, batch, out); });
    run("rows U4 1024x512 nt", [&](const u32x4* p) { row_stream<4, true, 8><<<1024, 512>>>(p, batch, out); });
    run("rows U8 512x512 nt", [&](const u32x4* p) { row_stream<8, true, 8><<<512, 512>>>(p, batch, out); });
  }
  return 0;
}
