// Streaming ceiling of the SGD round body, per-launch vs persistent multi-round (A/B in one
// process, hipEvent timing). 100k-row × 2000-B bf16 batches (200 MB) rotating through a 4 GB
// buffer; full per-row math (packed fp32 dot + axpy, wave sum, logistic multiplier).
// persistent: ONE launch runs R batches; between batches every block adds its partial row into
// an accumulator (float atomics), draws a ticket, the last block "updates" coef (sc1 stores) and
// publishes a round counter, the others prefetch the next batch's first rows and wait on it.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float wsum_dpp(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xA, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xC, 0xF, false));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
template <typename A> __device__ __forceinline__ void st_agent(A* p, A v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename A> __device__ __forceinline__ A ld_agent(const A* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

constexpr int D = 1000, NCH = 125;

template <int U, int DEPTH>
struct Body {
  // processes this wave's rows r0, r0+W, ... < rows (rows already prefetched into ring[0] if pre)
  f2 w2[2][4], acc2[2][4];
  float ls;
  __device__ void load(const u32x4* x, long r0, long W, long rows, u32x4 (&d)[U][2], int c0, int c1) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long r = r0 + u * W;
      r = r < rows ? r : rows - 1;
      d[u][0] = __builtin_nontemporal_load(x + r * NCH + c0);
      d[u][1] = __builtin_nontemporal_load(x + r * NCH + c1);
    }
  }
  __device__ void use(u32x4 (&d)[U][2], long r0, long W, long rows) {
    f2 f[U][2][4];
    float dot[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f2 s[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const unsigned v = d[u][h][q];
          f[u][h][q] = f2{__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
          s[q & 1] = __builtin_elementwise_fma(f[u][h][q], w2[h][q], s[q & 1]);
        }
      const f2 t = s[0] + s[1];
      dot[u] = t.x + t.y;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) dot[u] = wsum_dpp(dot[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float ys = (u & 1) ? 1.f : -1.f;
      const float z = -dot[u] * ys;
      const float tt = __builtin_amdgcn_exp2f(-fabsf(z) * 1.4426950408889634f);
      const float rc = __builtin_amdgcn_rcpf(1.f + tt);
      const bool ok = r0 + u * W < rows;
      ls += ok ? fmaxf(z, 0.f) + __builtin_amdgcn_logf(1.f + tt) * 0.6931471805599453f : 0.f;
      const float m = ok ? -ys * (z > 0.f ? rc : tt * rc) : 0.f;
      const f2 m2 = {m, m};
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc2[h][q] = __builtin_elementwise_fma(m2, f[u][h][q], acc2[h][q]);
    }
  }
};

template <int U, bool PERSIST>
__global__ __launch_bounds__(512, 2) void round_probe(const u32x4* x, long batch, int P, int R, float* coef, float* acc,
                                                      int* cnt, float* out) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long W = (long)gridDim.x * 8;
  const long gw = (long)blockIdx.x * 8 + wave;
  const int c0 = lane, c1 = lane + 64 < NCH ? lane + 64 : NCH - 1;
  __shared__ float sred[8][D + 8];
  __shared__ int sflag;
  Body<U, 2> b;
  u32x4 a[U][2], bb[U][2];
  const int base = PERSIST ? ld_agent(cnt + 1) : 0;
  int e = ld_agent(cnt + 2);
  bool pre = false;
  const long step = (long)U * W;
  for (int rr = 0; rr < R; ++rr) {
    const u32x4* xb = x + (size_t)(e % P) * batch * NCH;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = h ? c1 : c0;
        b.w2[h][q] = f2{ld_agent(coef + c * 8 + 2 * q), ld_agent(coef + c * 8 + 2 * q + 1)};
        b.acc2[h][q] = f2{0.f, 0.f};
      }
    b.ls = 0.f;
    long r = gw;
    if (!pre) b.load(xb, r, W, batch, a, c0, c1);
    while (true) {
      b.load(xb, r + step, W, batch, bb, c0, c1);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      b.use(a, r, W, batch);
      r += step;
      if (r >= batch) break;
      b.load(xb, r + step, W, batch, a, c0, c1);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      b.use(bb, r, W, batch);
      r += step;
      if (r >= batch) break;
    }
    // block reduce (LDS) + float atomics + ticket
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = h ? lane + 64 : lane;
      if (c < NCH)
#pragma unroll
        for (int q = 0; q < 4; ++q) { sred[wave][c * 8 + 2 * q] = b.acc2[h][q].x; sred[wave][c * 8 + 2 * q + 1] = b.acc2[h][q].y; }
    }
    if (lane == 0) sred[wave][D] = b.ls;
    __syncthreads();
    for (int c = threadIdx.x; c < D + 1; c += 512) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) v += sred[q][c];
      atomicAdd(acc + c, v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) sflag = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
    __syncthreads();
    const bool last = sflag;
    if (last) {
      if (threadIdx.x == 0) st_agent(cnt, 0);
      for (int c = threadIdx.x; c < D; c += 512) {
        const float g = ld_agent(acc + c);
        st_agent(acc + c, 0.f);
        st_agent(coef + c, ld_agent(coef + c) * 0.999f + g * 1e-9f);
      }
      if (threadIdx.x == 0) { st_agent(acc + D, 0.f); st_agent(cnt + 2, e + 1); }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (PERSIST && threadIdx.x == 0) __hip_atomic_fetch_add(cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!PERSIST) return;
    if (rr + 1 >= R) return;
    ++e;
    const u32x4* xn = x + (size_t)(e % P) * batch * NCH;
    b.load(xn, gw, W, batch, a, c0, c1);
    pre = true;
    if (threadIdx.x == 0) {
      long it = 0;
      while (ld_agent(cnt + 1) < base + rr + 1 && ++it < (1L << 24)) __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  (void)out;
}

int main() {
  const long rows_total = 2000000, batch = 100000;
  const size_t bytes = (size_t)rows_total * 2000;
  u32x4* x;
  float *out, *coef, *acc;
  int* cnt;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&coef, 4096 * 4));
  CK(hipMalloc(&acc, 4096 * 4));
  CK(hipMalloc(&cnt, 64));
  CK(hipMemset(x, 0x3c, bytes));
  CK(hipMemset(coef, 0, 4096 * 4));
  CK(hipMemset(acc, 0, 4096 * 4));
  CK(hipMemset(cnt, 0, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int P = (int)(rows_total / batch);
  const double gb = batch * 2000.0 / 1e9;
  auto run = [&](const char* name, int per_launch, auto launch) -> int {
    for (int i = 0; i < 4; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int launches = 200 / per_launch;
    for (int i = 0; i < launches; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / (launches * per_launch);
    printf("%-36s %8.2f us/round %8.0f GB/s\n", name, us, gb / (us * 1e-6));
    fflush(stdout);
    return 0;
  };
  for (int rep = 0; rep < 2; ++rep) {
    run("per-launch U2 256x512", 1, [&] { round_probe<2, false><<<256, 512>>>(x, batch, P, 1, coef, acc, cnt, out); });
    run("per-launch U1 256x512", 1, [&] { round_probe<1, false><<<256, 512>>>(x, batch, P, 1, coef, acc, cnt, out); });
    run("per-launch U2 512x512", 1, [&] { round_probe<2, false><<<512, 512>>>(x, batch, P, 1, coef, acc, cnt, out); });
    run("persist R10 U2 256x512", 10, [&] { round_probe<2, true><<<256, 512>>>(x, batch, P, 10, coef, acc, cnt, out); });
    run("persist R10 U1 256x512", 10, [&] { round_probe<1, true><<<256, 512>>>(x, batch, P, 10, coef, acc, cnt, out); });
    run("persist R20 U2 256x512", 20, [&] { round_probe<2, true><<<256, 512>>>(x, batch, P, 20, coef, acc, cnt, out); });

    run("persist R10 U4 256x512", 10, [&] { round_probe<4, true><<<256, 512>>>(x, batch, P, 10, coef, acc, cnt, out); });
  }
  return 0;
}
