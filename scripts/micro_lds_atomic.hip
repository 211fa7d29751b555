// LDS accumulate throughput on gfx950: 6.4M (key, value) pairs (random keys in a 4096-slot slab)
// summed into LDS by 256 blocks of 1024 threads, by mode:
//   0 ds_add_f32 (atomicAdd float, no return)   1 ds_add_u32 (int, no return)
//   2 ds_add_rtn_u32 (int, with return)          3 plain ds_write (no accumulate: the floor)
//   4 ds_add_f32 with the keys sorted inside each wave's 64 (fewer bank/address collisions)
// Prints one JSON line per mode: µs per launch (events over 50 launches).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

constexpr int NT = 1024, SLAB = 4096;

template <int MODE>
__global__ __launch_bounds__(NT) void k(const uint16_t* __restrict__ key, const float* __restrict__ val, long n,
                                        float* __restrict__ out) {
  __shared__ float slab[SLAB];
  for (int i = threadIdx.x; i < SLAB; i += NT) slab[i] = 0.f;
  __syncthreads();
  const long per = (n + gridDim.x - 1) / gridDim.x;
  const long b0 = blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
  int acc = 0;
  for (long q0 = b0; q0 < b1; q0 += 8 * NT) {
    uint16_t kk[8];
    float vv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long q = q0 + threadIdx.x + u * NT;
      const long qq = q < b1 ? q : b0;
      kk[u] = key[qq] & (SLAB - 1);
      vv[u] = val[qq];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (q0 + threadIdx.x + u * NT >= b1) continue;
      if (MODE == 0 || MODE == 4) atomicAdd(&slab[kk[u]], vv[u]);
      if (MODE == 1) atomicAdd(reinterpret_cast<unsigned*>(&slab[kk[u]]), 1u);
      if (MODE == 2) acc += atomicAdd(reinterpret_cast<int*>(&slab[kk[u]]), 1);
      if (MODE == 3) slab[kk[u]] = vv[u];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < SLAB; i += NT) out[(long)blockIdx.x * SLAB + i] = slab[i] + (float)acc;
}

template <int MODE>
float run(const uint16_t* key, const float* val, long n, float* out) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(NT), 0, 0, key, val, n, out);
  (void)hipEventRecord(a);
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(NT), 0, 0, key, val, n, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / 50;
}

int main() {
  const long n = 6400000;
  std::vector<uint16_t> hk(n), hs(n);
  std::vector<float> hv(n);
  std::mt19937 g(1);
  for (long i = 0; i < n; ++i) {
    hk[i] = g() & (SLAB - 1);
    hv[i] = (g() & 1023) / 1024.f;
  }
  hs = hk;
  for (long i = 0; i + 64 <= n; i += 64) std::sort(hs.begin() + i, hs.begin() + i + 64);
  uint16_t *dk, *ds;
  float *dv, *out;
  (void)hipMalloc(&dk, n * 2);
  (void)hipMalloc(&ds, n * 2);
  (void)hipMalloc(&dv, n * 4);
  (void)hipMalloc(&out, 256L * SLAB * 4);
  (void)hipMemcpy(dk, hk.data(), n * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, hs.data(), n * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dv, hv.data(), n * 4, hipMemcpyHostToDevice);
  printf("{\"mode\": \"ds_add_f32\", \"us\": %.2f}\n", run<0>(dk, dv, n, out));
  printf("{\"mode\": \"ds_add_u32\", \"us\": %.2f}\n", run<1>(dk, dv, n, out));
  printf("{\"mode\": \"ds_add_rtn_u32\", \"us\": %.2f}\n", run<2>(dk, dv, n, out));
  printf("{\"mode\": \"ds_write\", \"us\": %.2f}\n", run<3>(dk, dv, n, out));
  printf("{\"mode\": \"ds_add_f32_wave_sorted\", \"us\": %.2f}\n", run<4>(ds, dv, n, out));
  (void)hipDeviceSynchronize();
  return 0;
}
