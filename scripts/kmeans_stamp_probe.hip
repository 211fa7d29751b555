// Phase stamps of the pipelined MFMA assign (kmeans.hip kmeans_assign_bf16_pipe_kernel<8, true>)
// at the north-star shard shape, 12.5M x 128 rows vs k = 1024, random bf16 data. A diagnostic
// build: every wave's lane 0 records s_memtime at kernel entry (4), rows + first two tiles ready
// (0 → 1 after the wait), tile loop done (2) and labels stored (3), plus s_memrealtime beside each
// (slots + 8), into a buffer no other code reads. Prints where a wave's life goes
// (profiles/r4/kmeans_assign_phase_stamps.log).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kmeans_stamp_probe scripts/kmeans_stamp_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr long PROBE_MAX_WAVES = 200000;
__device__ unsigned long long g_km_st[PROBE_MAX_WAVES * 16];
#define KM_STAMP(i_)                                                                      \
  if ((threadIdx.x & 63) == 0 && (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6) < PROBE_MAX_WAVES) { \
    const long w_ = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);             \
    g_km_st[w_ * 16 + (i_)] = __builtin_amdgcn_s_memtime();                               \
    g_km_st[w_ * 16 + 8 + (i_)] = __builtin_amdgcn_s_memrealtime();                       \
  }
#include "../flink_ml_amd/ops/csrc/kmeans.hip"

__global__ void fill_bf16(unsigned short* p, long n, unsigned seed, float scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const float v = (float)(h & 0xffffff) * (1.0f / 16777216.0f) * scale;
    p[i] = (unsigned short)(__float_as_uint(v) >> 16);
  }
}
__global__ void fill_f32(float* p, long n, float base) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    p[i] = base + (float)(i % 97) * 0.01f;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(q * (v.size() - 1))];
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 12500000, D = 128;
  const int k = 1024, kpad = 1024;
  unsigned short *X, *Cb;
  float* cn;
  int* labels;
  CK(hipMalloc(&X, n * D * 2));
  CK(hipMalloc(&Cb, (long)kpad * D * 2));
  CK(hipMalloc(&cn, kpad * 4));
  CK(hipMalloc(&labels, n * 4));
  uint2* baug;
  CK(hipMalloc(&baug, kpad * 8));
  fill_bf16<<<4096, 256>>>(X, n * D, 1234u, 1.0f);
  fill_bf16<<<256, 256>>>(Cb, (long)kpad * D, 99u, -2.0f);  // the tile image is pre-scaled by -2
  fill_f32<<<4, 256>>>(cn, kpad, 40.0f);
  hipLaunchKernelGGL(kmeans_baug_kernel, dim3((kpad + 255) / 256), dim3(256), 0, 0, cn, kpad, baug);
  CK(hipDeviceSynchronize());
  const int blocks = (int)((n + 255) / 256);
  const long waves = (long)blocks * 4;
  const bool stamps = waves <= PROBE_MAX_WAVES;  // larger runs: timings only
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms = 0;
  for (int it = 0; it < 6; ++it) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((kmeans_assign_bf16_pipe_kernel<8, true>), dim3(blocks), dim3(256), 0, 0,
                       (const bf16_t*)X, D, n, (const bf16_t*)Cb, baug, kpad, labels);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("launch %d: %.3f ms\n", it, ms);
  }
  {
    std::vector<int> h(n);
    CK(hipMemcpy(h.data(), labels, n * 4, hipMemcpyDeviceToHost));
    unsigned long long cs = 1469598103934665603ull;
    for (long i = 0; i < n; ++i) cs = (cs ^ (unsigned)h[i]) * 1099511628211ull;
    std::printf("labels checksum %016llx\n", cs);
  }
  if (!stamps) return 0;
  std::vector<unsigned long long> st(waves * 16);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_km_st), waves * 16 * 8));
  std::vector<double> life, start, loop, tail, clk;
  unsigned long long t_min = ~0ull, t_max = 0;
  double busy = 0;
  for (long w = 0; w < waves; ++w) {
    const unsigned long long* s = &st[w * 16];
    life.push_back((double)(s[3] - s[4]));
    start.push_back((double)(s[1] - s[4]));
    loop.push_back((double)(s[2] - s[1]));
    tail.push_back((double)(s[3] - s[2]));
    const double rt = (double)(s[8 + 3] - s[8 + 4]);  // 100 MHz ticks
    if (rt > 0) clk.push_back((double)(s[3] - s[4]) / rt * 0.1);
    t_min = std::min(t_min, s[8 + 4]);
    t_max = std::max(t_max, s[8 + 3]);
    busy += rt;
  }
  double sl = 0, ss = 0, sp = 0, stl = 0;
  for (size_t i = 0; i < life.size(); ++i) {
    sl += life[i];
    ss += start[i];
    sp += loop[i];
    stl += tail[i];
  }
  std::printf("waves %ld, kernel span %.3f ms (realtime), last launch %.3f ms\n", waves, (t_max - t_min) * 1e-5, ms);
  std::printf("in-kernel clock (median over waves) %.3f GHz\n", pct(clk, 0.5));
  std::printf("wave life cycles: median %.0f p10 %.0f p90 %.0f\n", pct(life, 0.5), pct(life, 0.1), pct(life, 0.9));
  std::printf("  entry -> rows+tiles ready: median %.0f p10 %.0f p90 %.0f  (%.1f %% of life)\n", pct(start, 0.5),
              pct(start, 0.1), pct(start, 0.9), 100 * ss / sl);
  std::printf("  tile loop (32 tiles):      median %.0f p10 %.0f p90 %.0f  (%.1f %% of life, %.0f cyc/tile)\n",
              pct(loop, 0.5), pct(loop, 0.1), pct(loop, 0.9), 100 * sp / sl, pct(loop, 0.5) / 32);
  std::printf("  labels:                    median %.0f p10 %.0f p90 %.0f  (%.1f %% of life)\n", pct(tail, 0.5),
              pct(tail, 0.1), pct(tail, 0.9), 100 * stl / sl);
  std::printf("resident waves on average: %.1f per CU (wave-time / span / 256)\n",
              busy * 1e-5 / ((t_max - t_min) * 1e-5) / 256.0);
  return 0;
}
