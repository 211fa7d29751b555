// Micro-benchmark: the cost of element-granular 4-byte gathers on one MI355X, to price the sparse
// GLM round (glm.hip glm_csr_fwd_kernel gathers coef[idx] per non-zero, glm_csc_bwd_kernel
// gathers mult[row] per non-zero; 6.4M of each per 100k x 64-nnz batch).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/micro_gather scripts/micro_gather.hip
// Cases (N = 6.4M gathers, all with the index stream read coalesced):
//   stream    — sum idx + val only (no gather)
//   seq       — table[idx] with idx = i mod T (coalesced)
//   random    — idx uniform over a table of T floats
//   sorted<k> — random idx sorted within runs of k entries (lanes of a run share cache lines)
// One JSON line per case with µs (median of 20 launches) and the line-request estimate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

// MODE: 0 plain load, 1 non-temporal load, 2 buffer load with aux bits AUX (cache policy)
template <int K, bool GATHER, int MODE = 0, int AUX = 0>
__global__ __launch_bounds__(256) void gather_kernel(const int* __restrict__ idx, const float* __restrict__ val,
                                                     const float* __restrict__ table, long n, float* __restrict__ out) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)table, (short)0, 0x7fffffff, 0x00020000);
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long T = (long)gridDim.x * blockDim.x;
  float s = 0;
  for (long b = tid; b < n; b += T * K) {
    int ii[K];
    float vv[K];
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const long j = b + t * T;
      const long jj = j < n ? j : 0;
      ii[t] = __builtin_nontemporal_load(idx + jj);
      vv[t] = __builtin_nontemporal_load(val + jj);
    }
#pragma unroll
    for (int t = 0; t < K; ++t) {
      if (GATHER && MODE == 0)
        s += vv[t] * table[ii[t]];
      else if (GATHER && MODE == 1)
        s += vv[t] * __builtin_nontemporal_load(table + ii[t]);
      else if (GATHER && MODE == 2)
        s += vv[t] * __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, ii[t] * 4, 0, AUX));
      else
        s += vv[t] * (float)ii[t];
    }
  }
  if (s == 12345.678f) out[0] = s;  // keep the work
}

template <int K, bool GATHER, int MODE = 0, int AUX = 0>
static float run(const int* idx, const float* val, const float* table, long n, float* out, int blocks) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ts;
  for (int r = 0; r < 23; ++r) {
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((gather_kernel<K, GATHER, MODE, AUX>), dim3(blocks), dim3(256), 0, 0, idx, val, table, n, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r >= 3) ts.push_back(ms * 1000.f);
  }
  std::sort(ts.begin(), ts.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
  const long n = 6400000;
  const long T = argc > 1 ? atol(argv[1]) : 1000000;  // table floats (1M = the SVC coef vector)
  std::mt19937 rng(7);
  std::uniform_int_distribution<int> U(0, (int)T - 1);
  std::vector<int> rnd(n), seq(n);
  for (long i = 0; i < n; ++i) { rnd[i] = U(rng); seq[i] = (int)(i % T); }
  int *d_idx;
  float *d_val, *d_tab, *d_out;
  CK(hipMalloc(&d_idx, n * 4));
  CK(hipMalloc(&d_val, n * 4));
  CK(hipMalloc(&d_tab, T * 4));
  CK(hipMalloc(&d_out, 4));
  CK(hipMemset(d_val, 0, n * 4));
  CK(hipMemset(d_tab, 0, T * 4));
  const int runs[] = {0, 1, 4096, 32768};
  for (int ri = 0; ri < 4; ++ri) {
    const int k = runs[ri];
    std::vector<int> h = k == 0 ? seq : rnd;
    if (k > 1)
      for (long s = 0; s < n; s += k) std::sort(h.begin() + s, h.begin() + std::min(n, s + k));
    // distinct 64-B lines touched per wave-instruction summed (an estimate of line requests)
    long lines = 0;
    for (long s = 0; s < n; s += 64) {
      long prev = -1, c = 0;
      std::vector<long> ls;
      for (long i = s; i < std::min(n, s + 64); ++i) ls.push_back(h[i] / 16);
      std::sort(ls.begin(), ls.end());
      for (long x : ls) { if (x != prev) ++c; prev = x; }
      lines += c;
    }
    CK(hipMemcpy(d_idx, h.data(), n * 4, hipMemcpyHostToDevice));
    for (int blocks : {2048, 8192}) {
      const float g1 = run<1, true>(d_idx, d_val, d_tab, n, d_out, blocks);
      const float g4 = run<4, true>(d_idx, d_val, d_tab, n, d_out, blocks);
      const float s4 = run<4, false>(d_idx, d_val, d_tab, n, d_out, blocks);
      const float nt = run<4, true, 1>(d_idx, d_val, d_tab, n, d_out, blocks);
      const float b0 = run<4, true, 2, 0>(d_idx, d_val, d_tab, n, d_out, blocks);
      const float b1 = run<4, true, 2, 1>(d_idx, d_val, d_tab, n, d_out, blocks);
      const float b2 = run<4, true, 2, 2>(d_idx, d_val, d_tab, n, d_out, blocks);
      const float b3 = run<4, true, 2, 3>(d_idx, d_val, d_tab, n, d_out, blocks);
      printf("{\"case\": \"%s\", \"run\": %d, \"table\": %ld, \"blocks\": %d, \"us_gather_k1\": %.2f, "
             "\"us_gather_k4\": %.2f, \"us_stream_k4\": %.2f, \"us_nt_k4\": %.2f, \"us_buf_aux0\": %.2f, "
             "\"us_buf_aux1\": %.2f, \"us_buf_aux2\": %.2f, \"us_buf_aux3\": %.2f, \"lines_per_wave_instr\": %.2f}\n",
             k == 0 ? "seq" : (k == 1 ? "random" : "sorted"), k, T, blocks, g1, g4, s4, nt, b0, b1, b2, b3,
             (double)lines / ((n + 63) / 64));
      fflush(stdout);
    }
  }
  CK(hipFree(d_idx));
  CK(hipFree(d_val));
  CK(hipFree(d_tab));
  CK(hipFree(d_out));
  return 0;
}
