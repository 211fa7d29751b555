// Online (unbounded-stream) training kernels: FTRL local gradients / update and the OnlineKMeans
// decayed local update + weighted global merge (SURVEY §2.1 K10–K12).
//
// Reference: LIB/classification/logisticregression/OnlineLogisticRegression.java:331-383
// (CalculateLocalGradient: dense and sparse branches), :271-301 (UpdateModel, FTRL-proximal),
// LIB/clustering/kmeans/OnlineKMeans.java:292-321 (ModelDataLocalUpdater), :188-211
// (ModelDataGlobalReducer).
//
// MI355X design. Every global mini-batch is ONE all-reduce of a fixed-size payload whose last
// element is a "batch present" flag (1 per rank that had a local batch): the update kernels run
// predicated on ALL ranks having contributed (flag sum == world), so the host never needs a
// separate end-of-stream collective and can queue round r+1 before it reads round r's flag
// (models/online.py, VersionedModelStream). Predicated-off rounds change nothing and do not
// advance the device model version.
#include "common.h"

namespace {

__device__ __forceinline__ bool all_present(const float* flag, int world) { return *flag > (float)world - 0.5f; }
__device__ __forceinline__ bool all_present(const double* flag, int world) { return *flag > (double)world - 0.5; }

// ---- FTRL: sparse local gradient (the reference's sparse branch). One wave per CSR row: the
// gathered dot is a wave sum, then every lane scatter-adds (p − y)·x_j into grad[j] and the row
// weight into wsum[j] (float atomics: order-dependent last bits). payload = [grad d | wsum d | flag],
// zeroed by the launcher (one memset node) before this kernel.
template <typename A>
__global__ __launch_bounds__(256) void ftrl_grad_csr_kernel(const long* __restrict__ indptr,
                                                            const int* __restrict__ idx, const A* __restrict__ val,
                                                            const A* __restrict__ y, const A* __restrict__ wt,
                                                            const A* __restrict__ coef, long n, long d,
                                                            A* __restrict__ payload) {
  const int lane = threadIdx.x & 63;
  const long W = (long)gridDim.x * (blockDim.x >> 6);
  A* grad = payload;
  A* wsum = payload + d;
  for (long r = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += W) {
    const long p0 = indptr[r], p1 = indptr[r + 1];
    A dot = 0;
    for (long p = p0 + lane; p < p1; p += 64) dot += val[p] * coef[idx[p]];
    dot = wave_sum(dot);
    const A m = (A)1 / ((A)1 + exp(-dot)) - y[r];
    const A w = wt ? wt[r] : (A)1;
    for (long p = p0 + lane; p < p1; p += 64) {
      const int j = idx[p];
      atomicAdd(grad + j, m * val[p]);
      atomicAdd(wsum + j, w);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) payload[2 * d] = (A)1;
}

// ---- FTRL-proximal update (UpdateModel), predicated on the batch flag. wsum_stride 0: one
// weight sum for every coordinate (the dense branch's Σ 1.0 per row).
template <typename A>
__global__ __launch_bounds__(256) void ftrl_update_kernel(const A* __restrict__ grad, const A* __restrict__ wsum,
                                                          long wsum_stride, const A* __restrict__ flag, int world,
                                                          A* __restrict__ coef, A* __restrict__ z, A* __restrict__ nn,
                                                          long* __restrict__ version, long d, A alpha, A beta, A l1,
                                                          A l2) {
  if (flag && !all_present(flag, world)) return;
  if (version && blockIdx.x == 0 && threadIdx.x == 0) *version += 1;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < d; i += (long)gridDim.x * blockDim.x) {
    A g = grad[i];
    const A ws = wsum[i * wsum_stride];
    if (ws != (A)0) g = g / ws;
    const A n0 = nn[i];
    const A sigma = (sqrt(n0 + g * g) - sqrt(n0)) / alpha;
    const A zi = z[i] + g - sigma * coef[i];
    const A ni = n0 + g * g;
    z[i] = zi;
    nn[i] = ni;
    coef[i] = fabs(zi) <= l1 ? (A)0 : ((zi < (A)0 ? (A)-1 : (A)1) * l1 - zi) / ((beta + sqrt(ni)) / alpha + l2);
  }
}

// ---- OnlineKMeans local update (ModelDataLocalUpdater) → the merge payload. red = this rank's
// [k·D sums | k counts] of the batch; one block per cluster:
//   W' = W·decay/P; if count > 0: W' += count, λ = count / W', c' = (1 − λ)·c + (λ / count)·sum
// and the payload row is [c'·W' | W'] so that the all-reduce + division is the weighted average
// of ModelDataGlobalReducer. The block of cluster 0 writes the flag.
template <typename A>
__global__ __launch_bounds__(256) void okm_local_update_kernel(const A* __restrict__ red, const A* __restrict__ C,
                                                               const A* __restrict__ Wt, int k, int D, A decay_over_p,
                                                               A* __restrict__ out) {
  const int j = blockIdx.x;
  const A cnt = red[(long)k * D + j];
  A w = Wt[j] * decay_over_p;
  A lam = 0, scale = 0;
  if (cnt > (A)0) {
    w += cnt;
    lam = cnt / w;
    scale = lam / cnt;
  }
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    const A cj = C[(long)j * D + c];
    const A v = cnt > (A)0 ? cj * ((A)1 - lam) + red[(long)j * D + c] * scale : cj;
    out[(long)j * D + c] = v * w;
  }
  if (threadIdx.x == 0) {
    out[(long)k * D + j] = w;
    if (j == 0) out[(long)k * D + k] = (A)1;
  }
}

// ---- global merge, predicated: C = Σ c·w / max(Σ w, 1e-16), W = Σ w, plus the bf16 (−2-scaled)
// centroid image and norms the next batch's MFMA assign consumes (as kmeans_finalize).
template <typename A>
__global__ __launch_bounds__(256) void okm_merge_kernel(const A* __restrict__ m, int k, int D, int world,
                                                        A* __restrict__ C, A* __restrict__ Wt,
                                                        bf16_t* __restrict__ Cb, int DP, float* __restrict__ cnorm_bf16,
                                                        A* __restrict__ cnorm_acc, long* __restrict__ version) {
  if (!all_present(m + (long)k * D + k, world)) return;
  const int j = blockIdx.x;
  if (version && j == 0 && threadIdx.x == 0) *version += 1;
  const A w = m[(long)k * D + j];
  const A inv = (A)1 / (w > (A)1e-16 ? w : (A)1e-16);
  float nb = 0.f;
  A na = 0;
  for (int c = threadIdx.x; c < DP; c += blockDim.x) {
    const A v = c < D ? m[(long)j * D + c] * inv : (A)0;
    if (c < D) C[(long)j * D + c] = v;
    if (Cb) {
      const bf16_t bv = f32_to_bf16((float)v);
      const float fb = bf16_to_f32(bv);
      Cb[(long)j * DP + c] = f32_to_bf16(-2.f * fb);
      nb += fb * fb;
    }
    na += v * v;
  }
  __shared__ float smb[256];
  __shared__ A sma[256];
  smb[threadIdx.x] = nb;
  sma[threadIdx.x] = na;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tb = 0.f;
    A ta = 0;
    for (int i = 0; i < (int)blockDim.x; ++i) { tb += smb[i]; ta += sma[i]; }
    if (cnorm_bf16) cnorm_bf16[j] = tb;
    if (cnorm_acc) cnorm_acc[j] = sqrt(ta);
    Wt[j] = w;
  }
}

int grid_for(long work, int per_block, int cap) {
  long b = (work + per_block - 1) / per_block;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

FMLX_API int fmlx_ftrl_grad_csr(int acc_f64, const long* indptr, const int* idx, const void* val, const void* y,
                                const void* wt, const void* coef, long n, long d, void* payload, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const size_t bytes = (size_t)(2 * d + 1) * (acc_f64 ? 8 : 4);
  hipError_t e = hipMemsetAsync(payload, 0, bytes, s);
  if (e != hipSuccess) return (int)e;
  const int blocks = grid_for(n, 4, 16384);
  if (acc_f64)
    hipLaunchKernelGGL(ftrl_grad_csr_kernel<double>, dim3(blocks), dim3(256), 0, s, indptr, idx, (const double*)val,
                       (const double*)y, (const double*)wt, (const double*)coef, n, d, (double*)payload);
  else
    hipLaunchKernelGGL(ftrl_grad_csr_kernel<float>, dim3(blocks), dim3(256), 0, s, indptr, idx, (const float*)val,
                       (const float*)y, (const float*)wt, (const float*)coef, n, d, (float*)payload);
  return (int)hipGetLastError();
}

// flag: the payload's batch-present slot (null = unconditional); version: int64 device counter
// advanced by every update that runs (may be null).
FMLX_API int fmlx_ftrl_update2(int acc_f64, const void* grad, const void* wsum, long wsum_stride, const void* flag,
                               int world, void* coef, void* z, void* n, long* version, long d, double alpha, double beta,
                               double l1, double l2, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int blocks = grid_for(d, 256, 2048);
  if (acc_f64)
    hipLaunchKernelGGL(ftrl_update_kernel<double>, dim3(blocks), dim3(256), 0, s, (const double*)grad,
                       (const double*)wsum, wsum_stride, (const double*)flag, world, (double*)coef, (double*)z,
                       (double*)n, version, d, alpha, beta, l1, l2);
  else
    hipLaunchKernelGGL(ftrl_update_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)grad,
                       (const float*)wsum, wsum_stride, (const float*)flag, world, (float*)coef, (float*)z,
                       (float*)n, version, d, (float)alpha, (float)beta, (float)l1, (float)l2);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_okm_local_update(int acc_f64, const void* red, const void* C, const void* W, int k, int D,
                                   double decay_over_p, void* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (acc_f64)
    hipLaunchKernelGGL(okm_local_update_kernel<double>, dim3(k), dim3(256), 0, s, (const double*)red,
                       (const double*)C, (const double*)W, k, D, decay_over_p, (double*)out);
  else
    hipLaunchKernelGGL(okm_local_update_kernel<float>, dim3(k), dim3(256), 0, s, (const float*)red, (const float*)C,
                       (const float*)W, k, D, (float)decay_over_p, (float*)out);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_okm_merge(int acc_f64, const void* m, int k, int D, int world, void* C, void* W, void* Cb, int DP,
                            float* cnorm_bf16, void* cnorm_acc, long* version, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (acc_f64)
    hipLaunchKernelGGL(okm_merge_kernel<double>, dim3(k), dim3(256), 0, s, (const double*)m, k, D, world, (double*)C,
                       (double*)W, (bf16_t*)Cb, DP, cnorm_bf16, (double*)cnorm_acc, version);
  else
    hipLaunchKernelGGL(okm_merge_kernel<float>, dim3(k), dim3(256), 0, s, (const float*)m, k, D, world, (float*)C,
                       (float*)W, (bf16_t*)Cb, DP, cnorm_bf16, (float*)cnorm_acc, version);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
