// FTRL-proximal update: reference
// LIB/classification/logisticregression/OnlineLogisticRegression.java:271-301 (UpdateModel).
// One fused elementwise pass over the model: normalise the all-reduced gradient by its
// per-coordinate weight sum, update z and n, and solve the closed-form coefficient.
#include "common.h"

namespace {
template <typename A>
__global__ __launch_bounds__(256) void ftrl_update_kernel(const A* __restrict__ grad, const A* __restrict__ wsum,
                                                          A* __restrict__ coef, A* __restrict__ z, A* __restrict__ nn,
                                                          long d, A alpha, A beta, A l1, A l2) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < d; i += (long)gridDim.x * blockDim.x) {
    A g = grad[i];
    const A ws = wsum[i];
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
}  // namespace

FMLX_API int fmlx_ftrl_update(int acc_f64, const void* grad, const void* wsum, void* coef, void* z, void* n, long d,
                              double alpha, double beta, double l1, double l2, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int blocks = (int)((d + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) return 0;
  if (acc_f64)
    hipLaunchKernelGGL(ftrl_update_kernel<double>, dim3(blocks), dim3(256), 0, s, (const double*)grad,
                       (const double*)wsum, (double*)coef, (double*)z, (double*)n, d, alpha, beta, l1, l2);
  else
    hipLaunchKernelGGL(ftrl_update_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)grad,
                       (const float*)wsum, (float*)coef, (float*)z, (float*)n, d, (float)alpha, (float)beta,
                       (float)l1, (float)l2);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
