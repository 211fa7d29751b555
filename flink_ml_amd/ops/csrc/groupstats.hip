// Grouped column statistics: for a row-major [n, d] matrix, per-group weighted
// column sums S[g][c] = Σ_{r: group(r)=g} w_r · x_rc together with the plain column sum Σ x_rc and
// Σ x_rc², all accumulated in fp64 in one pass over X.
//
// Used by ANOVATest (group = class index, w = 1: per-class sums; reference ANOVATest.java:120-200)
// and FValueTest (one group, w = y - ȳ: the centred cross-moment; FValueTest.java:150-260).
//
// Layout: a block owns a contiguous row range. Its 256 threads form R row-lanes × C column lanes
// (C = 64·ceil(min(d,256)/64), R = 256/C) so narrow matrices still keep every lane busy; each
// thread accumulates its column's group sums in its own LDS slots (no atomics, no bank sharing
// between threads), the R row-lanes are folded through LDS at the end, and one fp64 partial
// record [G·d | d | d] per block is combined in block order by a second kernel (deterministic).
#include "common.h"

namespace {
constexpr int kThreads = 256;
constexpr int kMaxGroups = 32;

template <typename T>
__global__ __launch_bounds__(kThreads) void group_stats_partial_kernel(
    const T* __restrict__ X, long ld, long n, int d, const int* __restrict__ gidx, int G,
    const double* __restrict__ w, long rows_per_block, int C, double* __restrict__ part) {
  __shared__ double acc[kMaxGroups * kThreads];
  __shared__ double s1[kThreads];
  __shared__ double s2[kThreads];
  const int tid = threadIdx.x;
  const int R = kThreads / C;
  const int lane_c = tid % C, lane_r = tid / C;
  const long r0 = (long)blockIdx.x * rows_per_block;
  long r1 = r0 + rows_per_block;
  if (r1 > n) r1 = n;
  const int rec = (G + 2) * d;
  double* out = part + (long)blockIdx.x * rec;
  for (int c0 = 0; c0 < d; c0 += C) {
    const int c = c0 + lane_c;
    const bool active = lane_r < R && c < d;
    for (int g = 0; g < G; ++g) acc[g * kThreads + tid] = 0.0;
    double s = 0.0, q = 0.0;
    if (active) {
      for (long r = r0 + lane_r; r < r1; r += R) {
        const double x = (double)Ld<T>::f(X[r * ld + c]);
        const int g = gidx ? gidx[r] : 0;
        const double wx = w ? w[r] * x : x;
        acc[g * kThreads + tid] += wx;
        s += x;
        q += x * x;
      }
    }
    s1[tid] = s;
    s2[tid] = q;
    __syncthreads();
    if (lane_r == 0 && c < d) {
      for (int rr = 1; rr < R; ++rr) {
        const int o = rr * C + lane_c;
        s += s1[o];
        q += s2[o];
      }
      for (int g = 0; g < G; ++g) {
        double v = acc[g * kThreads + tid];
        for (int rr = 1; rr < R; ++rr) v += acc[g * kThreads + rr * C + lane_c];
        out[(long)g * d + c] = v;
      }
      out[(long)G * d + c] = s;
      out[(long)(G + 1) * d + c] = q;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void group_stats_combine_kernel(const double* __restrict__ part, int nb, int rec,
                                                                  double* __restrict__ res) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rec) return;
  double v = 0.0;
  for (int b = 0; b < nb; ++b) v += part[(long)b * rec + i];
  res[i] = v;
}

template <typename T>
int launch(const void* X, long ld, long n, int d, const int* gidx, int G, const double* w, double* part, int nb,
           double* res, hipStream_t s) {
  int C = d < kThreads ? ((d + 63) / 64) * 64 : kThreads;
  if (C > kThreads) C = kThreads;
  const long rpb = (n + nb - 1) / nb;
  hipLaunchKernelGGL((group_stats_partial_kernel<T>), dim3(nb), dim3(kThreads), 0, s, (const T*)X, ld, n, d, gidx, G,
                     w, rpb, C, part);
  const int rec = (G + 2) * d;
  hipLaunchKernelGGL(group_stats_combine_kernel, dim3((rec + 255) / 256), dim3(256), 0, s, part, nb, rec, res);
  return (int)hipGetLastError();
}
}  // namespace

// part: scratch [nb][(G+2)*d] fp64; res: [(G+2)*d] fp64 = S[G][d] | Σx[d] | Σx²[d].
// gidx (int32 [n], values in [0, G)) and w (fp64 [n]) may be null. Requires 1 <= G <= 32.
FMLX_API int fmlx_group_colstats(int dtype, const void* X, long ld, long n, int d, const int* gidx, int G,
                                 const double* w, double* part, int nb, double* res, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (G < 1 || G > kMaxGroups || nb < 1 || d < 1) return -1;
  if (dtype == DT_F32) return launch<float>(X, ld, n, d, gidx, G, w, part, nb, res, s);
  if (dtype == DT_F64) return launch<double>(X, ld, n, d, gidx, G, w, part, nb, res, s);
  if (dtype == DT_BF16) return launch<bf16_t>(X, ld, n, d, gidx, G, w, part, nb, res, s);
  return -1;
}

FMLX_DEFINE_PRELOAD()
