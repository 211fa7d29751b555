// One-shot small-message all-reduce over xGMI peer memory (SURVEY §5 "Distributed communication
// backend", §7.4 hard part 6).
//
// Reference: the per-round feedback all-reduce of SGD (LIB/common/optimizer/SGD.java:125-132 →
// CORE/common/datastream/AllReduceImpl.java:54-302: 4096-double chunks, reduce-scatter to the
// chunk owner, all-gather back) and the KMeans/OnlineKMeans/OnlineLR gather-to-one reduces
// (LIB/clustering/kmeans/KMeans.java:166-173). Their payloads are 0.8 KB – 0.5 MB: latency
// bound, where a ring pays 2·(P−1) dependent link hops.
//
// MI355X design (layout and protocol: xgmi.h): a call is ONE kernel per rank with
// grid = ceil(n / CHUNK) independent blocks. Block b copies chunk b of my input into my
// exchange buffer, raises tag (slot, b), waits for every peer's tag (slot, b) and sums chunk b
// of ranks 0..P−1 in rank order: bit-identical results on every rank, and the P−1 pulls use
// P−1 different xGMI links at once. Block b only depends on block b of the peers, never on
// another block of its own grid, so nothing assumes co-residency. Every spin is bounded; a
// timeout sets the error word that the host checks (parallel/xgmi.py), so a lost peer cannot
// hang the GPU; a block whose wait gave up writes NaN instead of a partial sum.
#include "xgmi.h"

namespace {

template <typename A>
__global__ __launch_bounds__(xgmi::THREADS) void xar_oneshot_kernel(xgmi::Ctx x, const A* src, A* dst, long n,
                                                                   const int* __restrict__ state) {
  using namespace xgmi;
  if (state) {  // predicated like the GLM round kernels: a finished iteration skips on every rank
    const int e = state[0];
    if (state[1 + (e & 1)] == 0) return;
  }
  const int b = blockIdx.x;
  const int g = x.gen[b];
  const int slot = g & 1;
  const long base = (long)b * CHUNK;
  const long rec = DATA + ((long)slot * MAX_BLOCKS + b) * CHUNK * (long)sizeof(A);
  A* mine = at<A>(x.peers[x.rank], rec);
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const long j = (long)i * THREADS + threadIdx.x;
    if (base + j < n) st_sys(mine + j, src[base + j]);
  }
  const bool ok = signal_and_wait(x, FLAGS, slot * MAX_BLOCKS + b, g + 1);
  A out[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) out[i] = ok ? sum_ranks<A>(x, rec, (long)i * THREADS + threadIdx.x) : poison<A>();
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const long j = (long)i * THREADS + threadIdx.x;
    if (base + j < n) dst[base + j] = out[i];
  }
  if (threadIdx.x == 0) x.gen[b] = g + 1;  // every thread read gen[b] before the first barrier
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// host API (flat C ABI, driven from flink_ml_amd/parallel/xgmi.py)
// ---------------------------------------------------------------------------------------------
FMLX_API long fmlx_xar_total_bytes() { return xgmi::TOTAL; }
FMLX_API int fmlx_xar_chunk() { return xgmi::CHUNK; }
FMLX_API int fmlx_xar_max_blocks() { return xgmi::MAX_BLOCKS; }
FMLX_API int fmlx_xar_max_ranks() { return xgmi::MAX_RANKS; }
FMLX_API int fmlx_xar_gen_size() { return xgmi::GEN_SIZE; }
FMLX_API int fmlx_xar_glm_max() { return xgmi::GLM_MAX; }
FMLX_API int fmlx_xar_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// Allocates `bytes` of uncached device memory on the current device, zeroes it and exports its
// IPC handle (64 bytes) into out_handle.
FMLX_API int fmlx_xar_alloc(long bytes, void** out_ptr, void* out_handle) {
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, (size_t)bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) {
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, p);
    if (e == hipSuccess) __builtin_memcpy(out_handle, &h, sizeof(h));
  }
  if (e != hipSuccess) {
    (void)hipFree(p);
    return (int)e;
  }
  *out_ptr = p;
  return 0;
}

FMLX_API int fmlx_xar_open(const void* handle, void** out_ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out_ptr, h, hipIpcMemLazyEnablePeerAccess);
}

FMLX_API int fmlx_xar_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

// Host-mapped, coherent (fine-grained) int32 words for device→host status flags: the device
// writes them with system-scope stores and the host reads them without synchronising.
FMLX_API int fmlx_host_flags_alloc(int n, void** host_ptr, void** dev_ptr) {
  void* h = nullptr;
  hipError_t e = hipHostMalloc(&h, (size_t)n * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return (int)e;
  __builtin_memset(h, 0, (size_t)n * sizeof(int));
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    return (int)e;
  }
  *host_ptr = h;
  *dev_ptr = d;
  return 0;
}
FMLX_API int fmlx_host_flags_free(void* h) { return (int)hipHostFree(h); }
FMLX_API int fmlx_xar_free(void* p) { return (int)hipFree(p); }

// In-place allowed (dst == src). dtype: 0 = f32, 1 = f64. state: optional SGD round state that
// predicates the call (skipped uniformly once the iteration has terminated).
FMLX_API int fmlx_xar_allreduce(int dtype, void* const* peers_dev, int world, int rank, const void* src, void* dst,
                                long n, int* gen, int* err, const int* state, long spin_limit, void* stream) {
  if (world < 1 || world > xgmi::MAX_RANKS || rank < 0 || rank >= world) return -1;
  const long nb = (n + xgmi::CHUNK - 1) / xgmi::CHUNK;
  if (nb > xgmi::MAX_BLOCKS) return -3;
  if (nb == 0) return 0;
  xgmi::Ctx x{peers_dev, world, rank, gen, err, spin_limit};
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(xar_oneshot_kernel<float>, dim3((unsigned)nb), dim3(xgmi::THREADS), 0, s, x,
                       (const float*)src, (float*)dst, n, state);
  else
    hipLaunchKernelGGL(xar_oneshot_kernel<double>, dim3((unsigned)nb), dim3(xgmi::THREADS), 0, s, x,
                       (const double*)src, (double*)dst, n, state);
  return (int)hipGetLastError();
}
