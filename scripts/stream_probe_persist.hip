// Floor of the SGD round's launch structure (VERDICT r3 next #2b). The flagship round streams a
// fresh 100k-row × 2000-B bf16 batch (200 MB) per round; rounds depend on each other (round e+1
// needs w_{e+1}, i.e. every block of round e), so between rounds there is either a kernel boundary
// or a grid-wide barrier. Three structures, same row body (one wave per row, rows interleaved over
// the grid's waves, U rows per step, 2 steps in flight, trivial consumer), 20 batches per timing:
//   launches  — 20 launches back to back, directly and as one captured hipGraph;
//   persist   — ONE launch streams the 20 batches with a counter grid barrier between them;
//   persist+pf— the same, but waves 1..7 of every block issue their first 2 steps of batch i+1
//               BEFORE waiting at barrier i (the next batch's rows do not depend on the barrier),
//               so early blocks keep HBM busy while the stragglers finish; wave 0 polls.
// Bounded spins: a barrier that waits > ~50 ms sets a timeout word and the kernel stops.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/sp_persist scripts/stream_probe_persist.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr long ROWS = 100000;   // rows per batch
constexpr int CH = 125;         // 16-B chunks per 2000-B row
constexpr int NBATCH = 20;

template <int U>
struct Body {
  const u32x4* x;
  long W, gw;
  int c0, c1;
  float s = 0.f;
  __device__ void load(long r0, u32x4 (&d)[U][2]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long r = r0 + u * W;
      r = r < ROWS ? r : ROWS - 1;
      d[u][0] = __builtin_nontemporal_load(x + r * CH + c0);
      d[u][1] = __builtin_nontemporal_load(x + r * CH + c1);
    }
  }
  __device__ void use(u32x4 (&d)[U][2]) {
#pragma unroll
    for (int u = 0; u < U; ++u) s += __uint_as_float(d[u][0].x) + __uint_as_float(d[u][1].w);
  }
  // streams the batch; a and b may already hold steps 0 and 1 (pre = true)
  __device__ void run(u32x4 (&a)[U][2], u32x4 (&b)[U][2], bool pre) {
    const long step = (long)U * W;
    long r = gw;
    if (!pre) load(r, a);
    bool have_b = pre;
    while (true) {
      if (!have_b) load(r + step, b);
      have_b = false;
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      use(a);
      r += step;
      if (r >= ROWS) break;
      load(r + step, a);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      use(b);
      r += step;
      if (r >= ROWS) break;
    }
  }
};

template <int U, int WPB>
__global__ __launch_bounds__(WPB * 64) void one_batch(const u32x4* x, float* out) {
  Body<U> B{x, (long)gridDim.x * WPB, (long)blockIdx.x * WPB + (threadIdx.x >> 6), (int)(threadIdx.x & 63),
            (int)((threadIdx.x & 63) + 64 < CH ? (threadIdx.x & 63) + 64 : CH - 1)};
  u32x4 a[U][2], b[U][2];
  B.run(a, b, false);
  if (B.s == 1234.5f) out[0] = B.s;
}

// counter barrier: every wave drained, one lane arrives (relaxed agent atomic), wave 0 lane 0
// polls relaxed with s_sleep, the block's raw s_barrier releases the other waves
__device__ __forceinline__ bool bar_arrive(unsigned* bar) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}
__device__ __forceinline__ bool bar_wait(unsigned* bar, unsigned target, unsigned* tmo) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    int good = 1;
    for (unsigned spin = 0;; ++spin) {
      const unsigned v = __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int)(v - target) >= 0) break;
      if (spin > (1u << 22)) {  // ~50+ ms
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        good = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    ok = good;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  return ok != 0;
}

template <int U, int WPB, bool PF>
__global__ __launch_bounds__(WPB * 64) void persist(const u32x4* x, long batch_stride, unsigned* bar, unsigned* tmo,
                                                    float* out) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  Body<U> B{x, (long)gridDim.x * WPB, (long)blockIdx.x * WPB + wave, (int)(threadIdx.x & 63),
            (int)((threadIdx.x & 63) + 64 < CH ? (threadIdx.x & 63) + 64 : CH - 1)};
  u32x4 a[U][2], b[U][2];
  bool pre = false;
  for (int i = 0; i < NBATCH; ++i) {
    B.x = x + (long)i * batch_stride;
    B.run(a, b, pre);
    bar_arrive(bar);
    pre = false;
    if (i + 1 < NBATCH) {
      if (PF && wave != 0) {
        const Body<U> nb{x + (long)(i + 1) * batch_stride, B.W, B.gw, B.c0, B.c1};
        Body<U> tmp = nb;
        tmp.load(B.gw, a);
        tmp.load(B.gw + (long)U * B.W, b);
        pre = true;
      }
      if (!bar_wait(bar, (unsigned)(i + 1) * gridDim.x, tmo)) break;
      if (PF && wave == 0) pre = false;
    }
  }
  if (B.s == 1234.5f) out[0] = B.s;
}

int main() {
  const long rows_total = 2000000;
  const size_t bytes = (size_t)rows_total * 2000;
  u32x4* x;
  float* out;
  unsigned* sync;
  CK(hipMalloc(&x, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMalloc(&sync, 256));
  CK(hipMemset(x, 0x3c, bytes));
  CK(hipMemset(sync, 0, 256));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const long bstride = ROWS * CH;
  const int P = (int)(rows_total / ROWS);
  const double gb = ROWS * 2000.0 / 1e9;
  int start = 0;  // rotate the 20-batch window through the 4 GB buffer (no cache reuse)
  auto timeit = [&](const char* name, auto launch) -> int {
    double best = 1e30, sum = 0;
    const int reps = 8;
    for (int rep = 0; rep < reps + 2; ++rep) {
      const u32x4* base = x + (size_t)(start % (P - NBATCH + 1)) * bstride;
      start += NBATCH;
      CK(hipMemsetAsync(sync, 0, 256, st));
      CK(hipEventRecord(e0, st));
      if (launch(base)) return 1;
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipGetLastError());
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned t = 0;
      CK(hipMemcpy(&t, sync + 32, 4, hipMemcpyDeviceToHost));
      if (t) { printf("%s: barrier timeout\n", name); return 1; }
      if (rep < 2) continue;  // warm-up
      const double us = ms * 1e3 / NBATCH;
      sum += us;
      best = us < best ? us : best;
    }
    printf("%-40s mean %7.2f  best %7.2f us/batch  (%5.0f GB/s mean)\n", name, sum / reps, best, gb / (sum / reps * 1e-6));
    fflush(stdout);
    return 0;
  };
  for (int blocks : {224, 256}) {
    char nm[96];
    snprintf(nm, sizeof nm, "launches x20 U2 %d blk", blocks);
    if (timeit(nm, [&](const u32x4* p) {
          for (int i = 0; i < NBATCH; ++i) one_batch<2, 8><<<blocks, 512, 0, st>>>(p + (long)i * bstride, out);
          return 0;
        })) return 1;
    // the same 20 launches captured once per base pointer would freeze the pointers: capture a
    // graph over a fixed window and time replays of it
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < NBATCH; ++i) one_batch<2, 8><<<blocks, 512, 0, st>>>(x + (long)i * bstride, out);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    snprintf(nm, sizeof nm, "graph(20 launches) U2 %d blk", blocks);
    if (timeit(nm, [&](const u32x4*) { return hipGraphLaunch(ge, st) != hipSuccess; })) return 1;
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    snprintf(nm, sizeof nm, "persist U2 %d blk", blocks);
    if (timeit(nm, [&](const u32x4* p) {
          persist<2, 8, false><<<blocks, 512, 0, st>>>(p, bstride, sync, sync + 32, out);
          return 0;
        })) return 1;
    snprintf(nm, sizeof nm, "persist+pf U2 %d blk", blocks);
    if (timeit(nm, [&](const u32x4* p) {
          persist<2, 8, true><<<blocks, 512, 0, st>>>(p, bstride, sync, sync + 32, out);
          return 0;
        })) return 1;
  }
  return 0;
}
