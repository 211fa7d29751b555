// Layout and device helpers of the one-shot xGMI exchange (xgmi_allreduce.hip, glm.hip).
//
// Every rank owns ONE exchange buffer allocated uncached (fine-grained) and exported through a
// dmabuf IPC handle; every rank maps every peer's buffer (flink_ml_amd/parallel/xgmi.py). A
// payload is published with system-scope stores into the owner's own buffer, then a tag word is
// raised; consumers poll the peers' tag words over xGMI (one lane per peer, relaxed, bounded,
// s_sleep between polls) and read the peers' payloads with system-scope loads.
//
// Byte layout of one rank's buffer:
//   FLAGS      int32 [2][MAX_BLOCKS]             generic all-reduce, one tag per (slot, chunk)
//   GLM_FLAGS  int32 [2] (256-B block)           fused GLM round feedback exchange
//   DATA       [2][MAX_BLOCKS][CHUNK] x 8 B      generic records (f32 or f64 elements)
//   GLM_DATA   [2][GLM_MAX] x 8 B                fused GLM feedback record [grad | Σw | Σloss]
//   TS_*                                         two-shot all-reduce regions (below)
// Slot = tag parity; tags are per-channel counters kept in LOCAL memory (gen[]), advanced by the
// consuming block itself, so every rank — issuing the same call sequence — uses the same tags and
// hipGraph replays keep advancing them (they are read from memory, never frozen arguments).
// Two slots make reuse safe: a block that writes slot s in call k+2 has seen every peer publish
// call k+1, which that peer issued only after its call k (stream order) finished reading slot s.
#pragma once
#include <cstdlib>

#include "common.h"

namespace xgmi {

constexpr int THREADS = 256;
constexpr int VEC = 4;
constexpr int CHUNK = THREADS * VEC;  // elements per generic record / block
constexpr int MAX_RANKS = 8;          // one node: 8 GPUs, fully connected by xGMI
constexpr int MAX_BLOCKS = 1024;      // => up to 1M elements per generic all-reduce
constexpr int GLM_MAX = 4104;         // d + 2 for the register-resident GLM path (d <= 4096)

constexpr long FLAGS = 0;
constexpr long GLM_FLAGS = FLAGS + 2L * MAX_BLOCKS * 4;
constexpr long DATA = GLM_FLAGS + 256;
constexpr long GLM_DATA = DATA + 2L * MAX_BLOCKS * CHUNK * 8;
// Two-shot all-reduce (xgmi_allreduce.hip, 1-8 MB payloads): block b of every rank handles the
// chunk group {b·P … b·P + P − 1}; chunk c is reduced by rank c mod P.
//   TS_PFLAGS  int32 [2][TS_MAX_BLOCKS]          "my copy of group b is published"
//   TS_RFLAGS  int32 [2][TS_MAX_BLOCKS]          "my reduced chunk of group b is published"
//   TS_DATA    [2][TS_MAX_ELEMS] x 8 B           every rank's full input (published copies)
//   TS_RED     [2][TS_MAX_ELEMS] x 8 B           reduced chunks, at their own positions
constexpr long TS_MAX_ELEMS = 2L << 20;  // 2M elements: 8 MB f32 / 16 MB f64
constexpr int TS_MAX_BLOCKS = (int)(TS_MAX_ELEMS / CHUNK);
constexpr long TS_PFLAGS = GLM_DATA + 2L * GLM_MAX * 8;
constexpr long TS_RFLAGS = TS_PFLAGS + 2L * TS_MAX_BLOCKS * 4;
constexpr long TS_DATA = TS_RFLAGS + 2L * TS_MAX_BLOCKS * 4;
constexpr long TS_RED = TS_DATA + 2L * TS_MAX_ELEMS * 8;
constexpr long TOTAL = TS_RED + 2L * TS_MAX_ELEMS * 8;
constexpr int GEN_GLM = MAX_BLOCKS;   // index of the fused-GLM counter in gen[]
constexpr int GEN_TS = MAX_BLOCKS + 1;  // first two-shot block counter in gen[]
constexpr int GEN_SIZE = GEN_TS + TS_MAX_BLOCKS;

// FMLX_XGMI_STRICT_FENCE=1 (read once per process, host side): signal_and_wait brackets the tag
// with system-scope release/acquire fences (an L2 write-back per exchanging block) instead of
// the vmcnt drain + workgroup acquire that suffice while every record word moves with
// system-scope stores/loads on the uncached buffers. The switch for a first run on a topology
// where the relaxed hand-off has not been validated (GPU tests run in both modes).
// The host may switch the fences on later (fmlx_xar_set_strict_fence: bench.py after an exchange
// that failed its verification); a Ctx reads the flag when it is built, i.e. per launch.
inline int& strict_fence_flag() {
  static int v = [] {
    const char* e = getenv("FMLX_XGMI_STRICT_FENCE");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return v;
}
inline int strict_fence() { return strict_fence_flag(); }

// Kernel-argument bundle. `peers` is a DEVICE array of `world` buffer pointers (mine at `rank`).
struct Ctx {
  void* const* peers;
  int world, rank;
  int* gen;         // int32[GEN_SIZE], local memory
  int* err;         // int32[1] in host-mapped coherent memory: set to 1 when a peer never
                    // arrived (the host reads it without a device sync, parallel/xgmi.py)
  long spin_limit;  // polls before giving up
  int strict = strict_fence();  // FMLX_XGMI_STRICT_FENCE=1: system-scope release/acquire fences
};

__device__ __forceinline__ int ld_sys(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename A>
__device__ __forceinline__ A ld_sys(const A* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename A>
__device__ __forceinline__ void st_sys(A* p, A v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <typename T>
__device__ __forceinline__ T* at(void* buf, long byte_off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(buf) + byte_off);
}

// Called by EVERY thread of the block after it stored its share of this rank's record with
// st_sys: drain every wave's stores, raise my tag, then wait until every peer raised the same
// tag (one polling lane per peer, bounded). Returns true (block-uniform) when every peer
// arrived: the peers' records are then readable. On a timeout the error word is raised and the
// caller must NOT sum (it poisons its output with NaN instead), so a partial exchange can never
// pass for a result.
// Every record word crosses with system-scope stores / loads on the uncached buffers, so the
// hand-off needs the stores DONE, not a cache write-back: a vmcnt(0) drain before the tag (a
// system-scope release fence here wrote back the whole L2 once per block — twice per block per
// two-shot call, ~1,000 write-backs for a 4 MB payload) and a workgroup-scope acquire after it.
__device__ __forceinline__ bool signal_and_wait(const Ctx& x, long flag_off, int idx, int tag) {
  __shared__ int s_timeout;
  if (threadIdx.x == 0) s_timeout = 0;
  if (x.strict)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: stores done + L2 written back
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) st_sys(at<int>(x.peers[x.rank], flag_off) + idx, tag);
  if ((int)threadIdx.x < x.world && (int)threadIdx.x != x.rank) {
    const int* f = at<int>(x.peers[threadIdx.x], flag_off) + idx;
    long it = 0;
    while (ld_sys(f) != tag) {
      // (an exchange of this context already gave up: the error word is raised and every result
      // is discarded — stop after a short poll instead of a full spin limit per call)
      if (++it > x.spin_limit || ((it & 1023) == 0 && ld_sys(x.err) != 0)) {
        st_sys(x.err, 1);  // plain system-scope store (host memory: no PCIe atomics needed)
        s_timeout = 1;     // any writer, same value
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (x.strict)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: stale cached lines invalidated
  else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the record loads below stay below the wait
  return s_timeout == 0;
}

template <typename A>
__device__ __forceinline__ A poison() {
  return (A)__builtin_nan("");
}

// Σ over ranks 0..world-1, in rank order, of element `i` of the records at byte offset `off`
// (element type A): identical bits on every rank. All MAX_RANKS loads are issued
// unconditionally (ranks past `world` re-read my own record and are masked out of the sum) so
// they are in flight together instead of one xGMI round trip per rank.
template <typename A>
__device__ __forceinline__ A sum_ranks(const Ctx& x, long off, long i) {
  A v[MAX_RANKS];
#pragma unroll
  for (int r = 0; r < MAX_RANKS; ++r) {
    const int rr = r < x.world ? r : x.rank;
    v[r] = ld_sys(at<A>(x.peers[rr], off) + i);
  }
  A s = (A)0;
#pragma unroll
  for (int r = 0; r < MAX_RANKS; ++r) s += r < x.world ? v[r] : (A)0;
  return s;
}

}  // namespace xgmi
