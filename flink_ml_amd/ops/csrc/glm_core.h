// Shared device helpers of the GLM kernels (glm.hip: dense rounds; glm_sparse.hip: CSR rounds):
// loss/multiplier of the reference's loss functions, the device round state, the SGD update with
// elastic-net regularisation and the agent-scope hand-off primitives.
#pragma once
#include "common.h"

namespace {

enum { LOSS_LOGISTIC = 0, LOSS_HINGE = 1, LOSS_LSQ = 2, LOSS_FTRL = 3 };
enum { ST_ROUND = 0, ST_RUN0 = 1, ST_ARRIVE = 3, ST_EXECUTED = 4, ST_ROUND_ALT = 5, ST_DONE = 6 };
enum { TAIL_PARTIALS = 0, TAIL_FEEDBACK = 1, TAIL_UPDATE = 2, TAIL_XGMI = 3 };
constexpr int TAIL_GROUP = 32;  // block partials summed per group finisher
constexpr int TAIL_MAXG = 16;   // groups of the deterministic tail (=> at most 512 blocks)
constexpr int TAIL_TOP = 64;    // index of the top-level ticket (atomic tail: up to 64 groups)

// fp32 (bf16/fp32 data): one v_exp, one v_log, one v_rcp per row instead of the accurate libm
// expf/log1pf/division sequences (~100 VALU instructions per row, wave-uniform work that cost
// 6 µs of the 200 MB round body, measured); fp64 parity mode keeps the accurate path below.
//   logistic, z = −dot·ys, t = e^(−|z|) ∈ (0, 1]:  softplus(z) = max(z, 0) + log(1 + t),
//   mult = −ys / (e^(−z) + 1) = −ys · (z > 0 ? 1 : t) / (1 + t)
__device__ __forceinline__ void loss_and_mult(int loss, float dot, float y, float wt, float& l, float& m) {
  if (loss == LOSS_LOGISTIC) {
    const float ys = 2.f * y - 1.f;
    const float z = -dot * ys;
    // raw v_exp_f32 / v_log_f32 (base 2): t ∈ (0, 1] and 1 + t ∈ (1, 2] need none of the
    // denormal range fix-ups of expf/logf; v_rcp_f32 (1 ulp), not the IEEE division sequence
    const float t = __builtin_amdgcn_exp2f(-fabsf(z) * 1.4426950408889634f);
    const float r = __builtin_amdgcn_rcpf(1.f + t);
    l = wt * (fmaxf(z, 0.f) + __builtin_amdgcn_logf(1.f + t) * 0.6931471805599453f);
    m = wt * (-ys) * (z > 0.f ? r : t * r);
  } else if (loss == LOSS_HINGE) {
    const float ys = 2.f * y - 1.f;
    const float h = 1.f - ys * dot;
    const bool pos = h > 0.f;
    l = pos ? wt * h : 0.f;
    m = pos ? -ys * wt : 0.f;
  } else if (loss == LOSS_FTRL) {
    m = __builtin_amdgcn_rcpf(1.f + __expf(-dot)) - y;
    l = 0.f;
  } else {
    const float r = dot - y;
    l = wt * 0.5f * r * r;
    m = r * wt;
  }
}

template <typename A>
__device__ __forceinline__ void loss_and_mult(int loss, A dot, A y, A wt, A& l, A& m) {
  if (loss == LOSS_LOGISTIC) {
    A ys = (A)2 * y - (A)1;
    A z = -dot * ys;
    // wt*log(1+exp(z)), stable softplus
    A sp = z > (A)0 ? z + log1p(exp(-z)) : log1p(exp(z));
    l = wt * sp;
    m = wt * (-ys / (exp(dot * ys) + (A)1));
  } else if (loss == LOSS_HINGE) {
    A ys = (A)2 * y - (A)1;
    A h = (A)1 - ys * dot;
    if (h > (A)0) { l = wt * h; m = -ys * wt; } else { l = (A)0; m = (A)0; }
  } else if (loss == LOSS_FTRL) {
    // OnlineLogisticRegression local gradient (OnlineLogisticRegression.java:344-368, dense
    // branch): (sigmoid(dot) - label) · x, weight ignored; the weight slot counts rows.
    m = (A)1 / ((A)1 + exp(-dot)) - y;
    l = (A)0;
  } else {
    A r = dot - y;
    l = wt * (A)0.5 * r * r;
    m = r * wt;
  }
}

__device__ __forceinline__ bool round_running(const int* st, int& e) {
  e = st[ST_ROUND];
  return st[ST_RUN0 + (e & 1)] != 0;
}

// apply the SGD step + elastic-net regularisation to one coefficient (SGD.java:231-243,
// RegularizationUtils.java:47-91). The reg loss only feeds the discarded totalLoss slot in the
// reference, so it is not materialised here.
template <typename A>
__device__ __forceinline__ A sgd_apply(A w, A g, A W, A lr, A reg, A en) {
  if (!(W > (A)0)) return w;
  w = w - lr / W * g;
  if (reg == (A)0) return w;
  if (en == (A)0) return w * ((A)1 - lr * reg);
  A sg = w > (A)0 ? (A)1 : (w < (A)0 ? (A)-1 : (A)0);
  if (en == (A)1) return w - lr * en * reg * sg;
  return w - lr * (en * reg * sg + ((A)1 - en) * reg * w);
}

// Write-through (sc1) hand-off of the partial rows (cdna_hip_programming.md Guideline 16, the
// sc1 form of the split-K combine): every handed-off value is stored with an agent-scope store
// (global_store … sc1) and loaded with an agent-scope load (global_load … sc1), so no release
// fence (an L2 write-back per block: ~20 µs over 512 blocks, measured) and no acquire fence
// are needed — only the drain before the ticket.
template <typename A>
__device__ __forceinline__ void st_agent(A* p, A v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename A>
__device__ __forceinline__ A ld_agent(const A* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every wave drains its sc1 stores, lane 0 draws a ticket; the block drawing the last one
// proceeds (returns true there only).
__device__ __forceinline__ bool arrive_last(int* cnt, int expected, int* sflag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sflag = t == expected - 1;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the sc1 loads below the ticket
  return *sflag != 0;
}

// last-arriving block advances the round state (Guideline 16 counter form).
__device__ __forceinline__ void arrive_and_advance(int* state, int e, bool cont, int executed_inc) {
  __syncthreads();
  // No data is handed between blocks here: every block has already consumed its read of the
  // state words (its control flow depended on them) before its ticket add, so the last arriver
  // may overwrite them; the next kernel sees the writes through the kernel boundary.
  if (threadIdx.x == 0) {
    const int nblocks = (int)(gridDim.x * gridDim.y);
    int t = __hip_atomic_fetch_add(&state[ST_ARRIVE], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == nblocks - 1) {
      state[ST_RUN0 + ((e + 1) & 1)] = cont ? 1 : 0;
      state[ST_EXECUTED] += executed_inc;
      state[ST_ROUND] = e + 1;
      state[ST_ARRIVE] = 0;
    }
  }
}

constexpr long LDS_PER_CU = 160 * 1024;
constexpr int NUM_CU = 256;

}  // namespace
