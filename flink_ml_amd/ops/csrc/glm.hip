// Fused generalized-linear-model kernels for SGD training and prediction (SURVEY §2.1 K4–K7).
//
// Reference hot loop (per row, fp64, Java): LIB/common/optimizer/SGD.java:275-279 calling
// LIB/common/lossfunc/{BinaryLogisticLoss,HingeLoss,LeastSquareLoss}.java — dot(x, w), loss,
// then axpy(mult, x, grad). Update + regularisation: SGD.java:231-243 and
// RegularizationUtils.java:47-91.
//
// MI355X design
//  * glm_grad_partials: ONE pass over the minibatch rows in HBM. A wave owns a row at a
//    time (two rows in flight for ILP when registers allow); each lane owns a fixed set of
//    EPC-element chunks (16-byte loads), so the coefficient slice AND the gradient
//    accumulator for those columns live in that lane's registers for the whole kernel: the
//    row is read exactly once, dot → wave butterfly → loss/multiplier → axpy, no LDS, no
//    atomics. Waves of a block combine by a fixed-order LDS tree, each block writes one
//    partial row [grad(d) | Σweight | Σloss] → deterministic, bit-reproducible.
//  * The round's reduction is fused into the same launch (glm_round_tail): each block publishes
//    its partial row and draws an arrival ticket (agent-scope release/acquire, Guideline 16);
//    the last block of every group of 32 sums the group's partials in fixed order, the last
//    group finisher sums the ≤16 group rows in fixed order and then, by mode,
//      TAIL_FEEDBACK  writes the (d+2) feedback (N GPUs over RCCL: all-reduce → glm_update),
//      TAIL_UPDATE    (1 GPU) evaluates TerminateOnMaxIterOrTol, applies w -= lr/Σw·g plus
//                     elastic-net regularisation and advances the device round state,
//      TAIL_XGMI      (N GPUs) exchanges the feedback with every peer over xGMI (xgmi.h: one
//                     record per rank, bounded tag waits, rank-order sum → bit-identical on all
//                     ranks) and then updates like TAIL_UPDATE.
//    So one SGD round is ONE kernel launch on 1 GPU and on N GPUs: no host synchronisation,
//    no separate reduce kernels, the whole round capturable in a hipGraph.
//  * Legacy split path (glm_reduce_stage1 → glm_reduce_update / glm_reduce) kept for the FTRL
//    local-gradient call and A/B measurements.
//  * Device round state (int32[8]): [0] round e, [1..2] running flag ping-pong
//    (running[e&1] gates round e), [3] arrival ticket, [4] rounds executed.
//    The batch of round e is rows [(e mod P)·B, min(+B, n)), P = ceil(n/B): exactly the
//    reference's sequential slicing with reset-to-0 (SGD.java:263-268).
#include "common.h"
#include "xgmi.h"
#include "glm_core.h"

FMLX_API void fmlx_glm_sparse_set_trace(void* trace);  // glm_sparse.hip

namespace {


// ------------------------------------------------------------------------------------------
// Fused round tail (after every block wrote its partial row)
// ------------------------------------------------------------------------------------------
struct GlmTail {
  int mode;        // TAIL_*
  int max_iter;
  int det;         // 1: deterministic fixed-order group tree; 0: float atomics into `acc`
  int flat_lds;    // atomic tail with the one-barrier [WPB][d] LDS image (set by the launcher)
  int nbatch;      // ceil(n / B) (set by the launcher)
  int* cnt;        // int32[TAIL_TOP + 1] arrival tickets: zero-initialised once, re-armed by the
                   // last arrivers, so every launch (and hipGraph replay) starts from zero
  void* acc;       // [d+2] zero-initialised accumulator of the atomic tail (re-zeroed by it)
  void* stage1;    // [ngroups][d+2] accumulator rows
  void* feedback;  // [d+2]: output of TAIL_FEEDBACK, a copy of the global feedback otherwise
  double tol, lr, reg, en;
  xgmi::Ctx x;     // TAIL_XGMI only
  int red_off;     // byte offset of the grouped row path's per-wave reduction scratch in LDS
  int acc_reps;    // atomic tail: replicas of `acc` (block b adds into replica b mod acc_reps)
  long acc_ld;     // elements between replicas (d + 2 rounded up to whole 256-B lines)
  int ticket2;     // atomic tail: two-level arrival tickets (per-residue groups, then a top one)
  int defer;       // deferred completion (TAIL_UPDATE / TAIL_XGMI, atomic flat tail): see defer_prologue
  int parity;      // deferred: this launch reads its round number from state[parity ? ALT : ROUND]
  void* cw;        // deferred: [2][d] coefficients of the last two rounds
  int wl_off;      // deferred: byte offset of the block's [d] coefficient image in LDS
  int ring_off;    // LDS-DMA row path: byte offset of the [WPB][DEPTH][U][2 KiB] row ring
  int xb_off;      // deferred TAIL_XGMI: byte offset of the lead block's [d+2] exchange row in LDS
  long long* trace;  // diagnostics (null = off): per block {start, rows done, end, hw id} in
                     // 100 MHz s_memrealtime ticks (scripts/trace_glm_blocks.py)
};
constexpr int ACC_MAX_REPS = 8;


// Replaces this rank's feedback fb[0..stride) (in LDS) by the rank-order sum over all ranks.
template <typename A>
__device__ void glm_xgmi_exchange(const xgmi::Ctx& x, A* fb, long stride) {
  using namespace xgmi;
  const int g = x.gen[GEN_GLM];
  const int slot = g & 1;
  const long rec = GLM_DATA + (long)slot * GLM_MAX * (long)sizeof(A);
  A* mine = at<A>(x.peers[x.rank], rec);
  for (long c = threadIdx.x; c < stride; c += blockDim.x) st_sys(mine + c, fb[c]);
  const bool ok = signal_and_wait(x, GLM_FLAGS, slot, g + 1);
  // a timed-out exchange poisons the feedback: with a NaN Σw the update is skipped and the
  // termination test (L/W > tol) fails, so the iteration stops on the last good coefficients;
  // the host raises on the error word (parallel/xgmi.py)
  for (long c = threadIdx.x; c < stride; c += blockDim.x) fb[c] = ok ? sum_ranks<A>(x, rec, c) : poison<A>();
  __syncthreads();
  if (threadIdx.x == 0) x.gen[GEN_GLM] = g + 1;
}

// Completes the round once sbuf[0..d+2) holds this rank's reduced feedback. In one-pass layouts
// (d + 2 <= 2·blockDim) the caller has prefetched coef[tid], coef[tid + blockDim] into wa, wb.
template <typename A>
__device__ void glm_round_finish(const GlmTail& tl, A* sbuf, int d, A* coef, int* state, int e, bool one_pass, A wa,
                                 A wb) {
  const long stride = d + 2;
  const int nt = blockDim.x;
  __syncthreads();
  if (tl.mode == TAIL_XGMI) glm_xgmi_exchange<A>(tl.x, sbuf, stride);
  A* fb = (A*)tl.feedback;
  if (tl.mode == TAIL_FEEDBACK) {
    for (long c = threadIdx.x; c < stride; c += nt) fb[c] = sbuf[c];
    return;
  }
  const A W = sbuf[d], L = sbuf[d + 1];
  const bool cont = (e + 1 < tl.max_iter) && (L / W > (A)tl.tol);
  const A lr = (A)tl.lr, reg = (A)tl.reg, en = (A)tl.en;
  const long ca = threadIdx.x, cb = threadIdx.x + nt;
  if (one_pass) {
    if (ca < d) coef[ca] = sgd_apply<A>(wa, sbuf[ca], W, lr, reg, en);
    if (cb < d) coef[cb] = sgd_apply<A>(wb, sbuf[cb], W, lr, reg, en);
  } else {
    for (long c = threadIdx.x; c < d; c += nt) coef[c] = sgd_apply<A>(coef[c], sbuf[c], W, lr, reg, en);
  }
  if (fb)
    for (long c = threadIdx.x; c < stride; c += nt) fb[c] = sbuf[c];
  if (threadIdx.x == 0) {
    // every block of this launch read the state words before its first ticket
    state[ST_RUN0 + ((e + 1) & 1)] = cont ? 1 : 0;
    state[ST_EXECUTED] += 1;
    state[ST_ROUND] = e + 1;
  }
}

// Deterministic tail: block partial rows → per-group fixed-order sums → fixed-order total.
template <typename A>
__device__ void glm_round_tail_det(const GlmTail& tl, const A* partials, int d, A* coef, int* state, int e, A* sbuf,
                                   int* sflag) {
  const long stride = d + 2;
  const int nb = gridDim.x;
  const int nt = blockDim.x;
  const int ngroups = (nb + TAIL_GROUP - 1) / TAIL_GROUP;
  const int g = blockIdx.x / TAIL_GROUP;
  const int g0 = g * TAIL_GROUP;
  const int gs = nb - g0 < TAIL_GROUP ? nb - g0 : TAIL_GROUP;
  A* st1 = (A*)tl.stage1;
  // ---- ticket 1: the group's last block sums its partial rows (fixed order). Two columns per
  // thread per pass with all their loads in flight together: one memory latency per pass.
  if (!arrive_last(&tl.cnt[g], gs, sflag)) return;
  for (long c0 = threadIdx.x; c0 < stride; c0 += 2 * nt) {
    const long c1 = c0 + nt < stride ? c0 + nt : c0;
    A v0[TAIL_GROUP], v1[TAIL_GROUP];
#pragma unroll
    for (int q = 0; q < TAIL_GROUP; ++q) {
      const A* row = partials + (long)(g0 + (q < gs ? q : 0)) * stride;
      v0[q] = ld_agent(row + c0);
      v1[q] = ld_agent(row + c1);
    }
    A s0 = (A)0, s1 = (A)0;
#pragma unroll
    for (int q = 0; q < TAIL_GROUP; ++q) {
      s0 += q < gs ? v0[q] : (A)0;
      s1 += q < gs ? v1[q] : (A)0;
    }
    st_agent(st1 + (long)g * stride + c0, s0);
    if (c1 != c0) st_agent(st1 + (long)g * stride + c1, s1);
  }
  if (threadIdx.x == 0) tl.cnt[g] = 0;  // all gs arrivals of this launch are in: re-arm
  // ---- ticket 2: the last group finisher sums the group rows and completes the round
  if (!arrive_last(&tl.cnt[TAIL_TOP], ngroups, sflag)) return;
  if (threadIdx.x == 0) tl.cnt[TAIL_TOP] = 0;
  const bool one_pass = stride <= 2L * nt && tl.mode != TAIL_FEEDBACK;
  A wa = (A)0, wb = (A)0;
  for (long c0 = threadIdx.x; c0 < stride; c0 += 2 * nt) {
    const long c1 = c0 + nt < stride ? c0 + nt : c0;
    A v0[TAIL_MAXG], v1[TAIL_MAXG];
#pragma unroll
    for (int q = 0; q < TAIL_MAXG; ++q) {
      const A* row = st1 + (long)(q < ngroups ? q : 0) * stride;
      v0[q] = ld_agent(row + c0);
      v1[q] = ld_agent(row + c1);
    }
    if (one_pass) {  // the coefficients come in the same memory latency
      wa = coef[threadIdx.x < d ? threadIdx.x : 0];
      wb = coef[threadIdx.x + nt < d ? threadIdx.x + nt : 0];
    }
    A s0 = (A)0, s1 = (A)0;
#pragma unroll
    for (int q = 0; q < TAIL_MAXG; ++q) {
      s0 += q < ngroups ? v0[q] : (A)0;
      s1 += q < ngroups ? v1[q] : (A)0;
    }
    sbuf[c0] = s0;
    sbuf[c1] = s1;
  }
  glm_round_finish<A>(tl, sbuf, d, coef, state, e, one_pass, wa, wb);
}

// Atomic tail: every block adds its row (LDS, 256 contiguous bytes per wave-instruction) into
// `acc` with no-return float atomics, drains, and draws a ticket (per group of 32, then a top
// ticket: no single counter takes all arrivals). The last block reads `acc` once, re-zeroes it
// for the next launch and completes the round. Summation order varies run to run (last bits);
// every rank of a multi-GPU job still ends identical (xGMI sums the published values in rank
// order).
template <typename A>
__device__ void glm_round_tail_atomic(const GlmTail& tl, int d, A* coef, int* state, int e, A* sbuf, int* sflag) {
  // (the caller has added this block's row into tl.acc with no-return atomics)
  const long stride = d + 2;
  const int nt = blockDim.x;
  A* acc = (A*)tl.acc;
  const int R = tl.acc_reps > 1 ? tl.acc_reps : 1;
  const long ald = tl.acc_ld > 0 ? tl.acc_ld : stride;
  if (tl.ticket2) {
    // two levels: the blocks of one residue class b mod R (one XCD under round-robin dispatch)
    // share a counter, the last of each class draws the top ticket — no counter takes more than
    // ceil(nb / R) arrivals at once
    const int nb = gridDim.x;
    const int g = blockIdx.x % R;
    const int gs = nb / R + (g < nb % R ? 1 : 0);
    if (!arrive_last(&tl.cnt[g], gs, sflag)) return;
    if (threadIdx.x == 0) st_agent(&tl.cnt[g], 0);
    if (!arrive_last(&tl.cnt[TAIL_TOP], nb < R ? nb : R, sflag)) return;
    if (threadIdx.x == 0) st_agent(&tl.cnt[TAIL_TOP], 0);
  } else {
    // one ticket over all blocks: arrivals are spread over the blocks' finishing times, so a
    // single counter costs the last block one atomic round trip instead of two
    if (!arrive_last(&tl.cnt[0], gridDim.x, sflag)) return;
    if (threadIdx.x == 0) tl.cnt[0] = 0;
  }
  const bool one_pass = stride <= 2L * nt && tl.mode != TAIL_FEEDBACK;
  A wa = (A)0, wb = (A)0;
  // Σ of the replicas in a fixed order (all R loads of a column in flight together), then re-zero
  auto take = [&](long c) -> A {
    A v[ACC_MAX_REPS];
#pragma unroll
    for (int q = 0; q < ACC_MAX_REPS; ++q) v[q] = q < R ? ld_agent(acc + q * ald + c) : (A)0;
    A t = (A)0;
#pragma unroll
    for (int q = 0; q < ACC_MAX_REPS; ++q) t += v[q];
#pragma unroll
    for (int q = 0; q < ACC_MAX_REPS; ++q)
      if (q < R) st_agent(acc + q * ald + c, (A)0);
    return t;
  };
  if (one_pass) {
    const long ca = threadIdx.x, cb = threadIdx.x + nt;
    wa = coef[ca < d ? ca : 0];
    wb = coef[cb < d ? cb : 0];
    if (ca < stride) sbuf[ca] = take(ca);
    if (cb < stride) sbuf[cb] = take(cb);
  } else {
    for (long c = threadIdx.x; c < stride; c += nt) sbuf[c] = take(c);
  }
  glm_round_finish<A>(tl, sbuf, d, coef, state, e, one_pass, wa, wb);
}

// Deferred round completion (1 GPU, TAIL_UPDATE with the atomic tail). Launch e first completes
// round e − 1: every block sums the replicas of that round's accumulator slot (fixed order, as
// the ticketed tail does), evaluates TerminateOnMaxIterOrTol and applies the SGD update into an
// LDS image of w_e; then it computes round e's gradient with w_e and adds it into slot e % 3 with
// no-return atomics — no arrival ticket and no serial last-block tail remain on the critical
// path. Ring of 3 slots: launch e reads slot (e − 1) % 3, adds into e % 3, zeroes (e + 1) % 3
// (read by launch e − 1, added into by launch e + 1; kernel boundaries order all three). Block 0
// publishes w_e (cw[e & 1] for launch e + 1, coef for the host) and the round counter into the
// state word the NEXT launch reads (launches alternate between two words, so no block of this
// launch can observe the update). Returns true (for every thread) when the iteration ended.
template <typename A>
__device__ bool defer_prologue(const GlmTail& tl, A* coef, int* state, int e, int d, A* wl) {
  const int nt = blockDim.x, tid = threadIdx.x;
  const int R = tl.acc_reps > 1 ? tl.acc_reps : 1;
  const long ald = tl.acc_ld;
  const long slot = (long)ACC_MAX_REPS * ald;
  A* ring = (A*)tl.acc;
  A* cw = (A*)tl.cw;
  A* fb = (A*)tl.feedback;
  const bool lead = blockIdx.x == 0;
  bool stop = false;
  if (e == 0) {
    for (long c = tid; c < d; c += nt) wl[c] = coef[c];
  } else {
    const A* prev = ring + (long)((e + 2) % 3) * slot;
    A vw[ACC_MAX_REPS], vl[ACC_MAX_REPS];
#pragma unroll
    for (int q = 0; q < ACC_MAX_REPS; ++q) {
      vw[q] = q < R ? ld_agent(prev + q * ald + d) : (A)0;
      vl[q] = q < R ? ld_agent(prev + q * ald + d + 1) : (A)0;
    }
    A W = (A)0, L = (A)0;
#pragma unroll
    for (int q = 0; q < ACC_MAX_REPS; ++q) {
      W += vw[q];
      L += vl[q];
    }
    stop = !(e < tl.max_iter && L / W > (A)tl.tol);
    const A lr = (A)tl.lr, reg = (A)tl.reg, en = (A)tl.en;
    const A* wp = cw + (long)((e - 1) & 1) * d;
    for (long c = tid; c < d; c += nt) {
      A v[ACC_MAX_REPS];
#pragma unroll
      for (int q = 0; q < ACC_MAX_REPS; ++q) v[q] = q < R ? ld_agent(prev + q * ald + c) : (A)0;
      const A w0 = wp[c];
      A g = (A)0;
#pragma unroll
      for (int q = 0; q < ACC_MAX_REPS; ++q) g += v[q];
      wl[c] = sgd_apply<A>(w0, g, W, lr, reg, en);
      if (lead && fb) fb[c] = g;
    }
    if (lead && fb && tid == 0) {
      fb[d] = W;
      fb[d + 1] = L;
    }
  }
  A* nxt = ring + (long)((e + 1) % 3) * slot;
  for (long i = (long)blockIdx.x * nt + tid; i < slot; i += (long)gridDim.x * nt) nxt[i] = (A)0;
  __syncthreads();
  if (lead) {
    A* wc = cw + (long)(e & 1) * d;
    for (long c = tid; c < d; c += nt) {
      wc[c] = wl[c];
      coef[c] = wl[c];  // launch 0: the value every block just read
    }
    if (tid == 0) {
      state[tl.parity ? ST_ROUND : ST_ROUND_ALT] = e + 1;
      if (e > 0) state[ST_EXECUTED] += 1;
      if (stop) state[ST_DONE] = 1;
    }
  }
  return stop;
}

// Deferred round completion across ranks (TAIL_XGMI with the atomic flat tail; SGD.java:246-255
// applies round e's update at the start of round e + 1). Launch e's blocks add round e's gradient
// into this rank's accumulator slot e % 3 and exit — no ticket, no serial last-block tail. Launch
// e + 1's LEAD block (block 0) sums that slot's replicas (fixed order), exchanges the row with
// every peer over xGMI (one record per rank, rank-order sum: bit-identical on every rank),
// evaluates TerminateOnMaxIterOrTol, applies the update into cw[e' & 1] (write-through) and raises
// a flag word; every other block keeps its first row steps in flight, waits for the flag (one
// polling lane, bounded) and reads w_{e'} from cw. So the exchange latency overlaps the next
// round's first row loads instead of following the last block's arrival. Returns true (for every
// thread) when the iteration ended.
constexpr int WFLAG_IDX = 120;  // tl.cnt word: (round << 1) | stop, published by the lead block
template <typename A>
__device__ bool defer_prologue_xgmi(const GlmTail& tl, A* coef, int* state, int e, int d, A* wl) {
  const int nt = blockDim.x, tid = threadIdx.x;
  const int R = tl.acc_reps > 1 ? tl.acc_reps : 1;
  const long ald = tl.acc_ld;
  const long slot = (long)ACC_MAX_REPS * ald;
  const long stride = d + 2;
  A* ring = (A*)tl.acc;
  A* cw = (A*)tl.cw;
  A* fb = (A*)tl.feedback;
  int* wflag = tl.cnt + WFLAG_IDX;
  __shared__ int s_stop;
  const bool lead = blockIdx.x == 0;
  if (e == 0) {
    for (long c = tid; c < d; c += nt) wl[c] = coef[c];
    if (tid == 0) s_stop = 0;
  } else if (lead) {
    extern __shared__ __align__(16) unsigned char smem_x[];
    A* xr = reinterpret_cast<A*>(smem_x + tl.xb_off);
    const A* prev = ring + (long)((e + 2) % 3) * slot;
    for (long c = tid; c < stride; c += nt) {
      A v[ACC_MAX_REPS];
#pragma unroll
      for (int q = 0; q < ACC_MAX_REPS; ++q) v[q] = q < R ? ld_agent(prev + q * ald + c) : (A)0;
      A g = (A)0;
#pragma unroll
      for (int q = 0; q < ACC_MAX_REPS; ++q) g += v[q];
      xr[c] = g;
    }
    __syncthreads();
    glm_xgmi_exchange<A>(tl.x, xr, stride);  // xr ← Σ over ranks (NaN-poisoned on a timeout)
    const A W = xr[d], L = xr[d + 1];
    const bool stop = !(e < tl.max_iter && L / W > (A)tl.tol);
    const A lr = (A)tl.lr, reg = (A)tl.reg, en = (A)tl.en;
    const A* wp = cw + (long)((e - 1) & 1) * d;
    A* wc = cw + (long)(e & 1) * d;
    for (long c = tid; c < d; c += nt) {
      const A w = sgd_apply<A>(wp[c], xr[c], W, lr, reg, en);
      wl[c] = w;
      st_agent(wc + c, w);
      coef[c] = w;
      if (fb) fb[c] = xr[c];
    }
    if (tid == 0) {
      if (fb) {
        fb[d] = W;
        fb[d + 1] = L;
      }
      s_stop = stop;
    }
    // every wave's write-through stores of w drained, then the flag (write-through, agent scope)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) st_agent(wflag, (e << 1) | (stop ? 1 : 0));
  } else {
    if (tid == 0) {
      int v = 0;
      long it = 0;
      for (;;) {
        v = ld_agent(wflag);
        if ((v >> 1) == e) break;
        if (++it > 4 * tl.x.spin_limit || ((it & 1023) == 0 && xgmi::ld_sys(tl.x.err) != 0)) {
          // the lead never published (or an exchange already gave up): stop, and say so
          xgmi::st_sys(tl.x.err, 1);
          v = (e << 1) | 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      s_stop = v & 1;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the sc1 loads below the wait
    if (!s_stop) {
      const A* wc = cw + (long)(e & 1) * d;
      for (long c = tid; c < d; c += nt) wl[c] = ld_agent(wc + c);
    }
  }
  __syncthreads();
  const bool stop = s_stop != 0;
  A* nxt = ring + (long)((e + 1) % 3) * slot;
  for (long i = (long)blockIdx.x * nt + tid; i < slot; i += (long)gridDim.x * nt) nxt[i] = (A)0;
  if (lead && tid == 0) {
    state[tl.parity ? ST_ROUND : ST_ROUND_ALT] = e + 1;
    if (e > 0) state[ST_EXECUTED] += 1;
    if (stop) state[ST_DONE] = 1;
  }
  if (lead && e == 0)  // launch 0: w_0 (the value every block just read) for launch 1's lead
    for (long c = tid; c < d; c += nt) cw[c] = wl[c];
  return stop;
}

// ------------------------------------------------------------------------------------------
// K4/K5/K6 — fused minibatch loss + gradient partials
// ------------------------------------------------------------------------------------------
// Sum over aligned segments of L lanes (L = 8 or 16) with DPP; every lane of a segment gets the
// segment's total. Quad xor1 / xor2 → row_half_mirror (8) → row_mirror (16).
template <int L>
__device__ __forceinline__ float seg_sum_dpp(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror: quads of an 8-lane half swap
  if constexpr (L == 16) v += dpp_mov<0x140>(v);  // row_mirror: 8-lane halves of a row swap
  return v;
}

// register-light shapes are capped at 128 VGPRs (4 waves per SIMD) so that two 8-wave blocks
// share a CU (the 512-block grids); everything else keeps the compiler's choice and runs one
// block per CU — under the 128 cap the row loop spills to scratch, and every spill reload is a
// vmcnt(0) in the loop. (Round 5's code-object audit found the old 64-byte one-row cap spilling
// 171–235 VGPRs for bf16 rows of 1025–4096 and fp64 rows; fp64 accumulators never take the cap.)
template <typename T, int EPC, int CPL, int U>
constexpr int glm_min_waves() {
  return sizeof(T) <= 4 && ((U == 1 && CPL * EPC * (int)sizeof(T) <= 32) || (U == 2 && CPL * EPC * (int)sizeof(T) <= 16))
             ? 4
             : 1;
}

// One 16-byte-per-lane LDS-DMA load (global_load_lds_dwordx4 … nt): lane i's 16 bytes land at LDS
// byte address lds + 16·i; no VGPR is written, the load counts in vmcnt and the caller waits for
// it itself (hipcc does not count asm loads). M0 (the LDS base) is compiler-reserved: saved and
// restored inside the same statement (cdna_hip_programming.md §5.7, LDS-DMA recipe).
__device__ __forceinline__ void dma16_nt(const void* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds)
               : "memory");
}

// X / y / wt are deliberately NOT __restrict__: with restrict the compiler may move the row
// prefetch loads below the compiler fence that pins them ahead of the math (see the row loop).
//
// Row schedule: wave slot gw = b·WPB + wave of the W = NB·WPB slots reads rows start + gw + j·W,
// U rows per step, two steps in flight. (Round 3 measured, and removed again, four alternatives
// on the flagship shape — a dynamic chunk-claim schedule, claimed row pairs after a static prefix,
// per-XCD L2 accumulator replicas, and a tail prefetch of the next round's rows; all exact, all
// slower: profiles/r3/lr_{dyn_schedule,pair_schedule,l2acc,tail_prefetch_timegated}_ab_1gpu.jsonl.)
template <typename T, int EPC, int CPL, int U, int WPB, bool NT, int DEPTH = 0>
__global__ __launch_bounds__(WPB * 64, (glm_min_waves<T, EPC, CPL, U>())) void glm_round_kernel(
    const T* X, long ld, const typename AccOf<T>::type* y,
    const typename AccOf<T>::type* wt, typename AccOf<T>::type* coef,
    long n, int d, long B, int loss, int* state, typename AccOf<T>::type* partials, GlmTail tl) {
  typedef typename AccOf<T>::type A;
  const long long t_start = tl.trace ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
  int e;
  if (tl.defer) {
    if (state[ST_DONE]) return;
    e = state[tl.parity ? ST_ROUND_ALT : ST_ROUND];
  } else if (!round_running(state, e)) return;
  long start = 0, end = 0;  // a rank with no rows (or a zero local batch) still joins the tail
  if (n > 0 && B > 0) {
    // batches per pass: precomputed by the launcher (a 64-bit division per wave otherwise)
    const unsigned P = tl.nbatch > 0 ? (unsigned)tl.nbatch : (unsigned)((n + B - 1) / B);
    start = (long)((unsigned)e % P) * B;
    end = start + B < n ? start + B : n;
  }

  const int lane = threadIdx.x & 63;
  // wave id made provably wave-uniform so row indices are scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = d / EPC;
  const long W = (long)gridDim.x * WPB;
  const long gw = (long)blockIdx.x * WPB + wave;

  // bf16 rows: packed fp32 math on {lo, hi} pairs (one dword = two bf16, widened exactly by a
  // shift / a mask): the dot and the gradient axpy are one v_pk_fma_f32 per pair each
  constexpr bool kPacked = sizeof(T) == 2 && EPC % 2 == 0;
  typedef float f2_t __attribute__((ext_vector_type(2)));
  constexpr int EP = kPacked ? EPC / 2 : 1;
  A w[CPL][EPC];
  A acc[CPL][EPC];
  f2_t w2[CPL][EP], acc2[CPL][EP];  // packed-pair views used by the bf16 path
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
#pragma unroll
    for (int i = 0; i < EPC; ++i) acc[k][i] = (A)0;
#pragma unroll
    for (int i = 0; i < EP; ++i) acc2[k][i] = f2_t{0.f, 0.f};
  }
  // coefficient slices (L2-hot), fetched after the first row loads are on their way
  extern __shared__ __align__(16) unsigned char smem_w[];
  A* wdef = reinterpret_cast<A*>(smem_w + tl.wl_off);  // deferred mode: w_e, built by the prologue
  // the same image through an LDS-typed pointer: generic (flat) loads would count in vmcnt AND
  // lgkmcnt, and one still pending at the row loop's header turns its counted waits into vmcnt(0)
  typedef __attribute__((address_space(3))) A lds_acc_t;
  const lds_acc_t* wlds = (const lds_acc_t*)(smem_w + tl.wl_off);
  auto load_w = [&]() {
    if (tl.defer) {
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        if constexpr (kPacked) {
#pragma unroll
          for (int i = 0; i < EP; ++i)
            w2[k][i] = c < nch ? f2_t{(float)wlds[c * EPC + 2 * i], (float)wlds[c * EPC + 2 * i + 1]} : f2_t{0.f, 0.f};
        } else {
#pragma unroll
          for (int i = 0; i < EPC; ++i) w[k][i] = c < nch ? wlds[c * EPC + i] : (A)0;
        }
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = lane + 64 * k;
      if constexpr (kPacked) {
#pragma unroll
        for (int i = 0; i < EP; ++i)
          w2[k][i] = c < nch ? f2_t{(float)coef[c * EPC + 2 * i], (float)coef[c * EPC + 2 * i + 1]} : f2_t{0.f, 0.f};
      } else {
#pragma unroll
        for (int i = 0; i < EPC; ++i) w[k][i] = c < nch ? coef[c * EPC + i] : (A)0;
      }
    }
  };
  A wsum = 0, lsum = 0;

  // Software pipeline, manually unrolled by two so the compiler keeps the next batch's loads in
  // flight under counted vmcnt waits (a loop-carried register copy, or a conditional load, would
  // force vmcnt(0)). All loads are unconditional: rows past the batch end are clamped to the
  // wave's current (just-read, L2-hot) row and masked by a zero weight; lanes past the last
  // chunk read an in-row chunk and meet a zero coefficient / are never written back.
  Chunk<T, EPC> xa[U][CPL], xb[U][CPL];
  A ya[U], wa[U], yb[U], wb[U];
  bool va[U], vb[U];
  const bool has_wt = wt != nullptr;
  const A* wsrc = has_wt ? wt : y;
  // Labels and weights of this wave's rows j = 0, 1, ... (row r_first + j·W) arrive 64 at a
  // time, one per lane, by ONE vector load each, and are read out with readlane. Scalar loads
  // per row would put every label behind an lgkmcnt(0) drain (SMEM returns out of order), i.e.
  // a full memory latency per row pair; the vector loads are ordered with the row loads.
  const long r_first = start + gw;
  A ylab = (A)0, wlab = (A)1;
  auto load_labels = [&](long j0) {
    long rr = r_first + (j0 + lane) * W;
    rr = rr < end ? rr : (end > 0 ? end - 1 : 0);
    ylab = y[rr];
    wlab = wsrc[rr];  // wsrc = wt, or y as a harmless stand-in (replaced by 1 in process)
  };
  auto lane_val = [&](A v, int l) -> A {
    if constexpr (sizeof(A) == 4) {
      return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
    } else {
      const long long b = __double_as_longlong(v);
      const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
      const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
      return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    }
  };
  // rows r0 + u·W (u < U) are rows j0 + u of this wave; U divides 64, so a batch never
  // straddles a label refill
  auto load_rows = [&](long r0, long j0, long rsafe, Chunk<T, EPC> (&dst)[U][CPL], A (&yy)[U], A (&ww)[U],
                       bool (&vv)[U]) {
    if ((j0 & 63) == 0 && j0 > 0) load_labels(j0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long ru0 = r0 + u * W;
      const bool ok = ru0 < end;
      const long ru = ok ? ru0 : rsafe;
      vv[u] = ok;
      const T* row = X + ru * ld;
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        if constexpr (NT) load_chunk_nt<T, EPC>(row + (c < nch ? c : nch - 1) * EPC, dst[u][k]);
        else load_chunk<T, EPC>(row + (c < nch ? c : nch - 1) * EPC, dst[u][k]);
      }
    }
    // after the row loads: reading the labels waits only for the (older) label load
#pragma unroll
    for (int u = 0; u < U; ++u) {
      yy[u] = lane_val(ylab, (int)((j0 + u) & 63));
      ww[u] = lane_val(wlab, (int)((j0 + u) & 63));
    }
  };
  auto process = [&](Chunk<T, EPC> (&x)[U][CPL], A (&yy)[U], A (&ww)[U], bool (&vv)[U]) {
    if constexpr (kPacked) {
      f2_t xf[U][CPL][EP];
      A dot[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        f2_t s2[2] = {{0.f, 0.f}, {0.f, 0.f}};  // two chains: half the dependent-FMA latency
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const uint32_t* q = reinterpret_cast<const uint32_t*>(x[u][k].v);
#pragma unroll
          for (int i = 0; i < EP; ++i) {
            xf[u][k][i] = f2_t{__uint_as_float(q[i] << 16), __uint_as_float(q[i] & 0xffff0000u)};
            s2[i & 1] = __builtin_elementwise_fma(xf[u][k][i], w2[k][i], s2[i & 1]);
          }
        }
        const f2_t st = s2[0] + s2[1];
        dot[u] = st.x + st.y;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) dot[u] = wave_sum_dpp(dot[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        A l, m;
        const A wu = has_wt ? ww[u] : (A)1;
        loss_and_mult(loss, dot[u], yy[u], wu, l, m);
        if (!vv[u]) { l = (A)0; m = (A)0; }
        wsum += vv[u] ? wu : (A)0;
        lsum += l;
        const f2_t m2 = {m, m};
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
          for (int i = 0; i < EP; ++i) acc2[k][i] = __builtin_elementwise_fma(m2, xf[u][k][i], acc2[k][i]);
      }
    } else {
      A dot[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        A s = 0;
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
          for (int i = 0; i < EPC; ++i) s += (A)Ld<T>::f(x[u][k].v[i]) * w[k][i];
        dot[u] = s;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) dot[u] = wave_sum_dpp(dot[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        A l, m;
        const A wu = has_wt ? ww[u] : (A)1;
        loss_and_mult(loss, dot[u], yy[u], wu, l, m);
        if (!vv[u]) { l = (A)0; m = (A)0; }
        wsum += vv[u] ? wu : (A)0;
        lsum += l;
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
          for (int i = 0; i < EPC; ++i) acc[k][i] += m * (A)Ld<T>::f(x[u][k].v[i]);
      }
    }
  };
  if constexpr (DEPTH > 0) {
    // ---- LDS-DMA row path (bf16 rows of 65–128 16-byte chunks). Each wave owns a ring of DEPTH
    // steps × U rows × 2 KiB in LDS; row loads are global_load_lds_dwordx4 … nt (two per row:
    // chunks lane and lane + 64), so DEPTH − 1 steps stay in flight through the math whatever
    // the registers hold, and the loads never write VGPRs (the streaming probe: 31.7 µs per 200 MB
    // batch vs 33.3 for 16-byte register loads, profiles/r4/lr_probe_lds.log). A step's rows are
    // read back with ds_read_b128 into the same per-lane chunk layout the register path uses.
    static_assert(sizeof(T) == 2 && EPC == 8 && CPL == 2, "LDS-DMA ring: bf16 rows of 65-128 chunks");
    extern __shared__ __align__(16) unsigned char smem_r[];
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) u32x4_t lds_u4_t;
    unsigned char* ring_w = smem_r + tl.ring_off + (long)wave * (DEPTH * U * 2048);
    const unsigned ring_a = __builtin_amdgcn_readfirstlane((unsigned)(size_t)ring_w);
    const long nrw = r_first < end ? (end - r_first + W - 1) / W : 0;  // rows of this wave
    const long nst = (nrw + U - 1) / U;                                 // steps of this wave
    const int c1 = lane + 64 < nch ? lane + 64 : nch - 1;
    auto issue = [&](long t) {
      const unsigned base = ring_a + (unsigned)((t % DEPTH) * U) * 2048u;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long ru = r_first + (t * U + u) * W;
        ru = ru < end ? ru : r_first;  // past the wave's rows: a valid row again, masked below
        const T* row = X + ru * ld;
        dma16_nt(row + lane * EPC, base + u * 2048u);
        dma16_nt(row + c1 * EPC, base + u * 2048u + 1024u);
      }
    };
    auto read = [&](long t, Chunk<T, EPC> (&x)[U][CPL], A (&yy)[U], A (&ww)[U], bool (&vv)[U]) {
      const long j0 = t * U;
      if ((j0 & 63) == 0 && j0 > 0) load_labels(j0);
      const unsigned char* sl = ring_w + (t % DEPTH) * U * 2048;
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const u32x4_t v = *(const lds_u4_t*)(sl + u * 2048 + k * 1024 + lane * 16);
          __builtin_memcpy(x[u][k].v, &v, 16);
        }
        vv[u] = j0 + u < nrw;
        yy[u] = lane_val(ylab, (int)((j0 + u) & 63));
        ww[u] = lane_val(wlab, (int)((j0 + u) & 63));
      }
    };
    if (nst > 0) {
      load_labels(0);
#pragma unroll
      for (int t = 0; t < DEPTH - 1; ++t)
        if (t < nst) issue(t);
    }
    if (tl.defer && (tl.mode == TAIL_XGMI ? defer_prologue_xgmi<A>(tl, coef, state, e, d, wdef)
                                          : defer_prologue<A>(tl, coef, state, e, d, wdef))) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the wave exits
      return;
    }
    if (nst > 0) {
      load_w();
      for (long t = 0; t < nst; ++t) {
        // step t + DEPTH − 1 goes into the slot step t − 1 was read from (its ds_reads are done:
        // their values fed step t − 1's math)
        if (t + DEPTH - 1 < nst) {
          issue(t + DEPTH - 1);
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * U * (DEPTH - 1)) : "memory");  // step t landed
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        read(t, xa, ya, wa, va);
        process(xa, ya, wa, va);
      }
    }
    // the epilogue's LDS buffers alias the ring: every wave of the block is past its last read
    __syncthreads();
  } else {
  const long step = (long)U * W;
  long r = start + gw;
  // (Round 4 also measured issuing a buffer's next loads right after widening its bf16 step to
  // fp32 pairs, before the step's math: 38.35 vs 38.33 µs — the loop is not limited by where the
  // loads go out, profiles/r4/lr_early_issue_ab_1gpu.jsonl.)
  // steps of U rows this wave owns; the loop runs them in pairs (xa, xb) with ONE exit test per
  // pair at the latch. (A `break` after each half gives the structurizer a flow block whose
  // conditional back edge carries the first half's pending loads into the header, where the
  // waitcnt pass then puts a vmcnt(0) at the top of EVERY iteration: round 3's loop had it, so the
  // next step's loads only went out once the current step had landed.)
  const long nst = r < end ? ((end - r + W - 1) / W + U - 1) / U : 0;
  if (nst > 0) {
    // the first TWO steps go out before the deferred prologue, whose sc1 reads of the previous
    // round's accumulator and SGD update take a few microseconds: HBM streams meanwhile
    load_labels(0);  // first: load_rows reads the labels right after issuing its row loads
    load_rows(r, 0, r, xa, ya, wa, va);
    load_rows(r + step, U, r, xb, yb, wb, vb);
  }
  // deferred mode: complete the previous round while the first rows are in flight
  if (tl.defer && (tl.mode == TAIL_XGMI ? defer_prologue_xgmi<A>(tl, coef, state, e, d, wdef)
                                        : defer_prologue<A>(tl, coef, state, e, d, wdef)))
    return;
  if (nst > 0) {
    load_w();
    // nothing in flight at the loop header but the back edge's own loads (the deferred prologue
    // has already waited for these)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    long t = 0;
    for (; t + 2 <= nst; t += 2) {
      // steps t (xa) and t + 1 (xb) are loaded; a buffer's next step (t + 2, t + 3) goes out as
      // soon as its math is done (rows past the wave's last one are clamped to a valid row and
      // masked). The empty asm + sched_barrier pin each load batch between the two math blocks:
      // without them the compiler sinks loads into the math to recycle registers.
      process(xa, ya, wa, va);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      load_rows(r + 2 * step, (t + 2) * U, r, xa, ya, wa, va);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      process(xb, yb, wb, vb);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      load_rows(r + 3 * step, (t + 3) * U, r, xb, yb, wb, vb);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      r += 2 * step;
    }
    if (t < nst) process(xa, ya, wa, va);  // odd step count: the last step is in xa
  }
  }

  if (tl.trace) {
    // every wave's rows are in: stamp once the whole block got here (the LDS reduction below
    // has its own barrier)
    __syncthreads();
    if (threadIdx.x == 0) {
      long long* tr = tl.trace + (long)blockIdx.x * 4;
      tr[0] = t_start;
      tr[1] = (long long)__builtin_amdgcn_s_memrealtime();
      unsigned hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      unsigned xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      tr[3] = ((long long)xcc << 32) | hw;
    }
  }
  if constexpr (kPacked) {
#pragma unroll
    for (int k = 0; k < CPL; ++k)
#pragma unroll
      for (int i = 0; i < EP; ++i) {
        acc[k][2 * i] = acc2[k][i].x;
        acc[k][2 * i + 1] = acc2[k][i].y;
      }
  }

  extern __shared__ __align__(16) unsigned char smem_raw[];
  A* buf = reinterpret_cast<A*>(smem_raw);          // [WPB][d] (flat) or [WPB/2][d] (tree)
  const bool flat = tl.mode != TAIL_PARTIALS && !tl.det && tl.flat_lds;
  A* lw = buf + (flat ? WPB : WPB / 2) * (long)d;   // [WPB][2]
  int* sflag = reinterpret_cast<int*>(lw + WPB * 2);
  if (lane == 0) { lw[wave * 2] = wsum; lw[wave * 2 + 1] = lsum; }
  if (flat) {
    // atomic tail, one barrier: every wave parks its row in LDS, then each thread sums its
    // columns over the waves (fixed order) and adds them to tl.acc (256 contiguous bytes per
    // wave-instruction)
    A* mine = buf + (long)wave * d;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = lane + 64 * k;
      if (c < nch)
#pragma unroll
        for (int i = 0; i < EPC; ++i) mine[c * EPC + i] = acc[k][i];
    }
    __syncthreads();
    // replica b mod acc_reps: at most ceil(nb / reps) adders per address (float atomics keep
    // their full rate up to ~32 adders per address; 256 on one 4 KB row serialise)
    const int rep = (int)(blockIdx.x % (tl.acc_reps > 1 ? tl.acc_reps : 1));
    A* gacc = (A*)tl.acc + (long)rep * tl.acc_ld + (tl.defer ? (long)(e % 3) * ACC_MAX_REPS * tl.acc_ld : 0L);
    const long stride = d + 2;
    for (long c = threadIdx.x; c < stride; c += blockDim.x) {
      A v = (A)0;
      if (c < d) {
#pragma unroll
        for (int q = 0; q < WPB; ++q) v += buf[(long)q * d + c];
      } else {
#pragma unroll
        for (int q = 0; q < WPB; ++q) v += lw[q * 2 + (int)(c - d)];
      }
      atomicAdd(gacc + c, v);
    }
    if (tl.trace) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) tl.trace[(long)blockIdx.x * 4 + 2] = (long long)__builtin_amdgcn_s_memrealtime();
    }
    if (tl.defer) return;  // launch e + 1 completes this round
    glm_round_tail_atomic<A>(tl, d, coef, state, e, buf, sflag);
    return;
  }
  // fixed-order tree across the block's waves through LDS
#pragma unroll
  for (int half = WPB / 2; half >= 1; half >>= 1) {
    if (wave >= half && wave < 2 * half) {
      A* dst = buf + (long)(wave - half) * d;
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        if (c < nch)
#pragma unroll
          for (int i = 0; i < EPC; ++i) dst[c * EPC + i] = acc[k][i];
      }
    }
    __syncthreads();
    if (wave < half) {
      const A* src = buf + (long)wave * d;
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        if (c < nch)
#pragma unroll
          for (int i = 0; i < EPC; ++i) acc[k][i] += src[c * EPC + i];
      }
    }
    __syncthreads();
  }
  if (tl.mode != TAIL_PARTIALS && !tl.det) {
    // atomic tail (rows too wide for the flat LDS image): the tree's result goes to LDS row 0,
    // then to `acc`
    if (wave == 0) {
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        if (c < nch)
#pragma unroll
          for (int i = 0; i < EPC; ++i) buf[c * EPC + i] = acc[k][i];
      }
      if (lane == 0) {
        A ws = 0, ls = 0;
        for (int q = 0; q < WPB; ++q) { ws += lw[q * 2]; ls += lw[q * 2 + 1]; }
        buf[d] = ws;
        buf[d + 1] = ls;
      }
    }
    __syncthreads();
    A* gacc = (A*)tl.acc + (long)(blockIdx.x % (tl.acc_reps > 1 ? tl.acc_reps : 1)) * tl.acc_ld;
    for (long c = threadIdx.x; c < d + 2; c += blockDim.x) atomicAdd(gacc + c, buf[c]);
    glm_round_tail_atomic<A>(tl, d, coef, state, e, buf, sflag);
    return;
  }
  if (wave == 0) {
    A* out = partials + (long)blockIdx.x * (d + 2);
    // sc1 (write-through) stores when the fused tail consumes the row inside this launch
    const bool wt1 = tl.mode != TAIL_PARTIALS;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = lane + 64 * k;
      if (c < nch)
#pragma unroll
        for (int i = 0; i < EPC; ++i) {
          if (wt1) st_agent(out + c * EPC + i, acc[k][i]);
          else out[c * EPC + i] = acc[k][i];
        }
    }
    if (lane == 0) {
      A ws = 0, ls = 0;
      for (int q = 0; q < WPB; ++q) { ws += lw[q * 2]; ls += lw[q * 2 + 1]; }
      if (wt1) {
        st_agent(out + d, ws);
        st_agent(out + d + 1, ls);
      } else {
        out[d] = ws;
        out[d + 1] = ls;
      }
    }
  }
  if (tl.mode == TAIL_PARTIALS) return;
  glm_round_tail_det<A>(tl, partials, d, coef, state, e, buf, sflag);
}

// ------------------------------------------------------------------------------------------
// Deterministic two-stage reduction of the block partials [nparts][d+2]:
//  stage 1 (many blocks): column c of row-group g = Σ_{p in group g, fixed order} partials[p][c]
//  stage 2 (fused with the update): Σ_g stage1[g][c] in fixed order.
// Every load in a stage is independent (fully unrolled) so each stage costs ~one memory latency.
// ------------------------------------------------------------------------------------------
constexpr int RED_G = 32;  // partial rows per stage-1 group (<= 512 partials -> <= 16 groups)

template <typename A>
__global__ __launch_bounds__(256) void glm_reduce_stage1_kernel(const A* __restrict__ partials, int nparts, int d,
                                                                A* __restrict__ stage1, const int* __restrict__ state) {
  int e;
  if (!round_running(state, e)) return;
  const long stride = d + 2;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= stride) return;
  const int p0 = blockIdx.y * RED_G;
  A v[RED_G];
#pragma unroll
  for (int q = 0; q < RED_G; ++q) v[q] = (p0 + q < nparts) ? partials[(long)(p0 + q) * stride + c] : (A)0;
  A s = 0;
#pragma unroll
  for (int q = 0; q < RED_G; ++q) s += v[q];
  stage1[(long)blockIdx.y * stride + c] = s;
}

template <typename A>
__device__ __forceinline__ A sum_groups(const A* __restrict__ stage1, int ngroups, long stride, long c) {
  A v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = q < ngroups ? stage1[(long)q * stride + c] : (A)0;
  A s = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) s += v[q];
  return s;
}


template <typename A>
__global__ __launch_bounds__(256) void glm_reduce_update_kernel(
    const A* __restrict__ stage1, int ngroups, int d, A* __restrict__ coef, A* __restrict__ feedback,
    int* __restrict__ state, int max_iter, A tol, A lr, A reg, A en) {
  int e;
  const bool run = round_running(state, e);
  if (!run) {
    arrive_and_advance(state, e, false, 0);
    return;
  }
  const long stride = d + 2;
  const int c = blockIdx.x * 256 + threadIdx.x;
  // Σweight / Σloss: two lanes of wave 0 reduce them (fixed order) while every thread reduces its
  // own column; broadcast through LDS
  __shared__ A wl[2];
  if (threadIdx.x < 2) wl[threadIdx.x] = sum_groups(stage1, ngroups, stride, d + threadIdx.x);
  const A g = c < d ? sum_groups(stage1, ngroups, stride, c) : (A)0;
  __syncthreads();
  const A W = wl[0];
  const A L = wl[1];
  const bool cont = (e + 1 < max_iter) && (L / W > tol);
  if (c < d) {
    coef[c] = sgd_apply<A>(coef[c], g, W, lr, reg, en);
    if (feedback) feedback[c] = g;
  }
  if (feedback && blockIdx.x == 0 && threadIdx.x == 0) { feedback[d] = W; feedback[d + 1] = L; }
  arrive_and_advance(state, e, cont, 1);
}

template <typename A>
__global__ __launch_bounds__(256) void glm_reduce_kernel(const A* __restrict__ stage1, int ngroups, int d,
                                                         A* __restrict__ feedback, const int* __restrict__ state) {
  int e;
  if (!round_running(state, e)) return;
  const long stride = d + 2;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < stride) feedback[c] = sum_groups(stage1, ngroups, stride, c);
}

template <typename A>
__global__ __launch_bounds__(256) void glm_update_kernel(const A* __restrict__ feedback, int d, A* __restrict__ coef,
                                                         int* __restrict__ state, int max_iter, A tol, A lr, A reg,
                                                         A en) {
  int e;
  const bool run = round_running(state, e);
  if (!run) {
    arrive_and_advance(state, e, false, 0);
    return;
  }
  const A W = feedback[d];
  const A L = feedback[d + 1];
  const bool cont = (e + 1 < max_iter) && (L / W > tol);
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < d; c += gridDim.x * blockDim.x)
    coef[c] = sgd_apply<A>(coef[c], feedback[c], W, lr, reg, en);
  arrive_and_advance(state, e, cont, 1);
}

// ------------------------------------------------------------------------------------------
// prediction: dot + model-specific epilogue (LogisticRegressionModel.java:165-169,
// LinearSVCModel.java:170-174, LinearRegressionModel.java:158-160)
// mode 0: LR   pred = dot>=0, raw = [1-p, p], p = 1-1/(1+e^dot)
// mode 1: SVC  pred = dot>=thr, raw = [dot, -dot]
// mode 2: LinReg pred = dot (raw unused)
// ------------------------------------------------------------------------------------------
template <typename T, int EPC, int CPL>
__global__ __launch_bounds__(256) void glm_predict_kernel(const T* __restrict__ X, long ld, long n, int d,
                                                          const typename AccOf<T>::type* __restrict__ coef, int mode,
                                                          double thr, double* __restrict__ pred,
                                                          double* __restrict__ raw) {
  typedef typename AccOf<T>::type A;
  const int lane = threadIdx.x & 63;
  const long gw = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long W = ((long)gridDim.x * blockDim.x) >> 6;
  const int nch = d / EPC;
  A w[CPL][EPC];
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c = lane + 64 * k;
#pragma unroll
    for (int i = 0; i < EPC; ++i) w[k][i] = c < nch ? coef[c * EPC + i] : (A)0;
  }
  for (long r = gw; r < n; r += W) {
    const T* row = X + r * ld;
    A s = 0;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = lane + 64 * k;
      if (c < nch) {
        Chunk<T, EPC> x;
        load_chunk<T, EPC>(row + c * EPC, x);
#pragma unroll
        for (int i = 0; i < EPC; ++i) s += (A)Ld<T>::f(x.v[i]) * w[k][i];
      }
    }
    s = wave_sum(s);
    if (lane == 0) {
      const double dot = (double)s;
      if (mode == 0) {
        const double p = 1.0 - 1.0 / (1.0 + exp(dot));
        pred[r] = dot >= 0 ? 1.0 : 0.0;
        raw[2 * r] = 1.0 - p;
        raw[2 * r + 1] = p;
      } else if (mode == 1) {
        pred[r] = dot >= thr ? 1.0 : 0.0;
        raw[2 * r] = dot;
        raw[2 * r + 1] = -dot;
      } else {
        pred[r] = dot;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Wide dense rows: a block's 8 waves split every row's columns
// ------------------------------------------------------------------------------------------
// Rows wider than one wave's registers hold (bf16 d > 4096, fp32 > 2048, fp64 > 1024) are cut
// into 8 column slices, one per wave of the block, each slice up to 64·CPL chunks of EPC: the block
// walks its rows (block b: rows b, b + G, …) RU at a time (2; 1 for 8 chunks per lane, whose two
// row buffers would spill), two steps in flight, every wave loads and dots its slice,
// the 8 partial dots meet in LDS (one barrier per step, double-buffered) and are summed in
// wave order, so every wave holds the same dot, multiplier and loss; each wave then accumulates
// its slice of the gradient in registers. At the end the slices (disjoint) form the block's
// gradient row in LDS and go into the accumulator with coalesced no-return atomics; the atomic
// tail (ticket, last block) completes the round. One read of the batch per round, against two
// library GEMVs (X_b·w, then X_bᵀ·m) plus loss and sum kernels on the path this replaces.
constexpr int WIDE_WAVES = 8;

template <typename T, int EPC, int CPL, int RU>
__global__ __launch_bounds__(WIDE_WAVES * 64) void glm_round_wide_kernel(
    const T* __restrict__ X, long ld, const typename AccOf<T>::type* __restrict__ y,
    const typename AccOf<T>::type* __restrict__ wt, typename AccOf<T>::type* __restrict__ coef, long n, int d, long B,
    int loss, int* __restrict__ state, GlmTail tl) {
  typedef typename AccOf<T>::type A;
  extern __shared__ __align__(16) unsigned char smem_wide[];
  A* sbuf = reinterpret_cast<A*>(smem_wide);  // [d + 2]: the block's gradient row, then the tail's
  int* sflag = reinterpret_cast<int*>(sbuf + d + 2);
  __shared__ A pdot[2][WIDE_WAVES][RU];
  int e;
  if (!round_running(state, e)) return;
  long start = 0, end = 0;
  if (n > 0 && B > 0) {
    const unsigned P = tl.nbatch > 0 ? (unsigned)tl.nbatch : (unsigned)((n + B - 1) / B);
    start = (long)((unsigned)e % P) * B;
    end = start + B < n ? start + B : n;
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = d / EPC;
  const int per = (nch + WIDE_WAVES - 1) / WIDE_WAVES;  // chunks per slice (≤ 64·CPL: host-checked)
  const int c0 = wave * per;
  const int c1 = c0 + per < nch ? c0 + per : nch;
  A w[CPL][EPC], acc[CPL][EPC];
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c = c0 + lane + 64 * k;
#pragma unroll
    for (int i = 0; i < EPC; ++i) {
      w[k][i] = c < c1 ? coef[c * EPC + i] : (A)0;
      acc[k][i] = (A)0;
    }
  }
  const long G = gridDim.x;
  const long r0 = start + blockIdx.x;
  const long nrows = r0 < end ? (end - r0 + G - 1) / G : 0;  // this block's rows
  const bool has_wt = wt != nullptr;
  A wsum = 0, lsum = 0;
  Chunk<T, EPC> xa[RU][CPL], xb[RU][CPL];
  auto load = [&](long j, Chunk<T, EPC> (&x)[RU][CPL]) {  // rows j … j + RU − 1 of this block
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const long jj = j + u < nrows ? j + u : (nrows > 0 ? nrows - 1 : 0);
      const T* row = X + (r0 + jj * G) * ld;
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int c = c0 + lane + 64 * k;
        load_chunk_nt<T, EPC>(row + (c < c1 ? c : (c0 < c1 ? c0 : 0)) * EPC, x[u][k]);
      }
    }
  };
  auto process = [&](long j, Chunk<T, EPC> (&x)[RU][CPL], int par) {
    A part[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      A s = 0;
#pragma unroll
      for (int k = 0; k < CPL; ++k)
#pragma unroll
        for (int i = 0; i < EPC; ++i) s += (A)Ld<T>::f(x[u][k].v[i]) * w[k][i];
      part[u] = wave_sum(s);
    }
    if (lane == 0)
#pragma unroll
      for (int u = 0; u < RU; ++u) pdot[par][wave][u] = part[u];
    __syncthreads();  // (double-buffered by step parity: one barrier per step)
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      A dot = 0;
#pragma unroll
      for (int q = 0; q < WIDE_WAVES; ++q) dot += pdot[par][q][u];
      const bool ok = j + u < nrows;
      const long r = r0 + (j + u) * G;
      A l, m;
      const A wu = ok ? (has_wt ? wt[r] : (A)1) : (A)0;
      loss_and_mult(loss, dot, ok ? y[r] : (A)0, wu, l, m);
      if (!ok) { l = (A)0; m = (A)0; }
      if (wave == 0) {
        wsum += wu;
        lsum += l;
      }
#pragma unroll
      for (int k = 0; k < CPL; ++k)
#pragma unroll
        for (int i = 0; i < EPC; ++i) acc[k][i] += m * (A)Ld<T>::f(x[u][k].v[i]);
    }
  };
  if (nrows > 0) {  // (nrows is block-uniform: every wave makes the same barrier calls)
    load(0, xa);
    load(RU, xb);
    int par = 0;
    for (long j = 0; j < nrows; j += 2 * RU) {
      process(j, xa, par);
      par ^= 1;
      load(j + 2 * RU, xa);  // rows past the block's last are clamped to it and masked
      if (j + RU < nrows) {
        process(j + RU, xb, par);
        par ^= 1;
        load(j + 3 * RU, xb);
      }
    }
  }
  // the block's gradient row: the waves' disjoint slices, then Σweight / Σloss
  for (long c = threadIdx.x; c < d + 2; c += blockDim.x) sbuf[c] = (A)0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c = c0 + lane + 64 * k;
    if (c < c1)
#pragma unroll
      for (int i = 0; i < EPC; ++i) sbuf[c * EPC + i] = acc[k][i];
  }
  if (wave == 0 && lane == 0) {  // (every lane of wave 0 summed the same row values)
    sbuf[d] = wsum;
    sbuf[d + 1] = lsum;
  }
  __syncthreads();
  const int rep = (int)(blockIdx.x % (tl.acc_reps > 1 ? tl.acc_reps : 1));
  A* gacc = (A*)tl.acc + (long)rep * tl.acc_ld;
  for (long c = threadIdx.x; c < d + 2; c += blockDim.x) atomicAdd(gacc + c, sbuf[c]);
  glm_round_tail_atomic<A>(tl, d, coef, state, e, sbuf, sflag);
}

// ---------------------------- host-side dispatch ------------------------------------------
constexpr int WPB = 8;

// Grid spreading: the dispatcher may stack up to 32 waves of this kernel on one CU while others
// idle; requesting enough LDS per block that at most ceil(nblocks / 256) blocks fit a CU makes
// every CU take its equal share (measured −11 % round time at 512 blocks). g_lds_pad < 0 = auto.
// Non-temporal row loads (`flags & 1`) for batches streamed once per pass (−12 %, measured).
static long g_lds_pad = -1;
static int g_nt = -1;
static int g_acc_reps = 4;  // atomic-tail accumulator replicas (A/B knob, <= ACC_MAX_REPS)
static int g_ticket2 = 0;   // two-level tickets (A/B knob)
static long long* g_trace = nullptr;  // per-block timestamps of the next launches (diagnostics)

static int g_dma_depth = 0;  // LDS-DMA row ring depth in steps (0 = 16-byte register loads)

template <typename T, int EPC, int CPL, int U, int DEPTH>
int launch_grad_k(const void* X, long ld, const void* y, const void* wt, void* coef, long n, int d, long B, int loss,
                  int* state, void* partials, int nblocks, GlmTail t2, bool nt, hipStream_t s) {
  typedef typename AccOf<T>::type A;
  // epilogue LDS: [WPB or WPB/2][d] wave rows | [WPB][2] | ticket flag; the DMA ring (if any)
  // starts at 0 and the epilogue buffers alias it; the deferred mode's w image follows both
  const size_t tail = (size_t)(t2.flat_lds ? WPB : WPB / 2) * d * sizeof(A) + WPB * 2 * sizeof(A) + 16;
  const size_t ring = (size_t)WPB * DEPTH * U * 2048;
  size_t shmem = tail > ring ? tail : ring;
  t2.ring_off = 0;
  if (t2.defer) {
    t2.wl_off = (int)((shmem + 15) & ~(size_t)15);
    shmem = (size_t)t2.wl_off + (size_t)d * sizeof(A);
    if (t2.mode == TAIL_XGMI) {  // the lead block's exchange row (never aliased with the ring)
      t2.xb_off = (int)((shmem + 15) & ~(size_t)15);
      shmem = (size_t)t2.xb_off + (size_t)(d + 2) * sizeof(A);
    }
  }
  if (g_lds_pad >= 0) {
    shmem += (size_t)g_lds_pad;
  } else {
    const long per_cu = (nblocks + NUM_CU - 1) / NUM_CU;
    if (per_cu <= 3) {
      const size_t want = (size_t)(LDS_PER_CU / (per_cu + 1) + 1024);
      if (shmem < want) shmem = want;
    }
  }
  if (shmem > (size_t)LDS_PER_CU) return -8;
  if constexpr (EPC * sizeof(T) == 16 && sizeof(T) == 2) {
    if (nt) {
      hipLaunchKernelGGL((glm_round_kernel<T, EPC, CPL, U, WPB, true, DEPTH>), dim3(nblocks), dim3(WPB * 64), shmem, s,
                         (const T*)X, ld, (const A*)y, (const A*)wt, (A*)coef, n, d, B, loss, state, (A*)partials, t2);
      return (int)hipGetLastError();
    }
  }
  if constexpr (DEPTH == 0) {
    hipLaunchKernelGGL((glm_round_kernel<T, EPC, CPL, U, WPB, false>), dim3(nblocks), dim3(WPB * 64), shmem, s,
                       (const T*)X, ld, (const A*)y, (const A*)wt, (A*)coef, n, d, B, loss, state, (A*)partials, t2);
    return (int)hipGetLastError();
  }
  return -9;
}

template <typename T, int EPC, int CPL, int U>
int launch_grad_u(const void* X, long ld, const void* y, const void* wt, void* coef, long n, int d, long B, int loss,
                  int* state, void* partials, int nblocks, const GlmTail& tl, int flags, hipStream_t s) {
  typedef typename AccOf<T>::type A;
  GlmTail t2 = tl;
  t2.nbatch = (n > 0 && B > 0) ? (int)((n + B - 1) / B) : 0;
  t2.flat_lds = tl.mode != TAIL_PARTIALS && !tl.det && (size_t)WPB * d * sizeof(A) <= 64 * 1024;
  // the deferred prologue needs the flat atomic tail
  if (t2.defer && (!t2.flat_lds || (tl.mode != TAIL_UPDATE && tl.mode != TAIL_XGMI) || tl.det || tl.cw == nullptr))
    return -7;
  const bool nt = g_nt >= 0 ? g_nt != 0 : (flags & 1) != 0;
  // LDS-DMA ring: bf16 rows of 65–128 16-byte chunks (d 513–1024), 16-byte aligned, non-temporal
#ifndef FMLX_ISA_PROBE_U
  if constexpr (sizeof(T) == 2 && EPC == 8 && CPL == 2) {
    if (g_dma_depth > 0 && nt) {
      switch (g_dma_depth) {
        case 2: return launch_grad_k<T, EPC, CPL, U, 2>(X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, t2, nt, s);
        case 3: return launch_grad_k<T, EPC, CPL, U, 3>(X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, t2, nt, s);
        default: return launch_grad_k<T, EPC, CPL, U, 4>(X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, t2, nt, s);
      }
    }
  }
#endif
  return launch_grad_k<T, EPC, CPL, U, 0>(X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, t2, nt, s);
}

// rows in flight per wave = 2·U (software pipeline); u == 0 picks the default for the shape
template <typename T, int EPC, int CPL>
int launch_grad(int u, const void* X, long ld, const void* y, const void* wt, void* coef, long n, int d, long B,
                int loss, int* state, void* partials, int nblocks, const GlmTail& tl, int flags, hipStream_t s) {
  constexpr int BYTES = CPL * EPC * (int)sizeof(T);
  // default: 4 rows in flight per wave (U = 2) up to 32 bytes per lane, 2 above. Flagship
  // 1000 × bf16 (32 bytes per lane) with the deferred tail, round 3: U=2 on 256 blocks 38.97 µs
  // vs U=1 on 512 blocks 40.09 µs (ops/glm.py round_blocks picks the grid; round 1, before the
  // deferred tail, had measured U=1 faster: 37.9 vs 39.1 µs)
  if (u <= 0) u = BYTES <= 32 ? 2 : 1;
#ifdef FMLX_ISA_PROBE_U  // one row-loop variant only (ISA inspection)
  return launch_grad_u<T, EPC, CPL, FMLX_ISA_PROBE_U>(X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
#endif
  // (compile-time guards: the multi-row variants of wide rows would only exist to spill)
  if constexpr (BYTES <= 32) {
    if (u >= 4)
      return launch_grad_u<T, EPC, CPL, 4>(X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
  }
  if constexpr (BYTES <= 32) {
    if (u >= 2)
      return launch_grad_u<T, EPC, CPL, 2>(X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
  }
  return launch_grad_u<T, EPC, CPL, 1>(X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
}

#ifndef FMLX_ISA_PROBE
template <typename T, int EPC>
int launch_grad_cpl(int cpl, int u, const void* X, long ld, const void* y, const void* wt, void* coef, long n, int d,
                    long B, int loss, int* state, void* partials, int nblocks, const GlmTail& tl, int flags,
                    hipStream_t s) {
  switch (cpl) {
    case 1: return launch_grad<T, EPC, 1>(u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
    case 2: return launch_grad<T, EPC, 2>(u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
    case 4: return launch_grad<T, EPC, 4>(u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
    case 8: return launch_grad<T, EPC, 8>(u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
  }
  return -1;
}

int launch_round(int dtype, int epc, int cpl, int u, const void* X, long ld, const void* y, const void* wt, void* coef,
                 long n, int d, long B, int loss, int* state, void* partials, int nblocks, const GlmTail& tl, int flags,
                 hipStream_t s) {
  if (dtype == DT_BF16) {
    if (epc == 8) return launch_grad_cpl<bf16_t, 8>(cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
    if (epc == 4) return launch_grad_cpl<bf16_t, 4>(cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
    if (epc == 2) return launch_grad_cpl<bf16_t, 2>(cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
    if (epc == 1) return launch_grad_cpl<bf16_t, 1>(cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
  } else if (dtype == DT_F32) {
    if (epc == 4) return launch_grad_cpl<float, 4>(cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
    if (epc == 2) return launch_grad_cpl<float, 2>(cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
    if (epc == 1) return launch_grad_cpl<float, 1>(cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
  } else if (dtype == DT_F64) {
    if (epc == 2) return launch_grad_cpl<double, 2>(cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
    if (epc == 1) return launch_grad_cpl<double, 1>(cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl, flags, s);
  }
  return -1;
}

template <typename T, int EPC, int CPL>
int launch_pred(const void* X, long ld, long n, int d, const void* coef, int mode, double thr, double* pred,
                double* raw, hipStream_t s) {
  long waves = n;
  int blocks = (int)((waves + 3) / 4);
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((glm_predict_kernel<T, EPC, CPL>), dim3(blocks), dim3(256), 0, s, (const T*)X, ld, n, d,
                     (const typename AccOf<T>::type*)coef, mode, thr, pred, raw);
  return (int)hipGetLastError();
}

template <typename T, int EPC>
int launch_pred_cpl(int cpl, const void* X, long ld, long n, int d, const void* coef, int mode, double thr,
                    double* pred, double* raw, hipStream_t s) {
  switch (cpl) {
    case 1: return launch_pred<T, EPC, 1>(X, ld, n, d, coef, mode, thr, pred, raw, s);
    case 2: return launch_pred<T, EPC, 2>(X, ld, n, d, coef, mode, thr, pred, raw, s);
    case 4: return launch_pred<T, EPC, 4>(X, ld, n, d, coef, mode, thr, pred, raw, s);
    case 8: return launch_pred<T, EPC, 8>(X, ld, n, d, coef, mode, thr, pred, raw, s);
  }
  return -1;
}

#endif  // FMLX_ISA_PROBE
}  // namespace

#ifdef FMLX_ISA_PROBE
// ISA inspection builds (hipcc --offload-device-only -S -DFMLX_ISA_PROBE): only the flagship round
// kernel's variants are instantiated, so the .s comes out in seconds, not minutes
FMLX_API int fmlx_glm_isa_probe(int u, const void* X, long ld, const void* y, void* coef, int* state, const GlmTail* tl) {
  return launch_grad<bf16_t, 8, 2>(u, X, ld, y, nullptr, coef, 1, 1000, 1, 0, state, nullptr, 224, *tl, 1, 0);
}
#else

// epc = elements per 16/8/4/2-byte chunk chosen by the host so that d % epc == 0 and rows are
// aligned; cpl = chunks per lane (power of two, 64*cpl*epc >= d).
FMLX_API int fmlx_glm_set_tuning(long lds_pad, int nt) {
  g_lds_pad = lds_pad;
  g_nt = nt;
  return 0;
}

// diagnostics: launches record per-block timestamps into trace[nblocks][4] (null: off)
FMLX_API void fmlx_glm_set_trace(void* trace) {
  g_trace = (long long*)trace;
  fmlx_glm_sparse_set_trace(trace);
}

// ints of the fused round's counter block: the arrival tickets (TAIL_TOP + 1, padded to 128)
FMLX_API int fmlx_glm_cnt_elems() { return 128; }

// LDS-DMA row ring of the fused round (bf16 rows of d 513–1024): depth in steps, 0 = off
FMLX_API int fmlx_glm_set_dma(int depth) {
  if (depth < 0 || depth > 4 || depth == 1) return -1;
  g_dma_depth = depth;
  return 0;
}

FMLX_API int fmlx_glm_set_tail_tuning(int acc_reps, int ticket2) {
  if (acc_reps < 1 || acc_reps > ACC_MAX_REPS) return -1;
  g_acc_reps = acc_reps;
  g_ticket2 = ticket2;
  return 0;
}

// elements of the atomic-tail accumulator for row width d + 2: the deferred mode's ring of 3
// slots of ACC_MAX_REPS replicas (the ticketed tail uses slot 0)
FMLX_API long fmlx_glm_acc_elems(int d) { return 3L * ACC_MAX_REPS * (((long)d + 2 + 63) / 64 * 64); }

FMLX_API int fmlx_glm_grad_partials(int dtype, int epc, int cpl, int u, const void* X, long ld, const void* y,
                                    const void* wt, const void* coef, long n, int d, long B, int loss, const int* state,
                                    void* partials, int nblocks, void* stream) {
  GlmTail tl{};
  tl.mode = TAIL_PARTIALS;
  return launch_round(dtype, epc, cpl, u, X, ld, y, wt, const_cast<void*>(coef), n, d, B, loss,
                      const_cast<int*>(state), partials, nblocks, tl, 0, (hipStream_t)stream);
}

// One whole SGD round in one launch (see the header comment). cnt: int32[17] zero-initialised;
// stage1: [ceil(nblocks/32)][d+2]; feedback: [d+2] (may be null for TAIL_UPDATE / TAIL_XGMI).
// peers/gen/err/spin_limit: the xGMI exchange (TAIL_XGMI only, see parallel/xgmi.py).
FMLX_API int fmlx_glm_round(int dtype, int epc, int cpl, int u, const void* X, long ld, const void* y, const void* wt,
                            void* coef, long n, int d, long B, int loss, int* state, void* partials, int nblocks,
                            int mode, int det, int* cnt, void* acc, void* stage1, void* feedback, int max_iter,
                            double tol, double lr,
                            double reg, double en, void* const* peers, int world, int rank, int* gen, int* err,
                            long spin_limit, int flags, int rounds, int defer, int parity, void* cw,
                            void* stream) {
  if (mode != TAIL_PARTIALS && cnt == nullptr) return -4;
  if (mode != TAIL_PARTIALS && det && (nblocks > TAIL_GROUP * TAIL_MAXG || stage1 == nullptr)) return -4;
  if (mode != TAIL_PARTIALS && !det && (nblocks > TAIL_GROUP * TAIL_TOP || acc == nullptr)) return -4;
  if (mode == TAIL_FEEDBACK && feedback == nullptr) return -5;
  if (mode == TAIL_XGMI && (d + 2 > xgmi::GLM_MAX || peers == nullptr || world > xgmi::MAX_RANKS)) return -6;
  GlmTail tl{};
  tl.mode = mode;
  tl.max_iter = max_iter;
  tl.det = det;
  tl.cnt = cnt;
  tl.acc = acc;
  tl.acc_reps = g_acc_reps;
  tl.acc_ld = ((long)d + 2 + 63) / 64 * 64;
  tl.ticket2 = g_ticket2;
  tl.stage1 = stage1;
  tl.feedback = feedback;
  tl.tol = tol;
  tl.lr = lr;
  tl.reg = reg;
  tl.en = en;
  tl.x = xgmi::Ctx{peers, world, rank, gen, err, spin_limit};
  tl.defer = defer;
  tl.cw = cw;
  tl.trace = g_trace;
  // `rounds` consecutive rounds, one launch each (a kernel boundary, ~1.5 µs, is cheaper than an
  // in-kernel grid-wide round barrier: measured, scripts/stream_probe2.hip)
  for (int i = 0; i < (rounds > 0 ? rounds : 1); ++i) {
    tl.parity = (parity + i) & 1;  // deferred mode: launches alternate their round-number word
    const int rc = launch_round(dtype, epc, cpl, u, X, ld, y, wt, coef, n, d, B, loss, state, partials, nblocks, tl,
                                flags, (hipStream_t)stream);
    if (rc) return rc;
  }
  return 0;
}

template <typename T, int EPC, int CPL>
static int launch_wide(const void* X, long ld, const void* y, const void* wt, void* coef, long n, int d, long B,
                       int loss, int* state, int nblocks, const GlmTail& tl, hipStream_t s) {
  typedef typename AccOf<T>::type A;
  const size_t lds = (size_t)(d + 2) * sizeof(A) + 16;
  if (lds > (size_t)LDS_PER_CU) return -8;
  hipLaunchKernelGGL((glm_round_wide_kernel<T, EPC, CPL, CPL >= 8 ? 1 : 2>), dim3(nblocks), dim3(WIDE_WAVES * 64), lds,
                     s, (const T*)X,
                     ld, (const A*)y, (const A*)wt, (A*)coef, n, d, B, loss, state, tl);
  return (int)hipGetLastError();
}

template <typename T, int EPC>
static int launch_wide_cpl(int cpl, const void* X, long ld, const void* y, const void* wt, void* coef, long n, int d,
                           long B, int loss, int* state, int nblocks, const GlmTail& tl, hipStream_t s) {
  switch (cpl) {
    case 1: return launch_wide<T, EPC, 1>(X, ld, y, wt, coef, n, d, B, loss, state, nblocks, tl, s);
    case 2: return launch_wide<T, EPC, 2>(X, ld, y, wt, coef, n, d, B, loss, state, nblocks, tl, s);
    case 4: return launch_wide<T, EPC, 4>(X, ld, y, wt, coef, n, d, B, loss, state, nblocks, tl, s);
    case 8: return launch_wide<T, EPC, 8>(X, ld, y, wt, coef, n, d, B, loss, state, nblocks, tl, s);
  }
  return -1;
}

// One SGD round on rows too wide for one wave (see glm_round_wide_kernel): 16-byte chunks of EPC
// elements, the row's chunks split over 8 waves, cpl = chunks per lane of a slice (1, 2, 4 or 8).
// mode TAIL_UPDATE (1 GPU) or TAIL_FEEDBACK (the caller all-reduces `feedback` and updates).
FMLX_API int fmlx_glm_round_wide(int dtype, int epc, int cpl, const void* X, long ld, const void* y, const void* wt,
                                 void* coef, long n, int d, long B, int loss, int* state, int nblocks, int mode,
                                 int* cnt, void* acc, void* feedback, int max_iter, double tol, double lr, double reg,
                                 double en, void* stream) {
  if (mode != TAIL_UPDATE && mode != TAIL_FEEDBACK) return -3;
  if (cnt == nullptr || acc == nullptr || nblocks < 1 || nblocks > TAIL_GROUP * TAIL_TOP) return -4;
  if (mode == TAIL_FEEDBACK && feedback == nullptr) return -5;
  if (d % epc != 0 || (d / epc + WIDE_WAVES - 1) / WIDE_WAVES > 64 * cpl) return -6;
  GlmTail tl{};
  tl.mode = mode;
  tl.max_iter = max_iter;
  tl.cnt = cnt;
  tl.acc = acc;
  tl.acc_reps = g_acc_reps;
  tl.acc_ld = ((long)d + 2 + 63) / 64 * 64;
  tl.ticket2 = g_ticket2;
  tl.feedback = feedback;
  tl.tol = tol;
  tl.lr = lr;
  tl.reg = reg;
  tl.en = en;
  tl.nbatch = (n > 0 && B > 0) ? (int)((n + B - 1) / B) : 0;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DT_BF16 && epc == 8) return launch_wide_cpl<bf16_t, 8>(cpl, X, ld, y, wt, coef, n, d, B, loss, state, nblocks, tl, s);
  if (dtype == DT_F32 && epc == 4) return launch_wide_cpl<float, 4>(cpl, X, ld, y, wt, coef, n, d, B, loss, state, nblocks, tl, s);
  if (dtype == DT_F64 && epc == 2) return launch_wide_cpl<double, 2>(cpl, X, ld, y, wt, coef, n, d, B, loss, state, nblocks, tl, s);
  return -1;
}

// stage1 scratch: [ceil(nparts/16)][d+2] of the accumulator type (nparts <= 512)
template <typename A>
static int launch_stage1(const void* partials, int nparts, int d, void* stage1, const int* state, hipStream_t s) {
  dim3 grid((d + 2 + 255) / 256, (nparts + RED_G - 1) / RED_G);
  hipLaunchKernelGGL(glm_reduce_stage1_kernel<A>, grid, dim3(256), 0, s, (const A*)partials, nparts, d, (A*)stage1,
                     state);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_glm_reduce_update(int acc_f64, const void* partials, int nparts, int d, void* stage1, void* coef,
                                    void* feedback, int* state, int max_iter, double tol, double lr, double reg,
                                    double en, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int ngroups = (nparts + RED_G - 1) / RED_G;
  if (ngroups > 16) return -2;
  int rc = acc_f64 ? launch_stage1<double>(partials, nparts, d, stage1, state, s)
                   : launch_stage1<float>(partials, nparts, d, stage1, state, s);
  if (rc) return rc;
  int blocks = (d + 255) / 256;
  if (acc_f64)
    hipLaunchKernelGGL(glm_reduce_update_kernel<double>, dim3(blocks), dim3(256), 0, s, (const double*)stage1,
                       ngroups, d, (double*)coef, (double*)feedback, state, max_iter, tol, lr, reg, en);
  else
    hipLaunchKernelGGL(glm_reduce_update_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)stage1, ngroups,
                       d, (float*)coef, (float*)feedback, state, max_iter, (float)tol, (float)lr, (float)reg,
                       (float)en);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_glm_reduce(int acc_f64, const void* partials, int nparts, int d, void* stage1, void* feedback,
                             const int* state, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int ngroups = (nparts + RED_G - 1) / RED_G;
  if (ngroups > 16) return -2;
  int rc = acc_f64 ? launch_stage1<double>(partials, nparts, d, stage1, state, s)
                   : launch_stage1<float>(partials, nparts, d, stage1, state, s);
  if (rc) return rc;
  int blocks = (d + 2 + 255) / 256;
  if (acc_f64)
    hipLaunchKernelGGL(glm_reduce_kernel<double>, dim3(blocks), dim3(256), 0, s, (const double*)stage1, ngroups, d,
                       (double*)feedback, state);
  else
    hipLaunchKernelGGL(glm_reduce_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)stage1, ngroups, d,
                       (float*)feedback, state);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_glm_update(int acc_f64, const void* feedback, int d, void* coef, int* state, int max_iter,
                             double tol, double lr, double reg, double en, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int blocks = (d + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (acc_f64)
    hipLaunchKernelGGL(glm_update_kernel<double>, dim3(blocks), dim3(256), 0, s, (const double*)feedback, d,
                       (double*)coef, state, max_iter, tol, lr, reg, en);
  else
    hipLaunchKernelGGL(glm_update_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)feedback, d,
                       (float*)coef, state, max_iter, (float)tol, (float)lr, (float)reg, (float)en);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_glm_predict(int dtype, int epc, int cpl, const void* X, long ld, long n, int d, const void* coef,
                              int mode, double thr, double* pred, double* raw, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return 0;
  if (dtype == DT_BF16) {
    if (epc == 8) return launch_pred_cpl<bf16_t, 8>(cpl, X, ld, n, d, coef, mode, thr, pred, raw, s);
    if (epc == 4) return launch_pred_cpl<bf16_t, 4>(cpl, X, ld, n, d, coef, mode, thr, pred, raw, s);
    if (epc == 2) return launch_pred_cpl<bf16_t, 2>(cpl, X, ld, n, d, coef, mode, thr, pred, raw, s);
    if (epc == 1) return launch_pred_cpl<bf16_t, 1>(cpl, X, ld, n, d, coef, mode, thr, pred, raw, s);
  } else if (dtype == DT_F32) {
    if (epc == 4) return launch_pred_cpl<float, 4>(cpl, X, ld, n, d, coef, mode, thr, pred, raw, s);
    if (epc == 2) return launch_pred_cpl<float, 2>(cpl, X, ld, n, d, coef, mode, thr, pred, raw, s);
    if (epc == 1) return launch_pred_cpl<float, 1>(cpl, X, ld, n, d, coef, mode, thr, pred, raw, s);
  } else if (dtype == DT_F64) {
    if (epc == 2) return launch_pred_cpl<double, 2>(cpl, X, ld, n, d, coef, mode, thr, pred, raw, s);
    if (epc == 1) return launch_pred_cpl<double, 1>(cpl, X, ld, n, d, coef, mode, thr, pred, raw, s);
  }
  return -1;
}

#endif  // FMLX_ISA_PROBE

FMLX_DEFINE_PRELOAD()
