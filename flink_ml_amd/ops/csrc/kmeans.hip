// KMeans kernels (SURVEY §2.1 K8–K10).
//
// Reference: LIB/clustering/kmeans/KMeans.java:269-300 (per point findClosest + axpy + count),
// :200-212 (divide by counts), CORE/common/distance/EuclideanDistanceMeasure.java:53-73
// (norm-based distance with lower-bound pruning, strict '<' → lowest index wins ties),
// Cosine/ManhattanDistanceMeasure.java.
//
// MI355X design
//  * kmeans_assign_bf16: the distance "GEMM" X·Cᵀ on MFMA (v_mfma_f32_32x32x16_bf16) with the
//    argmin fused into the epilogue — the n×k distance matrix is never written. Each wave owns
//    MT·32 rows whose A fragments (16-byte row chunks) stay in registers for the whole kernel;
//    centroid tiles of 32 are register-staged into a double-buffered, padded (bank-conflict-free)
//    LDS image shared by the block's 4 waves, so every centroid byte is read once per block
//    (from L2: C is tiny) while the block streams its 128–256 rows from HBM exactly once.
//    The tile is stored pre-scaled by −2 (exact in bf16) and the accumulators start at a
//    (slightly biased) ‖x‖², so the MFMA yields ‖x‖² − 2·x·c; the epilogue adds ‖c‖² (packed),
//    inserts the tile number into the low mantissa bits of the now strictly positive distance
//    and keeps an unsigned min per accumulator register (3 VALU ops per row×centroid pair, was
//    AGPR read + compare + 2 selects), then a 32-lane butterfly (ties → lower index) per row.
//  * kmeans_assign_generic<T>: fp32/fp64 (parity) path, one thread per row, centroids in LDS,
//    exact reference semantics for euclidean (incl. pruning), manhattan and cosine.
//  * Centroid update without atomics, deterministic: rows are ordered by label (stable sort),
//    cut into ≤CH-row chunks that never straddle clusters; kmeans_chunk_sum gathers each chunk's
//    rows (fixed order) into a partial; kmeans_cluster_sum adds a cluster's chunk partials in
//    order → [k·D sums ‖ k counts], the exact payload of the cross-GPU all-reduce (C3 → RCCL).
//  * kmeans_finalize: c = sum·(1/count) (KMeans.java:205), weights = counts, and the padded bf16
//    copy + ‖c‖² used by the next round's MFMA assign.
#include "common.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

constexpr int KM_CH = 256;  // rows per gather chunk

// in-kernel phase stamps of the pipelined assign, for scripts/kmeans_stamp_probe.hip only (the
// library build defines nothing here: no stamp executes in the shipped kernel)
#ifndef KM_STAMP
#define KM_STAMP(i_)
#endif

// ------------------------------------------------------------------------------------------
// MFMA assign (euclidean, bf16)
// ------------------------------------------------------------------------------------------
template <int KS, bool FULL>
// Cb / cnorm are not __restrict__ so the compiler fence after each tile prefetch keeps the
// loads where they are issued (with restrict they get sunk next to their use, after the MFMAs).
__global__ __launch_bounds__(256, 1) void kmeans_assign_bf16_kernel(const bf16_t* __restrict__ X, long ld, long n,
                                                                 int D, const bf16_t* Cb, const float* cnorm,
                                                                 int kpad, int* __restrict__ labels) {
  constexpr int MT = KS <= 8 ? 2 : 1;     // 32-row m-tiles per wave
  constexpr int DP = KS * 16;             // padded feature dim
  constexpr int ROWB = DP * 2 + 16;       // padded LDS row stride (bytes): conflict-free b128 reads
  constexpr int CHUNKS = 32 * DP / 8;     // 16-byte chunks per 32-centroid tile
  constexpr int CPT = (CHUNKS + 255) / 256;
  constexpr int LDSB = 2 * 32 * ROWB;
  __shared__ __align__(16) unsigned char lds[LDSB];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const long ngroups = (n + 4 * 32 * MT - 1) / (4 * 32 * MT);
  for (long grp = blockIdx.x; grp < (long)blockIdx.x + 1 && grp < ngroups; grp += gridDim.x) {
  const long rowbase = grp * (4 * 32 * MT) + (long)wave * 32 * MT;

  // ---- A fragments: this wave's MT x 32 rows, whole padded K, in registers. FULL (D == 16·KS,
  // 16-B aligned rows): unconditional 16-B loads of clamped rows, all in flight together — a
  // per-fragment branch would make every load wait for the previous one (16 round trips).
  bf16x8_t a[MT][KS];
  if constexpr (FULL) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const long row = rowbase + m * 32 + r32;
      const bf16_t* xr = X + (row < n ? row : n - 1) * ld;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        union { uint4 u; bf16x8_t v; } t;
        t.u = *reinterpret_cast<const uint4*>(xr + 16 * s + 8 * h);
        a[m][s] = t.v;
      }
    }
  } else {
    const bool aligned16 = (ld & 7) == 0;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const long row = rowbase + m * 32 + r32;
      const bf16_t* xr = X + (row < n ? row : 0) * ld;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int k0 = 16 * s + 8 * h;
        union { uint4 u; bf16x8_t v; uint16_t e[8]; } t;
        t.u = make_uint4(0, 0, 0, 0);
        if (row < n) {
          if (k0 + 8 <= D) {
            if (aligned16) {
              t.u = *reinterpret_cast<const uint4*>(xr + k0);
            } else {
              const uint32_t* p = reinterpret_cast<const uint32_t*>(xr + k0);
              t.u = make_uint4(p[0], p[1], p[2], p[3]);
            }
          } else {
            for (int j = 0; j < 8; ++j) t.e[j] = (k0 + j < D) ? xr[k0 + j] : (uint16_t)0;
          }
        }
        a[m][s] = t.v;
      }
    }
  }

  // Consume the fragments once here: the waits for their loads then sit before the tile loop
  // instead of inside it, where the (static) counts would also drain the next tile's prefetch.
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" ::"v"(a[m][s]));

  // Row norms ‖x‖² (of the bf16 values), biased by 2^-10·‖x‖² so every computed distance is
  // strictly positive (the fp32 rounding of ‖x‖² + ‖c‖² − 2x·c is ~2^-15·(‖x‖²+‖c‖²) and cancels
  // only when x ≈ c, i.e. ‖c‖² ≈ ‖x‖²); a per-row constant does not move the argmin. They seed
  // the MFMA accumulators, so with the tile pre-scaled by −2 the MFMA yields ‖x‖²' − 2x·c.
  f32x16_t xnb[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    float p = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = (float)a[m][s][j];
        p = __builtin_fmaf(f, f, p);
      }
    p += __shfl_xor(p, 32, 64);  // both K-halves of row r32
    p *= 1.0f + 0x1p-10f;
    // register r of half h holds row (r&3) + 8(r>>2) + 4h: two wave-uniform readlanes + a select
    // per register (was one ds_bpermute each)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int src = (r & 3) + 8 * (r >> 2);
      const float a0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), src));
      const float a1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), src + 4));
      xnb[m][r] = h ? a1 : a0;
    }
  }

  // Running argmin as one u32 key per accumulator register: the positive distance's bits with the
  // tile number in the low TB mantissa bits (relative quantisation 2^(TB-24)). Unsigned order =
  // float order for positive values, and on equal distances the lower tile — the lower centroid
  // index, since the lane is the column — wins: per (row, centroid) the epilogue is one packed add
  // (+‖c‖²), one bit-insert and one unsigned min (was compare + two selects + AGPR reads).
  const int ntiles = kpad / 32;
  int TB = 0;
  while ((1 << TB) < ntiles) ++TB;
  const unsigned tmask = (1u << TB) - 1u;
  // the keep-mask lives in a VGPR: with it in an SGPR next to the SGPR tile number, gfx9's
  // one-scalar-operand limit splits the v_and_or_b32 into two instructions
  unsigned vkeep;
  asm volatile("v_mov_b32 %0, %1" : "=v"(vkeep) : "s"(~tmask));
  unsigned best[MT][16];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) best[m][r] = 0xFFFFFFFFu;

  // register-staged tile loader: chunk q of the tile = (row q / (DP/8), 16B piece q % (DP/8)).
  // Loads are unconditional (clamped to the last chunk) so the next tile stays in flight under
  // this tile's MFMAs; the LDS write is the masked part. (Plain code, no lambdas: a captured
  // staging array was demoted to scratch, and its spill store waited for the prefetch.)
#define KM_LD1(I_, T_)                                                                 \
  if constexpr (CPT > (I_)) {                                                          \
    int q = threadIdx.x + 256 * (I_);                                                  \
    if (CHUNKS % 256 != 0) q = q < CHUNKS ? q : CHUNKS - 1;                            \
    st##I_ = reinterpret_cast<const uint4*>(Cb + (long)(T_) * 32 * DP)[q];             \
  }
#define KM_ST1(I_, BUF_)                                                               \
  if constexpr (CPT > (I_)) {                                                          \
    const int q = threadIdx.x + 256 * (I_);                                            \
    if (CHUNKS % 256 == 0 || q < CHUNKS) {                                             \
      const int rr = q / (DP / 8), cc = q % (DP / 8);                                  \
      *reinterpret_cast<uint4*>(lds + (BUF_) * 32 * ROWB + rr * ROWB + cc * 16) = st##I_; \
    }                                                                                  \
  }
#define KM_GLOAD(T_) \
  KM_LD1(0, T_) KM_LD1(1, T_) KM_LD1(2, T_) KM_LD1(3, T_) cn_next = cnorm[(T_) * 32 + r32];
#define KM_SWRITE(BUF_) KM_ST1(0, BUF_) KM_ST1(1, BUF_) KM_ST1(2, BUF_) KM_ST1(3, BUF_)
  static_assert(CPT <= 4, "tile staging supports up to 4 chunks per thread");
  uint4 st0, st1, st2, st3;  // named registers (an indexed array was demoted to scratch)
  float cn_next;
  KM_GLOAD(0)
  KM_SWRITE(0)
  float cn = cn_next;
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < ntiles;
    const int tn = more ? t + 1 : t;  // the last tile re-fetches itself (unconditional loads)
    KM_GLOAD(tn)
    asm volatile("" ::: "memory");
    f32x16_t acc[MT];
    const unsigned char* tb = lds + cur * 32 * ROWB + r32 * ROWB + h * 16;
    bf16x8_t bfr[KS];  // all B fragments in flight before the first MFMA needs one
#pragma unroll
    for (int s = 0; s < KS; ++s) bfr[s] = *reinterpret_cast<const bf16x8_t*>(tb + s * 32);
    const unsigned tt = (unsigned)t;
    typedef float f32x2_t __attribute__((ext_vector_type(2)));
    const f32x2_t c2 = {cn, cn};
    // epilogue of accumulator registers r, r+1 of m-tile m: + ‖c‖² (packed), tile id into the low
    // mantissa bits, unsigned running min — 5 VALU instructions
#define KM_EPI2(M_, R_)                                                        \
    {                                                                          \
      f32x2_t v = {acc[M_][R_], acc[M_][(R_) + 1]};                            \
      v = v + c2;                                                              \
      const unsigned k0 = (__float_as_uint(v[0]) & vkeep) | tt;                \
      const unsigned k1 = (__float_as_uint(v[1]) & vkeep) | tt;                \
      best[M_][R_] = k0 < best[M_][R_] ? k0 : best[M_][R_];                    \
      best[M_][(R_) + 1] = k1 < best[M_][(R_) + 1] ? k1 : best[M_][(R_) + 1]; \
    }
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        acc[m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m][s], bfr[s], s == 0 ? xnb[m] : acc[m], 0, 0, 0);
    // (a software-pipelined variant — tile t's MFMAs interleaved with tile t-1's epilogue on a
    // second accumulator set — measured slower: 4.46 ms at 256 VGPRs vs 4.02 ms for this loop at
    // 190 VGPRs; two resident waves per SIMD already overlap one's MFMAs with the other's VALU.
    // An interleaved MFMA/epilogue schedule and LDS-DMA-staged rows measured 4.07 vs 3.95-4.00 ms
    // and within noise, and were removed in round 5.)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 16; r += 2) KM_EPI2(m, r)
#undef KM_EPI2
    // unconditional (after the last tile it rewrites the idle buffer with the re-fetched last
    // tile, which nobody reads): a branch here split the tile body into two scheduling regions
    KM_SWRITE(cur ^ 1)
    cn = cn_next;
    __syncthreads();
  }
#undef KM_GLOAD
#undef KM_SWRITE
#undef KM_LD1
#undef KM_ST1

  // ---- row argmin across the 32 lanes of each half (equal keys → lower column). Per row: the
  // minimum key of each 32-lane half by 4 DPP steps within 16-lane rows plus one swap of the
  // 16-lane halves, then the lowest lane holding it from a ballot (the key carries the tile, the
  // lane is the column) — ~10 instructions and one LDS-permute per row, where a butterfly of
  // (key, index) pairs took 10 dependent ds_bpermutes
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    int mine = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned v0 = best[m][r];
      unsigned v = v0;
      v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));   // quad xor 1
      v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));   // quad xor 2
      v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
      v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));  // row_mirror
      v = min(v, (unsigned)__shfl_xor((int)v, 16, 64));                                      // 16-lane halves
      const unsigned long long hit = __ballot(v0 == v);
      const unsigned lo = (unsigned)hit, hi = (unsigned)(hit >> 32);
      const int l0 = __builtin_ctz(lo | 0x80000000u), l1 = __builtin_ctz(hi | 0x80000000u);
      const int id = (int)(v & tmask) * 32 + (h ? l1 : l0);
      if (r32 == r) mine = id;
    }
    if (r32 < 16) {
      const long row = rowbase + m * 32 + (r32 & 3) + 8 * (r32 >> 2) + 4 * h;
      if (row < n) labels[row] = mine;
    }
  }
  }  // row groups
}

// ------------------------------------------------------------------------------------------
// MFMA assign, pipelined (euclidean, bf16, whole 16-B aligned rows, D = 64 or 128)
// ------------------------------------------------------------------------------------------
// Counters of the kernel above at 12.5M x 128, k = 1024 (profiles/r2/kmeans_assign_plain_pmc.json; the variant: kmeans_assign_pipe_pmc.json):
// MFMA busy 44 % of SIMD cycles; per wave and 32-centroid tile 16 MFMAs (512 cycles) but ≈110
// VALU (≈570 cycles of vector issue, the MFMAs' own 8 issue cycles included) that run AFTER the
// MFMAs; a register-staged centroid load waited on right before every barrier; and a label
// stage of 32 dependent ds_bpermute round trips plus exec-masked selects per wave. This variant:
//  * folds BOTH norms into the matrix core: one extra k-step of 16 per m-tile multiplies
//    A_aug = [1, 1, 1, x_h, x_m, x_l, 0…] (the biased ‖x‖² split into three truncated bf16s,
//    exact to fp32) by B_aug = [c_h, c_m, c_l, 1, 1, 1, 0…] (‖c‖², same split), so with the
//    tile pre-scaled by −2 the MFMA chain alone yields ‖x‖²' + ‖c‖² − 2x·c, strictly positive,
//    from a zero seed: the epilogue is one bit-insert (tile id into the low mantissa bits) and
//    one unsigned min per (row, centroid) — 2 VALU instead of 3, and no ‖x‖² seed registers
//    (+12.5 % MFMA work, −40 % epilogue VALU: the tile becomes MFMA-bound);
//  * centroid tiles (and their ‖c‖²) land in LDS by LDS-DMA TWO tiles ahead into a 3-slot
//    ring — no staging registers, no ds_write; the per-tile wait only covers a load issued a
//    tile earlier. Unpadded XOR-swizzled image (16-B slot s of row r holds chunk s ^ (r mod
//    2·KS)): the B-fragment ds_read_b128s are bank-conflict free;
//  * each m-tile's epilogue runs in the MFMA gaps of the OTHER m-tile's chain (tile t's
//    m-tile-0 MFMAs carry tile t−1's m-tile-1 epilogue, its m-tile-1 MFMAs carry tile t's
//    m-tile-0 epilogue), so the VALU hides under the matrix core instead of following it;
//  * labels: every wave transposes its 64×32 final keys through LDS so that each lane owns one
//    row and scans its 32 column keys (min3 tree, then the lowest column holding the minimum):
//    ≈100 VALU and 40 LDS ops per wave, no cross-lane round trips.
// Same keys and tie rule as kmeans_assign_bf16_kernel (lower tile, then lower column = lower
// centroid index); the distances differ from it only by fp32 summation order.
// B_aug row of a centroid from its ‖c‖² (fp32 bits): [c_h, c_m, c_l, 1, 1, 1, 0, 0], ‖c‖² split
// into three truncated bf16s (exact to fp32; +inf padding rows give inf/NaN words, whose keys lose
// to every finite distance). Built once per assign by kmeans_baug_kernel, not per tile per lane;
// only the first two words vary, so a centroid's row is 8 bytes (the rest is constant).
__device__ __forceinline__ uint2 km_baug_words(uint32_t cb) {
  const float c = __uint_as_float(cb);
  const float c1 = c - __uint_as_float(cb & 0xffff0000u);
  const uint32_t c1b = __float_as_uint(c1);
  const float c2 = c1 - __uint_as_float(c1b & 0xffff0000u);
  uint2 q;
  q.x = (cb >> 16) | (c1b & 0xffff0000u);
  q.y = (__float_as_uint(c2) >> 16) | 0x3F800000u;
  return q;
}

__global__ __launch_bounds__(256) void kmeans_baug_kernel(const float* __restrict__ cnorm, int kpad,
                                                          uint2* __restrict__ baug) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < kpad) baug[j] = km_baug_words(__float_as_uint(cnorm[j]));
}

template <int KS, int NW = 4>
__global__ __launch_bounds__(NW * 64, 8 / NW) void kmeans_assign_bf16_pipe_kernel(const bf16_t* __restrict__ X, long ld,
                                                                         long n, const bf16_t* Cb,
                                                                         const uint2* baug, int kpad,
                                                                         int* __restrict__ labels) {
  static_assert(KS == 4 || KS == 8, "pipelined assign: D = 64 or 128");
  constexpr int MT = 2;
  constexpr int DP = KS * 16;
  constexpr int ROWB = DP * 2;            // bytes per centroid row in LDS (unpadded, swizzled)
  constexpr int NS = 2 * KS;              // 16-B slots per row
  constexpr int TILEB = 32 * ROWB;        // bytes per 32-centroid tile
  constexpr int PW = TILEB / 1024 / NW;   // 1-KiB LDS-DMA pieces per wave per tile (1 or 2)
  static_assert(PW >= 1 && PW * NW * 1024 == TILEB, "tile pieces must split evenly over the waves");
  // + the tile's 32 B_aug rows (8 B each), one copy per wave, + the constant B_aug half [1, 1, 0, 0]
  // that the K-half-1 lanes read (written once at entry; the ring's DMAs never touch it)
  constexpr int SLOTB = TILEB + NW * 256 + 16;
  constexpr int BCONST = TILEB + NW * 256;
  // label transpose: words per row (4·LSTR ≡ 32 mod 64 banks). (A 36-word stride — 36 KB blocks,
  // so a gather-sum block of the previous row part fits beside four assign blocks — measured the
  // same round time as this 40 KB layout, split or not: profiles/r4/kmeans_assign_lds_split_ab.jsonl.)
  constexpr int LSTR = 40;
  constexpr int LDSB = 3 * SLOTB > NW * 64 * LSTR * 4 ? 3 * SLOTB : NW * 64 * LSTR * 4;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  typedef short s16x4_t __attribute__((ext_vector_type(4)));
  __shared__ __align__(16) unsigned char lds[LDSB];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const long rowbase = (long)blockIdx.x * (NW * 32 * MT) + (long)wave * 32 * MT;
  const int ntiles = kpad / 32;
  KM_STAMP(4)

  // tile T → ring slot B: piece p = wave + 4i covers tile rows [p·1024/ROWB, …); lane l of the
  // piece lands at LDS byte p·1024 + 16·l = (row, slot) and fetches chunk slot ^ (row mod NS);
  // then the tile's 32 norms (one copy per wave). Issued by inline asm, not
  // __builtin_amdgcn_global_load_lds: with the builtin the compiler cannot tell the ring slots
  // apart and puts a vmcnt(0) in front of every ds_read of the current slot, draining the tile
  // in flight; here the ordering is explicit (vmcnt + barrier at the end of every tile). The
  // compiler's own vmcnt waits stay correct: VMEM ops it does not know of can only make them
  // over-wait. M0 is reserved for the compiler, which warns that a clobber of it is not
  // guaranteed to be honoured: nothing else in this kernel reads or writes M0 (checked in the
  // ISA: the only M0 writes are these blocks'), so no compiler-held M0 value can be disturbed.
  const unsigned lds_base = (unsigned)(uintptr_t)(lds_ptr_t)lds;
#define KP_DMA(T_, B_)                                                                                  \
  {                                                                                                     \
    const char* tsrc_ = reinterpret_cast<const char*>(Cb) + (long)(T_) * TILEB; /* uniform */          \
    _Pragma("unroll") for (int i_ = 0; i_ < PW; ++i_) {                                                 \
      const unsigned dst_ = dma_dst[i_] + (unsigned)((B_) * SLOTB); /* scalar */                        \
      asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(dma_off[i_]), "s"(tsrc_), "s"(dst_) \
                   : "memory", "m0");                                                                   \
    }                                                                                                   \
    const uint2* csrc_ = baug + (long)(T_) * 32; /* uniform */                                           \
    const unsigned cdst_ = dma_cdst + (unsigned)((B_) * SLOTB); /* scalar */                           \
    asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dword %0, %1" ::"v"(dma_noff), "s"(csrc_), "s"(cdst_) \
                 : "memory", "m0");                                                                     \
  }

  // per-lane byte offsets of the pieces inside a tile (and of the norms): the loads take the
  // tile's address as a scalar base (saddr form), so no per-tile 64-bit address math in VALU
  unsigned dma_off[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int off = (wave + NW * i) * 1024 + lane * 16;
    const int row = off / ROWB, slot = (off % ROWB) / 16;
    dma_off[i] = (unsigned)((row * DP + (slot ^ (row & (NS - 1))) * 8) * 2);
  }
  const unsigned dma_noff = (unsigned)lane * 4u;  // the tile's 32 x 8-byte B_aug rows
  // LDS destinations of slot 0 (wave-uniform, made scalar once: per tile only a scalar add)
  unsigned dma_dst[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) dma_dst[i] = __builtin_amdgcn_readfirstlane(lds_base + (wave + NW * i) * 1024);
  const unsigned dma_cdst = __builtin_amdgcn_readfirstlane(lds_base + TILEB + wave * 256);

  // the first two tiles go out before the row loads, so their L2 latency overlaps the rows' HBM one
  const int t1 = ntiles > 1 ? 1 : 0;
  KP_DMA(0, 0)
  KP_DMA(t1, 1)

  // A fragments: this wave's 2 x 32 rows, whole K, in registers (clamped rows, unconditional)
  bf16x8_t a[MT][KS];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const long row = rowbase + m * 32 + r32;
    const bf16_t* xr = X + (row < n ? row : n - 1) * ld;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      union { uint4 u; bf16x8_t v; } t;
      t.u = *reinterpret_cast<const uint4*>(xr + 16 * s + 8 * h);
      a[m][s] = t.v;
    }
  }

  // A_aug, the norm step's A operand (one v_mfma_f32_32x32x8_bf16: K = 8, half the cycles of a
  // K = 16 step): row [1, 1, 1, x_h, x_m, x_l, 0, 0] — lanes of half 0 hold k 0-3, half 1 k 4-7
  // (‖x‖² of the bf16 values, biased by 2^-10·‖x‖² so every distance is strictly positive — the
  // fp32 rounding of ‖x‖² + ‖c‖² − 2x·c is ~2^-15·(‖x‖²+‖c‖²) and cancels only when x ≈ c; a
  // per-row constant does not move the argmin). B_aug = [c_h, c_m, c_l, 1, 1, 1, 0, 0].
  s16x4_t aaug[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    float p = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      union { bf16x8_t v; uint32_t u[4]; } t;
      t.v = a[m][s];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
        union { uint32_t u; bf16x2_t v; } q;
        q.u = t.u[j];
        p = __builtin_amdgcn_fdot2_f32_bf16(q.v, q.v, p, false);
      }
    }
    p += __shfl_xor(p, 32, 64);  // both K-halves of row r32
    p *= 1.0f + 0x1p-10f;
    const uint32_t pb = __float_as_uint(p);
    const float r1 = p - __uint_as_float(pb & 0xffff0000u);
    const uint32_t r1b = __float_as_uint(r1);
    const float r2 = r1 - __uint_as_float(r1b & 0xffff0000u);
    union { uint32_t u[2]; s16x4_t v; } q;
    q.u[0] = h ? (r1b >> 16) | (__float_as_uint(r2) & 0xffff0000u) : 0x3F803F80u;  // x_m, x_l | 1, 1
    q.u[1] = h ? 0u : 0x3F80u | (pb & 0xffff0000u);                                 // 0, 0 | 1, x_h
    aaug[m] = q.v;
  }
#pragma unroll
  for (int m = 0; m < MT; ++m) {
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" ::"v"(a[m][s]));
    asm volatile("" ::"v"(aaug[m]));
  }

  int TB = 0;
  while ((1 << TB) < ntiles) ++TB;
  const unsigned tmask = (1u << TB) - 1u;
  unsigned vkeep;
  asm volatile("v_mov_b32 %0, %1" : "=v"(vkeep) : "s"(~tmask));
  unsigned best[MT][16];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) best[m][r] = 0xFFFFFFFFu;

  // one accumulator register: tile id into the low mantissa bits, unsigned running min (2 VALU)
#define KP_EPI(ACC_, M_, R_, TT_)                                         \
  {                                                                       \
    const unsigned k_ = (__float_as_uint(ACC_[R_]) & vkeep) | (TT_);      \
    best[M_][R_] = k_ < best[M_][R_] ? k_ : best[M_][R_];                 \
  }
  constexpr int EPG = 16 / (KS + 1) + 1;  // epilogue registers per MFMA gap (KS + 1 gaps)

  // m-tile-1 accumulator of the "previous tile" before tile 0: FLT_MAX keys lose to every
  // finite distance (NaN rows resolve to label 0 as in the plain kernel)
  f32x16_t acc0, acc1;
  const f32x16_t zero16 = {};
#pragma unroll
  for (int r = 0; r < 16; ++r) acc1[r] = 3.4028235e38f;
  unsigned tprev = 0;
  int s_cur = 0, s_n1 = 1, s_n2 = 2;  // ring slots of tiles t, t+1, t+2
  if (threadIdx.x < 3) *reinterpret_cast<uint2*>(lds + threadIdx.x * SLOTB + BCONST) = make_uint2(0x3F803F80u, 0u);
  // B_aug source of this lane in a slot: its centroid's row (half 0) or the constant (half 1)
  const int ba_off = h ? BCONST : TILEB + wave * 256 + r32 * 8;
  KM_STAMP(0)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // rows, tiles 0 and 1
  __syncthreads();
  KM_STAMP(1)

  // B fragments of a ring slot, and the tile's B_aug rows (half 1 multiplies A_aug's zeros)
#define KP_LDB(SLOT_, BF_, BA_)                                                                   \
  {                                                                                               \
    const unsigned char* tb_ = lds + (SLOT_) * SLOTB + r32 * ROWB;                                \
    BA_ = *reinterpret_cast<const s16x4_t*>(lds + (SLOT_) * SLOTB + ba_off);                      \
    _Pragma("unroll") for (int s_ = 0; s_ < KS; ++s_)                                             \
        BF_[s_] = *reinterpret_cast<const bf16x8_t*>(tb_ + (((2 * s_ + h) ^ (r32 & (NS - 1))) * 16)); \
  }
  // one m-tile chain: KS MFMAs + the norm step, carrying the OTHER accumulator's epilogue
#define KP_CHAIN(ACC_, M_, BF_, BA_, EACC_, EM_, ETT_)                                               \
  _Pragma("unroll") for (int s_ = 0; s_ <= KS; ++s_) {                                               \
    if (s_ < KS)                                                                                     \
      ACC_ = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[M_][s_], BF_[s_], s_ == 0 ? zero16 : ACC_, 0, 0, 0); \
    else                                                                                             \
      ACC_ = __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(aaug[M_], BA_, ACC_, 0, 0, 0);                 \
    _Pragma("unroll") for (int e_ = 0; e_ < EPG; ++e_) if (s_ * EPG + e_ < 16)                      \
        KP_EPI(EACC_, EM_, s_ * EPG + e_, ETT_)                                                      \
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                               \
    __builtin_amdgcn_sched_group_barrier(0x002, 2 * EPG, 0);                                         \
  }

  {
    // B fragments one tile ahead in registers: the ring wait + barrier sit between the two
    // chains of a tile, and the next tile's ds_reads are issued under the second chain, so no
    // chain ever starts on an LDS round trip. Two named register sets, loop unrolled by two.
    bf16x8_t bA[KS], bB[KS];
    s16x4_t gA, gB;
    KP_LDB(0, bA, gA)
#define KP_TILE(BF_, BA_, NBF_, NBA_)                                                     \
    {                                                                                           \
      const int t2_ = t + 2 < ntiles ? t + 2 : ntiles - 1; /* the tail re-fetches the last tile */ \
      KP_DMA(t2_, s_n2)                                                                         \
      const unsigned tt_ = (unsigned)t;                                                         \
      __builtin_amdgcn_sched_barrier(0);                                                        \
      KP_CHAIN(acc0, 0, BF_, BA_, acc1, 1, tprev)                                               \
      __builtin_amdgcn_sched_barrier(0);                                                        \
      /* tile t + 1 (issued a tile ago) complete for this wave, then for every wave */          \
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW + 1) : "memory");                             \
      __syncthreads();                                                                          \
      KP_LDB(s_n1, NBF_, NBA_)                                                                  \
      KP_CHAIN(acc1, 1, BF_, BA_, acc0, 0, tt_)                                                 \
      __builtin_amdgcn_sched_barrier(0);                                                        \
      tprev = tt_;                                                                              \
      const int s_old_ = s_cur;                                                                 \
      s_cur = s_n1;                                                                             \
      s_n1 = s_n2;                                                                              \
      s_n2 = s_old_;                                                                            \
    }
    int t = 0;
    while (true) {
      KP_TILE(bA, gA, bB, gB)
      if (++t == ntiles) break;
      KP_TILE(bB, gB, bA, gA)
      if (++t == ntiles) break;
    }
#undef KP_TILE
  }
#undef KP_CHAIN
#undef KP_LDB
#pragma unroll
  for (int r = 0; r < 16; ++r) KP_EPI(acc1, 1, r, tprev)
  KM_STAMP(2)
#undef KP_EPI
#undef KP_DMA
  // every wave's tail re-fetches landed before the ring is reused for the label transpose
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // labels: key of (row ρ, column c) → word (m·32 + ρ)·LSTR + c of this wave's region; register
  // r of half h holds row ρ = (r&3) + 8(r>>2) + 4h. Then lane L owns row L (m = L / 32).
  uint32_t* reg = reinterpret_cast<uint32_t*>(lds) + wave * 64 * LSTR;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      reg[(m * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * LSTR + r32] = best[m][r];
  // (no barrier: the region is this wave's own, and a wave's LDS accesses complete in order)
  unsigned key[32];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint4 v = *reinterpret_cast<const uint4*>(reg + lane * LSTR + 4 * j);
    key[4 * j] = v.x;
    key[4 * j + 1] = v.y;
    key[4 * j + 2] = v.z;
    key[4 * j + 3] = v.w;
  }
  unsigned mn = key[0];
#pragma unroll
  for (int c = 1; c < 31; c += 2) mn = min(min(mn, key[c]), key[c + 1]);
  mn = min(mn, key[31]);
  int col = 0;
#pragma unroll
  for (int c = 31; c >= 0; --c) col = key[c] == mn ? c : col;
  const long row = rowbase + lane;
  if (row < n) labels[row] = (int)(mn & tmask) * 32 + col;
  KM_STAMP(3)
}

// ------------------------------------------------------------------------------------------
// generic assign (fp32 / fp64): exact reference semantics
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void kmeans_assign_generic_kernel(const T* __restrict__ X, long ld, long n, int D,
                                                                    const T* __restrict__ C, const T* __restrict__ cnrm,
                                                                    int k, int metric, int use_lds,
                                                                    int* __restrict__ labels) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* Cs = reinterpret_cast<T*>(smem_raw);
  if (use_lds) {
    for (int i = threadIdx.x; i < k * D; i += blockDim.x) Cs[i] = C[i];
    __syncthreads();
  }
  const T* Cp = use_lds ? Cs : C;
  const long row = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  const T* x = X + row * ld;
  T pn2 = 0;
  for (int j = 0; j < D; ++j) pn2 += x[j] * x[j];
  const T pn = sqrt(pn2);
  int bi = metric == 0 ? 0 : -1;
  T best = metric == 0 ? (T)__builtin_huge_val() : (T)1.7976931348623157e308;
  for (int i = 0; i < k; ++i) {
    const T* c = Cp + (long)i * D;
    const T cn = cnrm[i];
    if (metric == 0) {
      const T lb = pn - cn;
      if (lb * lb >= best) continue;
      T dot = 0;
      for (int j = 0; j < D; ++j) dot += x[j] * c[j];
      T d2 = pn * pn + cn * cn - (T)2 * dot;
      d2 = d2 > (T)0 ? d2 : (T)0;
      if (d2 < best) { best = d2; bi = i; }
    } else if (metric == 1) {
      T s = 0;
      for (int j = 0; j < D; ++j) s += fabs(x[j] - c[j]);
      if (s < best) { best = s; bi = i; }
    } else {
      T dot = 0;
      for (int j = 0; j < D; ++j) dot += x[j] * c[j];
      const T dist = (T)1 - dot / pn / cn;
      if (dist < best) { best = dist; bi = i; }
    }
  }
  labels[row] = bi;
}

// ------------------------------------------------------------------------------------------
// generic assign v2 (fp32 / fp64): one wave per row, lanes split the feature dimension
// ------------------------------------------------------------------------------------------
// Each lane holds VPL = ceil(D/64) coalesced row elements in registers; for every group of KG
// centroids the lanes accumulate partial dot products / L1 sums and a wave butterfly (DPP for
// fp32) turns them into wave-uniform distances, so the argmin runs on uniform values (ties keep
// the lower index, strict '<' like DistanceMeasure.findClosest). X is read exactly once,
// coalesced; centroids come from LDS when k·D fits.
template <typename T>
__device__ __forceinline__ T wave_allsum(T v) {
  return wave_sum_dpp(v);
}

template <typename T, int VPL>
__global__ __launch_bounds__(256) void kmeans_assign_wave_kernel(const T* __restrict__ X, long ld, long n, int D,
                                                                 const T* __restrict__ C, const T* __restrict__ cnrm,
                                                                 int k, int metric, int use_lds,
                                                                 int* __restrict__ labels) {
  constexpr int KG = 8;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* Cs = reinterpret_cast<T*>(smem_raw);
  // centroid norms next to the centroids in LDS: as per-centroid scalar loads they would share
  // lgkmcnt with the LDS reads, so every LDS wait would also wait for an SMEM round trip
  T* Ns = Cs + (use_lds ? (long)k * D : 0);
  if (use_lds) {
    for (int i = threadIdx.x; i < k * D; i += blockDim.x) Cs[i] = C[i];
    for (int i = threadIdx.x; i < k; i += blockDim.x) Ns[i] = cnrm[i];
    __syncthreads();
  }
  const T* Cp = use_lds ? Cs : C;
  const T* Np = use_lds ? Ns : cnrm;
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long nwaves = (long)gridDim.x * (blockDim.x >> 6);
  // the next row's elements are loaded before this row's reductions start (one row of load
  // latency hidden behind the DPP chains; a wave otherwise waits a full HBM trip per row)
  T xv[VPL], xn[VPL];
  auto load_row = [&](long r, T (&dst)[VPL]) {
    const T* x = X + (r < n ? r : n - 1) * ld;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int c = lane + 64 * v;
      dst[v] = c < D ? x[c] : (T)0;
    }
  };
  if (wave < n) load_row(wave, xv);
  for (long row = wave; row < n; row += nwaves) {
    load_row(row + nwaves, xn);
    T pn2 = 0;
#pragma unroll
    for (int v = 0; v < VPL; ++v) pn2 += xv[v] * xv[v];
    pn2 = wave_allsum(pn2);
    const T pn = sqrt(pn2);
    int bi = metric == 0 ? 0 : -1;
    T best = metric == 0 ? (T)__builtin_huge_val() : (T)1.7976931348623157e308;
    for (int i0 = 0; i0 < k; i0 += KG) {
      T acc[KG];
#pragma unroll
      for (int g = 0; g < KG; ++g) {
        acc[g] = 0;
        const int i = i0 + g;
        if (i < k) {
          const T* c = Cp + (long)i * D;
#pragma unroll
          for (int v = 0; v < VPL; ++v) {
            const int cc = lane + 64 * v;
            const T cv = cc < D ? c[cc] : (T)0;
            if (metric == 1) acc[g] += cc < D ? (T)fabs(xv[v] - cv) : (T)0;
            else acc[g] += xv[v] * cv;
          }
        }
      }
#pragma unroll
      for (int g = 0; g < KG; ++g)
        if (i0 + g < k) acc[g] = wave_allsum(acc[g]);  // (k is uniform: no reductions of padding)
#pragma unroll
      for (int g = 0; g < KG; ++g) {
        const int i = i0 + g;
        if (i >= k) break;
        T dist;
        if (metric == 0) {
          const T cn = Np[i];
          dist = pn * pn + cn * cn - (T)2 * acc[g];
          dist = dist > (T)0 ? dist : (T)0;
        } else if (metric == 1) {
          dist = acc[g];
        } else {
          dist = (T)1 - acc[g] / pn / Np[i];
        }
        if (dist < best) {
          best = dist;
          bi = i;
        }
      }
    }
    if (lane == 0) labels[row] = bi;
#pragma unroll
    for (int v = 0; v < VPL; ++v) xv[v] = xn[v];
  }
}

// ------------------------------------------------------------------------------------------
// deterministic centroid accumulation: chunk gather-sum then per-cluster chunk reduction
// ------------------------------------------------------------------------------------------
template <typename T, int VPL>
__global__ __launch_bounds__(256) void kmeans_chunk_sum_kernel(const T* __restrict__ X, long ld, int D,
                                                               const long* __restrict__ order,
                                                               const long* __restrict__ offsets,  // [k+1]
                                                               const long* __restrict__ chunk_off,  // [k+1]
                                                               int k, typename AccOf<T>::type* __restrict__ partial) {
  typedef typename AccOf<T>::type A;
  const long b = blockIdx.x;
  if (b >= chunk_off[k]) return;
  // cluster j with chunk_off[j] <= b < chunk_off[j+1]
  int lo = 0, hi = k;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (chunk_off[mid] <= b) lo = mid; else hi = mid;
  }
  const int j = lo;
  const long q = b - chunk_off[j];
  const long p0 = offsets[j] + q * KM_CH;
  long p1 = p0 + KM_CH;
  if (p1 > offsets[j + 1]) p1 = offsets[j + 1];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  A acc[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) acc[v] = 0;
  for (long p = p0 + wave; p < p1; p += 4) {
    const T* xr = X + order[p] * ld;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int c = lane + 64 * v;
      if (c < D) acc[v] += (A)Ld<T>::f(xr[c]);
    }
  }
  __shared__ A sm[4][64 * VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) sm[wave][lane + 64 * v] = acc[v];
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) partial[b * D + c] = ((sm[0][c] + sm[1][c]) + sm[2][c]) + sm[3][c];
}

// bf16 rows, D = 8·LPR with LPR | 64: one 16-byte load per lane per row (LPR lanes cover a row,
// 64/LPR rows per wave-step). The chunk's row indices are staged in LDS first so the gathers are
// independent loads (4 in flight per lane), not an index→row dependent pair per row. Fixed
// summation order (lane stripe, xor tree, wave order): deterministic.
template <int LPR>
__global__ __launch_bounds__(256) void kmeans_chunk_sum_bf16v_kernel(const bf16_t* __restrict__ X, long ld, int D,
                                                                     const int* __restrict__ order,
                                                                     const long* __restrict__ offsets,
                                                                     const long* __restrict__ chunk_off, int k,
                                                                     float* __restrict__ partial) {
  constexpr int RPW = 64 / LPR;  // rows per wave-step
  const long b = blockIdx.x;
  if (b >= chunk_off[k]) return;
  int lo = 0, hi = k;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (chunk_off[mid] <= b) lo = mid; else hi = mid;
  }
  const int j = lo;
  const long p0 = offsets[j] + (b - chunk_off[j]) * KM_CH;
  long p1 = p0 + KM_CH;
  if (p1 > offsets[j + 1]) p1 = offsets[j + 1];
  const int nrow = (int)(p1 - p0);
  __shared__ int rows_s[KM_CH];
  __shared__ float sm[4][512];
  if ((int)threadIdx.x < nrow) rows_s[threadIdx.x] = order[p0 + threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane / LPR, cl = lane % LPR;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  constexpr int STEP = 4 * RPW;  // rows per block-step
  for (int q0 = 0; q0 < nrow; q0 += 4 * STEP) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = q0 + u * STEP + wave * RPW + sub;
      const int qc = q < nrow ? q : 0;  // unconditional load (row 0 of the chunk), masked below
      v[u] = *reinterpret_cast<const uint4*>(X + (long)rows_s[qc] * ld + cl * 8);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = q0 + u * STEP + wave * RPW + sub < nrow;
      const unsigned int w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        acc[2 * h] += ok ? __uint_as_float(w4[h] << 16) : 0.f;
        acc[2 * h + 1] += ok ? __uint_as_float(w4[h] & 0xffff0000u) : 0.f;
      }
    }
  }
#pragma unroll
  for (int off = LPR; off < 64; off <<= 1)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += __shfl_xor(acc[i], off, 64);
  if (sub == 0)
#pragma unroll
    for (int i = 0; i < 8; ++i) sm[wave][cl * 8 + i] = acc[i];
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) partial[b * D + c] = ((sm[0][c] + sm[1][c]) + sm[2][c]) + sm[3][c];
}

// Cluster boundaries from the sorted labels, no host sync: offsets[c] = first position of a
// label ≥ c (binary search, one thread per cluster), chunk_off = exclusive scan of
// ceil(count / KM_CH) (one block, fixed order). Replaces bincount + cumsum (bincount's min/max
// range check synchronised the host every round).
__global__ __launch_bounds__(1024) void kmeans_offsets_kernel(const int* __restrict__ keys_sorted, long n, int k,
                                                              long* __restrict__ offsets, long* __restrict__ chunk_off) {
  __shared__ long warp_tot[16];
  __shared__ long carry;
  if (threadIdx.x == 0) carry = 0;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // 1. offsets[c] = lower_bound(keys_sorted, c) for c = 0..k, every cluster's search in parallel
  for (int c = threadIdx.x; c <= k; c += 1024) {
    long lo = 0, hi = n;
    while (lo < hi) {
      const long mid = (lo + hi) >> 1;
      if (keys_sorted[mid] < c) lo = mid + 1; else hi = mid;
    }
    offsets[c] = lo;
  }
  __syncthreads();  // this block's global writes are visible to the block after the barrier
  // 2. chunk_off = exclusive scan of ceil(count / KM_CH), fixed order (wave prefix, wave totals,
  // carry across 1024-cluster passes); counts from neighbouring offsets — one binary search per
  // cluster instead of two dependent ones
  for (int base = 0; base <= k; base += 1024) {
    const int c = base + threadIdx.x;
    const long chunks = c < k ? (offsets[c + 1] - offsets[c] + KM_CH - 1) / KM_CH : 0;
    long incl = chunks;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const long o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    if (lane == 63) warp_tot[wv] = incl;
    __syncthreads();
    long wpre = 0;
    for (int i = 0; i < wv; ++i) wpre += warp_tot[i];
    const long excl = carry + wpre + incl - chunks;
    if (c <= k) chunk_off[c] = excl;
    __syncthreads();
    if (threadIdx.x == 1023) carry = excl + chunks;
    __syncthreads();
  }
}

template <typename A>
__global__ __launch_bounds__(256) void kmeans_cluster_sum_kernel(const A* __restrict__ partial, int D,
                                                                 const long* __restrict__ offsets,
                                                                 const long* __restrict__ chunk_off, int k,
                                                                 A* __restrict__ out /* [k*D sums | k counts] */) {
  const int j = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  const long q0 = chunk_off[j], q1 = chunk_off[j + 1];
  if (c < D) {
    A s8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s8[i] = 0;
    long q = q0;
    for (; q + 8 <= q1; q += 8)
#pragma unroll
      for (int i = 0; i < 8; ++i) s8[i] += partial[(q + i) * D + c];
    for (int i = 0; q < q1; ++q, ++i) s8[i] += partial[q * D + c];
    A s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += s8[i];
    out[(long)j * D + c] = s;
  }
  if (blockIdx.y == 0 && threadIdx.x == 0) out[(long)k * D + j] = (A)(offsets[j + 1] - offsets[j]);
}

// centroids = sums * (1/count); padded bf16 copy + squared norms (of the bf16 values) for MFMA
template <typename A>
__global__ __launch_bounds__(256) void kmeans_finalize_kernel(const A* __restrict__ red, int D, int k,
                                                              A* __restrict__ cent, double* __restrict__ weights,
                                                              bf16_t* __restrict__ Cb, int DP,
                                                              float* __restrict__ cnorm_bf16,
                                                              A* __restrict__ cnorm_acc) {
  const int j = blockIdx.x;
  const A cnt = red[(long)k * D + j];
  const A inv = (A)1 / cnt;
  float nb = 0.f;
  A na = 0;
  for (int c = threadIdx.x; c < DP; c += blockDim.x) {
    A v = c < D ? red[(long)j * D + c] * inv : (A)0;
    if (c < D) cent[(long)j * D + c] = v;
    if (Cb) {
      const bf16_t bv = f32_to_bf16((float)v);
      const float fb = bf16_to_f32(bv);
      Cb[(long)j * DP + c] = f32_to_bf16(-2.f * fb);  // the assign kernel's −2-scaled tile (exact)
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
    if (weights) weights[j] = (double)cnt;
  }
}

// LDS-DMA centroid ring + cross-m-tile epilogue interleave (kmeans_assign_bf16_pipe_kernel, the
// B fragments prefetched one tile ahead): the shipped assign for D = 64 / 128; 0 = plain loop.
// History of the variants measured against it (all removed in round 5): one wave per SIMD via an
// LDS pad (90 KB): 3.68 vs 3.22 ms at 12.5M x 128, k = 1024 — the second wave covers
// part of the first's issue stalls. (Issuing the tile's LDS-DMA pieces inside the MFMA chain
// instead of ahead of it: 3.15 vs 3.15 ms, not kept. Dropping the per-tile barrier altogether —
// wrong labels, a diagnostic — ran 3.13-3.16 vs 3.17-3.19 ms: the barrier costs ~1 %; what is
// left is the per-wave issue budget, ≈86 VALU + 18 MFMA per 32-centroid tile. An epilogue over
// tile PAIRS — two bit-inserts + one v_min3_u32 per register, 75 VALU per tile at 244 VGPRs —
// ran 3.11-3.14 vs 3.17 ms there but 0.126 vs 0.105 ms at 2M x 64, k = 256: not kept. Round 4: a
// 4-slot ring, DMA three tiles ahead, 3.417-3.427 vs 3.407-3.430 ms — the DMA wait is not what
// the waves wait on (profiles/r4/kmeans_assign_ring4_ab.log); three blocks per CU (≤ 168 of the
// D = 128 kernel's ~207 VGPRs) spill 420-444 bytes per lane: neither kept. Phase stamps
// (scripts/kmeans_stamp_probe.hip): a wave spends 14 % of its life waiting for its rows and first
// tiles, 82 % in the tile loop at ~1,430 cycles per tile (2 waves per SIMD: ~80 % MFMA in the
// loop), 4 % on labels, at a 1.69-1.75 GHz in-kernel clock. A persistent grid (2 blocks per CU
// walking the row groups, the next group's rows loaded under the label transpose and its first
// tiles riding the ring's tail fetches; 256 VGPRs, identical labels) ran 3.12-3.22 vs 3.09-3.10 ms
// interleaved: the entry wait is already covered by the CU's other wave — not kept;
// profiles/r4/kmeans_assign_phase_stamps.log, kmeans_assign_persistent_ab.log. The tile norms
// fetched once per block by wave 0 instead of once per wave (3 of 12 LDS-DMA issues per tile
// saved): 1,566 vs 1,430 cycles per tile, 3.24-3.26 vs 3.17-3.18 ms — not kept;
// kmeans_assign_norm_once_ab.log. The tile loop is ISSUE-bound: per wave and tile ~98 VALU × 4
// cycles + 18 MFMA issue holds × 8 + 3 LDS-DMA issues, twice per SIMD, ≈ the measured 1,430
// cycles (the 36 MFMAs alone are 1,152). Kept: the LDS-DMA sources in the saddr form (scalar tile
// base + loop-invariant lane offsets: no 64-bit address math per tile) and B_aug rows built once
// per assign (kmeans_baug_kernel) instead of per tile and lane — 78 VALU per tile, 1,316 cycles
// per tile, 3.08-3.11 vs 3.21 ms at 12.5M x 128 and 23.3-23.4 vs 24.5-24.6 ms at 100M x 128,
// identical labels (kmeans_assign_saddr_baug_ab.log, kmeans_assign_100M_saddr_baug_ab.log; the
// saving returns partly as a lower clock, 1.70 vs 1.75 GHz). Unrolling the tile loop by six so the
// ring slots become immediates spills 150 VGPRs. LDS-DMA destinations made scalar once (no
// readfirstlane per tile): 1,285 vs 1,314 cycles per tile at the same wall time, 3.02-3.03 ms —
// the chip is power-bound here, a cycle saving comes back as clock; kmeans_assign_scalar_dst_ab.log.
// The norm step on v_mfma_f32_32x32x8_bf16 (K = 8: 5.6 % fewer MFMA cycles per tile, 74 VALU,
// 193 VGPRs): identical labels, 1,285 cycles per tile and the same wall time —
// kmeans_assign_k8_norm_ab.log; kept for the lighter kernel. 8-wave, 512-row blocks: within
// noise at k = 1024 and slower at k = 32. The pipelined kernel without the B prefetch: 3.23 vs
// 3.18 ms.)
int g_km_pipe = 1;

template <int KS>
int launch_assign_bf16(const void* X, long ld, long n, int D, const void* Cb, const float* cnorm, int kpad, int* labels,
                       void* baug, hipStream_t s) {
  constexpr int MT = KS <= 8 ? 2 : 1;
  const long rows_per_block = 4 * 32 * MT;
  const int blocks = (int)((n + rows_per_block - 1) / rows_per_block);
  if (blocks == 0) return 0;
  const bool full = D == 16 * KS && (ld % 8) == 0 && ((uintptr_t)X % 16) == 0;
  const bool pipe = full && g_km_pipe && baug != nullptr;
  if constexpr (KS == 4 || KS == 8) {
    if (pipe) {
      hipLaunchKernelGGL(kmeans_baug_kernel, dim3((kpad + 255) / 256), dim3(256), 0, s, cnorm, kpad, (uint2*)baug);
      hipLaunchKernelGGL((kmeans_assign_bf16_pipe_kernel<KS>), dim3(blocks), dim3(256), 0, s, (const bf16_t*)X, ld,
                         n, (const bf16_t*)Cb, (const uint2*)baug, kpad, labels);
      return (int)hipGetLastError();
    }
  }
  if (full)
    hipLaunchKernelGGL((kmeans_assign_bf16_kernel<KS, true>), dim3(blocks), dim3(256), 0, s, (const bf16_t*)X, ld, n, D,
                       (const bf16_t*)Cb, cnorm, kpad, labels);
  else
    hipLaunchKernelGGL((kmeans_assign_bf16_kernel<KS, false>), dim3(blocks), dim3(256), 0, s, (const bf16_t*)X, ld, n,
                       D, (const bf16_t*)Cb, cnorm, kpad, labels);
  return (int)hipGetLastError();
}

template <typename T, int VPL>
int launch_chunk_sum(const void* X, long ld, int D, const long* order, const long* offsets, const long* chunk_off,
                     int k, long max_chunks, void* partial, hipStream_t s) {
  if (max_chunks <= 0) return 0;
  hipLaunchKernelGGL((kmeans_chunk_sum_kernel<T, VPL>), dim3((unsigned)max_chunks), dim3(256), 0, s, (const T*)X, ld,
                     D, order, offsets, chunk_off, k, (typename AccOf<T>::type*)partial);
  return (int)hipGetLastError();
}

template <typename T>
int chunk_sum_vpl(const void* X, long ld, int D, const long* order, const long* offsets, const long* chunk_off, int k,
                  long max_chunks, void* partial, hipStream_t s) {
  if (D <= 64) return launch_chunk_sum<T, 1>(X, ld, D, order, offsets, chunk_off, k, max_chunks, partial, s);
  if (D <= 128) return launch_chunk_sum<T, 2>(X, ld, D, order, offsets, chunk_off, k, max_chunks, partial, s);
  if (D <= 256) return launch_chunk_sum<T, 4>(X, ld, D, order, offsets, chunk_off, k, max_chunks, partial, s);
  if (D <= 512) return launch_chunk_sum<T, 8>(X, ld, D, order, offsets, chunk_off, k, max_chunks, partial, s);
  if (D <= 1024) return launch_chunk_sum<T, 16>(X, ld, D, order, offsets, chunk_off, k, max_chunks, partial, s);
  return -3;
}

}  // namespace

// Assign schedule: 1 (default) = the pipelined kernel for D = 64 / 128 (other widths: plain loop),
// 0 = the plain loop everywhere (A/B and tests).
FMLX_API int fmlx_kmeans_set_sched(int mode) {
  g_km_pipe = mode != 0;
  return 0;
}

// KS = padded K-steps of 16 (one of 1..8,10,12,16; >= ceil(D/16)); Cb is [kpad][16*KS] zero-padded.
// baug: kpad x 8 bytes of scratch for the pipelined kernel's B_aug rows (nullptr: plain loop)
FMLX_API int fmlx_kmeans_assign_bf16(const void* X, long ld, long n, int D, int KS, const void* Cb, const float* cnorm,
                                     int kpad, int* labels, void* baug, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (KS * 16 < D) return -2;
  switch (KS) {
    case 1: return launch_assign_bf16<1>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 2: return launch_assign_bf16<2>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 3: return launch_assign_bf16<3>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 4: return launch_assign_bf16<4>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 5: return launch_assign_bf16<5>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 6: return launch_assign_bf16<6>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 7: return launch_assign_bf16<7>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 8: return launch_assign_bf16<8>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 10: return launch_assign_bf16<10>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 12: return launch_assign_bf16<12>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
    case 16: return launch_assign_bf16<16>(X, ld, n, D, Cb, cnorm, kpad, labels, baug, s);
  }
  return -2;  // unsupported D for the MFMA path
}

template <typename T, int VPL>
int launch_assign_wave(const void* X, long ld, long n, int D, const void* C, const void* cnrm, int k, int metric,
                       int* labels, hipStream_t s) {
  const size_t need = ((size_t)k * D + k) * sizeof(T);
  const int use_lds = need <= 64 * 1024;
  const size_t sh = use_lds ? need : 0;
  long waves = n;
  long blocks = (waves + 3) / 4;
  if (blocks > 2048) blocks = 2048;  // ≫ 256 CUs; each wave then loops over rows
  hipLaunchKernelGGL((kmeans_assign_wave_kernel<T, VPL>), dim3((unsigned)blocks), dim3(256), sh, s, (const T*)X, ld,
                     n, D, (const T*)C, (const T*)cnrm, k, metric, use_lds, labels);
  return (int)hipGetLastError();
}

template <typename T>
int assign_wave_vpl(const void* X, long ld, long n, int D, const void* C, const void* cnrm, int k, int metric,
                    int* labels, hipStream_t s) {
  if (D <= 64) return launch_assign_wave<T, 1>(X, ld, n, D, C, cnrm, k, metric, labels, s);
  if (D <= 128) return launch_assign_wave<T, 2>(X, ld, n, D, C, cnrm, k, metric, labels, s);
  if (D <= 256) return launch_assign_wave<T, 4>(X, ld, n, D, C, cnrm, k, metric, labels, s);
  if (D <= 512) return launch_assign_wave<T, 8>(X, ld, n, D, C, cnrm, k, metric, labels, s);
  return launch_assign_wave<T, 16>(X, ld, n, D, C, cnrm, k, metric, labels, s);
}

FMLX_API int fmlx_kmeans_assign_generic(int dtype, const void* X, long ld, long n, int D, const void* C,
                                        const void* cnrm, int k, int metric, int* labels, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) return 0;
  if (D <= 1024) {
    if (dtype == DT_F64) return assign_wave_vpl<double>(X, ld, n, D, C, cnrm, k, metric, labels, s);
    if (dtype == DT_F32) return assign_wave_vpl<float>(X, ld, n, D, C, cnrm, k, metric, labels, s);
    return -1;
  }
  const int blocks = (int)((n + 255) / 256);
  const size_t es = dtype == DT_F64 ? 8 : 4;
  const size_t need = (size_t)k * D * es;
  const int use_lds = need <= 64 * 1024;
  const size_t sh = use_lds ? need : 0;
  if (dtype == DT_F64)
    hipLaunchKernelGGL(kmeans_assign_generic_kernel<double>, dim3(blocks), dim3(256), sh, s, (const double*)X, ld, n,
                       D, (const double*)C, (const double*)cnrm, k, metric, use_lds, labels);
  else if (dtype == DT_F32)
    hipLaunchKernelGGL(kmeans_assign_generic_kernel<float>, dim3(blocks), dim3(256), sh, s, (const float*)X, ld, n, D,
                       (const float*)C, (const float*)cnrm, k, metric, use_lds, labels);
  else
    return -1;
  return (int)hipGetLastError();
}

FMLX_API int fmlx_kmeans_chunk_sum(int dtype, const void* X, long ld, int D, const long* order, const long* offsets,
                                   const long* chunk_off, int k, long max_chunks, void* partial, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == DT_BF16) return chunk_sum_vpl<bf16_t>(X, ld, D, order, offsets, chunk_off, k, max_chunks, partial, s);
  if (dtype == DT_F32) return chunk_sum_vpl<float>(X, ld, D, order, offsets, chunk_off, k, max_chunks, partial, s);
  if (dtype == DT_F64) return chunk_sum_vpl<double>(X, ld, D, order, offsets, chunk_off, k, max_chunks, partial, s);
  return -1;
}

// bf16 fast path of the centroid accumulation: int32 row order (from the radix sort),
// D in {8, 16, 32, 64, 128, 256, 512}, rows 16-byte aligned. Returns -2 for other shapes.
FMLX_API int fmlx_kmeans_chunk_sum_bf16v(const void* X, long ld, int D, const int* order, const long* offsets,
                                         const long* chunk_off, int k, long max_chunks, float* partial,
                                         void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (max_chunks <= 0) return 0;
  if ((ld % 8) != 0 || ((uintptr_t)X % 16) != 0) return -2;
  dim3 g((unsigned)max_chunks);
  const bf16_t* x = (const bf16_t*)X;
  switch (D) {
    case 8: hipLaunchKernelGGL(kmeans_chunk_sum_bf16v_kernel<1>, g, dim3(256), 0, s, x, ld, D, order, offsets, chunk_off, k, partial); break;
    case 16: hipLaunchKernelGGL(kmeans_chunk_sum_bf16v_kernel<2>, g, dim3(256), 0, s, x, ld, D, order, offsets, chunk_off, k, partial); break;
    case 32: hipLaunchKernelGGL(kmeans_chunk_sum_bf16v_kernel<4>, g, dim3(256), 0, s, x, ld, D, order, offsets, chunk_off, k, partial); break;
    case 64: hipLaunchKernelGGL(kmeans_chunk_sum_bf16v_kernel<8>, g, dim3(256), 0, s, x, ld, D, order, offsets, chunk_off, k, partial); break;
    case 128: hipLaunchKernelGGL(kmeans_chunk_sum_bf16v_kernel<16>, g, dim3(256), 0, s, x, ld, D, order, offsets, chunk_off, k, partial); break;
    case 256: hipLaunchKernelGGL(kmeans_chunk_sum_bf16v_kernel<32>, g, dim3(256), 0, s, x, ld, D, order, offsets, chunk_off, k, partial); break;
    case 512: hipLaunchKernelGGL(kmeans_chunk_sum_bf16v_kernel<64>, g, dim3(256), 0, s, x, ld, D, order, offsets, chunk_off, k, partial); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

FMLX_API int fmlx_kmeans_offsets(const int* keys_sorted, long n, int k, long* offsets, long* chunk_off, void* stream) {
  hipLaunchKernelGGL(kmeans_offsets_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, keys_sorted, n, k, offsets,
                     chunk_off);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_kmeans_cluster_sum(int acc_f64, const void* partial, int D, const long* offsets,
                                     const long* chunk_off, int k, void* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(k, (D + 255) / 256);
  if (acc_f64)
    hipLaunchKernelGGL(kmeans_cluster_sum_kernel<double>, grid, dim3(256), 0, s, (const double*)partial, D, offsets,
                       chunk_off, k, (double*)out);
  else
    hipLaunchKernelGGL(kmeans_cluster_sum_kernel<float>, grid, dim3(256), 0, s, (const float*)partial, D, offsets,
                       chunk_off, k, (float*)out);
  return (int)hipGetLastError();
}

FMLX_API int fmlx_kmeans_finalize(int acc_f64, const void* red, int D, int k, void* cent, double* weights, void* Cb,
                                  int DP, float* cnorm_bf16, void* cnorm_acc, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (acc_f64)
    hipLaunchKernelGGL(kmeans_finalize_kernel<double>, dim3(k), dim3(256), 0, s, (const double*)red, D, k,
                       (double*)cent, weights, (bf16_t*)Cb, DP, cnorm_bf16, (double*)cnorm_acc);
  else
    hipLaunchKernelGGL(kmeans_finalize_kernel<float>, dim3(k), dim3(256), 0, s, (const float*)red, D, k, (float*)cent,
                       weights, (bf16_t*)Cb, DP, cnorm_bf16, (float*)cnorm_acc);
  return (int)hipGetLastError();
}

FMLX_DEFINE_PRELOAD()
