// Double.toString + Guava murmur3_32 of `prefix + string` on the device (FeatureHasher's
// categorical numeric columns hash `col + "=" + value` for every row — reference
// FeatureHasher.java:184-194, StringIndexer.java:127-137 for the String.valueOf mapping).
//
// One thread per value, nothing materialised: the shortest round-trip decimal digits come from a
// Ryu-style fixed-point computation (128-bit multiplier tables built exactly on the host with
// Python integers and passed in), the Java layout rules turn them into characters, and every
// character is folded into the murmur3 state as a UTF-16 unit as it is produced. The result is
// bit-identical to the host path (ops/csrc/host/javastr.cpp: std::to_chars shortest digits, same
// layout): plain "123.45" / "0.001" for 1e-3 <= |v| < 1e7, "d.dddE±n" otherwise, "NaN",
// "Infinity", "-Infinity", "0.0", "-0.0".
#include "common.h"

namespace {

constexpr int kMantBits = 52;
constexpr int kBias = 1023;
constexpr int kPow5InvBits = 125;
constexpr int kPow5Bits = 125;

__device__ __forceinline__ uint32_t pow5bits(int32_t e) { return (uint32_t)(((uint32_t)e * 1217359u) >> 19) + 1u; }
__device__ __forceinline__ uint32_t log10_pow2(int32_t e) { return ((uint32_t)e * 78913u) >> 18; }
__device__ __forceinline__ uint32_t log10_pow5(int32_t e) { return ((uint32_t)e * 732923u) >> 20; }

__device__ __forceinline__ uint32_t pow5_factor(uint64_t v) {
  uint32_t c = 0;
  for (;;) {
    const uint64_t q = v / 5u;
    if ((uint32_t)(v - 5u * q) != 0u) break;
    v = q;
    ++c;
  }
  return c;
}

// (m · (hi:lo)) >> j for 64 < j < 128 (m < 2^55)
__device__ __forceinline__ uint64_t mul_shift64(uint64_t m, const uint64_t* mul, int32_t j) {
  const uint64_t h0 = __umul64hi(m, mul[0]);
  const uint64_t l1 = m * mul[1];
  uint64_t h1 = __umul64hi(m, mul[1]);
  const uint64_t sum = h0 + l1;
  h1 += sum < h0 ? 1u : 0u;
  const int d = j - 64;
  return (h1 << (64 - d)) | (sum >> d);
}

// shortest decimal (digits, exponent) with value = digits · 10^exp that rounds back to the double
// given by (mantissa, exponent) bits; nonzero finite inputs only
__device__ void shortest_decimal(uint64_t ieee_m, uint32_t ieee_e, const uint64_t* inv_tab, const uint64_t* pow_tab,
                                 uint64_t& out, int32_t& exp10) {
  // integers in [1, 2^53): exact, strip trailing decimal zeros
  {
    const uint64_t m2 = (1ull << kMantBits) | ieee_m;
    const int32_t e2 = (int32_t)ieee_e - kBias - kMantBits;
    if (ieee_e != 0 && e2 <= 0 && e2 >= -52) {
      const uint64_t mask = (1ull << -e2) - 1u;
      if ((m2 & mask) == 0u) {
        uint64_t v = m2 >> -e2;
        int32_t e = 0;
        for (;;) {
          const uint64_t q = v / 10u;
          if ((uint32_t)(v - 10u * q) != 0u) break;
          v = q;
          ++e;
        }
        out = v;
        exp10 = e;
        return;
      }
    }
  }
  int32_t e2;
  uint64_t m2;
  if (ieee_e == 0) {
    e2 = 1 - kBias - kMantBits - 2;
    m2 = ieee_m;
  } else {
    e2 = (int32_t)ieee_e - kBias - kMantBits - 2;
    m2 = (1ull << kMantBits) | ieee_m;
  }
  const bool accept_bounds = (m2 & 1u) == 0u;
  const uint64_t mv = 4u * m2;
  const uint32_t mm_shift = (ieee_m != 0u || ieee_e <= 1u) ? 1u : 0u;
  uint64_t vr, vp, vm;
  int32_t e10;
  bool vm_tz = false, vr_tz = false;
  if (e2 >= 0) {
    const uint32_t q = log10_pow2(e2) - (e2 > 3 ? 1u : 0u);
    e10 = (int32_t)q;
    const int32_t k = kPow5InvBits + (int32_t)pow5bits((int32_t)q) - 1;
    const int32_t i = -e2 + (int32_t)q + k;
    const uint64_t* mul = inv_tab + 2 * q;
    vr = mul_shift64(4u * m2, mul, i);
    vp = mul_shift64(4u * m2 + 2u, mul, i);
    vm = mul_shift64(4u * m2 - 1u - mm_shift, mul, i);
    if (q <= 21u) {
      if ((uint32_t)(mv % 5u) == 0u)
        vr_tz = pow5_factor(mv) >= q;
      else if (accept_bounds)
        vm_tz = pow5_factor(mv - 1u - mm_shift) >= q;
      else
        vp -= pow5_factor(mv + 2u) >= q ? 1u : 0u;
    }
  } else {
    const uint32_t q = log10_pow5(-e2) - (-e2 > 1 ? 1u : 0u);
    e10 = (int32_t)q + e2;
    const int32_t i = -e2 - (int32_t)q;
    const int32_t k = (int32_t)pow5bits(i) - kPow5Bits;
    const int32_t j = (int32_t)q - k;
    const uint64_t* mul = pow_tab + 2 * i;
    vr = mul_shift64(4u * m2, mul, j);
    vp = mul_shift64(4u * m2 + 2u, mul, j);
    vm = mul_shift64(4u * m2 - 1u - mm_shift, mul, j);
    if (q <= 1u) {
      vr_tz = true;
      if (accept_bounds)
        vm_tz = mm_shift == 1u;
      else
        --vp;
    } else if (q < 63u) {
      vr_tz = (mv & ((1ull << q) - 1u)) == 0u;
    }
  }
  int32_t removed = 0;
  uint32_t last = 0;
  uint64_t output;
  if (vm_tz || vr_tz) {
    for (;;) {
      const uint64_t vp10 = vp / 10u, vm10 = vm / 10u;
      if (vp10 <= vm10) break;
      const uint32_t vm_mod = (uint32_t)(vm - 10u * vm10);
      const uint64_t vr10 = vr / 10u;
      const uint32_t vr_mod = (uint32_t)(vr - 10u * vr10);
      vm_tz &= vm_mod == 0u;
      vr_tz &= last == 0u;
      last = vr_mod;
      vr = vr10;
      vp = vp10;
      vm = vm10;
      ++removed;
    }
    if (vm_tz) {
      for (;;) {
        const uint64_t vm10 = vm / 10u;
        if ((uint32_t)(vm - 10u * vm10) != 0u) break;
        const uint64_t vp10 = vp / 10u, vr10 = vr / 10u;
        const uint32_t vr_mod = (uint32_t)(vr - 10u * vr10);
        vr_tz &= last == 0u;
        last = vr_mod;
        vr = vr10;
        vp = vp10;
        vm = vm10;
        ++removed;
      }
    }
    if (vr_tz && last == 5u && (vr & 1u) == 0u) last = 4u;  // exact ...50..0: round half to even
    output = vr + (((vr == vm && (!accept_bounds || !vm_tz)) || last >= 5u) ? 1u : 0u);
  } else {
    bool round_up = false;
    const uint64_t vp100 = vp / 100u, vm100 = vm / 100u;
    if (vp100 > vm100) {
      const uint64_t vr100 = vr / 100u;
      round_up = (uint32_t)(vr - 100u * vr100) >= 50u;
      vr = vr100;
      vp = vp100;
      vm = vm100;
      removed += 2;
    }
    for (;;) {
      const uint64_t vp10 = vp / 10u, vm10 = vm / 10u;
      if (vp10 <= vm10) break;
      const uint64_t vr10 = vr / 10u;
      round_up = (uint32_t)(vr - 10u * vr10) >= 5u;
      vr = vr10;
      vp = vp10;
      vm = vm10;
      ++removed;
    }
    output = vr + ((vr == vm || round_up) ? 1u : 0u);
  }
  out = output;
  exp10 = e10 + removed;
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t mix_k1(uint32_t k1) { return rotl32(k1 * 0xcc9e2d51u, 15) * 0x1b873593u; }
__device__ __forceinline__ uint32_t mix_h1(uint32_t h1, uint32_t k1) { return rotl32(h1 ^ k1, 13) * 5u + 0xe6546b64u; }

// murmur3_32 over a stream of UTF-16 units (Guava hashUnencodedChars)
struct Murmur16 {
  uint32_t h1 = 0, pend = 0;
  int n = 0;
  __device__ __forceinline__ void put(uint32_t c) {
    if (n & 1)
      h1 = mix_h1(h1, mix_k1(pend | (c << 16)));
    else
      pend = c;
    ++n;
  }
  __device__ __forceinline__ int32_t finish() {
    uint32_t h = h1;
    if (n & 1) h ^= mix_k1(pend);
    h ^= (uint32_t)(2 * n);
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return (int32_t)h;
  }
};

__device__ __forceinline__ void put_str(Murmur16& m, const char* s) {
  for (; *s; ++s) m.put((uint32_t)(unsigned char)*s);
}

__device__ void hash_java_double(Murmur16& m, double v, const uint64_t* inv_tab, const uint64_t* pow_tab) {
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  const bool neg = (bits >> 63) != 0u;
  const uint32_t ieee_e = (uint32_t)((bits >> kMantBits) & 0x7FFu);
  const uint64_t ieee_m = bits & ((1ull << kMantBits) - 1u);
  if (ieee_e == 0x7FFu) {
    if (ieee_m != 0u) {
      put_str(m, "NaN");
    } else {
      put_str(m, neg ? "-Infinity" : "Infinity");
    }
    return;
  }
  if (ieee_e == 0u && ieee_m == 0u) {
    put_str(m, neg ? "-0.0" : "0.0");
    return;
  }
  uint64_t dig;
  int32_t e10;
  shortest_decimal(ieee_m, ieee_e, inv_tab, pow_tab, dig, e10);
  char d[20];
  int nd = 0;
  for (uint64_t x = dig; x != 0u; x /= 10u) d[nd++] = (char)('0' + (int)(x % 10u));  // least significant first
  const int E = e10 + nd - 1;  // scientific exponent
  if (neg) m.put('-');
  const double a = fabs(v);
  if (a >= 1e-3 && a < 1e7) {
    if (E >= 0) {
      for (int i = 0; i <= E; ++i) m.put(i < nd ? (uint32_t)d[nd - 1 - i] : (uint32_t)'0');
      m.put('.');
      if (nd > E + 1)
        for (int i = E + 1; i < nd; ++i) m.put((uint32_t)d[nd - 1 - i]);
      else
        m.put('0');
    } else {
      m.put('0');
      m.put('.');
      for (int i = 0; i < -E - 1; ++i) m.put('0');
      for (int i = 0; i < nd; ++i) m.put((uint32_t)d[nd - 1 - i]);
    }
  } else {
    m.put((uint32_t)d[nd - 1]);
    m.put('.');
    if (nd > 1)
      for (int i = 1; i < nd; ++i) m.put((uint32_t)d[nd - 1 - i]);
    else
      m.put('0');
    m.put('E');
    int x = E;
    if (x < 0) {
      m.put('-');
      x = -x;
    }
    char ed[4];
    int ne = 0;
    do {
      ed[ne++] = (char)('0' + x % 10);
      x /= 10;
    } while (x);
    while (ne) m.put((uint32_t)ed[--ne]);
  }
}

__global__ __launch_bounds__(256) void hash_prefixed_doubles_kernel(const uint16_t* __restrict__ prefix, int plen,
                                                                     const double* __restrict__ vals, long n,
                                                                     const uint64_t* __restrict__ inv_tab,
                                                                     const uint64_t* __restrict__ pow_tab,
                                                                     int32_t* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    Murmur16 m;
    for (int p = 0; p < plen; ++p) m.put(prefix[p]);
    hash_java_double(m, vals[i], inv_tab, pow_tab);
    out[i] = m.finish();
  }
}

}  // namespace

// out[i] = murmur3_32(prefix ++ Double.toString(vals[i])) over UTF-16 units, on the device.
// inv_tab: 342 × (lo, hi) u64 = ⌊2^(bitlen(5^q) − 1 + 125) / 5^q⌋ + 1; pow_tab: 326 × (lo, hi) u64 =
// 5^i scaled to 125 significant bits (tables built by ops/hashing.py).
FMLX_API int fmlx_hash_prefixed_doubles_dev(const uint16_t* prefix, int plen, const double* vals, long n,
                                            const uint64_t* inv_tab, const uint64_t* pow_tab, int32_t* out,
                                            void* stream) {
  if (n <= 0) return 0;
  if (plen < 0 || (plen > 0 && prefix == nullptr) || inv_tab == nullptr || pow_tab == nullptr) return -1;
  const long want = (n + 255) / 256;
  const int blocks = (int)(want < 8192 ? want : 8192);
  hipLaunchKernelGGL(hash_prefixed_doubles_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, prefix, plen, vals,
                     n, inv_tab, pow_tab, out);
  FMLX_CHECK_LAUNCH();
}

FMLX_DEFINE_PRELOAD()
