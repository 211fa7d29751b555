// Host-side Java-compatible random utilities (bit-exact with java.util.Random), used where the
// reference's results depend on the JVM RNG stream (SURVEY §7.4 "RNG compatibility"):
//   * reservoir sampling of DataStreamUtils.SamplingOperator (DataStreamUtils.java:633-704)
//   * bulk nextDouble / nextInt / nextGaussian streams (data generators, RandomSplitter, MinHash)
#include <cmath>
#include <cstdint>

namespace {
struct JRandom {
  uint64_t seed;
  bool have_gauss = false;
  double next_gauss = 0;
  explicit JRandom(int64_t s) : seed(((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1)) {}
  int32_t next(int bits) {
    seed = (seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
    return (int32_t)(int64_t)(seed >> (48 - bits));
  }
  int32_t next_int(int32_t bound) {
    int32_t r = next(31);
    int32_t m = bound - 1;
    if ((bound & m) == 0) return (int32_t)(((int64_t)bound * (int64_t)r) >> 31);
    // Java's rejection test relies on int overflow (u - r + m < 0): wrap explicitly (signed
    // overflow is undefined in C++ and an optimiser may drop the test)
    for (int32_t u = r; (int32_t)((uint32_t)u - (uint32_t)(r = u % bound) + (uint32_t)m) < 0; u = next(31)) {
    }
    return r;
  }
  double next_double() { return (double)(((int64_t)next(26) << 27) + next(27)) * (1.0 / (double)(1LL << 53)); }
  double next_gaussian() {
    if (have_gauss) { have_gauss = false; return next_gauss; }
    double v1, v2, s;
    do {
      v1 = 2 * next_double() - 1;
      v2 = 2 * next_double() - 1;
      s = v1 * v1 + v2 * v2;
    } while (s >= 1 || s == 0);
    double mul = std::sqrt(-2 * std::log(s) / s);
    next_gauss = v2 * mul;
    have_gauss = true;
    return v1 * mul;
  }
};
}  // namespace

extern "C" {

// Reservoir sample of k positions out of n (SamplingOperator.processElement semantics).
// Writes the chosen positions (in reservoir slot order) to out[0..min(n,k)); returns that count.
int fmlx_reservoir_sample(int64_t n, int32_t k, int64_t seed, int64_t* out) {
  JRandom rnd(seed);
  int64_t filled = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t count = (int32_t)(i + 1);
    if (filled < k) {
      out[filled++] = i;
    } else {
      int32_t idx = rnd.next_int(count);
      if (idx < k) out[idx] = i;
    }
  }
  return (int)filled;
}

// The sequential part of the device reservoir sampler (ops/datagen.py reservoir_sample_device):
// draw i (i = k .. n-1) is Random.nextInt(i + 1) on the stream after the draws before it. A
// position p of the raw next(31) stream can only be a rejected draw if u_p ≥ 2^31 − n (for
// every bound b ≤ n, u < 2^31 − b + 1 is accepted), so only those "candidates" are scanned here,
// in order: the draw at p is i = p + k − R with R the rejections before p; it is rejected iff b is
// not a power of two and u − u % b + b − 1 ≥ 2^31. Writes the rejected positions (ascending) to
// rej and returns their count; *done receives 1 if the scan proved that draw n − 1 happens before
// position `npos` (the generated stream was long enough), else 0.
int64_t fmlx_reservoir_rejections(int64_t n, int32_t k, int64_t npos, const int32_t* cand_p, const int32_t* cand_u,
                                  int64_t ncand, int64_t* rej, int32_t* done) {
  // The decision for a candidate depends on R through its bound; the dependency chain through
  // R would put a division on every step's critical path. Instead the next candidate's decision is
  // computed for both values R can take there (R, R + 1) while this one's is resolved — two
  // independent 32-bit divisions per step off the chain, one select on it (u < 2^31 and
  // b ≤ n < 2^31 keep everything in 32 bits).
  auto dec = [&](int64_t c, int64_t R) -> int {
    const uint32_t b = (uint32_t)((int64_t)cand_p[c] + k - R + 1);
    const uint32_t u = (uint32_t)cand_u[c];
    return ((b & (b - 1)) != 0) & ((uint64_t)(u - u % b) + b - 1 >= (1ULL << 31));
  };
  int64_t R = 0;
  int d = ncand > 0 ? dec(0, 0) : 0;
  for (int64_t c = 0; c < ncand; ++c) {
    if ((int64_t)cand_p[c] + k - R >= n) break;
    int n0 = 0, n1 = 0;
    if (c + 1 < ncand) {
      n0 = dec(c + 1, R);
      n1 = dec(c + 1, R + 1);
    }
    rej[R] = cand_p[c];  // kept only if d (R advances)
    R += d;
    d = d ? n1 : n0;
  }
  // the last draw (i = n − 1) sits at position n − 1 − k + R; it must be inside the stream
  *done = (n - 1 - k + R) < npos ? 1 : 0;
  return R;
}

void fmlx_java_next31(int64_t seed, int64_t start, int64_t n, int32_t* out) {
  JRandom rnd(seed);
  for (int64_t i = 0; i < start; ++i) rnd.next(31);
  for (int64_t i = 0; i < n; ++i) out[i] = rnd.next(31);
}

void fmlx_java_next_doubles(int64_t seed, int64_t n, double* out) {
  JRandom rnd(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = rnd.next_double();
}

void fmlx_java_next_gaussians(int64_t seed, int64_t n, double* out) {
  JRandom rnd(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = rnd.next_gaussian();
}

void fmlx_java_next_ints(int64_t seed, int64_t n, int32_t bound, int32_t* out) {
  JRandom rnd(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = rnd.next_int(bound);
}
}
