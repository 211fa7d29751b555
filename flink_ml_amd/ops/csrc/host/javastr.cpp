// Java string conversions of numbers + Guava murmur3_32 of the resulting UTF-16 strings, batched
// and multi-threaded on the host (FeatureHasher categorical columns hash `col + "=" + value` for
// every row, StringIndexer maps numbers through String.valueOf — reference
// FeatureHasher.java:126-129,184-194, StringIndexer.java:127-137).
//
// Double.toString: shortest round-trip digits (std::to_chars), printed plainly for
// 1e-3 <= |v| < 1e7 ("123.45", "0.001", always one fractional digit) and as "d.dddE±n" otherwise;
// "NaN", "Infinity", "-Infinity", "0.0", "-0.0" as in the JDK.
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {
inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t mix_k1(uint32_t k1) { return rotl(k1 * 0xcc9e2d51u, 15) * 0x1b873593u; }
inline uint32_t mix_h1(uint32_t h1, uint32_t k1) { return rotl(h1 ^ k1, 13) * 5u + 0xe6546b64u; }
inline uint32_t fmix(uint32_t h1, uint32_t length) {
  h1 ^= length;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  return h1 ^ (h1 >> 16);
}

// hashUnencodedChars over (prefix ++ ascii body) without materialising UTF-16
struct CharStream {
  const uint16_t* pre;
  int plen;
  const char* body;
  int blen;
  inline uint32_t at(int i) const { return i < plen ? pre[i] : (uint32_t)(unsigned char)body[i - plen]; }
};

inline int32_t hash_stream(const CharStream& s) {
  const int len = s.plen + s.blen;
  uint32_t h1 = 0;
  for (int i = 1; i < len; i += 2) h1 = mix_h1(h1, mix_k1(s.at(i - 1) | (s.at(i) << 16)));
  if (len & 1) h1 ^= mix_k1(s.at(len - 1));
  return (int32_t)fmix(h1, (uint32_t)(2 * len));
}

int java_double_string(double v, char* out) {
  if (std::isnan(v)) return (int)(std::memcpy(out, "NaN", 3), 3);
  if (std::isinf(v)) {
    if (v > 0) return (int)(std::memcpy(out, "Infinity", 8), 8);
    return (int)(std::memcpy(out, "-Infinity", 9), 9);
  }
  if (v == 0.0) {
    if (std::signbit(v)) return (int)(std::memcpy(out, "-0.0", 4), 4);
    return (int)(std::memcpy(out, "0.0", 3), 3);
  }
  char sci[64];
  auto res = std::to_chars(sci, sci + sizeof(sci), v, std::chars_format::scientific);
  *res.ptr = 0;
  // parse "-d.ddde[+-]XX"
  const char* p = sci;
  int o = 0;
  if (*p == '-') {
    out[o++] = '-';
    ++p;
  }
  char digits[32];
  int nd = 0;
  while (*p && *p != 'e') {
    if (*p != '.') digits[nd++] = *p;
    ++p;
  }
  int e = 0;
  if (*p == 'e') e = std::atoi(p + 1);
  const double a = std::fabs(v);
  if (a >= 1e-3 && a < 1e7) {
    if (e >= 0) {
      for (int i = 0; i <= e; ++i) out[o++] = i < nd ? digits[i] : '0';
      out[o++] = '.';
      if (nd > e + 1)
        for (int i = e + 1; i < nd; ++i) out[o++] = digits[i];
      else
        out[o++] = '0';
    } else {
      out[o++] = '0';
      out[o++] = '.';
      for (int i = 0; i < -e - 1; ++i) out[o++] = '0';
      for (int i = 0; i < nd; ++i) out[o++] = digits[i];
    }
  } else {
    out[o++] = digits[0];
    out[o++] = '.';
    if (nd > 1)
      for (int i = 1; i < nd; ++i) out[o++] = digits[i];
    else
      out[o++] = '0';
    out[o++] = 'E';
    o += std::sprintf(out + o, "%d", e);
  }
  return o;
}

template <typename F>
void parallel_for(int64_t n, int nthreads, F f) {
  if (nthreads <= 1 || n < 4096) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  const int64_t step = (n + nthreads - 1) / nthreads;
  for (int t = 0; t < nthreads; ++t) {
    const int64_t s = t * step, e = s + step < n ? s + step : n;
    if (s >= e) break;
    ts.emplace_back([=] { f(s, e); });
  }
  for (auto& t : ts) t.join();
}
}  // namespace

extern "C" {

// out_hash[i] = murmur3_32(prefix ++ Double.toString(vals[i])) (UTF-16 semantics)
void fmlx_hash_prefixed_doubles(const uint16_t* prefix, int32_t plen, const double* vals, int64_t n, int32_t* out_hash,
                                int32_t nthreads) {
  parallel_for(n, nthreads, [&](int64_t s, int64_t e) {
    char buf[64];
    for (int64_t i = s; i < e; ++i) {
      const int bl = java_double_string(vals[i], buf);
      out_hash[i] = hash_stream(CharStream{prefix, plen, buf, bl});
    }
  });
}

// Double.toString for a batch: writes the strings back to back into `chars` (capacity 32 per
// value) and their end offsets into `ends`.
void fmlx_java_double_strings(const double* vals, int64_t n, char* chars, int64_t* ends) {
  int64_t o = 0;
  for (int64_t i = 0; i < n; ++i) {
    o += java_double_string(vals[i], chars + o);
    ends[i] = o;
  }
}
}
