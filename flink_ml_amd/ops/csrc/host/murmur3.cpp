// Guava Hashing.murmur3_32() (seed 0) — bit-exact host implementation used by HashingTF,
// FeatureHasher and the StringIndexer/CountVectorizer hash tables (reference
// LIB/feature/hashingtf/HashingTF.java:165-194, LIB/feature/featurehasher/FeatureHasher.java:186).
#include <cstdint>
#include <cstring>

namespace {
inline uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t mix_k1(uint32_t k1) {
  k1 *= 0xcc9e2d51u;
  k1 = rotl(k1, 15);
  k1 *= 0x1b873593u;
  return k1;
}
inline uint32_t mix_h1(uint32_t h1, uint32_t k1) {
  h1 ^= k1;
  h1 = rotl(h1, 13);
  h1 = h1 * 5u + 0xe6546b64u;
  return h1;
}
inline uint32_t fmix(uint32_t h1, uint32_t length) {
  h1 ^= length;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  return h1;
}
inline int32_t hash_chars(const uint16_t* cs, int64_t len) {
  uint32_t h1 = 0;
  for (int64_t i = 1; i < len; i += 2) {
    uint32_t k1 = (uint32_t)cs[i - 1] | ((uint32_t)cs[i] << 16);
    h1 = mix_h1(h1, mix_k1(k1));
  }
  if (len & 1) h1 ^= mix_k1((uint32_t)cs[len - 1]);
  return (int32_t)fmix(h1, (uint32_t)(2 * len));
}
}  // namespace

extern "C" {
// strings given as UTF-16 code units, string i = units[offsets[i] .. offsets[i+1])
void fmlx_murmur3_chars(const uint16_t* units, const int64_t* offsets, int64_t n, int32_t* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = hash_chars(units + offsets[i], offsets[i + 1] - offsets[i]);
}
void fmlx_murmur3_ints(const int32_t* v, int64_t n, int32_t* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)fmix(mix_h1(0, mix_k1((uint32_t)v[i])), 4);
}
void fmlx_murmur3_longs(const int64_t* v, int64_t n, int32_t* out) {
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t x = (uint64_t)v[i];
    uint32_t h1 = mix_h1(0, mix_k1((uint32_t)x));
    h1 = mix_h1(h1, mix_k1((uint32_t)(x >> 32)));
    out[i] = (int32_t)fmix(h1, 8);
  }
}
}
