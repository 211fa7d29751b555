// Host string tables: many strings as one UTF-16 code-unit array + int64 offsets, with the batch
// operations the vocabulary stages need at high cardinality (StringIndexer, CountVectorizer,
// IndexToString, keyed vocabulary merges across ranks) done natively instead of per-string Python:
//
//   fmlx_str_hash64   64-bit content hash per string (rank-independent, keys the device shuffle)
//   fmlx_str_argsort  stable order by String.compareTo (lexicographic UTF-16 code units),
//                     ascending or descending (StringIndexer alphabet orders,
//                     StringIndexer.java:160-178)
//   fmlx_hashmap_order  java.util.HashMap iteration order from Java hashes (counting sort)
//   fmlx_str_lookup   for every query string, the index of the FIRST equal string of a dictionary
//                     or −1 (open-addressing table keyed by hash64; StringIndexerModel's
//                     HashMap<String, Integer> lookup, StringIndexerModel.java:140-160)
//
// Java String.hashCode stays in javastr.cpp (fmlx_java_string_hashes).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <thread>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdULL;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ULL;
  return h ^ (h >> 33);
}

// 4 code units per step (one 64-bit word), then the length: independent of the platform, so every
// rank computes the same key for the same string
inline uint64_t hash_units(const uint16_t* u, int64_t len) {
  uint64_t h = 0x9e3779b97f4a7c15ULL ^ (uint64_t)len;
  int64_t i = 0;
  for (; i + 4 <= len; i += 4) {
    uint64_t w;
    std::memcpy(&w, u + i, 8);
    h = mix64(h ^ w) + 0x9e3779b97f4a7c15ULL;
  }
  uint64_t t = 0;
  for (int64_t k = 0; i < len; ++i, ++k) t |= (uint64_t)u[i] << (16 * k);
  return mix64(h ^ t ^ ((uint64_t)len << 56));
}

inline bool units_less(const uint16_t* a, int64_t la, const uint16_t* b, int64_t lb) {
  const int64_t m = la < lb ? la : lb;
  for (int64_t i = 0; i < m; ++i)
    if (a[i] != b[i]) return a[i] < b[i];
  return la < lb;
}

inline bool units_equal(const uint16_t* a, int64_t la, const uint16_t* b, int64_t lb) {
  return la == lb && (la == 0 || std::memcmp(a, b, (size_t)la * 2) == 0);
}

template <typename F>
void parallel_for(int64_t n, int64_t grain, F&& f) {
  int nt = (int)std::min<int64_t>(std::max<int64_t>(1, n / grain), (int64_t)std::thread::hardware_concurrency());
  nt = std::max(1, std::min(nt, 16));
  if (nt == 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back([&, t] { f(n * t / nt, n * (t + 1) / nt); });
  for (auto& x : th) x.join();
}

}  // namespace

extern "C" {

void fmlx_str_hash64(const uint16_t* units, const int64_t* offs, int64_t n, uint64_t* out) {
  parallel_for(n, 1 << 16, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) out[i] = hash_units(units + offs[i], offs[i + 1] - offs[i]);
  });
}

// perm = a stable ordering of [0, n) by String.compareTo (descending: reversed comparison, still
// stable among equal strings). Chunks are sorted in parallel, then merged pairwise.
void fmlx_str_argsort(const uint16_t* units, const int64_t* offs, int64_t n, int descending, int64_t* perm) {
  std::iota(perm, perm + n, (int64_t)0);
  auto less = [&](int64_t x, int64_t y) {
    const uint16_t* a = units + offs[x];
    const uint16_t* b = units + offs[y];
    const int64_t la = offs[x + 1] - offs[x], lb = offs[y + 1] - offs[y];
    return descending ? units_less(b, lb, a, la) : units_less(a, la, b, lb);
  };
  const int64_t grain = 1 << 15;
  int nt = (int)std::min<int64_t>(std::max<int64_t>(1, n / grain), 16);
  std::vector<int64_t> bounds(nt + 1);
  for (int t = 0; t <= nt; ++t) bounds[t] = n * t / nt;
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t] { std::stable_sort(perm + bounds[t], perm + bounds[t + 1], less); });
    for (auto& x : th) x.join();
  }
  // pairwise merges keep stability: the left run precedes the right run
  for (int width = 1; width < nt; width *= 2) {
    std::vector<std::thread> th;
    for (int t = 0; t + width < nt; t += 2 * width) {
      const int64_t lo = bounds[t], mid = bounds[t + width], hi = bounds[std::min(t + 2 * width, nt)];
      th.emplace_back([&, lo, mid, hi] { std::inplace_merge(perm + lo, perm + mid, perm + hi, less); });
    }
    for (auto& x : th) x.join();
  }
}

// out[q] = index of the first dictionary string equal to query q, or −1
void fmlx_str_lookup(const uint16_t* du, const int64_t* doffs, int64_t nd, const uint16_t* qu, const int64_t* qoffs,
                     int64_t nq, int64_t* out) {
  int64_t cap = 16;
  while (cap < 2 * nd) cap <<= 1;
  std::vector<uint64_t> dh((size_t)nd);
  fmlx_str_hash64(du, doffs, nd, dh.data());
  std::vector<int64_t> slot((size_t)cap, -1);
  const uint64_t mask = (uint64_t)cap - 1;
  for (int64_t i = 0; i < nd; ++i) {  // in order: the first of equal strings keeps the slot
    uint64_t p = dh[i] & mask;
    while (true) {
      const int64_t s = slot[p];
      if (s < 0) {
        slot[p] = i;
        break;
      }
      if (dh[s] == dh[i] && units_equal(du + doffs[s], doffs[s + 1] - doffs[s], du + doffs[i], doffs[i + 1] - doffs[i]))
        break;
      p = (p + 1) & mask;
    }
  }
  parallel_for(nq, 1 << 15, [&](int64_t a, int64_t b) {
    for (int64_t q = a; q < b; ++q) {
      const uint16_t* u = qu + qoffs[q];
      const int64_t len = qoffs[q + 1] - qoffs[q];
      const uint64_t h = hash_units(u, len);
      uint64_t p = h & mask;
      int64_t r = -1;
      while (true) {
        const int64_t s = slot[p];
        if (s < 0) break;
        if (dh[s] == h && units_equal(du + doffs[s], doffs[s + 1] - doffs[s], u, len)) {
          r = s;
          break;
        }
        p = (p + 1) & mask;
      }
      out[q] = r;
    }
  });
}

// Gather strings idx[0..m) of a table into (out_units, out_offs); out_offs[m] = total units.
void fmlx_str_gather(const uint16_t* units, const int64_t* offs, const int64_t* idx, int64_t m, uint16_t* out_units,
                     int64_t* out_offs) {
  out_offs[0] = 0;
  for (int64_t i = 0; i < m; ++i) out_offs[i + 1] = out_offs[i] + (offs[idx[i] + 1] - offs[idx[i]]);
  parallel_for(m, 1 << 16, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      const int64_t len = out_offs[i + 1] - out_offs[i];
      if (len) std::memcpy(out_units + out_offs[i], units + offs[idx[i]], (size_t)len * 2);
    }
  });
}

// Iteration order of a java.util.HashMap (table capacity `cap`, a power of two) filled with keys
// of Java hashes h[0..n) in index order, no treeified bins: by bucket (h ^ h >>> 16) & (cap − 1),
// insertion order inside a bucket (HashMap.java putVal / resize keep it) — a counting sort.
void fmlx_hashmap_order(const int32_t* h, int64_t n, int64_t cap, int64_t* out) {
  std::vector<int64_t> start((size_t)cap + 1, 0);
  std::vector<uint32_t> b((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t x = (uint32_t)h[i];
    b[i] = (x ^ (x >> 16)) & (uint32_t)(cap - 1);
    ++start[b[i] + 1];
  }
  for (int64_t c = 0; c < cap; ++c) start[c + 1] += start[c];
  for (int64_t i = 0; i < n; ++i) out[start[b[i]]++] = i;
}

}  // extern "C"
