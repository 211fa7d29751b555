// Nearest-neighbour-chain agglomerative clustering core (reference
// AgglomerativeClustering.nnChainCore, flink-ml-lib/.../clustering/agglomerativeclustering/
// AgglomerativeClustering.java:360-460).
//
// The merge sequence of NN-chain depends on the order in which the live cluster labels are
// scanned (ties resolve to the first minimum), and the reference scans a java.util.HashSet<Integer>.
// LabelSet reproduces that iteration order exactly: buckets = label & (cap - 1) (Integer.hashCode
// spread by h ^ (h >>> 16), the identity for labels < 65536 and computed in full otherwise), each
// bucket a chain in insertion order, cap fixed after the initial fill like HashMap's resize rule.
//
// Distances live in the reference's condensed (2n-1)-node upper-triangular matrix so merged
// clusters get their own rows (Lance-Williams updates for single / complete / average / ward).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

namespace {

struct LabelSet {
  int64_t cap;
  std::vector<std::vector<int64_t>> buckets;
  int64_t count = 0;

  static int64_t table_size_for(int64_t n) {
    int64_t c = 1;
    while (c < n) c <<= 1;
    return c;
  }
  static uint32_t spread(int64_t v) {
    uint32_t h = (uint32_t)(int32_t)v;
    return h ^ (h >> 16);
  }
  explicit LabelSet(int64_t n) {
    // new HashSet<>(n): first put allocates tableSizeFor(n); resize while size > 0.75 * cap
    cap = table_size_for(n < 1 ? 1 : n);
    while ((double)n > 0.75 * (double)cap) cap <<= 1;
    buckets.resize((size_t)cap);
  }
  void add(int64_t v) {
    buckets[spread(v) & (cap - 1)].push_back(v);
    ++count;
  }
  void remove(int64_t v) {
    auto& b = buckets[spread(v) & (cap - 1)];
    for (size_t i = 0; i < b.size(); ++i)
      if (b[i] == v) {
        b.erase(b.begin() + (long)i);
        --count;
        return;
      }
  }
  bool contains(int64_t v) const {
    const auto& b = buckets[spread(v) & (cap - 1)];
    for (int64_t x : b)
      if (x == v) return true;
    return false;
  }
  template <typename F>
  void for_each(F f) const {
    for (const auto& b : buckets)
      for (int64_t x : b) f(x);
  }
  // first two elements in iteration order
  void first_two(int64_t* a, int64_t* b) const {
    int got = 0;
    for (const auto& bk : buckets)
      for (int64_t x : bk) {
        if (got == 0) *a = x;
        else if (got == 1) {
          *b = x;
          return;
        }
        ++got;
      }
  }
};

struct Condensed {
  int64_t n;
  std::vector<double> d;
  explicit Condensed(int64_t n_) : n(n_), d((size_t)(n_ * (n_ - 1) / 2)) {}
  inline size_t off(int64_t i, int64_t j) const {
    const int64_t s = i < j ? i : j, b = i < j ? j : i;
    return (size_t)((n * 2 - 1 - s) * s / 2 + (b - s - 1));
  }
  inline double get(int64_t i, int64_t j) const { return d[off(i, j)]; }
  inline void set(int64_t i, int64_t j, double v) { d[off(i, j)] = v; }
};

inline double lance_williams(double dik, double djk, double dij, double si, double sj, double sk, int linkage) {
  switch (linkage) {
    case 0:  // ward
      return std::sqrt(((si + sk) * dik * dik + (sj + sk) * djk * djk - sk * dij * dij) / (si + sj + sk));
    case 1:  // complete
      return dik > djk ? dik : djk;
    case 2:  // average
      return (si * dik + sj * djk) / (si + sj);
    default:  // single
      return dik < djk ? dik : djk;
  }
}

}  // namespace

extern "C" {

// pairwise: n*(n-1)/2 distances between the n points, row-major upper triangle (i < j).
// Outputs n-1 merges (a, b, merged label, distance) in NN-chain discovery order and the
// cluster sizes of all 2n-1 nodes. Returns the number of merges or -1 on bad input.
int64_t fmlx_nnchain(const double* pairwise, int64_t n, int32_t linkage, int64_t* out_a, int64_t* out_b,
                     int64_t* out_merged, double* out_dist, int64_t* sizes) {
  if (n < 1) return -1;
  if (n == 1) {
    sizes[0] = 1;
    return 0;
  }
  Condensed dm(2 * n - 1);
  {
    size_t k = 0;
    for (int64_t i = 0; i < n; ++i)
      for (int64_t j = i + 1; j < n; ++j) dm.set(i, j, pairwise[k++]);
  }
  LabelSet nodes(n);
  for (int64_t i = 0; i < n; ++i) nodes.add(i);
  for (int64_t i = 0; i < 2 * n - 1; ++i) sizes[i] = i < n ? 1 : 0;
  std::vector<int64_t> chain;
  chain.reserve((size_t)n);
  int64_t next_id = n, m = 0;
  int64_t a = 0, b = 0;
  while (nodes.count > 1) {
    if (chain.size() <= 3) {
      nodes.first_two(&a, &b);
      chain.clear();
      chain.push_back(a);
    } else {
      const size_t cs = chain.size();
      a = chain[cs - 4];
      b = chain[cs - 3];
      chain.resize(cs - 3);
    }
    while (chain.size() < 3 || chain[chain.size() - 3] != a) {
      double best = std::numeric_limits<double>::max();
      int64_t c = -1;
      nodes.for_each([&](int64_t x) {
        if (x == a) return;
        const double dax = dm.get(a, x);
        if (dax < best) {
          c = x;
          best = dax;
        }
      });
      if (best == dm.get(a, b) && nodes.contains(b)) c = b;
      b = a;
      a = c;
      chain.push_back(a);
    }
    const int64_t merged = next_id++;
    const double dab = dm.get(a, b);
    out_a[m] = a;
    out_b[m] = b;
    out_merged[m] = merged;
    out_dist[m] = dab;
    ++m;
    nodes.remove(a);
    nodes.remove(b);
    sizes[merged] = sizes[a] + sizes[b];
    const double sa = (double)sizes[a], sb = (double)sizes[b];
    nodes.for_each([&](int64_t x) {
      dm.set(x, merged, lance_williams(dm.get(a, x), dm.get(b, x), dab, sa, sb, (double)sizes[x], linkage));
    });
    nodes.add(merged);
  }
  return m;
}

}  // extern "C"
