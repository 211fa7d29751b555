// Greenwald–Khanna quantile summary kernels (reference LIB/common/util/QuantileSummary.java:39-414):
// the summary is three parallel arrays (value, g, delta) sorted by value; the Python object
// (flink_ml_amd/utils/quantile_summary.py) owns them and the head buffer and calls these for the
// O(n) passes. Semantics follow the reference exactly (delta rule at the ends of the merged
// sequence, backward compression keeping the minimum, merge with cross-summary delta penalties).
#include <cmath>
#include <cstdint>

extern "C" {

// Merge the sorted head buffer `h` into the samples; returns the new sample count (ns + nh).
int64_t fmlx_gk_insert(const double* sv, const int64_t* sg, const int64_t* sd, int64_t ns, const double* h,
                       int64_t nh, int64_t delta_base, double* ov, int64_t* og, int64_t* od) {
  int64_t o = 0, cur = 0;
  for (int64_t i = 0; i < nh; ++i) {
    while (cur < ns && sv[cur] <= h[i]) {
      ov[o] = sv[cur];
      og[o] = sg[cur];
      od[o] = sd[cur];
      ++o;
      ++cur;
    }
    int64_t delta = delta_base;
    if (o == 0 || (cur == ns && i == nh - 1)) delta = 0;
    ov[o] = h[i];
    og[o] = 1;
    od[o] = delta;
    ++o;
  }
  for (; cur < ns; ++cur, ++o) {
    ov[o] = sv[cur];
    og[o] = sg[cur];
    od[o] = sd[cur];
  }
  return o;
}

// Backward compression with merge threshold `thr`; writes the result front-aligned and returns
// its length. Output arrays may not alias the input.
int64_t fmlx_gk_compress(const double* v, const int64_t* g, const int64_t* d, int64_t n, double thr, double* ov,
                         int64_t* og, int64_t* od) {
  if (n == 0) return 0;
  // build back to front into the tail of the output, then shift to the front
  int64_t w = n;  // next free slot (exclusive) from the back
  double hv = v[n - 1];
  int64_t hg = g[n - 1], hd = d[n - 1];
  for (int64_t i = n - 2; i >= 1; --i) {
    if ((double)(g[i] + hg + hd) < thr) {
      hg += g[i];
    } else {
      --w;
      ov[w] = hv;
      og[w] = hg;
      od[w] = hd;
      hv = v[i];
      hg = g[i];
      hd = d[i];
    }
  }
  --w;
  ov[w] = hv;
  og[w] = hg;
  od[w] = hd;
  if (v[0] <= hv && n > 1) {
    --w;
    ov[w] = v[0];
    og[w] = g[0];
    od[w] = d[0];
  }
  const int64_t m = n - w;
  for (int64_t i = 0; i < m; ++i) {
    ov[i] = ov[w + i];
    og[i] = og[w + i];
    od[i] = od[w + i];
  }
  return m;
}

// Ordered merge of two summaries (before compression). add_a is added to a sample of `a` once
// any sample of `b` precedes it, and vice versa; the leftover tail is copied unchanged.
int64_t fmlx_gk_merge(const double* av, const int64_t* ag, const int64_t* ad, int64_t na, const double* bv,
                      const int64_t* bg, const int64_t* bd, int64_t nb, int64_t add_a, int64_t add_b, double* ov,
                      int64_t* og, int64_t* od) {
  int64_t i = 0, j = 0, o = 0;
  while (i < na && j < nb) {
    if (av[i] < bv[j]) {
      ov[o] = av[i];
      og[o] = ag[i];
      od[o] = ad[i] + (j > 0 ? add_a : 0);
      ++i;
    } else {
      ov[o] = bv[j];
      og[o] = bg[j];
      od[o] = bd[j] + (i > 0 ? add_b : 0);
      ++j;
    }
    ++o;
  }
  for (; i < na; ++i, ++o) {
    ov[o] = av[i];
    og[o] = ag[i];
    od[o] = ad[i];
  }
  for (; j < nb; ++j, ++o) {
    ov[o] = bv[j];
    og[o] = bg[j];
    od[o] = bd[j];
  }
  return o;
}

// Answers sorted percentiles `ps` (ascending) into `out` in the same order.
void fmlx_gk_query(const double* v, const int64_t* g, const int64_t* d, int64_t n, int64_t count, double rel_err,
                   const double* ps, int64_t np, double* out) {
  double target = (double)INT64_MIN;
  for (int64_t i = 0; i < n; ++i) target = std::fmax(target, (double)(d[i] + g[i]));
  target /= 2;
  int64_t index = 0, min_rank = g[0];
  for (int64_t q = 0; q < np; ++q) {
    const double p = ps[q];
    if (p <= rel_err) {
      out[q] = v[0];
    } else if (p >= 1 - rel_err) {
      out[q] = v[n - 1];
    } else {
      const int64_t rank = (int64_t)std::ceil(p * (double)count);
      int64_t mr = min_rank, i = index;
      bool found = false;
      while (i < n - 1) {
        const int64_t max_rank = mr + d[i];
        if ((double)max_rank - target < (double)rank && (double)rank <= (double)mr + target) {
          found = true;
          break;
        }
        ++i;
        mr += g[i];
      }
      if (found) {
        index = i;
        min_rank = mr;
        out[q] = v[i];
      } else {
        index = n - 1;
        min_rank = 0;
        out[q] = v[n - 1];
      }
    }
  }
}
}
