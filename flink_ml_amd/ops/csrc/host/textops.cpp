// Text-stage helpers over the DISTINCT strings of a dictionary-encoded column (the rows
// themselves stay device codes): Tokenizer's `toLowerCase()` + `String.split("\\s")` for a batch
// of strings with the produced tokens deduplicated into a vocabulary — the per-distinct-string
// host work that dominates high-cardinality columns (reference Tokenizer.java:55-66).
//
// ASCII only: a string with a byte >= 0x80 makes the call return -1 so the caller takes the
// general (Unicode-aware) path. Java semantics kept: `\s` = [ \t\n\x0B\f\r]; "" splits to [""];
// a leading delimiter yields a leading empty token; trailing empty tokens are removed.
#include <cstdint>
#include <cstring>
#include <vector>

namespace {
inline bool java_ws(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == 0x0B || c == '\f' || c == '\r'; }
inline char lower_ascii(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }

// 64-bit hash of a byte string (8 bytes per step)
inline uint64_t hash_bytes(const char* p, int64_t len) {
  uint64_t h = 0x9e3779b97f4a7c15ULL ^ (uint64_t)len;
  int64_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t w;
    std::memcpy(&w, p + i, 8);
    h = (h ^ w) * 0xff51afd7ed558ccdULL;
    h ^= h >> 32;
  }
  uint64_t t = 0;
  for (int64_t k = 0; i < len; ++i, ++k) t |= (uint64_t)(unsigned char)p[i] << (8 * k);
  h = (h ^ t) * 0xc4ceb9fe1a85ec53ULL;
  return h ^ (h >> 29);
}
}  // namespace

extern "C" {

// bytes/offs: n strings (offs[n+1]). Outputs: ntok[n] tokens per string, tok_ids[] (capacity
// tok_cap) the vocabulary id of every token in order, vocab_bytes (capacity = total bytes +
// tok_cap) the distinct tokens in first-seen order, each followed by '\n' (a token never contains
// one), with vocab_offs[] (capacity tok_cap + 1) their start offsets and *nvocab their count.
// Returns the total number of tokens, -1 for non-ASCII input, -2 when a capacity is too small.
// General form: split on a single-character class (`delim`, a 128-entry table over ASCII), `plus`
// = runs of delimiters are ONE delimiter (pattern `X+`), optional lowercasing, tokens shorter than
// `min_len` dropped (RegexTokenizer.java:74-90 with gaps = true on a one-character pattern).
int64_t fmlx_tokenize_class(const char* bytes, const int64_t* offs, int64_t n, const uint8_t* delim, int plus,
                            int lower, int min_len, int32_t* ntok, int32_t* tok_ids, int64_t tok_cap,
                            char* vocab_bytes, int64_t* vocab_offs, int64_t* nvocab) {
  auto isd = [&](unsigned char c) -> bool { return delim[c & 0x7f] != 0; };
  const int64_t total_bytes = offs[n];
  for (int64_t i = 0; i < total_bytes; ++i)
    if ((unsigned char)bytes[i] >= 0x80) return -1;
  // lowercased copy lives in vocab_bytes' scratch? no: tokens are views into a lowered buffer
  char* low = new char[total_bytes > 0 ? total_bytes : 1];
  for (int64_t i = 0; i < total_bytes; ++i) low[i] = lower ? lower_ascii(bytes[i]) : bytes[i];
  // token → id: open addressing over token hashes (ids index vocab_offs; a flat table is several
  // times faster than std::unordered_map at a million distinct tokens)
  int64_t cap = 16;
  while (cap < 2 * (n + 8)) cap <<= 1;
  std::vector<int32_t> slot((size_t)cap, -1);
  std::vector<uint64_t> vhash;
  vhash.reserve((size_t)n + 16);
  int64_t nt = 0, vb = 0, nv = 0;
  vocab_offs[0] = 0;
  auto grow = [&]() {
    cap <<= 1;
    std::vector<int32_t> ns((size_t)cap, -1);
    const uint64_t m2 = (uint64_t)cap - 1;
    for (int64_t v = 0; v < nv; ++v) {
      uint64_t q = vhash[v] & m2;
      while (ns[q] >= 0) q = (q + 1) & m2;
      ns[q] = (int32_t)v;
    }
    slot.swap(ns);
  };
  auto emit = [&](const char* p, int64_t len) -> bool {
    if (nt >= tok_cap) return false;
    const uint64_t h = hash_bytes(p, len);
    uint64_t q = h & ((uint64_t)cap - 1);
    int32_t id = -1;
    while (true) {
      const int32_t v = slot[q];
      if (v < 0) break;
      const int64_t vl = vocab_offs[v + 1] - vocab_offs[v] - 1;
      if (vhash[v] == h && vl == len && std::memcmp(vocab_bytes + vocab_offs[v], p, (size_t)len) == 0) {
        id = v;
        break;
      }
      q = (q + 1) & ((uint64_t)cap - 1);
    }
    if (id < 0) {
      std::memcpy(vocab_bytes + vb, p, (size_t)len);
      id = (int32_t)nv;
      slot[q] = id;
      vhash.push_back(h);
      vb += len;
      vocab_bytes[vb++] = '\n';
      vocab_offs[++nv] = vb;
      if (2 * nv > cap) grow();
    }
    tok_ids[nt++] = id;
    return true;
  };
  for (int64_t s = 0; s < n; ++s) {
    const char* p = low + offs[s];
    const int64_t len = offs[s + 1] - offs[s];
    const int64_t before = nt;
    if (len == 0) {  // no match: the (empty) string itself
      if (min_len <= 0 && !emit(p, 0)) { delete[] low; return -2; }
      ntok[s] = (int32_t)(nt - before);
      continue;
    }
    // trailing empty tokens are dropped: the last token ends at the last non-delimiter
    int64_t end = len;
    while (end > 0 && isd((unsigned char)p[end - 1])) --end;
    if (end == 0) {  // only delimiters: Java yields an empty array
      ntok[s] = 0;
      continue;
    }
    int64_t start = 0;
    for (int64_t i = 0; i <= end; ++i) {
      if (i == end || isd((unsigned char)p[i])) {
        if (i - start >= min_len && !emit(p + start, i - start)) { delete[] low; return -2; }
        if (plus)
          while (i + 1 < end && isd((unsigned char)p[i + 1])) ++i;  // a run is ONE delimiter
        start = i + 1;
      }
    }
    ntok[s] = (int32_t)(nt - before);
  }
  delete[] low;
  *nvocab = nv;
  return nt;
}

int64_t fmlx_tokenize_ws_lower(const char* bytes, const int64_t* offs, int64_t n, int32_t* ntok, int32_t* tok_ids,
                               int64_t tok_cap, char* vocab_bytes, int64_t* vocab_offs, int64_t* nvocab) {
  uint8_t ws[128] = {0};
  for (int c = 0; c < 128; ++c) ws[c] = java_ws((unsigned char)c) ? 1 : 0;
  return fmlx_tokenize_class(bytes, offs, n, ws, 0, 1, 0, ntok, tok_ids, tok_cap, vocab_bytes, vocab_offs, nvocab);
}
}

extern "C" {
// String.hashCode() of n strings given as UTF-16 code units (offs in units): s[0]·31^(n-1) + ...
void fmlx_java_string_hashes(const uint16_t* units, const int64_t* offs, int64_t n, int32_t* out) {
  for (int64_t s = 0; s < n; ++s) {
    uint32_t h = 0;
    for (int64_t i = offs[s]; i < offs[s + 1]; ++i) h = 31u * h + units[i];
    out[s] = (int32_t)h;
  }
}
}
