// Append-only record cache with memory segments that spill to files (the role of the reference's
// DataCacheWriter/DataCacheReader + MemorySegmentPool, ITER/datacache/nonkeyed/*.java: segments up
// to a size cap, kept in managed memory while the budget allows, written to the cache directory
// once it does not; readers replay records in order and can resume from any record).
//
// Records are opaque byte strings. Each record lives entirely inside one segment (a record larger
// than the segment size gets a segment of its own). Random access by record index: the index
// holds (segment, offset, length). Memory segments can be spilled explicitly (e.g. before a big
// device allocation) and the whole cache can be reopened from its directory via the manifest
// written by fmlx_dc_finish, which is what a checkpoint stores.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

namespace {
struct Segment {
  char* mem = nullptr;    // non-null while memory-resident
  int64_t cap = 0;        // allocated bytes (memory)
  int64_t used = 0;       // bytes written
  std::string file;       // non-empty once on disk
  int fd = -1;            // open for reading/appending when on disk
};

struct Rec {
  int32_t seg;
  int64_t off, len;
};

struct Cache {
  std::string dir;
  int64_t seg_bytes, mem_budget, mem_used = 0, file_bytes = 0;
  std::vector<Segment> segs;
  std::vector<Rec> recs;
  std::mutex mu;
  int next_file = 0;
};

std::string seg_path(Cache* c, int idx) {
  char buf[64];
  std::snprintf(buf, sizeof buf, "/segment-%06d", idx);
  return c->dir + buf;
}

bool write_all(int fd, const char* p, int64_t n) {
  while (n > 0) {
    const ssize_t w = ::write(fd, p, (size_t)(n > (1 << 30) ? (1 << 30) : n));
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= w;
  }
  return true;
}

bool read_all(int fd, char* p, int64_t n, int64_t off) {
  while (n > 0) {
    const ssize_t r = ::pread(fd, p, (size_t)(n > (1 << 30) ? (1 << 30) : n), off);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= r;
    off += r;
  }
  return true;
}

// moves a memory segment to its file; returns 0 on success
int spill(Cache* c, int idx) {
  Segment& s = c->segs[idx];
  if (!s.mem) return 0;
  s.file = seg_path(c, idx);
  s.fd = ::open(s.file.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0644);
  if (s.fd < 0) return -1;
  if (!write_all(s.fd, s.mem, s.used)) return -2;
  std::free(s.mem);
  s.mem = nullptr;
  c->mem_used -= s.cap;
  c->file_bytes += s.used;
  return 0;
}

int new_segment(Cache* c, int64_t need) {
  Segment s;
  const int64_t cap = need > c->seg_bytes ? need : c->seg_bytes;
  if (c->mem_used + cap <= c->mem_budget) {
    // page-aligned: the out-of-core trainers pin memory segments in place (hipHostRegister)
    void* p = nullptr;
    s.mem = ::posix_memalign(&p, 4096, (size_t)cap) == 0 ? (char*)p : nullptr;
    if (s.mem) {
      s.cap = cap;
      c->mem_used += cap;
    }
  }
  c->segs.push_back(s);
  const int idx = (int)c->segs.size() - 1;
  if (!c->segs[idx].mem) {  // budget exhausted or allocation failed: file-backed segment
    Segment& f = c->segs[idx];
    f.file = seg_path(c, idx);
    f.fd = ::open(f.file.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0644);
    if (f.fd < 0) return -1;
  }
  return idx;
}
}  // namespace

extern "C" {

void* fmlx_dc_open(const char* dir, int64_t seg_bytes, int64_t mem_budget) {
  ::mkdir(dir, 0755);
  Cache* c = new Cache();
  c->dir = dir;
  c->seg_bytes = seg_bytes > 0 ? seg_bytes : (int64_t)1 << 30;
  c->mem_budget = mem_budget;
  return c;
}

// Appends one record; returns its index (>= 0) or a negative error.
int64_t fmlx_dc_append(void* h, const void* data, int64_t n) {
  Cache* c = (Cache*)h;
  std::lock_guard<std::mutex> g(c->mu);
  int idx = (int)c->segs.size() - 1;
  bool fits = false;
  if (idx >= 0) {
    const Segment& s = c->segs[idx];
    fits = s.mem ? (s.used + n <= s.cap) : (s.used + n <= c->seg_bytes && s.used > 0);
  }
  if (!fits) {
    idx = new_segment(c, n);
    if (idx < 0) return -1;
  }
  Segment& s = c->segs[idx];
  if (s.mem) {
    std::memcpy(s.mem + s.used, data, (size_t)n);
  } else {
    if (::lseek(s.fd, s.used, SEEK_SET) < 0 || !write_all(s.fd, (const char*)data, n)) return -2;
    c->file_bytes += n;
  }
  c->recs.push_back(Rec{idx, s.used, n});
  s.used += n;
  return (int64_t)c->recs.size() - 1;
}

int64_t fmlx_dc_num_records(void* h) { return (int64_t)((Cache*)h)->recs.size(); }

int64_t fmlx_dc_record_size(void* h, int64_t i) {
  Cache* c = (Cache*)h;
  return (i < 0 || i >= (int64_t)c->recs.size()) ? -1 : c->recs[i].len;
}

// Copies record i into dst (capacity >= its size). Returns 0 or a negative error.
int fmlx_dc_read(void* h, int64_t i, void* dst) {
  Cache* c = (Cache*)h;
  if (i < 0 || i >= (int64_t)c->recs.size()) return -1;
  const Rec r = c->recs[i];
  const Segment& s = c->segs[r.seg];
  if (s.mem) {
    std::memcpy(dst, s.mem + r.off, (size_t)r.len);
    return 0;
  }
  return read_all(s.fd, (char*)dst, r.len, r.off) ? 0 : -2;
}

// Spills every memory segment to disk (returns 0 or a negative error).
// address of record i inside a memory segment (nullptr: the record lives in a file segment)
void* fmlx_dc_record_ptr(void* h, int64_t i) {
  Cache* c = (Cache*)h;
  if (i < 0 || i >= (int64_t)c->recs.size()) return nullptr;
  const Rec r = c->recs[i];
  const Segment& s = c->segs[r.seg];
  return s.mem ? (void*)(s.mem + r.off) : nullptr;
}

// memory segment idx: its base and capacity (0 / nullptr for file segments or a bad index)
void* fmlx_dc_segment_mem(void* h, int64_t idx, int64_t* cap) {
  Cache* c = (Cache*)h;
  *cap = 0;
  if (idx < 0 || idx >= (int64_t)c->segs.size() || !c->segs[idx].mem) return nullptr;
  *cap = c->segs[idx].cap;
  return c->segs[idx].mem;
}

int fmlx_dc_spill_all(void* h) {
  Cache* c = (Cache*)h;
  std::lock_guard<std::mutex> g(c->mu);
  for (int i = 0; i < (int)c->segs.size(); ++i) {
    const int rc = spill(c, i);
    if (rc) return rc;
  }
  return 0;
}

// stats[0..3] = memory bytes, file bytes, #segments, #memory segments
void fmlx_dc_stats(void* h, int64_t* stats) {
  Cache* c = (Cache*)h;
  int64_t m = 0;
  for (auto& s : c->segs) m += s.mem ? 1 : 0;
  stats[0] = c->mem_used;
  stats[1] = c->file_bytes;
  stats[2] = (int64_t)c->segs.size();
  stats[3] = m;
}

// Spills everything and writes `<dir>/MANIFEST` (binary: int64 nsegs, per segment int64 used;
// int64 nrecs, per record int32 seg + int64 off + int64 len). Afterwards the cache can be
// reopened with fmlx_dc_reopen (checkpoint/restore of cached inputs).
int fmlx_dc_finish(void* h) {
  Cache* c = (Cache*)h;
  int rc = fmlx_dc_spill_all(h);
  if (rc) return rc;
  for (auto& s : c->segs)
    if (s.fd >= 0) ::fsync(s.fd);
  const std::string tmp = c->dir + "/.MANIFEST.tmp", fin = c->dir + "/MANIFEST";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return -3;
  int64_t ns = (int64_t)c->segs.size(), nr = (int64_t)c->recs.size();
  std::fwrite(&ns, 8, 1, f);
  for (auto& s : c->segs) std::fwrite(&s.used, 8, 1, f);
  std::fwrite(&nr, 8, 1, f);
  for (auto& r : c->recs) {
    std::fwrite(&r.seg, 4, 1, f);
    std::fwrite(&r.off, 8, 1, f);
    std::fwrite(&r.len, 8, 1, f);
  }
  std::fclose(f);
  return std::rename(tmp.c_str(), fin.c_str()) == 0 ? 0 : -4;
}

void* fmlx_dc_reopen(const char* dir) {
  const std::string man = std::string(dir) + "/MANIFEST";
  FILE* f = std::fopen(man.c_str(), "rb");
  if (!f) return nullptr;
  Cache* c = new Cache();
  c->dir = dir;
  c->seg_bytes = (int64_t)1 << 30;
  c->mem_budget = 0;
  int64_t ns = 0, nr = 0;
  bool ok = std::fread(&ns, 8, 1, f) == 1;
  for (int64_t i = 0; ok && i < ns; ++i) {
    Segment s;
    ok = std::fread(&s.used, 8, 1, f) == 1;
    s.file = seg_path(c, (int)i);
    s.fd = ::open(s.file.c_str(), O_RDWR);
    ok = ok && s.fd >= 0;
    c->file_bytes += s.used;
    c->segs.push_back(s);
  }
  ok = ok && std::fread(&nr, 8, 1, f) == 1;
  for (int64_t i = 0; ok && i < nr; ++i) {
    Rec r;
    ok = std::fread(&r.seg, 4, 1, f) == 1 && std::fread(&r.off, 8, 1, f) == 1 && std::fread(&r.len, 8, 1, f) == 1;
    c->recs.push_back(r);
  }
  std::fclose(f);
  if (!ok) {
    for (auto& s : c->segs)
      if (s.fd >= 0) ::close(s.fd);
    delete c;
    return nullptr;
  }
  return c;
}

// Frees memory, closes files; deletes the segment files and manifest when `remove` is set.
void fmlx_dc_close(void* h, int remove) {
  Cache* c = (Cache*)h;
  for (auto& s : c->segs) {
    if (s.mem) std::free(s.mem);
    if (s.fd >= 0) ::close(s.fd);
    if (remove && !s.file.empty()) ::unlink(s.file.c_str());
  }
  if (remove) {
    ::unlink((c->dir + "/MANIFEST").c_str());
    ::rmdir(c->dir.c_str());
  }
  delete c;
}
}
