// Host read ingest (include/gqingest.h): BGZF/BAM -> SoA, MD tag -> MD events.
//
// Restates the reference's loading path (paths relative to
// /root/reference/src/main/scala/org/hammerlab/guacamole/):
//   Read.loadReadRDDAndSequenceDictionaryFromBAM + per-record filters   reads/Read.scala:368-451
//   Read.fromSAMRecord (isMapped, sample from RG, 0-based start)        reads/Read.scala:217-291
//   ReadSet.mappedReads                                                 ReadSet.scala:47-53
//   MappedRead: quals.length == sequence.length; end = start + padded reference length
//                                                                       reads/MappedRead.scala:50-51, 87
//   ADAM MdTag(md, start, cigar) as MappedRead.apply builds it          reads/MappedRead.scala:114-131
// guacamole_amd/reads.py (_load_bam) and soa.md_events are the Python statements of the same
// rules; tests/test_ingest.py checks both produce identical arrays.
//
// Layout of the work: the file is mapped; BGZF block boundaries are found by hopping over
// BSIZE fields; every block is inflated (raw deflate) in parallel straight into its slot of
// one contiguous buffer (ISIZE prefix sums), CRC32 checked.  Record boundaries are a
// sequential hop over block_size fields.  gq_bam_scan parses and filters the records in
// parallel chunks and keeps, per kept read, its record offset, MD position and read group;
// gq_bam_fill decodes the kept records straight into the caller's arrays (pool offsets from
// a per-block pre-pass), in file order when the file is coordinate-sorted and through a
// stable permutation otherwise.
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/gqingest.h"

namespace {

thread_local std::string g_err;

gqi_status fail(gqi_status s, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return s;
}

int threads_of(int32_t n) {
  if (n > 0) return n;
  const unsigned h = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(h ? h : 1u, 16u));
}

// fn(k) for k in [0, n) on up to nt threads, work handed out in order
template <class F>
void parallel_for(int64_t n, int nt, F fn) {
  if (n <= 0) return;
  nt = (int)std::min<int64_t>(nt, n);
  if (nt <= 1) {
    for (int64_t k = 0; k < n; ++k) fn(k);
    return;
  }
  std::atomic<int64_t> next{0};
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&]() {
      for (int64_t k; (k = next.fetch_add(1)) < n;) fn(k);
    });
  for (auto &x : th) x.join();
}

inline uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
inline int32_t rd32s(const uint8_t *p) { return (int32_t)rd32(p); }

// CIGAR op classes (htsjdk CigarOperator): M I D N S H P = X -> 0..8
constexpr uint32_t kConsumesRef = (1u << 0) | (1u << 2) | (1u << 3) | (1u << 7) | (1u << 8);
constexpr uint32_t kPaddedRef = kConsumesRef | (1u << 6);  // getPaddedReferenceLength also counts P
constexpr uint32_t kMdConsumed = (1u << 0) | (1u << 2) | (1u << 7) | (1u << 8);  // M D = X

// ------------------------------------------------------------------------------------------
// BGZF
struct Block {
  int64_t in_off;   // offset of the deflate payload in the file
  int64_t in_len;   // payload bytes
  int64_t out_off;  // offset of the inflated bytes
  uint32_t isize, crc;
};

// gzip member header at p (RFC 1952) -> payload offset; BGZF BSIZE in *bsize (or -1)
bool gzip_header(const uint8_t *p, int64_t avail, int64_t *payload, int64_t *bsize) {
  if (avail < 18 || p[0] != 31 || p[1] != 139 || p[2] != 8) return false;
  const uint8_t flg = p[3];
  int64_t o = 10;
  *bsize = -1;
  if (flg & 4) {
    const int64_t xlen = rd16(p + 10);
    o = 12;
    if (o + xlen > avail) return false;
    for (int64_t q = o; q + 4 <= o + xlen;) {
      const int slen = rd16(p + q + 2);
      if (p[q] == 66 && p[q + 1] == 67 && slen == 2) *bsize = (int64_t)rd16(p + q + 4) + 1;
      q += 4 + slen;
    }
    o += xlen;
  }
  if (flg & 8) {  // FNAME
    while (o < avail && p[o]) ++o;
    ++o;
  }
  if (flg & 16) {  // FCOMMENT
    while (o < avail && p[o]) ++o;
    ++o;
  }
  if (flg & 2) o += 2;  // FHCRC
  if (o > avail) return false;
  *payload = o;
  return true;
}

// whole gzip stream (one or more members), sequentially: a .gz without BGZF block sizes
gqi_status inflate_stream(const uint8_t *p, int64_t n, std::vector<uint8_t> &out) {
  z_stream z;
  memset(&z, 0, sizeof(z));
  if (inflateInit2(&z, 15 + 16) != Z_OK) return fail(GQI_E_NOMEM, "inflateInit2 failed");
  out.clear();
  std::vector<uint8_t> buf(1 << 20);
  int64_t in = 0;
  while (in < n) {
    int rc = Z_OK;
    z.next_in = const_cast<uint8_t *>(p + in);
    z.avail_in = (uInt)std::min<int64_t>(n - in, 1 << 30);
    const uInt given = z.avail_in;
    while (rc != Z_STREAM_END) {
      z.next_out = buf.data();
      z.avail_out = (uInt)buf.size();
      rc = inflate(&z, Z_NO_FLUSH);
      if (rc != Z_OK && rc != Z_STREAM_END) {
        inflateEnd(&z);
        return fail(GQI_E_FORMAT, "gzip stream: inflate error %d", rc);
      }
      out.insert(out.end(), buf.data(), buf.data() + (buf.size() - z.avail_out));
      if (rc == Z_OK && z.avail_in == 0 && z.avail_out != 0) break;  // needs more input
    }
    in += given - z.avail_in;
    if (rc == Z_STREAM_END) {
      inflateReset(&z);
    } else if (in >= n) {
      inflateEnd(&z);
      return fail(GQI_E_FORMAT, "gzip stream: truncated");
    }
  }
  inflateEnd(&z);
  return GQI_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------
struct Kept {  // a record that passed the filters
  int64_t rec;    // offset of its block_size field in the inflated stream
  int64_t md_at;  // offset of its MD value, -1: no MD tag
  int32_t md_len;
  int32_t rg;     // chunk-local RG id (global after gq_bam_scan), -1: none
};

struct Chunk {  // the records of one range of the file
  std::vector<Kept> kept;
  std::vector<std::string> rg_vals;  // chunk-local RG values, first appearance order
  std::vector<int64_t> rg_first;     // chunk-local kept index of each RG value's first read
  int64_t none_first = -1;           // ... and of the first kept read without an RG tag
  int64_t seq = 0, cigar = 0, md = 0, names = 0;  // pool totals of the kept reads
  bool sorted = true;                // kept reads in (contig, start) order within the chunk
  int32_t c0 = 0, c1 = 0;            // (contig, start) of the first and last kept read
  int64_t s0 = 0, s1 = 0;
  gqi_status err = GQI_OK;
  std::string err_msg;
};

struct gq_bam {
  int fd = -1;
  const uint8_t *map = nullptr;
  size_t map_len = 0;
  struct Bytes {  // inflated BAM stream: anonymous mapping on huge pages, faulted in by the inflate threads
    uint8_t *p = nullptr;
    int64_t n = 0;
    size_t cap = 0;
    bool alloc(int64_t len) {
      cap = (size_t)std::max<int64_t>(len, 1);
      void *m = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (m == MAP_FAILED) return false;
      madvise(m, cap, MADV_HUGEPAGE);
      p = (uint8_t *)m;
      n = len;
      return true;
    }
    ~Bytes() {
      if (p) munmap(p, cap);
    }
    uint8_t *data() { return p; }
    const uint8_t *data() const { return p; }
    size_t size() const { return (size_t)n; }
  } data;
  std::string text;
  std::vector<std::string> contig_names;
  std::vector<int64_t> contig_lengths;
  int64_t rec0 = 0;  // first alignment record
  // last scan
  std::vector<Kept> kept;  // every kept read, file order
  std::vector<std::string> rgs;
  std::vector<int64_t> rg_first;  // [1 + n_rg]: first kept read (file order) without RG, with RG k
  std::vector<int64_t> order;  // output read -> file-order read (empty: already sorted)
  gq_bam_sizes sizes{};
  bool scanned = false;
};

namespace {

// Raw-deflate backend for BGZF blocks: libdeflate when the system has it (a whole-buffer
// decoder, ~2x zlib's inflate here, and a folded CRC32), else zlib.  Both decode the same
// bytes; the choice only changes speed.  libdeflate ships without a header in this image,
// so its four entry points (stable since libdeflate 1.0) are resolved with dlsym.
struct Deflate {
  void *(*alloc)() = nullptr;
  int (*dec)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;
  uint32_t (*crc)(uint32_t, const void *, size_t) = nullptr;
};
const Deflate &deflate_lib() {
  static const Deflate lz = []() {
    Deflate x;
    if (getenv("GQ_INGEST_ZLIB")) return x;
    void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.alloc = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
    x.dec = (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(h, "libdeflate_deflate_decompress");
    x.crc = (uint32_t(*)(uint32_t, const void *, size_t))dlsym(h, "libdeflate_crc32");
    if (!x.alloc || !x.dec || !x.crc) x = Deflate();
    return x;
  }();
  return lz;
}

gqi_status inflate_bgzf(gq_bam *b, int nt) {
  const uint8_t *p = b->map;
  const int64_t n = (int64_t)b->map_len;
  std::vector<Block> blocks;
  int64_t off = 0, out = 0;
  bool bgzf = true;
  while (off < n) {
    int64_t payload, bsize;
    if (!gzip_header(p + off, n - off, &payload, &bsize))
      return fail(GQI_E_FORMAT, "not a BGZF/gzip member at file offset %lld", (long long)off);
    if (bsize < 0) {
      bgzf = false;
      break;
    }
    if (off + bsize > n || bsize < payload + 8)
      return fail(GQI_E_FORMAT, "truncated BGZF block at file offset %lld", (long long)off);
    Block k;
    k.in_off = off + payload;
    k.in_len = bsize - payload - 8;
    k.crc = rd32(p + off + bsize - 8);
    k.isize = rd32(p + off + bsize - 4);
    k.out_off = out;
    out += k.isize;
    blocks.push_back(k);
    off += bsize;
  }
  if (!bgzf) {
    std::vector<uint8_t> v;
    const gqi_status s = inflate_stream(p, n, v);
    if (s != GQI_OK) return s;
    if (!b->data.alloc((int64_t)v.size())) return fail(GQI_E_NOMEM, "inflated stream of %zu bytes", v.size());
    memcpy(b->data.p, v.data(), v.size());
    return GQI_OK;
  }
  if (!b->data.alloc(out)) return fail(GQI_E_NOMEM, "inflated stream of %lld bytes", (long long)out);
  const Deflate &lz = deflate_lib();
  std::atomic<int64_t> bad{-1};
  parallel_for((int64_t)blocks.size(), nt, [&](int64_t i) {
    const Block &k = blocks[i];
    uint8_t *dst = b->data.data() + k.out_off;
    bool ok;
    if (lz.dec) {  // libdeflate: whole-buffer decoder, no stream state
      thread_local void *d = nullptr;
      if (!d) d = lz.alloc();
      size_t got = 0;
      ok = d && lz.dec(d, p + k.in_off, (size_t)k.in_len, dst, k.isize, &got) == 0 && got == k.isize;
      if (ok) ok = lz.crc(0, dst, k.isize) == k.crc;
    } else {
      z_stream z;
      memset(&z, 0, sizeof(z));
      ok = inflateInit2(&z, -15) == Z_OK;
      if (ok) {
        z.next_in = const_cast<uint8_t *>(p + k.in_off);
        z.avail_in = (uInt)k.in_len;
        z.next_out = dst;
        z.avail_out = k.isize;
        const int rc = inflate(&z, Z_FINISH);
        ok = rc == Z_STREAM_END && z.total_out == k.isize;
        inflateEnd(&z);
      }
      if (ok) ok = (uint32_t)crc32(0L, dst, k.isize) == k.crc;
    }
    if (!ok) {
      int64_t cur = bad.load();
      while ((cur < 0 || i < cur) && !bad.compare_exchange_weak(cur, i)) {
      }
    }
  });
  if (bad.load() >= 0) {
    const Block &k = blocks[bad.load()];
    return fail(GQI_E_FORMAT, "corrupt BGZF block (inflate, ISIZE or CRC32) with payload at file offset %lld",
                (long long)k.in_off);
  }
  return GQI_OK;
}

gqi_status parse_header(gq_bam *b) {
  const uint8_t *d = b->data.data();
  const int64_t n = (int64_t)b->data.size();
  if (n < 12 || memcmp(d, "BAM\1", 4) != 0) return fail(GQI_E_FORMAT, "not a BAM file (magic)");
  int64_t o = 4;
  const int64_t l_text = rd32s(d + o);
  o += 4;
  if (l_text < 0 || o + l_text + 4 > n) return fail(GQI_E_FORMAT, "truncated BAM header");
  b->text.assign((const char *)d + o, (size_t)l_text);
  while (!b->text.empty() && b->text.back() == '\0') b->text.pop_back();
  o += l_text;
  const int32_t n_ref = rd32s(d + o);
  o += 4;
  for (int32_t i = 0; i < n_ref; ++i) {
    if (o + 4 > n) return fail(GQI_E_FORMAT, "truncated BAM reference dictionary");
    const int32_t l_name = rd32s(d + o);
    o += 4;
    if (l_name < 1 || o + l_name + 4 > n) return fail(GQI_E_FORMAT, "truncated BAM reference dictionary");
    b->contig_names.emplace_back((const char *)d + o, (size_t)(l_name - 1));
    o += l_name;
    b->contig_lengths.push_back(rd32s(d + o));
    o += 4;
  }
  b->rec0 = o;
  return GQI_OK;
}

// 2 bases per packed byte -> 2 ASCII bytes
struct SeqTable {
  uint16_t t[256];
  SeqTable() {
    const char *c = "=ACMGRSVTWYHKDBN";
    for (int v = 0; v < 256; ++v) t[v] = (uint16_t)((uint8_t)c[v >> 4] | ((uint16_t)(uint8_t)c[v & 15] << 8));
  }
};
const SeqTable kSeq;

bool loci_intersect(const gq_bam_filters *f, int32_t contig, int64_t s, int64_t e) {
  if (e <= s) return false;
  const int64_t b0 = f->loci_begin[contig], b1 = f->loci_begin[contig + 1];
  // first range with end > s (ranges sorted and disjoint: ends ascend)
  const int64_t *it = std::upper_bound(f->loci_end + b0, f->loci_end + b1, s);
  const int64_t k = it - f->loci_end;
  return k < b1 && f->loci_start[k] < e;
}

// plausible alignment record at o (every length field consistent with block_size)?
inline bool record_at(const uint8_t *d, int64_t n, int64_t o, int32_t n_ref) {
  if (o + 40 > n) return false;
  const int32_t bs = rd32s(d + o);
  if (bs < 32 || o + 4 + bs > n) return false;
  const uint8_t *p = d + o + 4;
  const int32_t ref_id = rd32s(p), pos = rd32s(p + 4), l_seq = rd32s(p + 16), next_ref = rd32s(p + 20);
  const uint32_t l_name = p[8], n_cig = rd16(p + 12);
  if (ref_id < -1 || ref_id >= n_ref || next_ref < -1 || next_ref >= n_ref || pos < -1 || l_seq < 0 || l_name < 1)
    return false;
  if (32 + (int64_t)l_name + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2 + l_seq > bs) return false;
  return p[32 + l_name - 1] == 0;
}

// Record boundaries: a hop over block_size fields is a dependent chain of cache misses, so
// the stream is cut into segments, each segment finds its first record by validating
// candidate offsets (a record must chain into 8 more plausible records) and hops to its end
// in parallel; a segment whose first record is not where the previous segment's chain lands
// (a false sync) is re-hopped from that landing point.  Segment 0 starts at the first record.
gqi_status record_offsets(const gq_bam *b, int nt, std::vector<int64_t> &recs) {
  const uint8_t *d = b->data.data();
  const int64_t n = (int64_t)b->data.size(), r0 = b->rec0;
  const int32_t n_ref = (int32_t)b->contig_names.size();
  const int64_t nseg = std::max<int64_t>(1, std::min<int64_t>(4 * nt, (n - r0) / (1 << 20)));
  const int64_t len = (n - r0 + nseg - 1) / std::max<int64_t>(nseg, 1);
  std::vector<std::vector<int64_t>> seg((size_t)nseg);
  std::vector<int64_t> land((size_t)nseg, -1);  // first offset >= the segment's end reached by its chain
  std::vector<int> bad((size_t)nseg, 0);
  auto hop = [&](int64_t o, int64_t stop, std::vector<int64_t> &out, int64_t *landed) -> bool {
    while (o < stop) {
      if (o + 4 > n) return false;
      const int32_t bs = rd32s(d + o);
      if (bs < 32 || o + 4 + bs > n) return false;
      out.push_back(o);
      o += 4 + bs;
    }
    *landed = o;
    return true;
  };
  parallel_for(nseg, nt, [&](int64_t k) {
    const int64_t a = r0 + k * len, e = std::min(n, a + len);
    if (a >= e) {
      land[k] = a;
      return;
    }
    int64_t o = a;
    if (k > 0) {  // sync: the first offset that chains into 8 more plausible records
      for (; o < e; ++o) {
        int64_t q = o;
        int ok = 0;
        while (ok < 9 && q < n && record_at(d, n, q, n_ref)) {
          q += 4 + rd32s(d + q);
          ++ok;
        }
        if (ok == 9 || (ok > 0 && q == n)) break;
      }
    }
    seg[k].reserve((size_t)((e - a) / 256 + 16));
    if (!hop(o, e, seg[k], &land[k])) bad[k] = 1;
  });
  recs.clear();
  int64_t at = r0;  // where the true chain stands
  for (int64_t k = 0; k < nseg; ++k) {
    const int64_t a = r0 + k * len, e = std::min(n, a + len);
    if (at >= e) continue;  // the previous chain already covered this segment
    if (!bad[k] && !seg[k].empty() && seg[k][0] == at) {
      recs.insert(recs.end(), seg[k].begin(), seg[k].end());
      at = land[k];
    } else if (!bad[k] && seg[k].empty() && land[k] == at) {
      continue;
    } else {  // false sync (or none): hop this segment from the true chain
      std::vector<int64_t> v;
      int64_t l = -1;
      if (!hop(at, e, v, &l))
        return fail(GQI_E_FORMAT, "truncated BAM record %lld", (long long)(recs.size() + v.size()));
      recs.insert(recs.end(), v.begin(), v.end());
      at = l;
    }
  }
  if (at != n) return fail(GQI_E_FORMAT, "truncated BAM record %lld", (long long)recs.size());
  return GQI_OK;
}

// scan pass over records [r0, r1): parse, filter, remember the kept ones and their sizes
void scan_chunk(const gq_bam *b, const std::vector<int64_t> &recs, int64_t r0, int64_t r1, const gq_bam_filters *f,
                Chunk &c) {
  const uint8_t *d = b->data.data();
  const int32_t n_ref = (int32_t)b->contig_names.size();
  std::unordered_map<std::string, int32_t> rg_local;
  auto error = [&](gqi_status s, const char *fmt, auto... args) {
    char buf[400];
    snprintf(buf, sizeof(buf), fmt, args...);
    c.err = s;
    c.err_msg = buf;
  };
  c.kept.reserve((size_t)(r1 - r0));
  for (int64_t r = r0; r < r1; ++r) {
    const int64_t o = recs[r], end = recs[r + 1];
    const uint8_t *p = d + o + 4;
    const int32_t ref_id = rd32s(p), pos = rd32s(p + 4);
    const uint32_t l_read_name = p[8];
    const uint32_t n_cig = rd16(p + 12), flag = rd16(p + 14);
    const int32_t l_seq = rd32s(p + 16);
    const int64_t cig_at = o + 36 + l_read_name;
    const int64_t qual_at = cig_at + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2;
    int64_t q = qual_at + l_seq;
    if (l_seq < 0 || l_read_name < 1 || q > end) {
      error(GQI_E_FORMAT, "truncated BAM record %lld", (long long)r);
      return;
    }
    // aux fields: MD and RG (every record's aux is parsed, as the Python statement does)
    int64_t md_at = -1, md_n = 0, rg_at = -1, rg_n = 0;
    while (q < end) {
      if (q + 3 > end) {
        error(GQI_E_FORMAT, "truncated aux field in BAM record %lld", (long long)r);
        return;
      }
      const uint8_t t0 = d[q], t1 = d[q + 1], ty = d[q + 2];
      q += 3;
      switch (ty) {
        case 'A': case 'c': case 'C': q += 1; break;
        case 's': case 'S': q += 2; break;
        case 'i': case 'I': case 'f': q += 4; break;
        case 'Z': case 'H': {
          const uint8_t *z = (const uint8_t *)memchr(d + q, 0, (size_t)(end - q));
          if (!z) {
            error(GQI_E_FORMAT, "unterminated aux string in BAM record %lld", (long long)r);
            return;
          }
          const int64_t len = z - (d + q);
          if (t0 == 'M' && t1 == 'D') md_at = q, md_n = len;
          else if (t0 == 'R' && t1 == 'G') rg_at = q, rg_n = len;
          q += len + 1;
          break;
        }
        case 'B': {
          if (q + 5 > end) {
            error(GQI_E_FORMAT, "truncated aux array in BAM record %lld", (long long)r);
            return;
          }
          const uint8_t sub = d[q];
          const int64_t cnt = rd32s(d + q + 1);
          int w = 0;
          switch (sub) {
            case 'c': case 'C': w = 1; break;
            case 's': case 'S': w = 2; break;
            case 'i': case 'I': case 'f': w = 4; break;
            default:
              error(GQI_E_RECORD, "bad aux array type '%c'", (char)sub);
              return;
          }
          if (cnt < 0 || q + 5 + cnt * w > end) {  // (a negative count would walk backwards)
            error(GQI_E_FORMAT, "truncated aux array in BAM record %lld", (long long)r);
            return;
          }
          q += 5 + cnt * w;
          break;
        }
        default:
          error(GQI_E_RECORD, "bad aux type '%c'", (char)ty);
          return;
      }
    }
    // Read.scala:411-418 record filters, then isMapped / hasMdTag (Read.scala:421-428)
    const bool unmapped = (flag & 0x4) || ref_id < 0;
    if (unmapped || pos < 0 || ref_id >= n_ref) continue;
    if (f->use_loci) {
      int64_t ref_len = 0;
      for (uint32_t k = 0; k < n_cig; ++k) {
        const uint32_t v = rd32(d + cig_at + 4 * k), op = v & 15;
        if (op < 9 && (kConsumesRef >> op) & 1) ref_len += v >> 4;
      }
      if (!loci_intersect(f, ref_id, pos, pos + ref_len)) continue;
    }
    if (f->non_duplicate && (flag & 0x400)) continue;
    if (f->passed_vendor_quality_checks && (flag & 0x200)) continue;
    if (f->is_paired && !(flag & 0x1)) continue;
    if (f->has_md_tag && md_at < 0) continue;
    // htsjdk: missing qualities (0xFF) -> empty array -> MappedRead's length assertion
    if (l_seq > 0 && d[qual_at] == 0xFF) {
      error(GQI_E_RECORD, "Base qualities have length 0 but sequence has length %d", l_seq);
      return;
    }
    const int64_t k = (int64_t)c.kept.size();
    int32_t rg = -1;
    if (rg_at >= 0) {
      std::string v((const char *)d + rg_at, (size_t)rg_n);
      auto it = rg_local.find(v);
      if (it == rg_local.end()) {
        it = rg_local.emplace(v, (int32_t)c.rg_vals.size()).first;
        c.rg_vals.push_back(v);
        c.rg_first.push_back(k);
      }
      rg = it->second;
    } else if (c.none_first < 0) {
      c.none_first = k;
    }
    if (k == 0) {
      c.c0 = ref_id;
      c.s0 = pos;
    } else if (ref_id < c.c1 || (ref_id == c.c1 && pos < c.s1)) {
      c.sorted = false;
    }
    c.c1 = ref_id;
    c.s1 = pos;
    c.kept.push_back(Kept{o, md_at, (int32_t)md_n, rg});
    c.seq += l_seq;
    c.cigar += n_cig;
    c.md += md_at >= 0 ? md_n : 0;
    c.names += l_read_name - 1;
  }
}

}  // namespace

extern "C" {

const char *gq_ingest_last_error(void) { return g_err.c_str(); }

gqi_status gq_bam_open(const char *path, int32_t n_threads, gq_bam **out) {
  *out = nullptr;
  gq_bam *b = new (std::nothrow) gq_bam;
  if (!b) return fail(GQI_E_NOMEM, "gq_bam");
  b->fd = open(path, O_RDONLY);
  if (b->fd < 0) {
    delete b;
    return fail(GQI_E_IO, "cannot open %s", path);
  }
  struct stat st;
  if (fstat(b->fd, &st) != 0 || st.st_size == 0) {
    close(b->fd);
    delete b;
    return fail(GQI_E_IO, "cannot stat (or empty) %s", path);
  }
  b->map_len = (size_t)st.st_size;
  void *m = mmap(nullptr, b->map_len, PROT_READ, MAP_PRIVATE | MAP_POPULATE, b->fd, 0);
  if (m == MAP_FAILED) {
    close(b->fd);
    delete b;
    return fail(GQI_E_IO, "cannot map %s", path);
  }
  b->map = (const uint8_t *)m;
  madvise(m, b->map_len, MADV_SEQUENTIAL);
  gqi_status s = inflate_bgzf(b, threads_of(n_threads));
  if (s == GQI_OK) s = parse_header(b);
  if (s != GQI_OK) {
    gq_bam_close(b);
    return s;
  }
  *out = b;
  return GQI_OK;
}

void gq_bam_close(gq_bam *b) {
  if (!b) return;
  if (b->map) munmap(const_cast<uint8_t *>(b->map), b->map_len);
  if (b->fd >= 0) close(b->fd);
  delete b;
}

const char *gq_bam_header_text(const gq_bam *b) { return b->text.c_str(); }
int32_t gq_bam_n_contigs(const gq_bam *b) { return (int32_t)b->contig_names.size(); }
const char *gq_bam_contig_name(const gq_bam *b, int32_t i) {
  return (i >= 0 && i < (int32_t)b->contig_names.size()) ? b->contig_names[i].c_str() : nullptr;
}
int64_t gq_bam_contig_length(const gq_bam *b, int32_t i) {
  return (i >= 0 && i < (int32_t)b->contig_lengths.size()) ? b->contig_lengths[i] : -1;
}
const char *gq_bam_rg(const gq_bam *b, int32_t k) {
  return (k >= 0 && k < (int32_t)b->rgs.size()) ? b->rgs[k].c_str() : nullptr;
}
int64_t gq_bam_rg_first(const gq_bam *b, int32_t k) {
  return (k >= -1 && k + 1 < (int32_t)b->rg_first.size()) ? b->rg_first[k + 1] : -1;
}

gqi_status gq_bam_scan(gq_bam *b, const gq_bam_filters *f, int32_t n_threads, gq_bam_sizes *sizes) {
  if (!b || !f || !sizes) return fail(GQI_E_ARG, "null argument");
  if (f->use_loci && (!f->loci_begin || (!f->loci_start && f->loci_begin[b->contig_names.size()] > 0)))
    return fail(GQI_E_ARG, "use_loci without loci arrays");
  const int nt = threads_of(n_threads);
  b->scanned = false;
  const uint8_t *d = b->data.data();
  const int64_t n = (int64_t)b->data.size();
  std::vector<int64_t> recs;
  gqi_status st = record_offsets(b, nt, recs);
  if (st != GQI_OK) return st;
  const int64_t nrec = (int64_t)recs.size();
  recs.push_back(n);
  const int64_t per = 1 << 14;
  const int64_t nch = std::max<int64_t>(1, (nrec + per - 1) / per);
  std::vector<Chunk> chunks((size_t)nch);
  parallel_for(nch, nt, [&](int64_t k) {
    scan_chunk(b, recs, k * per, std::min(nrec, (k + 1) * per), f, chunks[k]);
  });
  for (auto &c : chunks)
    if (c.err != GQI_OK) {  // the first failing record in file order (chunks are in order)
      g_err = c.err_msg;
      return c.err;
    }
  // global RG table (first appearance), sizes, sortedness, kept-read offsets per chunk
  gq_bam_sizes z{};
  b->rgs.clear();
  b->rg_first.assign(1, -1);
  std::unordered_map<std::string, int32_t> rg_glob;
  std::vector<int64_t> k0((size_t)nch + 1, 0);
  std::vector<std::vector<int32_t>> rg_map((size_t)nch);
  bool sorted = true;
  bool any = false;
  int32_t pc = 0;
  int64_t ps = 0;
  for (int64_t k = 0; k < nch; ++k) {
    const Chunk &c = chunks[k];
    rg_map[k].resize(c.rg_vals.size());
    for (size_t j = 0; j < c.rg_vals.size(); ++j) {
      auto it = rg_glob.find(c.rg_vals[j]);
      if (it == rg_glob.end()) {
        it = rg_glob.emplace(c.rg_vals[j], (int32_t)b->rgs.size()).first;
        b->rgs.push_back(c.rg_vals[j]);
        b->rg_first.push_back(z.n_reads + c.rg_first[j]);
      }
      rg_map[k][j] = it->second;
    }
    if (b->rg_first[0] < 0 && c.none_first >= 0) b->rg_first[0] = z.n_reads + c.none_first;
    if (!c.kept.empty()) {
      if (!c.sorted || (any && (c.c0 < pc || (c.c0 == pc && c.s0 < ps)))) sorted = false;
      any = true;
      pc = c.c1;
      ps = c.s1;
    }
    k0[k] = z.n_reads;
    z.n_reads += (int64_t)c.kept.size();
    z.seq_bytes += c.seq;
    z.cigar_len += c.cigar;
    z.md_bytes += c.md;
    z.name_bytes += c.names;
  }
  k0[nch] = z.n_reads;
  z.n_rg = (int32_t)b->rgs.size();
  b->kept.resize((size_t)z.n_reads);
  parallel_for(nch, nt, [&](int64_t k) {
    const Chunk &c = chunks[k];
    for (size_t i = 0; i < c.kept.size(); ++i) {
      Kept x = c.kept[i];
      x.rg = x.rg < 0 ? -1 : rg_map[k][x.rg];
      b->kept[k0[k] + i] = x;
    }
  });
  // not coordinate-sorted: a stable permutation (ties keep file order)
  b->order.clear();
  if (!sorted) {
    std::vector<std::pair<int32_t, int32_t>> key((size_t)z.n_reads);
    parallel_for(z.n_reads, nt, [&](int64_t i) {
      const uint8_t *p = d + b->kept[i].rec + 4;
      key[i] = {rd32s(p), rd32s(p + 4)};
    });
    b->order.resize((size_t)z.n_reads);
    std::iota(b->order.begin(), b->order.end(), 0);
    std::stable_sort(b->order.begin(), b->order.end(), [&](int64_t x, int64_t y) { return key[x] < key[y]; });
  }
  z.sorted = sorted ? 1 : 0;
  b->sizes = z;
  b->scanned = true;
  *sizes = z;
  return GQI_OK;
}

gqi_status gq_bam_fill(gq_bam *b, int32_t n_threads, const gq_bam_reads *R) {
  if (!b || !R) return fail(GQI_E_ARG, "null argument");
  if (!b->scanned) return fail(GQI_E_ARG, "gq_bam_fill before gq_bam_scan");
  const int nt = threads_of(n_threads);
  const int64_t N = b->sizes.n_reads;
  const uint8_t *d = b->data.data();
  auto kept_of = [&](int64_t r) -> const Kept & { return b->kept[b->order.empty() ? r : b->order[r]]; };
  // pass 1: pool sizes per block of output reads; pass 2: every field, straight from the records
  const int64_t per = 1 << 14;
  const int64_t nblk = (N + per - 1) / per;
  std::vector<int64_t> bs(nblk + 1, 0), bc(nblk + 1, 0), bm(nblk + 1, 0), bn(nblk + 1, 0);
  parallel_for(nblk, nt, [&](int64_t q) {
    int64_t s = 0, cg = 0, m = 0, nm = 0;
    for (int64_t r = q * per; r < std::min(N, (q + 1) * per); ++r) {
      const Kept &x = kept_of(r);
      const uint8_t *p = d + x.rec + 4;
      s += rd32s(p + 16);
      cg += rd16(p + 12);
      m += x.md_at >= 0 ? x.md_len : 0;
      nm += p[8] - 1;
    }
    bs[q + 1] = s;
    bc[q + 1] = cg;
    bm[q + 1] = m;
    bn[q + 1] = nm;
  });
  for (int64_t q = 0; q < nblk; ++q) {
    bs[q + 1] += bs[q];
    bc[q + 1] += bc[q];
    bm[q + 1] += bm[q];
    bn[q + 1] += bn[q];
  }
  parallel_for(nblk, nt, [&](int64_t q) {
    int64_t s = bs[q], cg = bc[q], m = bm[q], nm = bn[q];
    for (int64_t r = q * per; r < std::min(N, (q + 1) * per); ++r) {
      const Kept &x = kept_of(r);
      const uint8_t *p = d + x.rec + 4;
      const int32_t ref_id = rd32s(p), pos = rd32s(p + 4);
      const uint32_t l_name = p[8] - 1u, mapq = p[9], n_cig = rd16(p + 12), flag = rd16(p + 14);
      const int32_t l_seq = rd32s(p + 16);
      const uint8_t *name = p + 32, *cg_p = name + l_name + 1, *sq = cg_p + 4 * n_cig, *ql = sq + (l_seq + 1) / 2;
      int64_t padded = 0;
      for (uint32_t k = 0; k < n_cig; ++k) {
        const uint32_t v = rd32(cg_p + 4 * k), op = v & 15;
        if (op < 9 && (kPaddedRef >> op) & 1) padded += v >> 4;
      }
      R->contig[r] = ref_id;
      R->start[r] = pos;
      R->end[r] = pos + padded;
      R->mapq[r] = (uint8_t)mapq;
      R->flags[r] = (flag & 0x10) ? 1 : 0;
      R->rg[r] = x.rg;
      R->seq_off[r] = s;
      R->seq_len[r] = l_seq;
      R->cigar_off[r] = cg;
      R->n_cigar[r] = (int32_t)n_cig;
      R->md_off[r] = m;
      R->md_len[r] = x.md_at >= 0 ? x.md_len : -1;
      R->name_off[r] = nm;
      R->name_len[r] = (int32_t)l_name;
      uint8_t *os = R->seq + s;
      for (int32_t k = 0; k < l_seq / 2; ++k) memcpy(os + 2 * k, &kSeq.t[sq[k]], 2);
      if (l_seq & 1) os[l_seq - 1] = (uint8_t)(kSeq.t[sq[l_seq / 2]] & 0xFF);
      memcpy(R->qual + s, ql, (size_t)l_seq);
      memcpy(R->cigar + cg, cg_p, 4 * (size_t)n_cig);
      if (x.md_at >= 0 && x.md_len) memcpy(R->md + m, d + x.md_at, (size_t)x.md_len);
      if (l_name) memcpy(R->names + nm, name, l_name);
      s += l_seq;
      cg += n_cig;
      m += x.md_at >= 0 ? x.md_len : 0;
      nm += l_name;
    }
  });
  return GQI_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// MD events (soa.md_events)
namespace {

// k-th MD-consumed reference offset (M/=/X/D positions; N gaps skipped); past the CIGAR's
// last such position the offsets continue one by one.  k only grows, so a cursor suffices.
struct MdCursor {
  const uint32_t *cig;
  int32_t n;
  int32_t op = 0;    // current CIGAR op
  int64_t used = 0;  // MD positions consumed in ops before `op`
  int64_t ref = 0;   // reference offset at the start of `op`
  int64_t last = -1; // last MD-consumed offset seen (for k past the end)
  int64_t total = 0; // MD positions in all ops before `op`
  MdCursor(const uint32_t *c, int32_t nn) : cig(c), n(nn) {}
  int64_t at(int64_t k) {
    while (op < n) {
      const uint32_t v = cig[op], o = v & 15, ln = v >> 4;
      const bool md = o < 9 && ((kMdConsumed >> o) & 1);
      if (md && k < total + ln) return ref + (k - total);
      if (md) {
        total += ln;
        if (ln) last = ref + ln - 1;
      }
      if (o < 9 && ((kConsumesRef >> o) & 1)) ref += ln;
      ++op;
    }
    return last + (k - total + 1);
  }
};

// parse one MD string; emit(off, base) for each event; -> mismatches or -1 (error in err)
template <class Emit>
int64_t md_parse(const uint8_t *s, int64_t n, const uint32_t *cig, int32_t ncig, Emit emit, std::string *err) {
  if (n == 0) return 0;
  MdCursor cur(cig, ncig);
  int64_t i = 0, k = 0, mism = 0;
  auto up = [](uint8_t c) -> uint8_t { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; };
  auto bad = [&](const char *what) {
    char buf[300];
    snprintf(buf, sizeof(buf), "MdTag b'%.*s': %s at %lld", (int)std::min<int64_t>(n, 200), (const char *)s, what,
             (long long)i);
    *err = buf;
    return (int64_t)-1;
  };
  auto digits = [&]() -> bool {
    const int64_t j0 = i;
    int64_t v = 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') v = v * 10 + (s[i++] - '0');
    if (i == j0) return false;
    k += v;
    return true;
  };
  if (!digits()) return bad("digit expected");
  while (i < n) {
    const uint8_t ch = up(s[i]);
    if (ch == '^') {
      ++i;
      while (i < n && up(s[i]) >= 'A' && up(s[i]) <= 'Z') {
        emit(cur.at(k), up(s[i]));
        ++k;
        ++i;
      }
    } else if (ch >= 'A' && ch <= 'Z') {
      while (i < n && up(s[i]) >= 'A' && up(s[i]) <= 'Z') {
        emit(cur.at(k), up(s[i]));
        ++mism;
        ++k;
        ++i;
      }
    } else {
      *err = std::string("MdTag b'") + std::string((const char *)s, (size_t)std::min<int64_t>(n, 200)) +
             "': invalid character";
      return -1;
    }
    if (!digits()) return bad("digit expected");
  }
  return mism;
}

}  // namespace

extern "C" {

gqi_status gq_md_count(int64_t n, const int64_t *cigar_off, const int32_t *n_cigar, const uint32_t *cigar,
                       const int64_t *md_off, const int32_t *md_len, const uint8_t *md, int32_t n_threads,
                       int32_t *n_md, uint16_t *n_mismatch) {
  const int64_t per = 1 << 14;
  const int64_t nblk = (n + per - 1) / per;
  std::vector<int64_t> bad_at(nblk, -1);
  std::vector<std::string> bad_msg(nblk);
  parallel_for(nblk, threads_of(n_threads), [&](int64_t q) {
    for (int64_t r = q * per; r < std::min(n, (q + 1) * per); ++r) {
      if (md_len[r] < 0) {
        n_md[r] = -1;
        n_mismatch[r] = 0;
        continue;
      }
      int32_t cnt = 0;
      const int64_t mm = md_parse(md + md_off[r], md_len[r], cigar + cigar_off[r], n_cigar[r],
                                  [&](int64_t off, uint8_t) { cnt += off >= 0; }, &bad_msg[q]);
      if (mm < 0) {
        bad_at[q] = r;
        return;
      }
      n_md[r] = cnt;
      n_mismatch[r] = (uint16_t)std::min<int64_t>(mm, 65535);
    }
  });
  for (int64_t q = 0; q < nblk; ++q)
    if (bad_at[q] >= 0) return fail(GQI_E_MD, "%s", bad_msg[q].c_str());
  return GQI_OK;
}

gqi_status gq_md_fill(int64_t n, const int64_t *cigar_off, const int32_t *n_cigar, const uint32_t *cigar,
                      const int64_t *md_off, const int32_t *md_len, const uint8_t *md, const int64_t *md_ev_off,
                      int32_t n_threads, uint32_t *md_ev) {
  const int64_t per = 1 << 14;
  const int64_t nblk = (n + per - 1) / per;
  std::atomic<int> bad{0};
  parallel_for(nblk, threads_of(n_threads), [&](int64_t q) {
    std::string err;
    for (int64_t r = q * per; r < std::min(n, (q + 1) * per); ++r) {
      if (md_len[r] < 0) continue;
      uint32_t *o = md_ev + md_ev_off[r];
      if (md_parse(md + md_off[r], md_len[r], cigar + cigar_off[r], n_cigar[r],
                   [&](int64_t off, uint8_t base) {
                     if (off >= 0) *o++ = ((uint32_t)off << 8) | base;
                   },
                   &err) < 0)
        bad = 1;
    }
  });
  if (bad) return fail(GQI_E_MD, "MD parse error in gq_md_fill (gq_md_count was not called first?)");
  return GQI_OK;
}

}  // extern "C"
