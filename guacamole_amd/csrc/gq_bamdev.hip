// gq_bamdev.hip — a BAM file decoded in HBM (gqpileup.h: gq_bam_dev_*).
//
// The host loader (gq_ingest.cpp) spends its time inflating BGZF blocks and walking records;
// here the compressed file is the only host -> device copy and everything after it runs on
// the device:
//   bgzf_inflate   thread / BGZF block (Huffman tables in LDS): DEFLATE (RFC 1951) into the block's place in one
//                  inflated stream (offsets from the blocks' ISIZE footers, known on the host)
//   bgzf_crc       thread / block: CRC32 of the inflated bytes against the footer
//   rec_sync       wave / block: the first offset in the block that chains into 8 more
//                  plausible records (lanes test 64 offsets at a time)
//   rec_hop        thread / block: record count and landing offset from a start; the host
//                  checks that each block's chain lands on the next block's start and re-hops
//                  a block from the true chain where it does not (a false sync)
//   rec_list       thread / block: the record offsets
//   rec_parse      thread / record: fields, aux (MD, RG), Read.InputFilters, MD event count
//   rec_fill       16 lanes / kept record: the SoA scalars, sequence (4-bit -> ASCII),
//                  qualities, CIGAR, MD events
// then the sortedness check, contig_read_begin, pmax_end (max-scan) and the usual upload-time
// derivation (derive_shape).  The rules are the host loader's, record for record
// (Read.scala:217-291, :368-451; ReadSet.scala:47-53; MappedRead.scala:87, :114-131).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <zlib.h>

#include <chrono>
#include <climits>
#include <cstring>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gq_host.h"

using namespace gq;

namespace {

struct BgzfBlock {
  int64_t in_off;   // deflate payload in the file
  int64_t out_off;  // inflated bytes in the stream
  int32_t in_len;
  uint32_t isize, crc, pad;
};

// Huffman decoding: each lane's primary tables live in LDS, lane-minor (entry k of lane l at
// [k][l]): 8-bit literal/length codes (u16 entries: symbol << 4 | length) and 7-bit distance /
// code-length codes (u8 entries: symbol << 3 | length); 0 marks a longer code, which continues
// canonically from its first table-width bits against per-length limits in registers.  A
// workgroup is one wave with 32 lanes (blocks) active: 20 KiB of tables, and the 55 k blocks of
// a 3.6 GB stream make 1,720 waves, ~1.7 per SIMD, so two waves' dependent loads overlap and a
// wave waits on the slowest of 32 lanes, not 64 (measured: 64 lanes 127 ms, 32 lanes 103 ms,
// 16 lanes 120 ms for the chr20 30x BAM).
constexpr int kInfLanes = 32, kLitBits = 8, kDistBits = 7;  // lanes (blocks) per wave: see above
// per-lane global scratch (u16 units): per code (literal/length, distance): counts, first
// canonical code and first symbol index per length, symbols; then the code lengths (bytes)
constexpr int kLCount = 0, kLFirst = 16, kLIndex = 32, kLSym = 48, kDCount = kLSym + 288, kDFirst = kDCount + 16,
              kDIndex = kDFirst + 16, kDSym = kDIndex + 16, kTabEnd = kDSym + 32;
constexpr int kScratchBytes = 1536;
static_assert(kTabEnd * 2 + 352 <= kScratchBytes, "inflate scratch");

enum : int { E_OK = 0, E_INFLATE = 1, E_SIZE = 2, E_CRC = 3 };

__host__ __device__ __forceinline__ uint32_t ld32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
typedef uint32_t u32u __attribute__((aligned(1)));  // unaligned dword access (gfx950 global memory)

__host__ __device__ __forceinline__ uint32_t ld16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

struct BitIn {  // LSB-first bit reader over 32-bit words; zeros past the buffer's end.  The
                // stream comes in 16-byte chunks (one dwordx4 load each) and the next chunk is in
                // flight while the current one's four words are consumed: a refill waits on a load
                // only every fourth word, and that load was issued ~128 bits (~16 symbols) earlier.
                // (A one-word-ahead fetch waited on nearly every refill: the ~32 bits between
                // refills decode faster than a load returns.)
  const uint4 *p, *pend;  // the chunk after `nx`
  uint4 nx;               // in flight
  uint64_t q0, q1;        // the current chunk's words not yet taken (qn of them, lowest first)
  int qn;
  int64_t taken;          // words moved into bb
  uint64_t bb;
  int bc;
  __device__ __forceinline__ uint4 fetch16() {
    const uint4 v = p < pend ? *p : make_uint4(0u, 0u, 0u, 0u);
    ++p;
    return v;
  }
  __device__ __forceinline__ uint32_t word() {
    if (qn == 0) {
      q0 = (uint64_t)nx.x | ((uint64_t)nx.y << 32);
      q1 = (uint64_t)nx.z | ((uint64_t)nx.w << 32);
      qn = 4;
      nx = fetch16();
    }
    const uint32_t v = (uint32_t)q0;
    q0 = (q0 >> 32) | (q1 << 32);
    q1 >>= 32;
    --qn;
    return v;
  }
  // base 16-byte aligned; base_len: readable bytes (the caller's buffer is padded past its data)
  __device__ void init(const uint8_t *base, int64_t off, int64_t base_len) {
    pend = (const uint4 *)(base + (base_len & ~int64_t(15)));
    p = (const uint4 *)(base + (off & ~int64_t(15)));
    nx = fetch16();
    qn = 0;
    for (int k = (int)((off >> 2) & 3); k > 0; --k) word();  // (the chunk's words before off's)
    const int sk = (int)(off & 3);
    bb = (uint64_t)(word() >> (8 * sk));
    bc = 32 - 8 * sk;
    taken = 1;
  }
  __device__ __forceinline__ void need(int n) {  // n <= 32
    if (bc < n) {
      bb |= (uint64_t)word() << bc;
      bc += 32;
      ++taken;
    }
  }
  __device__ __forceinline__ void drop(int n) {
    bb >>= n;
    bc -= n;
  }
  __device__ __forceinline__ uint32_t get(int n) {
    need(n);
    const uint32_t v = (uint32_t)(bb & ((uint64_t(1) << n) - 1));
    drop(n);
    return v;
  }
};

// one canonical code of a lane: its symbols by (length, value) in global scratch, and for the
// lengths past the primary table, (limit << 16 | (index - first) & 0xFFFF) in registers (a code
// of length l is its symbol sym[code + index - first] when code < limit = first + count)
template <int kTb>
struct Code {
  uint16_t *sym;
  uint32_t lb[15 - kTb];
};

// 16 per-length 16-bit counters in four registers (no dynamically indexed arrays: those live in
// scratch memory, and a lane's slow build would stall its whole wave)
struct Pack16 {
  uint64_t w[4] = {0, 0, 0, 0};
  __device__ __forceinline__ uint32_t get(int l) const {
    const uint64_t x = l < 4 ? w[0] : l < 8 ? w[1] : l < 12 ? w[2] : w[3];
    return (uint32_t)(x >> (16 * (l & 3))) & 0xFFFF;
  }
  __device__ __forceinline__ void add(int l, uint32_t v) {
    const uint64_t d = (uint64_t)v << (16 * (l & 3));
    if (l < 4) w[0] += d;
    else if (l < 8) w[1] += d;
    else if (l < 12) w[2] += d;
    else w[3] += d;
  }
};

// canonical Huffman code from lengths: counts, first codes and indexes per length, symbols by
// (length, value) (for codes longer than the table), and the primary table (stride
// kInfLanes) of `tb` bits indexed by the next stream bits; entries (symbol << kShift) |
// length, 0 where the code is longer
template <class E, int kShift, int kTb>
__device__ bool huff_build(const uint8_t *len, int n, Code<kTb> &c, E *tab) {
  constexpr int tb = kTb;
  Pack16 cnt;
  for (int s = 0; s < n; ++s) cnt.add(len[s], 1);
  int left = 1;
  for (int l = 1; l < 16; ++l) {
    left = (left << 1) - (int)cnt.get(l);
    if (left < 0) return false;  // over-subscribed
  }
  Pack16 next, offs;  // next canonical code / next symbol slot per length
  int code = 0, idx = 0;
#pragma unroll
  for (int l = 1; l < 16; ++l) {
    const int k = (int)cnt.get(l);
    if (l > tb) c.lb[l - tb - 1] = ((uint32_t)(code + k) << 16) | ((uint32_t)(idx - code) & 0xFFFFu);
    next.add(l, (uint32_t)code);
    offs.add(l, (uint32_t)idx);
    idx += k;
    code = (code + k) << 1;
  }
  for (int k = 0; k < (1 << tb); ++k) tab[k * kInfLanes] = 0;
  for (int s = 0; s < n; ++s) {
    const int l = len[s];
    if (!l) continue;
    const int o = (int)offs.get(l);
    offs.add(l, 1);
    c.sym[o] = (uint16_t)s;
    if (l <= tb) {
      const int cd = (int)next.get(l);
      const int rev = (int)(__builtin_bitreverse32((uint32_t)cd) >> (32 - l));
      for (int k = rev; k < (1 << tb); k += 1 << l) tab[k * kInfLanes] = (E)((s << kShift) | l);
    }
    next.add(l, 1);
  }
  return true;
}

// a code longer than the primary table: its first kTb bits (stream order) reversed into code
// order, then one bit per length (RFC 1951 §3.2.2) against the register limits
template <int kTb>
__device__ __forceinline__ int huff_long(BitIn &in, const Code<kTb> &c) {
  in.need(16);
  int code = (int)(__builtin_bitreverse32((uint32_t)(in.bb & ((1u << kTb) - 1))) >> (32 - kTb));
  in.drop(kTb);
#pragma unroll
  for (int j = 0; j < 15 - kTb; ++j) {
    code = (code << 1) | (int)(in.bb & 1);
    in.drop(1);
    if (code < (int)(c.lb[j] >> 16)) return c.sym[code + (int)(int16_t)(c.lb[j] & 0xFFFF)];
  }
  return -1;
}

template <class E, int kShift, int kTb>
__device__ __forceinline__ int huff_decode(BitIn &in, const E *tab, const Code<kTb> &c) {
  in.need(16);
  const uint32_t e = tab[(in.bb & ((1u << kTb) - 1)) * kInfLanes];
  if (e) {
    in.drop((int)(e & ((1u << kShift) - 1)));
    return (int)(e >> kShift);
  }
  return huff_long<kTb>(in, c);
}

// one BGZF block's raw DEFLATE stream -> out[0, isize); E_OK or an error
__device__ int inflate_one(const uint8_t *comp, int64_t comp_len, const BgzfBlock &b, uint8_t *out, uint16_t *S,
                           uint16_t *lt, uint8_t *dt) {
  uint8_t *lens = (uint8_t *)(S + kTabEnd);
  uint8_t *cl = lens + 320;
  Code<kLitBits> lc;
  Code<kDistBits> dc;
  lc.sym = S + kLSym;
  dc.sym = S + kDSym;
  BitIn in;
  in.init(comp, b.in_off, comp_len);
  const int64_t osz = b.isize;
  int64_t op = 0;
  const int64_t in_bits = (int64_t)b.in_len * 8;
  const int sk = (int)(b.in_off & 3);
  auto used_bits = [&]() -> int64_t { return in.taken * 32 - in.bc - 8 * sk; };
  int final_blk = 0;
  do {
    if (used_bits() > in_bits) return E_INFLATE;
    final_blk = (int)in.get(1);
    const int type = (int)in.get(2);
    if (type == 0) {  // stored
      in.drop(in.bc & 7);
      const uint32_t ln = in.get(16), nln = in.get(16);
      if ((ln ^ 0xFFFFu) != nln || op + ln > osz) return E_INFLATE;
      for (uint32_t k = 0; k < ln; ++k) out[op++] = (uint8_t)in.get(8);
      continue;
    }
    if (type == 3) return E_INFLATE;
    if (type == 1) {  // fixed codes
      for (int s = 0; s < 288; ++s) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
      huff_build<uint16_t, 4, kLitBits>(lens, 288, lc, lt);
      for (int s = 0; s < 30; ++s) lens[s] = 5;
      huff_build<uint8_t, 3, kDistBits>(lens, 30, dc, dt);
    } else {  // dynamic codes
      const int hlit = (int)in.get(5) + 257, hdist = (int)in.get(5) + 1, hclen = (int)in.get(4) + 4;
      if (hlit > 286 || hdist > 30) return E_INFLATE;
      // RFC 1951 code-length order {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15},
      // 5 bits per entry (a constant array indexed by a lane value would go to scratch memory)
      const uint64_t ordA = 0x22caa324e804a30ull, ordB = 0x3c2e1346cull;
      for (int k = 0; k < 19; ++k) cl[k] = 0;
      for (int k = 0; k < hclen; ++k) cl[(k < 12 ? ordA >> (5 * k) : ordB >> (5 * (k - 12))) & 31] = (uint8_t)in.get(3);
      // the code-length code (lengths <= 7) in the distance table's place
      if (!huff_build<uint8_t, 3, kDistBits>(cl, 19, dc, dt)) return E_INFLATE;
      int i = 0;
      while (i < hlit + hdist) {
        const int s = huff_decode<uint8_t, 3, kDistBits>(in, dt, dc);
        if (s < 0) return E_INFLATE;
        if (s < 16) {
          lens[i++] = (uint8_t)s;
          continue;
        }
        int rep;
        uint8_t v = 0;
        if (s == 16) {
          if (i == 0) return E_INFLATE;
          v = lens[i - 1];
          rep = 3 + (int)in.get(2);
        } else if (s == 17) {
          rep = 3 + (int)in.get(3);
        } else {
          rep = 11 + (int)in.get(7);
        }
        if (i + rep > hlit + hdist) return E_INFLATE;
        for (int k = 0; k < rep; ++k) lens[i++] = v;
      }
      if (lens[256] == 0) return E_INFLATE;
      if (!huff_build<uint16_t, 4, kLitBits>(lens, hlit, lc, lt)) return E_INFLATE;
      if (!huff_build<uint8_t, 3, kDistBits>(lens + hlit, hdist, dc, dt)) return E_INFLATE;
    }
    for (;;) {  // symbols
      int sym = huff_decode<uint16_t, 4, kLitBits>(in, lt, lc);
      if (sym < 256) {
        if (sym < 0 || op >= osz) return E_INFLATE;
        out[op++] = (uint8_t)sym;
        continue;
      }
      if (sym == 256) break;
      sym -= 257;
      if (sym >= 29) return E_INFLATE;
      int len;
      if (sym < 8) {
        len = sym + 3;
      } else if (sym == 28) {
        len = 258;
      } else {
        const int ex = (sym - 4) >> 2;
        len = ((4 + (sym & 3)) << ex) + 3 + (int)in.get(ex);
      }
      const int dsym = huff_decode<uint8_t, 3, kDistBits>(in, dt, dc);
      if (dsym < 0 || dsym >= 30) return E_INFLATE;
      int dist;
      if (dsym < 4) {
        dist = dsym + 1;
      } else {
        const int ex = (dsym - 2) >> 1;
        dist = ((2 + (dsym & 1)) << ex) + 1 + (int)in.get(ex);
      }
      if (dist > op || op + len > osz) return E_INFLATE;
      uint8_t *o = out + op;
      const int64_t room = osz - op;  // bytes up to the block's end: chunks may over-store below it
      int i = 0;
      int d = dist;
      if (d < 8) {  // a run of period d: its first bytes one by one, then chunks at a multiple of d >= 8
        uint64_t pat = 0;
        for (int k = 0; k < d; ++k) pat |= (uint64_t)o[k - d] << (8 * k);
        const int first = min(len, d * ((8 + d - 1) / d));
        for (int k = 0; i < first; ++i) {
          o[i] = (uint8_t)(pat >> (8 * k));
          if (++k == d) k = 0;
        }
        d *= (8 + d - 1) / d;
      }
      if (d >= 32) {  // 32-byte chunks: every source byte precedes the chunk it lands in
        for (; i < len; i += 32) {
          if (i + 32 > room) {
            for (; i < len; ++i) o[i] = o[i - d];
            break;
          }
          const u32u *src = (const u32u *)(o + i - d);
          uint32_t t[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) t[k] = src[k];
          u32u *dst = (u32u *)(o + i);
#pragma unroll
          for (int k = 0; k < 8; ++k) dst[k] = t[k];
        }
      } else {  // 8 <= d < 32: 8-byte chunks
        for (; i < len; i += 8) {
          if (i + 8 > room) {
            for (; i < len; ++i) o[i] = o[i - d];
            break;
          }
          const u32u *src = (const u32u *)(o + i - d);
          const uint32_t t0 = src[0], t1 = src[1];
          u32u *dst = (u32u *)(o + i);
          dst[0] = t0;
          dst[1] = t1;
        }
      }
      op += len;
    }
  } while (!final_blk);
  if (used_bits() > in_bits) return E_INFLATE;
  return op == osz ? E_OK : E_SIZE;
}

__global__ void __launch_bounds__(kInfLanes) bgzf_inflate(const uint8_t *comp, int64_t comp_len,
                                                          const BgzfBlock *blk, int64_t n_blk, uint8_t *out,
                                                          uint16_t *scratch, int *status) {
  __shared__ uint16_t lt[(1 << kLitBits) * kInfLanes];
  __shared__ uint8_t dt[(1 << kDistBits) * kInfLanes];
  const int64_t b = (int64_t)blockIdx.x * kInfLanes + threadIdx.x;
  if (b >= n_blk) return;
  const BgzfBlock k = blk[b];
  status[b] = inflate_one(comp, comp_len, k, out + k.out_off, scratch + b * (kScratchBytes / 2), lt + threadIdx.x,
                          dt + threadIdx.x);
}

__global__ void __launch_bounds__(256) bgzf_crc(const uint8_t *out, const BgzfBlock *blk, int64_t n_blk, int *status) {
  __shared__ uint32_t tab[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    tab[i] = c;
  }
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_blk || status[b] != E_OK) return;
  const BgzfBlock k = blk[b];
  const uint8_t *p = out + k.out_off;
  uint32_t c = 0xFFFFFFFFu;
  int64_t i = 0;
  const int64_t n = k.isize;
  for (; i < n && ((k.out_off + i) & 3); ++i) c = tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  for (; i + 4 <= n; i += 4) {
    c ^= *(const uint32_t *)(p + i);
    c = tab[c & 0xFF] ^ (c >> 8);
    c = tab[c & 0xFF] ^ (c >> 8);
    c = tab[c & 0xFF] ^ (c >> 8);
    c = tab[c & 0xFF] ^ (c >> 8);
  }
  for (; i < n; ++i) c = tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  if ((c ^ 0xFFFFFFFFu) != k.crc) status[b] = E_CRC;
}

// ---- records ------------------------------------------------------------------------------
// plausible alignment record at o: every length field consistent with block_size (as the host
// loader's record_at)
// the fixed fields of a record at h (36 bytes readable: block_size and the 32-byte core) are
// plausible: references in the dictionary, a name, and a block size that holds the core's parts
__host__ __device__ __forceinline__ bool record_head_ok(const uint8_t *h, int32_t n_ref) {
  const int32_t bs = (int32_t)ld32(h);
  if (bs < 32) return false;
  const uint8_t *p = h + 4;
  const int32_t ref_id = (int32_t)ld32(p), pos = (int32_t)ld32(p + 4), l_seq = (int32_t)ld32(p + 16),
                next_ref = (int32_t)ld32(p + 20);
  const uint32_t l_name = p[8], n_cig = ld16(p + 12);
  if (ref_id < -1 || ref_id >= n_ref || next_ref < -1 || next_ref >= n_ref || pos < -1 || l_seq < 0 || l_name < 1)
    return false;
  return 32 + (int64_t)l_name + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2 + l_seq <= bs;
}

__host__ __device__ bool record_at(const uint8_t *d, int64_t n, int64_t o, int32_t n_ref) {
  if (o + 40 > n) return false;
  const int32_t bs = (int32_t)ld32(d + o);
  if (bs < 32 || o + 4 + bs > n) return false;
  const uint8_t *p = d + o + 4;
  const int32_t ref_id = (int32_t)ld32(p), pos = (int32_t)ld32(p + 4), l_seq = (int32_t)ld32(p + 16),
                next_ref = (int32_t)ld32(p + 20);
  const uint32_t l_name = p[8], n_cig = ld16(p + 12);
  if (ref_id < -1 || ref_id >= n_ref || next_ref < -1 || next_ref >= n_ref || pos < -1 || l_seq < 0 || l_name < 1)
    return false;
  if (32 + (int64_t)l_name + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2 + l_seq > bs) return false;
  return p[32 + l_name - 1] == 0;
}

// wave / block: first offset in [max(block start, rec0), block end) that chains into 8 more
// plausible records (or to the stream's end); -1 if none
__global__ void __launch_bounds__(256) rec_sync(const uint8_t *d, int64_t n, const BgzfBlock *blk, int64_t n_blk,
                                                int64_t rec0, int32_t n_ref, int64_t *first) {
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (b >= n_blk) return;
  const int64_t lo = max(blk[b].out_off, rec0), hi = blk[b].out_off + (int64_t)blk[b].isize;
  int64_t found = -1;
  for (int64_t base = lo; base < hi; base += 64) {
    const int64_t o = base + lane;
    bool ok9 = false;
    if (o < hi) {
      int64_t q = o;
      int ok = 0;
      while (ok < 9 && q < n && record_at(d, n, q, n_ref)) {
        q += 4 + (int32_t)ld32(d + q);
        ++ok;
      }
      ok9 = ok == 9 || (ok > 0 && q == n);
    }
    const uint64_t m = __ballot(ok9);
    if (m) {
      found = base + __builtin_ctzll(m);
      break;
    }
  }
  if (lane == 0) first[b] = found;
}

// thread / block with a start: records starting in the block and where the chain lands
// (>= the block's end); land = -2: a block_size runs past the stream
__global__ void __launch_bounds__(256) rec_hop(const uint8_t *d, int64_t n, const BgzfBlock *blk, int64_t b0,
                                               int64_t b1, const int64_t *start, int64_t *count, int64_t *land) {
  const int64_t b = b0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= b1) return;
  const int64_t s = start[b];
  if (s < 0) {
    count[b] = 0;
    land[b] = -1;
    return;
  }
  const int64_t hi = blk[b].out_off + (int64_t)blk[b].isize;
  int64_t o = s, c = 0;
  while (o < hi) {
    if (o + 4 > n) {
      o = -2;
      break;
    }
    const int32_t bs = (int32_t)ld32(d + o);
    if (bs < 32 || o + 4 + bs > n) {
      o = -2;
      break;
    }
    ++c;
    o += 4 + bs;
  }
  count[b] = c;
  land[b] = o;
}

__global__ void __launch_bounds__(256) rec_list(const uint8_t *d, const BgzfBlock *blk, int64_t n_blk,
                                                const int64_t *start, const int64_t *base, int64_t *rec) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_blk || start[b] < 0) return;
  const int64_t hi = blk[b].out_off + (int64_t)blk[b].isize;
  int64_t o = start[b], k = base[b];
  while (o < hi) {
    rec[k++] = o;
    o += 4 + (int32_t)ld32(d + o);
  }
}

// CIGAR op classes (htsjdk CigarOperator): M I D N S H P = X -> 0..8
constexpr uint32_t kConsumesRef = (1u << 0) | (1u << 2) | (1u << 3) | (1u << 7) | (1u << 8);
constexpr uint32_t kPaddedRef = kConsumesRef | (1u << 6);
constexpr uint32_t kMdConsumed = (1u << 0) | (1u << 2) | (1u << 7) | (1u << 8);

struct DevFilters {
  int32_t non_duplicate, passed_vendor, is_paired, has_md, use_loci, n_ref, n_rg;
  const int64_t *loci_begin, *loci_start, *loci_end;
  const uint8_t *rg_ids;      // n_rg NUL-terminated IDs back to back
  const int32_t *rg_id_off;   // [n_rg + 1]
};

struct RecInfo {  // one per record (file order)
  int64_t md_at;  // MD value offset in the stream, -1: no MD tag
  int32_t md_len, n_md;
  uint16_t n_mm;
  uint8_t rgc, keep;
  int32_t pad;
};

// error words: (record << 8 | code), minimum over records; codes below
enum : uint64_t { X_TRUNC = 1, X_AUX_TRUNC = 2, X_AUX_STR = 3, X_AUX_ARR = 4, X_AUX_ARR_TYPE = 5, X_AUX_TYPE = 6,
                  X_QUAL = 7, X_MD = 8 };

// k-th MD-consumed reference offset (M/=/X/D positions; N gaps skipped); past the CIGAR's
// last such position the offsets continue one by one (the host loader's MdCursor)
struct MdCursor {
  const uint8_t *cig;
  int32_t n, op = 0;
  int64_t ref = 0, last = -1, total = 0;
  __device__ int64_t at(int64_t k) {
    while (op < n) {
      const uint32_t v = ld32(cig + 4 * op), o = v & 15, ln = v >> 4;
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

// MdTag parse (the host loader's md_parse): emit(off, base) per event; -> mismatches or -1
template <class Emit>
__device__ int64_t md_parse(const uint8_t *s, int64_t n, const uint8_t *cig, int32_t ncig, Emit emit) {
  if (n == 0) return 0;
  MdCursor cur{cig, ncig};
  int64_t i = 0, k = 0, mism = 0;
  auto up = [](uint8_t c) -> uint8_t { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; };
  auto digits = [&]() -> bool {
    const int64_t j0 = i;
    int64_t v = 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') v = v * 10 + (s[i++] - '0');
    if (i == j0) return false;
    k += v;
    return true;
  };
  if (!digits()) return -1;
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
      return -1;
    }
    if (!digits()) return -1;
  }
  return mism;
}

__device__ bool loci_intersect(const DevFilters &f, int32_t contig, int64_t s, int64_t e) {
  if (e <= s) return false;
  int64_t lo = f.loci_begin[contig], hi = f.loci_begin[contig + 1];
  while (lo < hi) {  // first range with end > s
    const int64_t mid = (lo + hi) >> 1;
    if (f.loci_end[mid] > s) hi = mid;
    else lo = mid + 1;
  }
  return lo < f.loci_begin[contig + 1] && f.loci_start[lo] < e;
}

__device__ __forceinline__ void parse_one(const uint8_t *d, const int64_t *rec, int64_t n_rec, const DevFilters &f,
                                          RecInfo *info, int64_t *keep, int64_t *seq_k, int64_t *cig_k, int64_t *md_k,
                                          unsigned long long *err, int64_t r, int &cls, int64_t &span);

// thread / record: the host loader's scan_chunk + the MD event count of gq_md_count
__global__ void __launch_bounds__(256) rec_parse(const uint8_t *d, const int64_t *rec, int64_t n_rec, DevFilters f,
                                                 RecInfo *info, int64_t *keep, int64_t *seq_k, int64_t *cig_k,
                                                 int64_t *md_k, unsigned long long *rg_first,
                                                 unsigned long long *err, unsigned long long *span_max) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int cls = -1;  // the kept record's read-group class (for rg_first), -1: not kept
  int64_t span = 0;  // reference span of a mapped record (the region plan's halo check)
  parse_one(d, rec, n_rec, f, info, keep, seq_k, cig_k, md_k, err, r, cls, span);
  unsigned long long sm = (unsigned long long)span;
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long x = __shfl_xor(sm, o, 64);
    sm = x > sm ? x : sm;
  }
  if ((threadIdx.x & 63) == 0 && sm) atomicMax(span_max, sm);
  // first kept record per class: one atomic per (wave, class) — lanes hold increasing r
  for (;;) {
    const uint64_t m = __ballot(cls >= 0);
    if (!m) break;
    const int lead = __builtin_ctzll(m);
    const int c0 = __shfl(cls, lead);
    if ((int)(threadIdx.x & 63) == lead) atomicMin(rg_first + c0, (unsigned long long)r);
    if (cls == c0) cls = -1;
  }
}

__device__ __forceinline__ void parse_one(const uint8_t *d, const int64_t *rec, int64_t n_rec, const DevFilters &f,
                                          RecInfo *info, int64_t *keep, int64_t *seq_k, int64_t *cig_k, int64_t *md_k,
                                          unsigned long long *err, int64_t r, int &cls, int64_t &span) {
  if (r >= n_rec) return;
  RecInfo ri{-1, 0, 0, 0, 0, 0, 0};
  keep[r] = 0;
  seq_k[r] = cig_k[r] = md_k[r] = 0;
  const int64_t o = rec[r];
  const int64_t end = o + 4 + (int32_t)ld32(d + o);
  const uint8_t *p = d + o + 4;
  const int32_t ref_id = (int32_t)ld32(p), pos = (int32_t)ld32(p + 4);
  const uint32_t l_read_name = p[8];
  const uint32_t n_cig = ld16(p + 12), flag = ld16(p + 14);
  const int32_t l_seq = (int32_t)ld32(p + 16);
  const int64_t cig_at = o + 36 + l_read_name;
  const int64_t qual_at = cig_at + 4 * (int64_t)n_cig + ((int64_t)l_seq + 1) / 2;
  int64_t q = qual_at + l_seq;
  auto fail = [&](uint64_t code) {
    atomicMin(err, ((unsigned long long)r << 8) | code);
    info[r] = ri;
  };
  if (l_seq < 0 || l_read_name < 1 || q > end) return fail(X_TRUNC);
  int64_t md_at = -1, md_n = 0, rg_at = -1, rg_n = 0;
  while (q < end) {
    if (q + 3 > end) return fail(X_AUX_TRUNC);
    const uint8_t t0 = d[q], t1 = d[q + 1], ty = d[q + 2];
    q += 3;
    switch (ty) {
      case 'A': case 'c': case 'C': q += 1; break;
      case 's': case 'S': q += 2; break;
      case 'i': case 'I': case 'f': q += 4; break;
      case 'Z': case 'H': {
        int64_t z = q;
        while (z < end && d[z]) ++z;
        if (z >= end) return fail(X_AUX_STR);
        if (t0 == 'M' && t1 == 'D') md_at = q, md_n = z - q;
        else if (t0 == 'R' && t1 == 'G') rg_at = q, rg_n = z - q;
        q = z + 1;
        break;
      }
      case 'B': {
        if (q + 5 > end) return fail(X_AUX_ARR);
        const uint8_t sub = d[q];
        const int64_t cnt = (int32_t)ld32(d + q + 1);
        int w = 0;
        switch (sub) {
          case 'c': case 'C': w = 1; break;
          case 's': case 'S': w = 2; break;
          case 'i': case 'I': case 'f': w = 4; break;
          default: return fail(X_AUX_ARR_TYPE | ((uint64_t)0));
        }
        if (cnt < 0 || q + 5 + cnt * w > end) return fail(X_AUX_ARR);  // (a negative count would walk backwards)
        q += 5 + cnt * w;
        break;
      }
      default: return fail(X_AUX_TYPE);
    }
  }
  // Read.scala:411-418 record filters, then isMapped / hasMdTag (Read.scala:421-428)
  bool kept = !((flag & 0x4) || ref_id < 0) && pos >= 0 && ref_id < f.n_ref;
  if (kept) {
    int64_t ref_len = 0;
    for (uint32_t k = 0; k < n_cig; ++k) {
      const uint32_t v = ld32(d + cig_at + 4 * k), op = v & 15;
      if (op < 9 && (kConsumesRef >> op) & 1) ref_len += v >> 4;
    }
    span = ref_len;
    if (f.use_loci) kept = loci_intersect(f, ref_id, pos, pos + ref_len);
  }
  if (kept && f.non_duplicate && (flag & 0x400)) kept = false;
  if (kept && f.passed_vendor && (flag & 0x200)) kept = false;
  if (kept && f.is_paired && !(flag & 0x1)) kept = false;
  if (kept && f.has_md && md_at < 0) kept = false;
  if (!kept) {
    info[r] = ri;
    return;
  }
  // htsjdk: missing qualities (0xFF) -> empty array -> MappedRead's length assertion
  if (l_seq > 0 && d[qual_at] == 0xFF) return fail(X_QUAL);
  int rgc = f.n_rg;  // no RG tag, or an ID the header lacks: sample "default"
  if (rg_at >= 0) {
    for (int k = 0; k < f.n_rg; ++k) {
      const int32_t a = f.rg_id_off[k], ln = f.rg_id_off[k + 1] - a - 1;
      if (ln != rg_n) continue;
      bool eq = true;
      for (int j = 0; j < ln && eq; ++j) eq = f.rg_ids[a + j] == d[rg_at + j];
      if (eq) {
        rgc = k;
        break;
      }
    }
  }
  ri.md_at = md_at;
  ri.md_len = md_at >= 0 ? (int32_t)md_n : -1;
  ri.rgc = (uint8_t)rgc;
  ri.keep = 1;
  if (md_at >= 0) {
    int32_t cnt = 0;
    const int64_t mm = md_parse(d + md_at, md_n, d + cig_at, (int32_t)n_cig, [&](int64_t off, uint8_t) { cnt += off >= 0; });
    if (mm < 0) {
      atomicMin(err + 1, ((unsigned long long)r << 8) | X_MD);
      info[r] = ri;
      return;
    }
    ri.n_md = cnt;
    ri.n_mm = (uint16_t)min<int64_t>(mm, 65535);
  } else {
    ri.n_md = -1;
  }
  info[r] = ri;
  keep[r] = 1;
  cls = rgc;
  seq_k[r] = l_seq;
  cig_k[r] = n_cig;
  md_k[r] = max(ri.n_md, 0);
}

struct FillOut {
  int32_t *contig, *start, *end;
  uint8_t *mapq, *flags, *sample;
  int64_t *seq_off;
  int32_t *seq_len;
  int64_t *cigar_off;
  int32_t *n_cigar;
  int64_t *md_off;
  int32_t *n_md;
  uint16_t *n_mismatch;
  uint8_t *seq, *qual;
  uint32_t *cigar, *md_ev;
  uint64_t *end_key;  // contig << 32 | end, for the pmax_end scan
};

// 16 lanes / record (kept ones write): scalars + MD events by the group's first lane, the
// pools by all 16
__global__ void __launch_bounds__(256) rec_fill(const uint8_t *d, const int64_t *rec, int64_t n_rec,
                                                const RecInfo *info, const int64_t *kidx, const int64_t *seq_o,
                                                const int64_t *cig_o, const int64_t *md_o, const uint8_t *class_sample,
                                                FillOut F) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int g = threadIdx.x & 15;
  if (r >= n_rec) return;
  const RecInfo ri = info[r];
  if (!ri.keep) return;
  const int64_t i = kidx[r];
  const int64_t o = rec[r];
  const uint8_t *p = d + o + 4;
  const int32_t ref_id = (int32_t)ld32(p), pos = (int32_t)ld32(p + 4);
  const uint32_t l_name = p[8], mapq = p[9], n_cig = ld16(p + 12), flag = ld16(p + 14);
  const int32_t l_seq = (int32_t)ld32(p + 16);
  const uint8_t *cg = p + 32 + l_name, *sq = cg + 4 * n_cig, *ql = sq + (l_seq + 1) / 2;
  const int64_t so = seq_o[r], co = cig_o[r];
  if (g == 0) {
    int64_t padded = 0;
    for (uint32_t k = 0; k < n_cig; ++k) {
      const uint32_t v = ld32(cg + 4 * k), op = v & 15;
      if (op < 9 && (kPaddedRef >> op) & 1) padded += v >> 4;
    }
    const int32_t e = (int32_t)(pos + padded);
    F.contig[i] = ref_id;
    F.start[i] = pos;
    F.end[i] = e;
    F.end_key[i] = ((uint64_t)(uint32_t)ref_id << 32) | (uint32_t)e;
    F.mapq[i] = (uint8_t)mapq;
    F.flags[i] = (flag & 0x10) ? 1 : 0;
    F.sample[i] = class_sample[ri.rgc];
    F.seq_off[i] = so;
    F.seq_len[i] = l_seq;
    F.cigar_off[i] = co;
    F.n_cigar[i] = (int32_t)n_cig;
    F.md_off[i] = md_o[r];
    F.n_md[i] = ri.n_md;
    F.n_mismatch[i] = ri.md_at >= 0 ? ri.n_mm : 0;
    if (ri.md_at >= 0) {
      uint32_t *ev = F.md_ev + md_o[r];
      md_parse(d + ri.md_at, ri.md_len, cg, (int32_t)n_cig, [&](int64_t off, uint8_t base) {
        if (off >= 0) *ev++ = ((uint32_t)off << 8) | base;
      });
    }
  }
  const char *code = "=ACMGRSVTWYHKDBN";
  for (int k = g; k < (l_seq + 1) / 2; k += 16) {
    const uint8_t v = sq[k];
    F.seq[so + 2 * k] = (uint8_t)code[v >> 4];
    if (2 * k + 1 < l_seq) F.seq[so + 2 * k + 1] = (uint8_t)code[v & 15];
  }
  for (int k = g; k < l_seq; k += 16) F.qual[so + k] = ql[k];
  for (int k = g; k < (int)n_cig; k += 16) F.cigar[co + k] = ld32(cg + 4 * k);
}

// kept reads out of (contig, start) order -> flag; contig_read_begin at the contig changes
__global__ void __launch_bounds__(256) reads_order(const int32_t *contig, const int32_t *start, int64_t n,
                                                   int32_t n_contigs, int64_t *begin, int *unsorted) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  const int32_t c = i < n ? contig[i] : n_contigs;
  const int32_t pc = i > 0 ? contig[i - 1] : -1;
  if (i > 0 && i < n && (c < pc || (c == pc && start[i] < start[i - 1]))) atomicOr(unsorted, 1);
  for (int32_t k = pc + 1; k <= c && k <= n_contigs; ++k) begin[k] = i;
}

__global__ void __launch_bounds__(256) low32(const uint64_t *key, int64_t n, int32_t *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)(uint32_t)key[i];
}

struct U64Max {
  __device__ __forceinline__ uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; }
};

inline unsigned grid(int64_t n, int per) { return (unsigned)std::max<int64_t>(1, (n + per - 1) / per); }
inline float ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t).count();
}

bool gzip_member(const uint8_t *p, int64_t avail, int64_t *payload, int64_t *bsize) {
  if (avail < 18 || p[0] != 31 || p[1] != 139 || p[2] != 8) return false;
  const uint8_t flg = p[3];
  int64_t o = 10;
  *bsize = -1;
  auto rd16 = [&](int64_t q) { return (int64_t)p[q] | ((int64_t)p[q + 1] << 8); };
  if (flg & 4) {
    const int64_t xlen = rd16(10);
    o = 12;
    if (o + xlen > avail) return false;
    for (int64_t q = o; q + 4 <= o + xlen;) {
      const int64_t slen = rd16(q + 2);
      if (p[q] == 66 && p[q + 1] == 67 && slen == 2) *bsize = rd16(q + 4) + 1;
      q += 4 + slen;
    }
    o += xlen;
  }
  if (flg & 8) {
    while (o < avail && p[o]) ++o;
    ++o;
  }
  if (flg & 16) {
    while (o < avail && p[o]) ++o;
    ++o;
  }
  if (flg & 2) o += 2;
  if (o > avail) return false;
  *payload = o;
  return true;
}

}  // namespace

namespace {
// a planned segment (gq_bam_dev_plan): BGZF blocks [b0, b1) are inflated; its records run from
// offset `first` of block b0 up to block b1 - 1 (which only completes the last record), or to
// the end of the stream when `eof`
struct Seg {
  int64_t b0, first, b1;
  bool eof;
};
// host probe of one BGZF block: the key (contig << 32 | pos + 1) of the last record starting
// in it and the stream offset its chain lands on (the next record's start)
struct Probe {
  bool has = false;
  int64_t last = 0, land = 0;
};
}  // namespace

struct gq_bam_dev {
  gq_ctx *ctx = nullptr;
  int fd = -1;
  const uint8_t *map = nullptr;
  size_t map_len = 0;
  std::vector<BgzfBlock> blocks;
  std::vector<int64_t> foff;  // file offset of each block's gzip member
  int64_t n_out = 0, rec0 = 0;
  bool sorted = false;        // @HD SO:coordinate
  // region plan: segments, the probe cache, the linear index of the BAI (per contig)
  bool planned = false;
  std::vector<Seg> segs;
  std::vector<BgzfBlock> sel;  // the load's blocks (planned: segment by segment, stream offsets compacted)
  std::vector<int64_t> sel_seg0;  // first entry of each segment in `sel`
  std::map<int64_t, Probe> probes;  // (the plan probes on several host threads: probe_mu)
  std::mutex probe_mu;
  std::atomic<int64_t> n_probes{0};
  std::vector<std::vector<uint64_t>> bai_ioff;
  std::string text;
  std::vector<std::string> names;
  std::vector<int64_t> lengths;
  DevBuf comp, blk, out;  // compressed file, block table, inflated stream
  DevBuf scratch, status;  // inflate: per-block code tables and status
  // last scan
  DevBuf rec, info, kidx, seq_o, cig_o, md_o;
  int64_t n_rec = 0, n_keep = 0, seq_bytes = 0, cigar_len = 0, md_events = 0;
  bool scanned = false;
  gq_bam_dev_sizes sizes{};
  ~gq_bam_dev() {
    for (DevBuf *b : {&comp, &blk, &out, &scratch, &status, &rec, &info, &kidx, &seq_o, &cig_o, &md_o}) b->release();
    if (map) munmap(const_cast<uint8_t *>(map), map_len);
    if (fd >= 0) close(fd);
  }
};

namespace {

gq_status exclusive_sum(gq_ctx *c, const int64_t *in, int64_t *out, int64_t n, DevBuf &tmp) {
  size_t tb = 0;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, (int)n, c->stream));
  HIP_TRY(tmp.ensure(tb));
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, in, out, (int)n, c->stream));
  return GQ_OK;
}

gq_status d2h_i64(gq_ctx *c, const void *src, int64_t *dst) {
  HIP_TRY(hipMemcpyAsync(dst, src, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GQ_OK;
}

// ---- host side of the file: header, block probes, BAI, region plan -----------------------

// block k's raw DEFLATE payload inflated on the host (zlib), appended to `out`
bool host_inflate(const gq_bam_dev *b, int64_t k, std::vector<uint8_t> &out) {
  const BgzfBlock &blk = b->blocks[(size_t)k];
  const size_t at = out.size();
  out.resize(at + blk.isize);
  z_stream z;
  memset(&z, 0, sizeof(z));
  if (inflateInit2(&z, -15) != Z_OK) return false;
  z.next_in = const_cast<Bytef *>(b->map + blk.in_off);
  z.avail_in = (uInt)blk.in_len;
  z.next_out = out.data() + at;
  z.avail_out = (uInt)blk.isize;
  const int rc = inflate(&z, Z_FINISH);
  const bool ok = rc == Z_STREAM_END && z.total_out == blk.isize;
  inflateEnd(&z);
  return ok;
}

gq_status corrupt_block(const gq_bam_dev *b, int64_t k) {
  return set_err(GQ_E_BAM_FORMAT, "corrupt BGZF block (inflate, ISIZE or CRC32) with payload at file offset %lld",
                 (long long)b->blocks[(size_t)k].in_off);
}

// the BAM header (magic, SAM text, reference dictionary) from the first blocks, on the host;
// rec0 = the first alignment record's stream offset
gq_status parse_header(gq_bam_dev *b) {
  std::vector<uint8_t> h;
  int64_t k = 0;
  const int64_t nb = (int64_t)b->blocks.size();
  bool bad = false;
  auto need = [&](int64_t upto) -> bool {  // h holds >= upto bytes (false: the stream is shorter)
    while ((int64_t)h.size() < upto && k < nb) {
      if (!host_inflate(b, k, h)) {
        bad = true;
        return false;
      }
      ++k;
    }
    return (int64_t)h.size() >= upto;
  };
  auto fail = [&](const char *what) { return bad ? corrupt_block(b, k) : set_err(GQ_E_BAM_FORMAT, "%s", what); };
  if (!need(12) || memcmp(h.data(), "BAM\1", 4) != 0) return fail("not a BAM file (magic)");
  int64_t o = 4;
  int32_t l_text;
  memcpy(&l_text, h.data() + o, 4);
  o += 4;
  if (l_text < 0 || !need(o + l_text + 4)) return fail("truncated BAM header");
  b->text.assign((const char *)h.data() + o, (size_t)l_text);
  while (!b->text.empty() && b->text.back() == '\0') b->text.pop_back();
  o += l_text;
  int32_t n_ref;
  memcpy(&n_ref, h.data() + o, 4);
  o += 4;
  for (int32_t i = 0; i < n_ref; ++i) {
    int32_t l_name;
    if (!need(o + 4)) return fail("truncated BAM reference dictionary");
    memcpy(&l_name, h.data() + o, 4);
    o += 4;
    if (l_name < 1 || !need(o + l_name + 4)) return fail("truncated BAM reference dictionary");
    b->names.emplace_back((const char *)h.data() + o, (size_t)(l_name - 1));
    o += l_name;
    int32_t ln;
    memcpy(&ln, h.data() + o, 4);
    b->lengths.push_back(ln);
    o += 4;
  }
  b->rec0 = o;
  // SAM spec @HD SO:coordinate (the plan's binary searches need the sort order)
  const size_t hd = b->text.compare(0, 3, "@HD") == 0 ? 0 : b->text.find("\n@HD");
  if (hd != std::string::npos) {
    const size_t eol = b->text.find('\n', hd + 1);
    const std::string line = b->text.substr(hd, eol == std::string::npos ? std::string::npos : eol - hd);
    b->sorted = line.find("\tSO:coordinate") != std::string::npos;
  }
  return GQ_OK;
}

inline int64_t rec_key(int32_t ref, int32_t pos) {  // file order of a sorted BAM; unmapped last
  return ref < 0 ? INT64_MAX : ((int64_t)ref << 32) + (int64_t)pos + 1;
}

// Probe block k: inflate it (and the next blocks a record needs), find the first offset whose
// chain of plausible, key-sorted records runs through the block's end onto a plausible record
// (or the stream's end), and report the key of the chain's last record in the block and where
// it lands.  A false sync can only pass by merging into the true chain within the block, so the
// last record and the landing are true records.  has = false: no record starts in the block
// (header bytes only, an empty block, or one inside a longer record).
gq_status probe(gq_bam_dev *b, int64_t k, Probe &out) {
  {
    std::lock_guard<std::mutex> g(b->probe_mu);
    auto hit = b->probes.find(k);
    if (hit != b->probes.end()) {
      out = hit->second;
      return GQ_OK;
    }
  }
  Probe P;
  const BgzfBlock &blk = b->blocks[(size_t)k];
  const int64_t o0 = blk.out_off, hi = blk.isize, nb = (int64_t)b->blocks.size();
  const int32_t n_ref = (int32_t)b->names.size();
  if (hi > 0 && o0 + hi > b->rec0) {
    b->n_probes.fetch_add(1);
    std::vector<uint8_t> buf;
    if (!host_inflate(b, k, buf)) return corrupt_block(b, k);
    int64_t next = k + 1;
    auto extend = [&](int64_t upto) -> gq_status {  // buf holds >= upto bytes where the stream has them
      while ((int64_t)buf.size() < upto && next < nb && next <= k + 8)
        if (!host_inflate(b, next++, buf)) return corrupt_block(b, next - 1);
      return GQ_OK;
    };
    auto rec_ok = [&](int64_t q, int64_t &key, int64_t &len, gq_status &st) -> bool {
      // the fixed fields first: a false sync offset is nearly always rejected there, before its
      // (garbage) block size makes extend() inflate the following blocks
      if ((st = extend(q + 36))) return false;
      if (q + 36 > (int64_t)buf.size() || !record_head_ok(buf.data() + q, n_ref)) return false;
      const int32_t bs = (int32_t)ld32(buf.data() + q);
      if ((st = extend(q + 4 + bs))) return false;
      if (!record_at(buf.data(), (int64_t)buf.size(), q, n_ref)) return false;
      key = rec_key((int32_t)ld32(buf.data() + q + 4), (int32_t)ld32(buf.data() + q + 8));
      len = 4 + bs;
      return true;
    };
    const int64_t lo = std::max<int64_t>(0, b->rec0 - o0);
    const int64_t top = b->rec0 > o0 ? lo + 1 : hi;  // the block holding rec0: its first record is known
    for (int64_t o = lo; o < top && !P.has; ++o) {
      int64_t q = o, prev = INT64_MIN, key = 0, len = 0;
      gq_status st = GQ_OK;
      bool ok = true;
      while (ok && q < hi) {
        ok = rec_ok(q, key, len, st) && key >= prev;
        if (st) return st;
        prev = key;
        q += len;
      }
      if (!ok) continue;
      const int64_t last = prev;
      if ((st = extend(q + 4))) return st;
      if (q < (int64_t)buf.size() || next < nb) {  // not the stream's end: a record must start there
        if (!rec_ok(q, key, len, st) || key < last) {
          if (st) return st;
          continue;
        }
      }
      P.has = true;
      P.last = last;
      P.land = o0 + q;
    }
  }
  {
    std::lock_guard<std::mutex> g(b->probe_mu);
    b->probes[k] = P;
  }
  out = P;
  return GQ_OK;
}

// the last record key at or before block k (INT64_MIN: none — only header bytes so far)
gq_status key_upto(gq_bam_dev *b, int64_t k, int64_t &key, int64_t *land = nullptr, int64_t *blk = nullptr) {
  for (int64_t j = k; j >= 0; --j) {
    Probe P;
    gq_status st = probe(b, j, P);
    if (st) return st;
    if (P.has) {
      key = P.last;
      if (land) *land = P.land;
      if (blk) *blk = j;
      return GQ_OK;
    }
  }
  key = INT64_MIN;
  if (land) *land = b->rec0;
  if (blk) *blk = -1;
  return GQ_OK;
}

// smallest block b in [lo, nb) whose key_upto >= K (nb if none)
gq_status first_block_at(gq_bam_dev *b, int64_t lo, int64_t K, int64_t &out) {
  int64_t hi = (int64_t)b->blocks.size();
  while (lo < hi) {
    const int64_t m = lo + (hi - lo) / 2;
    int64_t key;
    gq_status st = key_upto(b, m, key);
    if (st) return st;
    if (key >= K) hi = m;
    else lo = m + 1;
  }
  out = lo;
  return GQ_OK;
}

// stream offset -> (block, offset in it)
void stream_pos(const gq_bam_dev *b, int64_t at, int64_t &blk, int64_t &off) {
  int64_t lo = 0, hi = (int64_t)b->blocks.size() - 1;
  while (lo < hi) {  // last block with out_off <= at
    const int64_t m = (lo + hi + 1) / 2;
    if (b->blocks[(size_t)m].out_off <= at) lo = m;
    else hi = m - 1;
  }
  // an offset at a block's end is the start of the next non-empty block
  while (lo + 1 < (int64_t)b->blocks.size() &&
         at >= b->blocks[(size_t)lo].out_off + (int64_t)b->blocks[(size_t)lo].isize)
    ++lo;
  blk = lo;
  off = at - b->blocks[(size_t)lo].out_off;
}

// the BAI's linear index (SAM spec §5.2): per reference, the virtual offset of the first
// record overlapping each 16 kb window.  false: no usable index (absent, older than the BAM,
// malformed, or for another dictionary).
bool load_bai(gq_bam_dev *b, const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  std::vector<uint8_t> v;
  {
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + k);
    fclose(f);
  }
  size_t o = 0;
  auto rd = [&](void *dst, size_t n) -> bool {
    if (o + n > v.size()) return false;
    memcpy(dst, v.data() + o, n);
    o += n;
    return true;
  };
  char magic[4];
  int32_t n_ref;
  if (!rd(magic, 4) || memcmp(magic, "BAI\1", 4) != 0 || !rd(&n_ref, 4) || n_ref != (int32_t)b->names.size())
    return false;
  b->bai_ioff.assign((size_t)n_ref, {});
  for (int32_t r = 0; r < n_ref; ++r) {
    int32_t n_bin;
    if (!rd(&n_bin, 4) || n_bin < 0) return false;
    for (int32_t i = 0; i < n_bin; ++i) {
      uint32_t bin;
      int32_t n_chunk;
      if (!rd(&bin, 4) || !rd(&n_chunk, 4) || n_chunk < 0 || o + 16 * (size_t)n_chunk > v.size()) return false;
      o += 16 * (size_t)n_chunk;
    }
    int32_t n_intv;
    if (!rd(&n_intv, 4) || n_intv < 0 || o + 8 * (size_t)n_intv > v.size()) return false;
    b->bai_ioff[(size_t)r].resize((size_t)n_intv);
    if (n_intv) memcpy(b->bai_ioff[(size_t)r].data(), v.data() + o, 8 * (size_t)n_intv);
    o += 8 * (size_t)n_intv;
  }
  return true;
}

// BGZF virtual offset -> (block, offset in its inflated bytes); false if it names no block
bool voff_pos(const gq_bam_dev *b, uint64_t v, int64_t &blk, int64_t &off) {
  const int64_t fo = (int64_t)(v >> 16), uo = (int64_t)(v & 0xFFFF);
  auto it = std::lower_bound(b->foff.begin(), b->foff.end(), fo);
  if (it == b->foff.end() || *it != fo) return false;
  blk = it - b->foff.begin();
  if (uo > (int64_t)b->blocks[(size_t)blk].isize) return false;
  stream_pos(b, b->blocks[(size_t)blk].out_off + uo, blk, off);
  return true;
}

}  // namespace

extern "C" {

gq_status gq_bam_dev_map_ex(const char *path, int32_t populate, gq_bam_dev **out) {
  if (!path || !out) return set_err(GQ_E_ARG, "gq_bam_dev_map: null argument");
  *out = nullptr;
  auto t0 = std::chrono::steady_clock::now();
  std::unique_ptr<gq_bam_dev> b(new gq_bam_dev());
  b->fd = open(path, O_RDONLY);
  if (b->fd < 0) return set_err(GQ_E_BAM_IO, "cannot open %s", path);
  struct stat st;
  if (fstat(b->fd, &st) != 0 || st.st_size == 0) return set_err(GQ_E_BAM_IO, "cannot stat (or empty) %s", path);
  b->map_len = (size_t)st.st_size;
  // (populate: the pages are faulted in by the block walk's threads below, in parallel, rather
  // than by MAP_POPULATE on this one thread)
  void *m = mmap(nullptr, b->map_len, PROT_READ, MAP_PRIVATE, b->fd, 0);
  if (m == MAP_FAILED) return set_err(GQ_E_BAM_IO, "cannot map %s", path);
  b->map = (const uint8_t *)m;
  const uint8_t *p = b->map;
  const int64_t n = (int64_t)b->map_len;
  // The block chain: each member's header gives the next member's offset.  Large files are
  // walked in parallel (the walk is page-fault bound on a file not yet in memory): chunk t > 0
  // starts at its first offset whose header chains through kVerify more members, each chunk's
  // walk runs to its first member at or past the chunk's end, and the chunks are stitched along
  // the true chain from offset 0 — a chunk whose guessed start is not where the previous chunk's
  // true walk lands is walked again from there, so the result (and any error) is the sequential
  // walk's.
  struct Mem {
    int64_t off;
    int32_t payload, bsize;
  };
  // one member at off: 1 a BGZF member (m filled), 0 not a member, -1 gzip without BGZF sizes,
  // -2 truncated
  auto member = [&](int64_t off, Mem &m) -> int {
    int64_t payload, bsize;
    if (!gzip_member(p + off, n - off, &payload, &bsize)) return 0;
    if (bsize < 0) return -1;
    if (off + bsize > n || bsize < payload + 8) return -2;
    m = Mem{off, (int32_t)payload, (int32_t)bsize};
    return 1;
  };
  auto walk = [&](int64_t off, int64_t stop, std::vector<Mem> &v) -> int64_t {  // true-chain walk
    Mem m;                                                                      // (-1: stopped on an error)
    while (off < n && off < stop) {
      if (member(off, m) != 1) return -1 - off;
      v.push_back(m);
      off += m.bsize;
    }
    return off;
  };
  constexpr int64_t kChunkMin = int64_t(64) << 20;
  constexpr int kVerify = 4;
  const char *env_nt = getenv("GQ_MAP_THREADS");  // (tests: 1 forces the sequential walk)
  const int64_t max_nt = env_nt && atoi(env_nt) > 0 ? atoi(env_nt) : 16;
  const int nt = (int)std::min<int64_t>(max_nt, std::max<int64_t>(1, n / kChunkMin));
  std::vector<std::vector<Mem>> part((size_t)nt);
  std::vector<int64_t> start((size_t)nt, -1), land((size_t)nt, -1);
  // populate: the file's pages mapped by 16 threads (a read per 4 KiB page), beside the walk
  std::vector<std::thread> touch;
  std::atomic<uint32_t> touched{0};
  if (populate) {
    const int ntt = (int)std::min<int64_t>(16, std::max<int64_t>(1, n >> 24));
    for (int t = 0; t < ntt; ++t)
      touch.emplace_back([&, t, ntt]() {  // (ntt by value: this block ends before the threads do)
        const int64_t a = n * t / ntt, e = n * (t + 1) / ntt;
        uint32_t acc = 0;
        for (int64_t o = a; o < e; o += 4096) acc += p[o];
        touched.fetch_add(acc, std::memory_order_relaxed);
      });
  }
  auto spec = [&](int t) {  // chunk t's speculative walk
    const int64_t c0 = n * t / nt, c1 = n * (t + 1) / nt;
    int64_t o = c0;
    if (t > 0) {
      for (; o < c1; ++o) {
        if (p[o] != 31 || p[o + 1 < n ? o + 1 : o] != 139) continue;
        Mem m;
        int64_t q = o;
        int k = 0;
        while (k < kVerify && q < n && member(q, m) == 1) {
          q += m.bsize;
          ++k;
        }
        if (k == kVerify || (k > 0 && q == n)) break;
      }
      if (o >= c1) return;
    }
    start[(size_t)t] = o;
    land[(size_t)t] = walk(o, c1, part[(size_t)t]);
  };
  {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(spec, t);
    spec(0);
    for (std::thread &x : th) x.join();
  }
  for (std::thread &x : touch) x.join();
  std::vector<Mem> mems;
  int64_t off = 0;
  for (int t = 0; t < nt && off >= 0 && off < n; ++t) {
    const int64_t c1 = n * (t + 1) / nt;
    if (start[(size_t)t] == off && land[(size_t)t] >= 0) {
      mems.insert(mems.end(), part[(size_t)t].begin(), part[(size_t)t].end());
      off = land[(size_t)t];
    } else if (off < c1) {
      off = walk(off, c1, mems);
    }
    part[(size_t)t] = std::vector<Mem>();
  }
  if (off < 0) {  // the true chain broke at -1 - off: the sequential walk's error
    const int64_t at = -1 - off;
    Mem m;
    const int w = member(at, m);
    if (w == -1) return set_err(GQ_E_NOT_BGZF, "%s: a gzip stream without BGZF block sizes", path);
    if (w == -2) return set_err(GQ_E_BAM_FORMAT, "truncated BGZF block at file offset %lld", (long long)at);
    return set_err(GQ_E_BAM_FORMAT, "not a BGZF/gzip member at file offset %lld", (long long)at);
  }
  int64_t outn = 0;
  b->blocks.reserve(mems.size());
  b->foff.reserve(mems.size());
  for (const Mem &m : mems) {
    BgzfBlock k{};
    k.in_off = m.off + m.payload;
    k.in_len = (int32_t)(m.bsize - m.payload - 8);
    memcpy(&k.crc, p + m.off + m.bsize - 8, 4);
    memcpy(&k.isize, p + m.off + m.bsize - 4, 4);
    if (k.isize > 65536) return set_err(GQ_E_BAM_FORMAT, "BGZF block ISIZE %u > 65536", k.isize);
    k.out_off = outn;
    outn += k.isize;
    b->blocks.push_back(k);
    b->foff.push_back(m.off);
  }
  b->n_out = outn;
  gq_status hs = parse_header(b.get());
  if (hs) return hs;
  const int64_t nb = (int64_t)b->blocks.size();
  gq_bam_dev_sizes &z = b->sizes;
  z.comp_bytes = n;
  z.bam_bytes = outn;
  z.n_blocks = nb;
  z.map_ms = ms_since(t0);
  *out = b.release();
  return GQ_OK;
}

gq_status gq_bam_dev_map(const char *path, gq_bam_dev **out) { return gq_bam_dev_map_ex(path, 1, out); }

gq_status gq_bam_dev_open(gq_ctx *c, const char *path, gq_bam_dev **out) {
  if (!c || !path || !out) return set_err(GQ_E_ARG, "gq_bam_dev_open: null argument");
  gq_bam_dev *m = nullptr;
  gq_status st = gq_bam_dev_map(path, &m);
  if (st) return st;
  st = gq_bam_dev_load(c, m);
  if (st) {
    gq_bam_dev_close(m);
    return st;
  }
  *out = m;
  return GQ_OK;
}

gq_status gq_bam_dev_plan(gq_bam_dev *b, const int64_t *loci_begin, const int64_t *loci_start, const int64_t *loci_end,
                          int64_t halo, const char *bai_path, gq_bam_dev_plan_info *info) {
  if (!b || !loci_begin || !info) return set_err(GQ_E_ARG, "gq_bam_dev_plan: null argument");
  if (b->ctx) return set_err(GQ_E_ARG, "gq_bam_dev_plan: after gq_bam_dev_load");
  const int32_t n_ref = (int32_t)b->names.size();
  if (loci_begin[n_ref] > 0 && (!loci_start || !loci_end)) return set_err(GQ_E_ARG, "gq_bam_dev_plan: loci arrays");
  if (halo < 0) return set_err(GQ_E_ARG, "gq_bam_dev_plan: halo < 0");
  if (!b->sorted) return set_err(GQ_E_PLAN, "the BAM header does not declare SO:coordinate");
  const int64_t nb = (int64_t)b->blocks.size();
  // the index, when it is at least as new as the BAM and describes its dictionary
  bool bai = false;
  if (bai_path && *bai_path) {
    struct stat sb, si;
    if (stat(bai_path, &si) == 0 && fstat(b->fd, &sb) == 0 && si.st_mtime >= sb.st_mtime) bai = load_bai(b, bai_path);
  }
  // the ranges (validated in order), then each range's segment on its own: the searches are
  // independent (the probe cache is shared), so they run on several host threads — without a
  // BAI, each is two binary searches of ~log2(blocks) probes, each probe a host inflate
  struct Range {
    int32_t c;
    int64_t S, E;
  };
  std::vector<Range> ranges;
  for (int32_t c = 0; c < n_ref; ++c) {
    for (int64_t i = loci_begin[c]; i < loci_begin[c + 1]; ++i) {
      const int64_t S = loci_start[i], E = loci_end[i];
      if (E <= S) continue;
      if (i > loci_begin[c] && S < loci_end[i - 1]) return set_err(GQ_E_ARG, "gq_bam_dev_plan: unsorted loci");
      ranges.push_back(Range{c, S, E});
    }
  }
  // the index's start for a range: 1 found, 0 none (no record overlaps the range), -1 unusable index
  auto bai_start = [&](const Range &r, Seg &g) -> int {
    const std::vector<uint64_t> &lx = b->bai_ioff[(size_t)r.c];
    const int64_t w = r.S >> 14;
    if (w >= (int64_t)lx.size()) return 0;  // no record overlaps a window from here on
    // the window's entry, or (an older writer's empty window) the first later one
    int64_t j = w;
    while (j < (int64_t)lx.size() && lx[(size_t)j] == 0) ++j;
    if (j >= (int64_t)lx.size()) return 0;
    return voff_pos(b, lx[(size_t)j], g.b0, g.first) ? 1 : -1;
  };
  if (bai) {  // an index naming a block that is not there is not used at all
    for (const Range &r : ranges) {
      Seg g{0, 0, 0, false};
      if (bai_start(r, g) < 0) {
        bai = false;
        b->bai_ioff.clear();
        break;
      }
    }
  }
  std::vector<Seg> per(ranges.size());
  std::vector<char> keep(ranges.size(), 0);
  std::vector<gq_status> sts(ranges.size(), GQ_OK);
  std::vector<std::string> msgs(ranges.size());
  auto plan_range = [&](size_t i) -> gq_status {
    const Range &r = ranges[i];
    Seg g{0, 0, 0, false};
    if (bai) {
      if (bai_start(r, g) == 0) return GQ_OK;
    } else {
      int64_t bs;
      gq_status st = first_block_at(b, 0, rec_key(r.c, (int32_t)std::max<int64_t>(0, r.S - halo)), bs);
      if (st) return st;
      if (bs >= nb) return GQ_OK;  // every record is before the range
      // the first record starting at or after the end of the last block before it
      int64_t kprev, land;
      if (bs > 0) {
        if ((st = key_upto(b, bs - 1, kprev, &land))) return st;
      } else {
        land = b->rec0;
      }
      stream_pos(b, land, g.b0, g.first);
    }
    // stop: the first block whose records all start at or past (c, E)
    int64_t be;
    gq_status st = first_block_at(b, g.b0, rec_key(r.c, (int32_t)std::min<int64_t>(r.E, INT32_MAX - 1)), be);
    if (st) return st;
    if (be + 1 >= nb) {
      g.b1 = nb;
      g.eof = true;
    } else {
      g.b1 = be + 2;  // records start up to block be; block be + 1 completes the last one
    }
    per[i] = g;
    keep[i] = 1;
    return GQ_OK;
  };
  {
    const int nt = (int)std::min<size_t>(ranges.size(), bai ? 1 : 16);
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i; (i = next.fetch_add(1)) < ranges.size();) {
        sts[i] = plan_range(i);
        if (sts[i]) msgs[i] = gq_last_error();  // (the message is thread-local)
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (std::thread &t : th) t.join();
  }
  std::vector<Seg> segs;
  for (size_t i = 0; i < ranges.size(); ++i) {
    if (sts[i]) return set_err(sts[i], "%s", msgs[i].c_str());
    if (keep[i]) segs.push_back(per[i]);
  }
  // file order, then merge segments whose blocks meet
  std::sort(segs.begin(), segs.end(), [](const Seg &x, const Seg &y) {
    return x.b0 != y.b0 ? x.b0 < y.b0 : x.first < y.first;
  });
  std::vector<Seg> merged;
  for (const Seg &g : segs) {
    if (!merged.empty() && g.b0 <= merged.back().b1) {
      Seg &m = merged.back();
      if (g.b1 > m.b1 || g.eof) {
        m.b1 = std::max(m.b1, g.b1);
        m.eof = m.eof || g.eof;
      }
    } else {
      merged.push_back(g);
    }
  }
  b->segs = merged;
  b->planned = true;
  info->n_segments = (int64_t)merged.size();
  info->n_blocks = info->comp_bytes = info->bam_bytes = 0;
  for (const Seg &g : merged) {
    info->n_blocks += g.b1 - g.b0;
    const int64_t f1 = g.b1 < nb ? b->foff[(size_t)g.b1] : (int64_t)b->map_len;
    info->comp_bytes += f1 - b->foff[(size_t)g.b0];
    for (int64_t k = g.b0; k < g.b1; ++k) info->bam_bytes += b->blocks[(size_t)k].isize;
  }
  info->probes = b->n_probes;
  info->used_index = bai ? 1 : 0;
  info->pad = 0;
  return GQ_OK;
}

gq_status gq_bam_dev_plan_segments(const gq_bam_dev *b, int64_t *first_block, int64_t *first_offset,
                                   int64_t *end_block, int32_t *to_eof) {
  if (!b || !first_block || !first_offset || !end_block || !to_eof)
    return set_err(GQ_E_ARG, "gq_bam_dev_plan_segments: null argument");
  for (size_t i = 0; i < b->segs.size(); ++i) {
    first_block[i] = b->segs[i].b0;
    first_offset[i] = b->segs[i].first;
    end_block[i] = b->segs[i].b1;
    to_eof[i] = b->segs[i].eof ? 1 : 0;
  }
  return GQ_OK;
}

gq_status gq_bam_dev_load(gq_ctx *c, gq_bam_dev *mapped) {
  if (!c || !mapped) return set_err(GQ_E_ARG, "gq_bam_dev_load: null argument");
  if (mapped->ctx) return set_err(GQ_E_ARG, "gq_bam_dev_load: already loaded");
  HIP_TRY(hipSetDevice(c->device));
  gq_bam_dev *b = mapped;
  b->ctx = c;
  const uint8_t *p = b->map;
  // the blocks to inflate and the file bytes to copy: the whole file, or the planned
  // segments back to back (their blocks' payload and stream offsets compacted)
  std::vector<std::pair<int64_t, int64_t>> pieces;  // (file offset, bytes) copied in order
  b->sel_seg0.clear();
  if (!b->planned) {
    b->sel = b->blocks;
    pieces.emplace_back(0, (int64_t)b->map_len);
  } else {
    b->sel.clear();
    int64_t in_acc = 0, out_acc = 0;
    const int64_t nb = (int64_t)b->blocks.size();
    for (const Seg &g : b->segs) {
      b->sel_seg0.push_back((int64_t)b->sel.size());
      const int64_t f0 = b->foff[(size_t)g.b0], f1 = g.b1 < nb ? b->foff[(size_t)g.b1] : (int64_t)b->map_len;
      for (int64_t k = g.b0; k < g.b1; ++k) {
        BgzfBlock x = b->blocks[(size_t)k];
        x.in_off = in_acc + (x.in_off - f0);
        x.out_off = out_acc;
        out_acc += x.isize;
        b->sel.push_back(x);
      }
      pieces.emplace_back(f0, f1 - f0);
      in_acc += f1 - f0;
    }
  }
  b->sel_seg0.push_back((int64_t)b->sel.size());
  int64_t n = 0, outn = 0;
  for (auto &pc : pieces) n += pc.second;
  for (const BgzfBlock &x : b->sel) outn += x.isize;
  b->n_out = outn;
  const int64_t nb = (int64_t)b->sel.size();
  gq_bam_dev_sizes &z = b->sizes;
  z.comp_bytes = n;
  z.bam_bytes = outn;
  z.n_blocks = nb;
  auto t0 = std::chrono::steady_clock::now();
  // the inflate's buffers are allocated on another host thread while this one copies the file
  hipError_t alloc_err = hipSuccess;
  std::thread alloc([&] {
    alloc_err = hipSetDevice(c->device);
    if (alloc_err == hipSuccess) alloc_err = b->out.ensure((size_t)outn + 64);
    if (alloc_err == hipSuccess) alloc_err = b->scratch.ensure((size_t)std::max<int64_t>(nb, 1) * kScratchBytes);
    if (alloc_err == hipSuccess) alloc_err = b->status.ensure(sizeof(int) * (size_t)std::max<int64_t>(nb, 1));
  });
  struct Join {
    std::thread &t;
    ~Join() {
      if (t.joinable()) t.join();
    }
  } join{alloc};
  // the file (or its segments) -> HBM (pinned chunks filled by host threads while the DMA drains
  // the other), then the inflate of every block at once.  (Launching each quarter of the blocks
  // on its own stream as its bytes landed measured slower: a launch lasts about one block's
  // decode whatever its size, and the extra streams cost their creation.)
  HIP_TRY(b->comp.ensure((size_t)n + 64));
  HIP_TRY(hipMemsetAsync((uint8_t *)b->comp.p + n, 0, 64, c->stream));
  HIP_TRY(b->blk.ensure(sizeof(BgzfBlock) * (size_t)std::max<int64_t>(nb, 1)));
  if (nb)
    HIP_TRY(hipMemcpyAsync(b->blk.p, b->sel.data(), sizeof(BgzfBlock) * (size_t)nb, hipMemcpyHostToDevice, c->stream));
  {
    H2DStager stager(c);
    HIP_TRY(stager.init());
    std::vector<int64_t> at(pieces.size() + 1, 0);  // logical offset of each piece
    for (size_t i = 0; i < pieces.size(); ++i) at[i + 1] = at[i] + pieces[i].second;
    HIP_TRY(stager.copy_from(b->comp.p, (size_t)n, [&](uint8_t *dst, size_t o, size_t k) {
      size_t i = (size_t)(std::upper_bound(at.begin(), at.end(), (int64_t)o) - at.begin()) - 1;
      while (k > 0) {
        const size_t in_piece = (size_t)(at[i + 1] - (int64_t)o);
        const size_t take = std::min(k, in_piece);
        memcpy(dst, p + pieces[i].first + ((int64_t)o - at[i]), take);
        dst += take;
        o += take;
        k -= take;
        ++i;
      }
    }));
    z.h2d_ms = ms_since(t0);
    t0 = std::chrono::steady_clock::now();
    alloc.join();
    HIP_TRY(alloc_err);
    HIP_TRY(hipMemsetAsync((uint8_t *)b->out.p + outn, 0, 64, c->stream));
    if (nb) {
      hipLaunchKernelGGL(bgzf_inflate, dim3(grid(nb, kInfLanes)), dim3(kInfLanes), 0, c->stream,
                         (const uint8_t *)b->comp.p, n + 64, (const BgzfBlock *)b->blk.p, nb, (uint8_t *)b->out.p,
                         (uint16_t *)b->scratch.p, (int *)b->status.p);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(bgzf_crc, dim3(grid(nb, 256)), dim3(256), 0, c->stream, (const uint8_t *)b->out.p,
                         (const BgzfBlock *)b->blk.p, nb, (int *)b->status.p);
      HIP_TRY(hipGetLastError());
    }
  }
  {
    DevBuf &status = b->status;
    std::vector<int> sth((size_t)nb);
    if (nb) HIP_TRY(hipMemcpyAsync(sth.data(), status.p, sizeof(int) * (size_t)nb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int64_t i = 0; i < nb; ++i)
      if (sth[(size_t)i] != E_OK) {  // report the block's payload offset in the file
        const int64_t fo = b->sel[(size_t)i].in_off;
        int64_t file_off = fo;
        if (b->planned) {
          size_t s = 0;
          while (s + 1 < b->segs.size() && b->sel_seg0[s + 1] <= i) ++s;
          const BgzfBlock &orig = b->blocks[(size_t)(b->segs[s].b0 + (i - b->sel_seg0[s]))];
          file_off = orig.in_off;
        }
        return set_err(GQ_E_BAM_FORMAT, "corrupt BGZF block (inflate, ISIZE or CRC32) with payload at file offset %lld",
                       (long long)file_off);
      }
  }
  z.inflate_ms = ms_since(t0);
  // the compressed bytes and the inflate tables are not read again (a later load re-uploads):
  // their HBM goes back before the scan and the SoA fill allocate (the load's peak)
  b->comp.release();
  b->scratch.release();
  return GQ_OK;
}

void gq_bam_dev_close(gq_bam_dev *b) { delete b; }
const char *gq_bam_dev_header_text(const gq_bam_dev *b) { return b ? b->text.c_str() : nullptr; }
int32_t gq_bam_dev_n_contigs(const gq_bam_dev *b) { return b ? (int32_t)b->names.size() : -1; }
const char *gq_bam_dev_contig_name(const gq_bam_dev *b, int32_t i) {
  return (b && i >= 0 && i < (int32_t)b->names.size()) ? b->names[(size_t)i].c_str() : nullptr;
}
int64_t gq_bam_dev_contig_length(const gq_bam_dev *b, int32_t i) {
  return (b && i >= 0 && i < (int32_t)b->lengths.size()) ? b->lengths[(size_t)i] : -1;
}

gq_status gq_bam_dev_scan(gq_bam_dev *b, const gq_bam_dev_filters *fl, int64_t *rg_first, gq_bam_dev_sizes *sizes) {
  if (!b || !fl || !rg_first || !sizes) return set_err(GQ_E_ARG, "gq_bam_dev_scan: null argument");
  gq_ctx *c = b->ctx;
  const int32_t n_ref = (int32_t)b->names.size();
  if (fl->use_loci && (!fl->loci_begin || (!fl->loci_start && fl->loci_begin[n_ref] > 0)))
    return set_err(GQ_E_ARG, "use_loci without loci arrays");
  if (fl->n_rg < 0 || fl->n_rg > 254 || (fl->n_rg > 0 && !fl->rg_ids)) return set_err(GQ_E_ARG, "bad read-group IDs");
  HIP_TRY(hipSetDevice(c->device));
  b->scanned = false;
  auto t0 = std::chrono::steady_clock::now();
  const uint8_t *d = (const uint8_t *)b->out.p;
  const int64_t n = b->n_out, nb = (int64_t)b->sel.size();
  const BgzfBlock *blk = (const BgzfBlock *)b->blk.p;
  // record boundaries: candidate starts per block, chains, the host walk of the true chain
  DevBuf first, cnt, land, base, tmp;
  const size_t nbb = sizeof(int64_t) * (size_t)(nb + 1);
  HIP_TRY(first.ensure(nbb));
  HIP_TRY(cnt.ensure(nbb));
  HIP_TRY(land.ensure(nbb));
  HIP_TRY(base.ensure(nbb));
  if (nb) {
    hipLaunchKernelGGL(rec_sync, dim3(grid(nb, 4)), dim3(256), 0, c->stream, d, n, blk, nb, b->planned ? 0 : b->rec0, n_ref,
                       (int64_t *)first.p);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(rec_hop, dim3(grid(nb, 256)), dim3(256), 0, c->stream, d, n, blk, (int64_t)0, nb,
                       (const int64_t *)first.p, (int64_t *)cnt.p, (int64_t *)land.p);
    HIP_TRY(hipGetLastError());
  }
  std::vector<int64_t> hf((size_t)nb), hc((size_t)nb), hl((size_t)nb);
  if (nb) {
    HIP_TRY(hipMemcpyAsync(hf.data(), first.p, sizeof(int64_t) * nb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(hc.data(), cnt.p, sizeof(int64_t) * nb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(hl.data(), land.p, sizeof(int64_t) * nb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  // the true chain, segment by segment (an unplanned load: one segment from the first record
  // to the stream's end)
  const std::vector<BgzfBlock> &sel = b->sel;
  int64_t n_rec = 0;
  int64_t rehops = 0;
  const size_t n_seg = b->planned ? b->segs.size() : 1;
  for (size_t s = 0; s < n_seg; ++s) {
    const int64_t k0 = b->planned ? b->sel_seg0[s] : 0, k1 = b->planned ? b->sel_seg0[s + 1] : nb;
    const bool eof = b->planned ? b->segs[s].eof : true;
    const int64_t kr = eof ? k1 : k1 - 1;  // blocks whose records are read (the last one only completes a record)
    int64_t at = b->planned ? sel[(size_t)k0].out_off + b->segs[s].first : b->rec0;
    for (int64_t k = k0; k < k1; ++k) {
      const int64_t hi = sel[(size_t)k].out_off + (int64_t)sel[(size_t)k].isize;
      if (k >= kr || at >= hi) {  // no record of the chain starts in this block
        hf[(size_t)k] = -1;
        hc[(size_t)k] = 0;
        continue;
      }
      if (hf[(size_t)k] != at || hl[(size_t)k] < 0) {  // a false sync (or none): re-hop from the chain
        ++rehops;
        hf[(size_t)k] = at;
        HIP_TRY(hipMemcpyAsync((int64_t *)first.p + k, &at, sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
        hipLaunchKernelGGL(rec_hop, dim3(1), dim3(64), 0, c->stream, d, n, blk, k, k + 1, (const int64_t *)first.p,
                           (int64_t *)cnt.p, (int64_t *)land.p);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(&hc[(size_t)k], (int64_t *)cnt.p + k, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(&hl[(size_t)k], (int64_t *)land.p + k, sizeof(int64_t), hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (hl[(size_t)k] < 0)
          return set_err(GQ_E_BAM_FORMAT, "truncated BAM record %lld", (long long)(n_rec + hc[(size_t)k]));
      }
      n_rec += hc[(size_t)k];
      at = hl[(size_t)k];
    }
    const int64_t seg_end = sel[(size_t)k1 - 1].out_off + (int64_t)sel[(size_t)k1 - 1].isize;
    if (eof && at != seg_end) return set_err(GQ_E_BAM_FORMAT, "truncated BAM record %lld", (long long)n_rec);
    if (!eof && at > seg_end)
      return set_err(GQ_E_PLAN, "a BAM record runs past the end of planned segment %lld", (long long)s);
  }
  std::vector<int64_t> hb((size_t)nb + 1, 0);
  for (int64_t k = 0; k < nb; ++k) hb[(size_t)k + 1] = hb[(size_t)k] + hc[(size_t)k];
  if (nb) {
    HIP_TRY(hipMemcpyAsync(first.p, hf.data(), sizeof(int64_t) * nb, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(base.p, hb.data(), sizeof(int64_t) * nb, hipMemcpyHostToDevice, c->stream));
  }
  HIP_TRY(b->rec.ensure(sizeof(int64_t) * (size_t)(n_rec + 1)));
  if (nb) {
    hipLaunchKernelGGL(rec_list, dim3(grid(nb, 256)), dim3(256), 0, c->stream, d, blk, nb, (const int64_t *)first.p,
                       (const int64_t *)base.p, (int64_t *)b->rec.p);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  b->sizes.records_ms = ms_since(t0);
  first.release();
  cnt.release();
  land.release();
  base.release();
  // parse + filter every record
  t0 = std::chrono::steady_clock::now();
  DevFilters f{};
  f.non_duplicate = fl->non_duplicate;
  f.passed_vendor = fl->passed_vendor_quality_checks;
  f.is_paired = fl->is_paired;
  f.has_md = fl->has_md_tag;
  f.use_loci = fl->use_loci;
  f.n_ref = n_ref;
  f.n_rg = fl->n_rg;
  DevBuf lb, lsb, leb, rgb, rgo, keep, seq_k, cig_k, md_k, rgf, errb;
  if (fl->use_loci) {
    const int64_t nl = fl->loci_begin[n_ref];
    HIP_TRY(lb.ensure(sizeof(int64_t) * (size_t)(n_ref + 1)));
    HIP_TRY(hipMemcpyAsync(lb.p, fl->loci_begin, sizeof(int64_t) * (size_t)(n_ref + 1), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(lsb.ensure(sizeof(int64_t) * (size_t)std::max<int64_t>(nl, 1)));
    HIP_TRY(leb.ensure(sizeof(int64_t) * (size_t)std::max<int64_t>(nl, 1)));
    if (nl) {
      HIP_TRY(hipMemcpyAsync(lsb.p, fl->loci_start, sizeof(int64_t) * (size_t)nl, hipMemcpyHostToDevice, c->stream));
      HIP_TRY(hipMemcpyAsync(leb.p, fl->loci_end, sizeof(int64_t) * (size_t)nl, hipMemcpyHostToDevice, c->stream));
    }
    f.loci_begin = (const int64_t *)lb.p;
    f.loci_start = (const int64_t *)lsb.p;
    f.loci_end = (const int64_t *)leb.p;
  }
  std::vector<int32_t> ro((size_t)fl->n_rg + 1, 0);
  {
    size_t q = 0;
    for (int k = 0; k < fl->n_rg; ++k) {
      ro[(size_t)k] = (int32_t)q;
      q += strlen(fl->rg_ids + q) + 1;
    }
    ro[(size_t)fl->n_rg] = (int32_t)q;
    HIP_TRY(rgb.ensure(std::max<size_t>(q, 1)));
    if (q) HIP_TRY(hipMemcpyAsync(rgb.p, fl->rg_ids, q, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(rgo.ensure(sizeof(int32_t) * ro.size()));
    HIP_TRY(hipMemcpyAsync(rgo.p, ro.data(), sizeof(int32_t) * ro.size(), hipMemcpyHostToDevice, c->stream));
    f.rg_ids = (const uint8_t *)rgb.p;
    f.rg_id_off = (const int32_t *)rgo.p;
  }
  const size_t n1 = sizeof(int64_t) * (size_t)(n_rec + 1);
  HIP_TRY(b->info.ensure(sizeof(RecInfo) * (size_t)std::max<int64_t>(n_rec, 1)));
  for (DevBuf *x : {&keep, &seq_k, &cig_k, &md_k}) {
    HIP_TRY(x->ensure(n1));
    HIP_TRY(hipMemsetAsync(x->p, 0, n1, c->stream));
  }
  HIP_TRY(rgf.ensure(sizeof(uint64_t) * (size_t)(fl->n_rg + 1)));
  HIP_TRY(hipMemsetAsync(rgf.p, 0xFF, sizeof(uint64_t) * (size_t)(fl->n_rg + 1), c->stream));
  HIP_TRY(errb.ensure(3 * sizeof(uint64_t)));
  HIP_TRY(hipMemsetAsync(errb.p, 0xFF, 2 * sizeof(uint64_t), c->stream));
  HIP_TRY(hipMemsetAsync((uint64_t *)errb.p + 2, 0, sizeof(uint64_t), c->stream));  // the largest span
  if (n_rec) {
    hipLaunchKernelGGL(rec_parse, dim3(grid(n_rec, 256)), dim3(256), 0, c->stream, d, (const int64_t *)b->rec.p, n_rec,
                       f, (RecInfo *)b->info.p, (int64_t *)keep.p, (int64_t *)seq_k.p, (int64_t *)cig_k.p,
                       (int64_t *)md_k.p, (unsigned long long *)rgf.p, (unsigned long long *)errb.p,
                       (unsigned long long *)errb.p + 2);
    HIP_TRY(hipGetLastError());
  }
  uint64_t err[3];
  HIP_TRY(hipMemcpyAsync(err, errb.p, sizeof(err), hipMemcpyDeviceToHost, c->stream));
  std::vector<uint64_t> rgh((size_t)fl->n_rg + 1);
  HIP_TRY(hipMemcpyAsync(rgh.data(), rgf.p, sizeof(uint64_t) * rgh.size(), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (err[0] != ~0ull) {
    const long long r = (long long)(err[0] >> 8);
    // the failing record's bytes, for the host loader's message details
    std::vector<uint8_t> rb;
    {
      int64_t ro = 0;
      int32_t bs = 0;
      if (hipMemcpy(&ro, (const int64_t *)b->rec.p + r, 8, hipMemcpyDeviceToHost) == hipSuccess &&
          hipMemcpy(&bs, d + ro, 4, hipMemcpyDeviceToHost) == hipSuccess && bs >= 32 && ro + 4 + bs <= n) {
        rb.resize((size_t)bs + 4);
        if (hipMemcpy(rb.data(), d + ro, rb.size(), hipMemcpyDeviceToHost) != hipSuccess) rb.clear();
      }
    }
    auto l_seq = [&]() -> int32_t {
      int32_t v = 0;
      if (rb.size() >= 24) memcpy(&v, rb.data() + 20, 4);
      return v;
    };
    auto bad_type = [&](bool array) -> char {  // the first aux type (or array sub-type) the scan rejects
      if (rb.size() < 36) return '?';
      int32_t ls;
      uint16_t nc;
      memcpy(&ls, rb.data() + 20, 4);
      memcpy(&nc, rb.data() + 16, 2);
      size_t q = 36 + rb[12] + 4 * (size_t)nc + (size_t)(ls + 1) / 2 + (size_t)ls;
      while (q + 3 <= rb.size()) {
        const char ty = (char)rb[q + 2];
        q += 3;
        if (strchr("AcC", ty)) q += 1;
        else if (strchr("sS", ty)) q += 2;
        else if (strchr("iIf", ty)) q += 4;
        else if (ty == 'Z' || ty == 'H') {
          while (q < rb.size() && rb[q]) ++q;
          ++q;
        } else if (ty == 'B') {
          if (q + 5 > rb.size()) return '?';
          const char sub = (char)rb[q];
          int32_t cnt;
          memcpy(&cnt, rb.data() + q + 1, 4);
          const int w = strchr("cC", sub) ? 1 : strchr("sS", sub) ? 2 : strchr("iIf", sub) ? 4 : 0;
          if (!w) return array ? sub : '?';
          q += 5 + (size_t)cnt * w;
        } else {
          return array ? '?' : ty;
        }
      }
      return '?';
    };
    switch (err[0] & 0xFF) {
      case X_TRUNC: return set_err(GQ_E_BAM_FORMAT, "truncated BAM record %lld", r);
      case X_AUX_TRUNC: return set_err(GQ_E_BAM_FORMAT, "truncated aux field in BAM record %lld", r);
      case X_AUX_STR: return set_err(GQ_E_BAM_FORMAT, "unterminated aux string in BAM record %lld", r);
      case X_AUX_ARR: return set_err(GQ_E_BAM_FORMAT, "truncated aux array in BAM record %lld", r);
      case X_AUX_ARR_TYPE: return set_err(GQ_E_BAM_RECORD, "bad aux array type '%c'", bad_type(true));
      case X_AUX_TYPE: return set_err(GQ_E_BAM_RECORD, "bad aux type '%c'", bad_type(false));
      default: return set_err(GQ_E_BAM_RECORD, "Base qualities have length 0 but sequence has length %d", l_seq());
    }
  }
  if (err[1] != ~0ull) return set_err(GQ_E_MD_PARSE, "MdTag parse error in BAM record %lld", (long long)(err[1] >> 8));
  for (int k = 0; k <= fl->n_rg; ++k) rg_first[k] = rgh[(size_t)k] == ~0ull ? -1 : (int64_t)rgh[(size_t)k];
  // kept-read indexes and pool offsets
  HIP_TRY(b->kidx.ensure(n1));
  HIP_TRY(b->seq_o.ensure(n1));
  HIP_TRY(b->cig_o.ensure(n1));
  HIP_TRY(b->md_o.ensure(n1));
  gq_status s;
  if ((s = exclusive_sum(c, (const int64_t *)keep.p, (int64_t *)b->kidx.p, n_rec + 1, tmp))) return s;
  if ((s = exclusive_sum(c, (const int64_t *)seq_k.p, (int64_t *)b->seq_o.p, n_rec + 1, tmp))) return s;
  if ((s = exclusive_sum(c, (const int64_t *)cig_k.p, (int64_t *)b->cig_o.p, n_rec + 1, tmp))) return s;
  if ((s = exclusive_sum(c, (const int64_t *)md_k.p, (int64_t *)b->md_o.p, n_rec + 1, tmp))) return s;
  if ((s = d2h_i64(c, (const int64_t *)b->kidx.p + n_rec, &b->n_keep))) return s;
  if ((s = d2h_i64(c, (const int64_t *)b->seq_o.p + n_rec, &b->seq_bytes))) return s;
  if ((s = d2h_i64(c, (const int64_t *)b->cig_o.p + n_rec, &b->cigar_len))) return s;
  if ((s = d2h_i64(c, (const int64_t *)b->md_o.p + n_rec, &b->md_events))) return s;
  b->n_rec = n_rec;
  b->sizes.parse_ms = ms_since(t0);
  b->sizes.n_records = n_rec;
  b->sizes.max_span = (int64_t)err[2];
  b->sizes.n_reads = b->n_keep;
  b->sizes.seq_bytes = b->seq_bytes;
  b->sizes.cigar_len = b->cigar_len;
  b->sizes.md_events = b->md_events;
  (void)rehops;
  b->scanned = true;
  *sizes = b->sizes;
  return GQ_OK;
}

gq_status gq_bam_dev_reads(gq_bam_dev *b, const uint8_t *class_sample, int32_t n_samples, const uint32_t *sample_hash,
                           gq_dev_reads **out, float *fill_ms) {
  if (!b || !class_sample || !out) return set_err(GQ_E_ARG, "gq_bam_dev_reads: null argument");
  if (!b->scanned) return set_err(GQ_E_ARG, "gq_bam_dev_reads before gq_bam_dev_scan");
  if (n_samples < 1 || n_samples > 8) return set_err(GQ_E_ARG, "n_samples must be in [1, 8]");
  gq_ctx *c = b->ctx;
  HIP_TRY(hipSetDevice(c->device));
  auto t0 = std::chrono::steady_clock::now();
  const int64_t n = b->n_keep;
  const int32_t n_ref = (int32_t)b->names.size();
  if (n_ref <= 0) return set_err(GQ_E_ARG, "bad read-set sizes");
  std::unique_ptr<gq_dev_reads> dr(new gq_dev_reads());
  gq_dev_reads *d = dr.get();
  d->ctx = c;
  auto alloc = [&](size_t bytes, void **p) -> hipError_t {
    *p = nullptr;
    hipError_t e = hipMalloc(p, std::max(bytes, (size_t)16));
    if (e == hipSuccess) d->owned.push_back(*p);
    return e;
  };
  struct Guard {  // frees the handle's buffers on an early return
    gq_dev_reads *d;
    ~Guard() {
      if (d)
        for (void *p : d->owned) (void)hipFree(p);
    }
  } guard{d};
  FillOut F{};
  void *p;
  DevBuf contig, ekey, cls, tmp, flag;
  const size_t n0 = (size_t)std::max<int64_t>(n, 1);
  HIP_TRY(contig.ensure(sizeof(int32_t) * n0));
  HIP_TRY(ekey.ensure(sizeof(uint64_t) * n0));
  F.contig = (int32_t *)contig.p;
  F.end_key = (uint64_t *)ekey.p;
  HIP_TRY(alloc(sizeof(int32_t) * n0, &p)); F.start = (int32_t *)p;
  HIP_TRY(alloc(sizeof(int32_t) * n0, &p)); F.end = (int32_t *)p;
  HIP_TRY(alloc(n0, &p)); F.mapq = (uint8_t *)p;
  HIP_TRY(alloc(n0, &p)); F.flags = (uint8_t *)p;
  HIP_TRY(alloc(n0, &p)); F.sample = (uint8_t *)p;
  HIP_TRY(alloc(sizeof(int64_t) * n0, &p)); F.seq_off = (int64_t *)p;
  HIP_TRY(alloc(sizeof(int32_t) * n0, &p)); F.seq_len = (int32_t *)p;
  HIP_TRY(alloc(sizeof(int64_t) * n0, &p)); F.cigar_off = (int64_t *)p;
  HIP_TRY(alloc(sizeof(int32_t) * n0, &p)); F.n_cigar = (int32_t *)p;
  HIP_TRY(alloc(sizeof(int64_t) * n0, &p)); F.md_off = (int64_t *)p;
  HIP_TRY(alloc(sizeof(int32_t) * n0, &p)); F.n_md = (int32_t *)p;
  HIP_TRY(alloc(sizeof(uint16_t) * n0, &p)); F.n_mismatch = (uint16_t *)p;
  HIP_TRY(alloc((size_t)b->seq_bytes + kSeqPad, &p)); F.seq = (uint8_t *)p;
  HIP_TRY(hipMemsetAsync(F.seq + b->seq_bytes, 0, kSeqPad, c->stream));
  HIP_TRY(alloc((size_t)b->seq_bytes + kSeqPad, &p)); F.qual = (uint8_t *)p;
  HIP_TRY(hipMemsetAsync(F.qual + b->seq_bytes, 0, kSeqPad, c->stream));
  HIP_TRY(alloc(sizeof(uint32_t) * (size_t)std::max<int64_t>(b->cigar_len, 1), &p)); F.cigar = (uint32_t *)p;
  HIP_TRY(alloc(sizeof(uint32_t) * (size_t)std::max<int64_t>(b->md_events, 1), &p)); F.md_ev = (uint32_t *)p;
  int32_t *pmax;
  HIP_TRY(alloc(sizeof(int32_t) * n0, &p)); pmax = (int32_t *)p;
  int64_t *begin;
  HIP_TRY(alloc(sizeof(int64_t) * (size_t)(n_ref + 1), &p)); begin = (int64_t *)p;
  const int n_cls = 256;
  HIP_TRY(cls.ensure(n_cls));
  HIP_TRY(hipMemsetAsync(cls.p, 0, n_cls, c->stream));
  HIP_TRY(hipMemcpyAsync(cls.p, class_sample, 255, hipMemcpyHostToDevice, c->stream));
  if (b->n_rec) {
    hipLaunchKernelGGL(rec_fill, dim3(grid(b->n_rec * 16, 256)), dim3(256), 0, c->stream, (const uint8_t *)b->out.p,
                       (const int64_t *)b->rec.p, b->n_rec, (const RecInfo *)b->info.p, (const int64_t *)b->kidx.p,
                       (const int64_t *)b->seq_o.p, (const int64_t *)b->cig_o.p, (const int64_t *)b->md_o.p,
                       (const uint8_t *)cls.p, F);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(flag.ensure(sizeof(int)));
  HIP_TRY(hipMemsetAsync(flag.p, 0, sizeof(int), c->stream));
  hipLaunchKernelGGL(reads_order, dim3(grid(n + 1, 256)), dim3(256), 0, c->stream, (const int32_t *)F.contig,
                     (const int32_t *)F.start, n, n_ref, begin, (int *)flag.p);
  HIP_TRY(hipGetLastError());
  if (n) {  // pmax_end: running max of (contig, end) keys; contigs are non-decreasing
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, tb, F.end_key, F.end_key, U64Max(), (int)n, c->stream));
    HIP_TRY(tmp.ensure(tb));
    HIP_TRY(hipcub::DeviceScan::InclusiveScan(tmp.p, tb, F.end_key, F.end_key, U64Max(), (int)n, c->stream));
    hipLaunchKernelGGL(low32, dim3(grid(n, 256)), dim3(256), 0, c->stream, (const uint64_t *)F.end_key, n, pmax);
    HIP_TRY(hipGetLastError());
  }
  int unsorted = 0;
  d->contig_read_begin.assign((size_t)n_ref + 1, 0);
  HIP_TRY(hipMemcpyAsync(&unsorted, flag.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(d->contig_read_begin.data(), begin, sizeof(int64_t) * (size_t)(n_ref + 1),
                         hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (unsorted)
    return set_err(GQ_E_UNSORTED, "the BAM's kept reads are not sorted by (contig, start) (the host loader sorts them)");
  DevReads &R = d->d;
  R.n_reads = n;
  R.n_contigs = n_ref;
  R.n_samples = n_samples;
  R.contig_read_begin = begin;
  R.start = F.start;
  R.end = F.end;
  R.pmax_end = pmax;
  R.mapq = F.mapq;
  R.flags = F.flags;
  R.sample = F.sample;
  R.seq_off = F.seq_off;
  R.seq_len = F.seq_len;
  R.cigar_off = F.cigar_off;
  R.n_cigar = F.n_cigar;
  R.md_off = F.md_off;
  R.n_md = F.n_md;
  R.n_mismatch = F.n_mismatch;
  R.seq = F.seq;
  R.qual = F.qual;
  R.cigar = F.cigar;
  R.md_ev = F.md_ev;
  R.seq_bytes = b->seq_bytes;
  R.seq_cap = b->seq_bytes + kSeqPad;
  R.cigar_len = b->cigar_len;
  R.md_len = b->md_events;
  if (sample_hash) {
    HIP_TRY(alloc(sizeof(uint32_t) * (size_t)n_samples, &p));
    HIP_TRY(hipMemcpy(p, sample_hash, sizeof(uint32_t) * (size_t)n_samples, hipMemcpyHostToDevice));
    R.sample_hash = (const uint32_t *)p;
  }
  d->seq_bytes = b->seq_bytes;
  contig.release();
  ekey.release();
  const float fill = ms_since(t0);
  d->h2d_ms = b->sizes.h2d_ms;
  const auto t1 = std::chrono::steady_clock::now();
  gq_status st = derive_shape(c, d, b->md_events);
  d->derive_ms = ms_since(t1);
  if (st) return st;
  if (fill_ms) *fill_ms = fill;
  guard.d = nullptr;
  *out = dr.release();
  return GQ_OK;
}

gq_status gq_reads_positions(const gq_dev_reads *r, int32_t *start, int32_t *end) {
  if (!r || (!start && !end)) return set_err(GQ_E_ARG, "gq_reads_positions: null argument");
  const size_t n = (size_t)r->d.n_reads;
  if (n == 0) return GQ_OK;
  HIP_TRY(hipSetDevice(r->ctx->device));
  if (start) HIP_TRY(hipMemcpyAsync(start, r->d.start, sizeof(int32_t) * n, hipMemcpyDeviceToHost, r->ctx->stream));
  if (end) HIP_TRY(hipMemcpyAsync(end, r->d.end, sizeof(int32_t) * n, hipMemcpyDeviceToHost, r->ctx->stream));
  HIP_TRY(hipStreamSynchronize(r->ctx->stream));
  return GQ_OK;
}

gq_status gq_reads_contig_begin(const gq_dev_reads *r, int64_t *out) {
  if (!r || !out) return set_err(GQ_E_ARG, "gq_reads_contig_begin: null argument");
  std::copy(r->contig_read_begin.begin(), r->contig_read_begin.end(), out);
  return GQ_OK;
}

gq_status gq_reads_download(const gq_dev_reads *r, const gq_reads *dst) {
  if (!r || !dst) return set_err(GQ_E_ARG, "gq_reads_download: null argument");
  HIP_TRY(hipSetDevice(r->ctx->device));
  const DevReads &R = r->d;
  const size_t n = (size_t)R.n_reads;
  hipStream_t st = r->ctx->stream;
  auto cp = [&](const void *h, const void *dv, size_t bytes) -> hipError_t {
    if (!h || !dv || !bytes) return hipSuccess;
    return hipMemcpyAsync(const_cast<void *>(h), dv, bytes, hipMemcpyDeviceToHost, st);
  };
  HIP_TRY(cp(dst->contig_read_begin, R.contig_read_begin, sizeof(int64_t) * (size_t)(R.n_contigs + 1)));
  HIP_TRY(cp(dst->start, R.start, sizeof(int32_t) * n));
  HIP_TRY(cp(dst->end, R.end, sizeof(int32_t) * n));
  HIP_TRY(cp(dst->pmax_end, R.pmax_end, sizeof(int32_t) * n));
  HIP_TRY(cp(dst->mapq, R.mapq, n));
  HIP_TRY(cp(dst->flags, R.flags, n));
  HIP_TRY(cp(dst->sample, R.sample, n));
  HIP_TRY(cp(dst->seq_off, R.seq_off, sizeof(int64_t) * n));
  HIP_TRY(cp(dst->seq_len, R.seq_len, sizeof(int32_t) * n));
  HIP_TRY(cp(dst->cigar_off, R.cigar_off, sizeof(int64_t) * n));
  HIP_TRY(cp(dst->n_cigar, R.n_cigar, sizeof(int32_t) * n));
  HIP_TRY(cp(dst->md_off, R.md_off, sizeof(int64_t) * n));
  HIP_TRY(cp(dst->n_md, R.n_md, sizeof(int32_t) * n));
  HIP_TRY(cp(dst->n_mismatch, R.n_mismatch, sizeof(uint16_t) * n));
  HIP_TRY(cp(dst->seq, R.seq, (size_t)R.seq_bytes));
  HIP_TRY(cp(dst->qual, R.qual, (size_t)R.seq_bytes));
  HIP_TRY(cp(dst->cigar, R.cigar, sizeof(uint32_t) * (size_t)R.cigar_len));
  HIP_TRY(cp(dst->md_ev, R.md_ev, sizeof(uint32_t) * (size_t)R.md_len));
  HIP_TRY(cp(dst->sample_hash, R.sample_hash, sizeof(uint32_t) * (size_t)R.n_samples));
  HIP_TRY(hipStreamSynchronize(st));
  return GQ_OK;
}

}  // extern "C"

namespace {
__global__ void warm_k() {}
}  // namespace
hipError_t gq::warm_bamdev(hipStream_t s) {
  hipLaunchKernelGGL(warm_k, dim3(1), dim3(64), 0, s);
  return hipGetLastError();
}
