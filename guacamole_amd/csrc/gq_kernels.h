// gq_kernels.h — device-side building blocks shared by the pileup kernels.
//
// Element semantics restate PileupElement.alignment / advanceToLocus
// (/root/reference/src/main/scala/org/hammerlab/guacamole/pileup/PileupElement.scala:68-248)
// and Pileup.referenceBaseAtLocus (pileup/Pileup.scala:157-165).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gq {

enum : int { OP_M = 0, OP_I = 1, OP_D = 2, OP_N = 3, OP_S = 4, OP_H = 5, OP_P = 6, OP_EQ = 7, OP_X = 8 };

__device__ __forceinline__ bool consumes_ref(int op) {
  return op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X;
}
__device__ __forceinline__ bool consumes_read(int op) {
  return op == OP_M || op == OP_I || op == OP_S || op == OP_EQ || op == OP_X;
}

// element kinds (pileup/Alignment.scala:32-94)
enum : int { K_SNV = 0, K_INS = 1, K_DEL = 2, K_MID = 3, K_CLIP = 4 };
// SNV = Match or Mismatch (decided against the pileup reference base later)

// Device view of a resident read set (device pointers).
struct DevReads {
  int64_t n_reads;
  int32_t n_contigs, n_samples;
  const int64_t *contig_read_begin;
  const int32_t *start, *end, *pmax_end;
  const uint8_t *mapq, *flags, *sample;
  const int64_t *seq_off;
  const int32_t *seq_len;
  const int64_t *cigar_off;
  const int32_t *n_cigar;
  const int64_t *md_off;
  const int32_t *n_md;
  const uint16_t *n_mismatch;
  const uint8_t *seq, *qual;
  const uint32_t *cigar, *md_ev;
  int64_t seq_bytes;
  int64_t seq_cap;  // readable bytes of the device seq allocation (>= seq_bytes; padded on upload)
  // derived at upload (read_shape):
  const int16_t *lead;   // leading soft clip of a [S|H]*(M|=|X)[S|H]* CIGAR, -1 otherwise
  const uint8_t *ev_rb;  // per MD event: the read's sequenced base at that position (0 for deletions)
};

// One locus tile: contiguous loci [L0, L1) of one contig, plus the index range
// [rb, re) of reads that can overlap it (pmax_end > L0, start < L1).
struct Tile {
  int64_t ordinal0;  // output ordinal of L0 (position in the concatenated loci ranges)
  int64_t rb, re;
  int32_t contig, L0, L1, range;
};

// Per-call record written by the germline kernels, sorted by `key` afterwards.
struct CallRec {
  uint64_t key;  // ordinal << 12 | sample << 4 | sub
  int32_t contig;
  int32_t pos;
  uint8_t sample, gt0, gt1, flags;
  uint16_t ref_len, alt_len;
  uint64_t allele;  // inline bytes (ref then alt) if ref_len + alt_len <= 8, else pool offset
};
static_assert(sizeof(CallRec) == 32, "CallRec layout");

struct ComplexItem {
  int32_t tile;
  int32_t pos;
  int32_t flags;  // bit0: queued unconditionally (wide tile): the complex kernel counts the visit
};

enum : int { ERR_NONE = 0 };

__device__ __forceinline__ void raise_error(int *err, int64_t *err_pos, int code, int64_t where) {
  if (atomicCAS(err, 0, code) == 0) *err_pos = where;
}

// Base categories: A=0, C=1, T=2, G=3, N=4, other=5.  For A/C/T/G the index is
// (b >> 1) & 3 of the ASCII byte, checked against the packed table 'A','C','T','G'.
__device__ __forceinline__ int base_cat(uint8_t b) {
  const uint32_t idx = ((uint32_t)b >> 1) & 3u;
  const uint32_t expect = (0x47544341u >> (8u * idx)) & 0xFFu;
  return ((uint32_t)b == expect) ? (int)idx : (b == 'N' ? 4 : 5);
}
__device__ __forceinline__ uint8_t cat_base(int c) {  // inverse of base_cat for 0..4
  return (uint8_t)((0x4E47544341ull >> (8 * c)) & 0xFFu);
}
__device__ __forceinline__ uint32_t std_bit(uint8_t b) {  // one bit per standard base (bit = category)
  const int c = base_cat(b);
  return c < 4 ? (1u << c) : 0u;
}
__device__ __forceinline__ uint8_t bit_base(uint32_t m) {  // lowest set bit of a std mask -> base
  return cat_base(__ffs((int)m) - 1);
}

// MD event lookup for reference offset `off` (events sorted by offset).
__device__ __forceinline__ int md_find(const uint32_t *ev, int32_t n, int32_t off) {
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    int32_t o = (int32_t)(ev[mid] >> 8);
    if (o < off) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && (int32_t)(ev[lo] >> 8) == off) return (int)(ev[lo] & 0xFFu);
  return -1;
}

// Bytes [b0, b1) of the sequence pool staged in LDS at `lds` (b0 16-aligned); empty when
// b1 <= b0.  A read whose chunk range lies inside is read from LDS, others from HBM.
struct StageView {
  const uint4 *lds;
  int64_t b0, b1;
};

// Fast path of walk_read_lane for CIGAR = [S|H]* (M|=|X) [S|H]* (one reference-consuming
// op: every element is a Match/Mismatch).  Two passes:
//   1. bases: the read's bytes over [max(s,L0), min(e,L1)) stream in as 16-byte aligned
//      chunks through a 4-deep rotating register prefetch; each dword goes to
//      sink.bases4(i, word, valid4) with no branch (bytes outside the read carry
//      valid = 0 and add nothing; i may fall in the sink's guard band);
//   2. MD events inside the window: sink.event_i(i, read base, MD reference base), with
//      the first four events and their read bases prefetched alongside the chunks.
template <class Sink>
__device__ __forceinline__ void walk_simple(const DevReads &R, int32_t s, int32_t e, int32_t lead, int64_t seq_off,
                                            int32_t nmd, int64_t md_off, int32_t L0, int32_t L1, uint8_t fl,
                                            Sink &sink, const StageView &sv) {
  const int32_t a = s > L0 ? s : L0;
  const int32_t b = e < L1 ? e : L1;
  const int64_t p0 = seq_off + lead + (a - s);
  const int64_t p1 = seq_off + lead + (b - s);
  const int64_t cb0 = p0 & ~(int64_t)15;
  const int nchunks = (int)((p1 - cb0 + 15) >> 4);
  const int32_t ioff = (a - L0) - (int32_t)(p0 - cb0);  // tile index of byte cb0
  const uint32_t *ev = R.md_ev + md_off;
  const uint8_t *evb = R.ev_rb + md_off;
  uint32_t e4[4], b4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    e4[k] = k < nmd ? ev[k] : 0xFFFFFFFFu;
    b4[k] = k < nmd ? evb[k] : 0u;
  }
  const int64_t cend = cb0 + 16 * (int64_t)nchunks;
  // ld(q): chunk q, clamped to the read's last chunk (every load in bounds).  Chunks are
  // loaded kChunkGroup at a time, all issued before the first is used: one memory latency
  // per group instead of one per few chunks.
  constexpr int kChunkGroup = 8;
  auto run = [&](auto ld) {
    const int32_t lo0 = (int32_t)(p0 - cb0);  // first valid byte of chunk 0
    for (int g = 0; g < nchunks; g += kChunkGroup) {
      uint4 c[kChunkGroup];
#pragma unroll
      for (int u = 0; u < kChunkGroup; ++u) c[u] = ld(g + u);
#pragma unroll
      for (int u = 0; u < kChunkGroup; ++u) {
        const int q = g + u;
        if (q < nchunks) {
          const int32_t lo = q == 0 ? lo0 : 0;
          const int64_t rem = p1 - (cb0 + 16 * (int64_t)q);
          const int32_t hi = rem < 16 ? (int32_t)rem : 16;
          const uint32_t vm = ((1u << hi) - 1u) & ~((1u << lo) - 1u);  // valid bytes [lo, hi)
          const int32_t ib = ioff + 16 * q;
          sink.bases4(ib, c[u].x, vm & 15u, fl);
          sink.bases4(ib + 4, c[u].y, (vm >> 4) & 15u, fl);
          sink.bases4(ib + 8, c[u].z, (vm >> 8) & 15u, fl);
          sink.bases4(ib + 12, c[u].w, (vm >> 12) & 15u, fl);
        }
      }
    }
  };
  if (cb0 >= sv.b0 && cend <= sv.b1) {  // staged in LDS
    const uint4 *base = sv.lds + ((cb0 - sv.b0) >> 4);
    run([&](int q) -> uint4 { return base[q < nchunks ? q : nchunks - 1]; });
  } else if (cend > R.seq_cap) {  // last read of an unpadded pool: byte loads
    for (int64_t p = p0; p < p1; ++p) {
      const int32_t i = ioff + (int32_t)(p - cb0);
      const int32_t sh = (int32_t)((p - cb0) & 3) * 8;
      sink.bases4(i - (sh >> 3), (uint32_t)R.seq[p] << sh, 1u << (sh >> 3), fl);
    }
  } else {
    const uint4 *base = reinterpret_cast<const uint4 *>(R.seq + cb0);
    run([&](int q) -> uint4 { return base[q < nchunks ? q : nchunks - 1]; });
  }
  // MD events inside [a - s, b - s): mismatching reference bases on this read
  for (int k = 0; k < nmd; ++k) {
    const uint32_t v = k < 4 ? (k == 0 ? e4[0] : k == 1 ? e4[1] : k == 2 ? e4[2] : e4[3]) : ev[k];
    const int32_t off = (int32_t)(v >> 8);
    if (off < a - s) continue;
    if (off >= b - s) break;
    const uint32_t rb = k < 4 ? (k == 0 ? b4[0] : k == 1 ? b4[1] : k == 2 ? b4[2] : b4[3]) : evb[k];
    sink.event_i(off + s - L0, (uint8_t)rb, (uint8_t)(v & 0xFFu), fl);
  }
}

// Per-lane walk of one read's CIGAR over the loci [L0, L1): every lane owns one
// read (64 reads in flight per wave).  `sink.elem(l, kind, base, mdb, ev, flags)`
// receives each pileup element: locus, kind, the sequenced base for SNV / anchor
// elements, the read's MD-derived reference base at l (MDTagUtils.getReference),
// and whether an MD event (mismatch or deleted base) sits at l.
//
// Fast path: CIGAR = [S|H]* (M|=|X) [S|H]* (one reference-consuming op), bases
// read as 16-byte aligned chunks.  General path: any CIGAR, byte loads.
template <class Sink>
__device__ __forceinline__ void walk_read_lane(const DevReads &R, int64_t r, int32_t L0, int32_t L1, Sink &sink,
                                               const StageView &sv = StageView{nullptr, 0, 0}) {
  const int32_t s = R.start[r];
  const int32_t e = R.end[r];
  if (e <= L0 || s >= L1) return;
  const int32_t nmd = R.n_md[r];
  if (nmd < 0) {  // MappedRead.mdTagReferenceBases on a read without MD (MappedRead.scala:57-60)
    sink.error(4 /*GQ_E_NO_MD*/, (int64_t)s);
    return;
  }
  const int64_t cig_off = R.cigar_off[r];
  const int32_t ncig = R.n_cigar[r];
  const uint32_t *ev = R.md_ev + R.md_off[r];
  const int64_t seq_off = R.seq_off[r];
  const int32_t slen = R.seq_len[r];
  const uint8_t fl = R.flags[r];

  const int32_t lead = R.lead[r];
  if (lead >= 0) {
    walk_simple(R, s, e, lead, seq_off, nmd, R.md_off[r], L0, L1, fl, sink, sv);
    return;
  }

  // general CIGAR
  int32_t ref = s;
  int32_t rpos = 0;
  bool lead_ins = false;  // I before any reference-consuming op on a read at locus 0 (PileupElement.scala:102-103, 240-245)
  bool seen_ref = false;
  int kev = 0;
  for (int k = 0; k < ncig; ++k) {
    const uint32_t c = R.cigar[cig_off + k];
    const int op = (int)(c & 15u);
    const int32_t len = (int32_t)(c >> 4);
    const int nextop = (k + 1 < ncig) ? (int)(R.cigar[cig_off + k + 1] & 15u) : -1;
    if (op == OP_I && !seen_ref && s == 0) lead_ins = true;
    if (op == OP_P) sink.error(1 /*GQ_E_ASSERT*/, (int64_t)ref);
    if (consumes_ref(op)) {
      seen_ref = true;
      const int32_t a = ref > L0 ? ref : L0;
      const int32_t b = (ref + len) < L1 ? (ref + len) : L1;
      while (kev < nmd && (int32_t)(ev[kev] >> 8) < a - s) ++kev;
      for (int32_t l = a; l < b; ++l) {
        const int32_t off = l - s;
        int mdv = -1;
        if (kev < nmd && (int32_t)(ev[kev] >> 8) == off) {
          mdv = (int)(ev[kev] & 0xFFu);
          ++kev;
        }
        if (op == OP_M || op == OP_EQ || op == OP_X) {
          const int32_t rp = rpos + (l - ref);
          uint8_t base = 0;
          if (rp < slen) base = R.seq[seq_off + rp];
          else sink.error(1, (int64_t)l);
          const bool fin = (l == ref + len - 1);
          int kind = K_SNV;
          if (lead_ins && l == 0) kind = K_INS;
          else if (fin && (op == OP_M || op == OP_EQ) && nextop == OP_I) kind = K_INS;
          else if (fin && nextop == OP_D) kind = K_DEL;
          sink.elem(l, kind, base, mdv >= 0 ? (uint8_t)mdv : base, mdv >= 0, fl);
        } else if (op == OP_D) {
          if (mdv < 0) sink.error(3 /*GQ_E_MD*/, (int64_t)l);
          sink.elem(l, K_MID, (uint8_t)0, mdv >= 0 ? (uint8_t)mdv : (uint8_t)'N', true, fl);
        } else {  // N: Clipped, MD-derived reference 'N'
          sink.elem(l, K_CLIP, (uint8_t)0, (uint8_t)'N', false, fl);
        }
      }
      ref += len;
    }
    if (consumes_read(op)) rpos += len;
    if (ref >= L1) break;
  }
}

// LDS histogram: seven u32 words per locus (SoA: word * S + guard + i, so consecutive loci
// sit on consecutive banks), each holding two 16-bit counters.  A sequenced base b has
// code (b >> 1) & 7, distinct for A 0, C 1, T 2, G 3, N 7; a base whose code does not
// map back to it is "other" (slot 4).  slot = word * 2 + half:
//   W_AC = A | C << 16, W_TG = T | G << 16, W_OX = other | complex << 16, W_NN = N << 16,
//   W_EAC / W_ETG = A C / T G counts of Match/Mismatch elements carrying an MD mismatch
//   event, W_MASK = OR of MD-derived standard reference bases of event / complex elements.
// Tiles whose read window could exceed 65535 reads never use this path (wide tiles).
enum : int { W_AC = 0, W_TG, W_OX, W_NN, W_EAC, W_ETG, W_MASK, W_N };
// LDS arrays carry a 16-entry guard band on each side (stride T + 32, index 16 + i), so
// the branch-free base pass may address i in [-16, T + 16) with a zero increment.
constexpr int kGuard = 16;

template <int T, int ABL = 0>
struct GermSink {
  uint32_t *cnt;  // W_N arrays of T + 2 * kGuard words
  int32_t L0;
  int *err;
  long long *err_pos;
  static constexpr int S = T + 2 * kGuard;
  uint32_t acc = 0;  // ABL & 4 only
  __device__ __forceinline__ ~GermSink() {
    if ((ABL & 4) && acc == 0x12345u) atomicAdd(cnt, 1u);
  }
  __device__ __forceinline__ uint32_t *at(int w, int i) const { return cnt + w * S + kGuard + i; }
  // four Match/Mismatch elements: the bytes of `w` at tile indices i..i+3 (valid4: bit per byte)
  __device__ __forceinline__ void bases4(int i, uint32_t w, uint32_t valid4, uint8_t) {
    const uint32_t code4 = (w >> 1) & 0x07070707u;
    const uint32_t exp4 = __builtin_amdgcn_perm(0x4E000000u, 0x47544341u, code4);  // 'A','C','T','G',0,0,0,'N'
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t bj = (w >> (8 * j)) & 0xFFu, ej = (exp4 >> (8 * j)) & 0xFFu, cj = (code4 >> (8 * j)) & 7u;
      const uint32_t slot = bj == ej ? cj : 4u;
      if (ABL & 4) {
        acc += ((valid4 >> j) & 1u) << ((slot & 1u) << 4);
        acc ^= slot;
      } else {
        atomicAdd(at((int)(slot >> 1), i + j), ((valid4 >> j) & 1u) << ((slot & 1u) << 4));
      }
    }
  }
  // an MD mismatch event on a Match/Mismatch element: read base b, MD reference base m
  __device__ __forceinline__ void event_i(int i, uint8_t b, uint8_t m, uint8_t) {
    if (ABL & 8) return;
    const int c = base_cat(b);
    if (c < 4) atomicAdd(at(W_EAC + (c >> 1), i), 1u << ((c & 1) << 4));
    const uint32_t bit = std_bit(m);
    if (bit) atomicOr(at(W_MASK, i), bit);
  }
  // general walker elements
  __device__ __forceinline__ void elem_i(int i, int kind, uint8_t base, uint8_t mdb, bool ev, uint8_t fl) {
    if (kind == K_SNV) {
      const int sh = (i & 3) * 8;
      bases4(i - (i & 3), (uint32_t)base << sh, 1u << (i & 3), fl);
      if (ev) event_i(i, base, mdb, fl);
    } else {
      atomicAdd(at(W_OX, i), 1u << 16);
      const uint32_t bit = std_bit(mdb);
      if (bit) atomicOr(at(W_MASK, i), bit);
    }
  }
  __device__ __forceinline__ void elem(int32_t l, int kind, uint8_t base, uint8_t mdb, bool ev, uint8_t fl) {
    elem_i(l - L0, kind, base, mdb, ev, fl);
  }
  __device__ __forceinline__ void error(int code, int64_t where) { raise_error(err, (int64_t *)err_pos, code, where); }
};

}  // namespace gq
