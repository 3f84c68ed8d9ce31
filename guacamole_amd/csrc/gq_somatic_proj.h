// gq_somatic_proj.h — somatic candidate loci over the read projections (somatic_proj), and
// the tumor's margin projection it reads (mproj_fill).  Included inside gq_somatic.hip's
// anonymous namespace.
//
// somatic_proj restates somatic_tile's per-locus test (SomaticStandardCaller.scala:184-206: the
// tumor pileup must hold a non-Match element, the normal pileup must be non-empty; loci whose
// tumor pileup provably has the hom-ref genotype as its maximum-likelihood genotype are dropped,
// hom_ref_margin_lane) on germline_proj's machinery: one wave per 512-locus tile, lane l owns the
// 8-locus column [B0 + 8l, B0 + 8l + 8), groups of 16 lanes walk the tumor reads of their
// 128-locus sub-span and add, per read and column, the projection's base codes (SWAR nibble
// counts) and the margin projection's 16-bit terms (saturating packed adds).  The tumor's MD
// events, N bases and complex ranges come from its sparse entries, the normal's depth from its
// reads' [start, end) intervals (every locus a read spans holds one of its elements,
// PileupElement.scala:68-135) as a difference array.  Tiles the projection cannot take go to
// somatic_tile (lane-per-read walker).
#pragma once

#include "gq_kernels.h"

// The margin term of one tumor element (hom_ref_margin_lane's t) in units of 1/8, rounded down
// with room for the FP32 rounding of t, so that a sum of terms never exceeds the margin it stands
// for: a sum that passes the bound proves what the FP32 sum proved.  Stored biased in a byte:
// 128 + term for terms in [-127, 127] (128: no element), kMargin8None (0) below -127/8 or for a
// quality outside the table — a slice holding one gets no bound at all (mnb).  A byte per element
// (half the int16 terms of round 3) halves somatic_proj's margin traffic; the coarser floor only
// sends a few more loci to the exact caller, whose decisions are the reference's.
constexpr uint8_t kMargin8None = 0, kMargin8Zero = 128;
__device__ __forceinline__ uint8_t margin_term8(bool match, int q, float em, float lsm) {
  constexpr float kLn2 = 0.69314718f;
  if (q < 0) return kMargin8None;  // outside the quality table: no bound
  const float eb = exp2f(-0.33219281f * (float)q);
  const float lsq = log1pf(-eb);
  const float f = eb + em - eb * em;  // 1 - pc
  const float t = match ? kLn2 + lsq + lsm - fmaxf(0.0f, kLn2 + __logf(f)) : __logf(f);
  const float v = floorf(t * 8.0f - 0.015625f);  // -1/64: room for the FP32 rounding of t
  if (!(v >= -127.0f)) return kMargin8None;
  return (uint8_t)(128 + (int)(v > 127.0f ? 127.0f : v));
}

// margin_term8 for every (mapq, quality 0-127, match) of one probability model: byte
// (mq << 8 | q << 1 | match), so the fill looks terms up instead of evaluating exp / log per
// element (the same function, so the same bytes).
__global__ void margin_table(int incl_align, uint8_t *__restrict__ tab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 256 * 256) return;
  const int mq = i >> 8, q = (i >> 1) & 127, match = i & 1;
  // probabilityCorrectIncludingAlignment (somatic tumor) or IgnoringAlignment (germline-standard)
  const float em = incl_align ? exp2f(-0.33219281f * (float)mq) : 0.0f;
  const float lsm = log1pf(-em);
  tab[i] = margin_term8(match != 0, q, em, lsm);
}

typedef uint64_t gq_u64m __attribute__((aligned(1)));  // unaligned 8-byte loads (gfx950 global memory)

// Piece setup of the margin fill: the read's descriptor and its MD events at the piece's loci as
// a bit mask (MD offsets are reference offsets from the read's start, sorted).  Reads the mapq
// filter drops (QualityAlignedReadsFilter, PileupElementsFilter.scala:25-36) are skipped: their
// loci keep the pool's kMargin8Zero fill.
__device__ __forceinline__ bool margin_setup(const DevReads &R, int min_mapq, int64_t md_off, PieceMeta &m) {
  if (min_mapq > 0 && (int)m.mq < min_mapq) return false;
  const int32_t nmd = (int32_t)(m.info & 0xFFFFu);
  const uint32_t *ev = R.md_ev + md_off;
  const int32_t o0 = 8 * m.s0 - m.s;  // offset of the piece's first locus
  uint32_t e0 = 0, e1 = 0, e2 = 0, e3 = 0;  // (registers: a dynamic index would go to scratch)
  auto mark = [&](uint32_t v) {
    const int32_t i = (int32_t)(v >> 8) - o0;
    if (i < 0 || i >= 128) return;
    const uint32_t bit = 1u << (i & 31);
    e0 |= (i >> 5) == 0 ? bit : 0u;
    e1 |= (i >> 5) == 1 ? bit : 0u;
    e2 |= (i >> 5) == 2 ? bit : 0u;
    e3 |= (i >> 5) == 3 ? bit : 0u;
  };
  if (nmd <= 4) {  // the common read: its (few) events in one round of loads
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = k < nmd ? ev[k] : 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nmd) mark(v[k]);
  } else {  // the first event at or past the piece's first locus, then the piece's events
    int k = 0, hi = nmd;
    while (k < hi) {
      const int mid = (k + hi) >> 1;
      if ((int32_t)(ev[mid] >> 8) < o0) k = mid + 1;
      else hi = mid;
    }
    for (; k < nmd; ++k) {
      const uint32_t v = ev[k];
      if ((int32_t)(v >> 8) - o0 >= 128) break;
      mark(v);
    }
  }
  m.ev[0] = e0;
  m.ev[1] = e1;
  m.ev[2] = e2;
  m.ev[3] = e3;
  return true;
}

// The margin word (8 loci, a byte each; hom_ref_margin_lane's terms in 1/8 units, biased) of read
// r at column col, from its piece m.  Loci outside the read's Match/Mismatch blocks hold
// kMargin8Zero.  margin_fetch loads the word's eight qualities (one 8-byte load inside a
// column-eligible read; a general CIGAR's word is complete here); margin_terms8 looks the terms up.
struct MarginRaw {
  uint64_t q;   // qualities, byte k = locus 8 col + k (eligible reads)
  uint2 word;   // general CIGAR: the word itself
  uint32_t valid, gen;  // valid: byte mask of loci inside the read
};
// lrow: the table row of mapping quality lmq staged in this wave's LDS (nullptr: none); a word of
// a read with that mapq looks its terms up there, others in the global table.
__device__ __forceinline__ uint2 margin_terms8(const PieceMeta &m, uint64_t q, uint32_t valid, uint32_t evb,
                                               const uint8_t *__restrict__ tab, const uint8_t *lrow = nullptr,
                                               uint32_t lmq = 0xFFFFFFFFu) {
  const uint8_t *tm = tab + (m.mq << 8);  // evb: the MD events at the word's loci
  const bool local = lrow && m.mq == lmq;
  uint32_t v[2] = {0x80808080u, 0x80808080u};
#pragma unroll
  for (int q8 = 0; q8 < 8; ++q8) {
    if (!((valid >> q8) & 1u)) continue;
    const int qv = (int)(int8_t)(uint8_t)(q >> (8 * q8));
    const int ti = (qv << 1) | ((evb >> q8) & 1u ? 0 : 1);
    const uint32_t t = qv < 0 ? (uint32_t)kMargin8None : local ? (uint32_t)lrow[ti] : (uint32_t)tm[ti];
    v[q8 >> 2] = (v[q8 >> 2] & ~(0xFFu << (8 * (q8 & 3)))) | (t << (8 * (q8 & 3)));
  }
  return make_uint2(v[0], v[1]);
}
// margin_terms8 for a wave whose words all look their terms up in the LDS row (no branches).
__device__ __forceinline__ uint2 margin_terms8_lds(uint64_t q, uint32_t valid, uint32_t evb, const uint8_t *lrow) {
  uint32_t v[2] = {0u, 0u};
#pragma unroll
  for (int q8 = 0; q8 < 8; ++q8) {
    const uint32_t b = (uint32_t)(q >> (8 * q8)) & 0xFFu;
    const uint32_t t0 = lrow[((b & 0x7Fu) << 1) | (((evb >> q8) & 1u) ^ 1u)];
    const uint32_t t1 = (b & 0x80u) ? (uint32_t)kMargin8None : t0;  // a quality outside the table
    const uint32_t t = ((valid >> q8) & 1u) ? t1 : (uint32_t)kMargin8Zero;
    v[q8 >> 2] |= t << (8 * (q8 & 3));
  }
  return make_uint2(v[0], v[1]);
}
__device__ __forceinline__ MarginRaw margin_fetch(const DevReads &R, int64_t r, const PieceMeta &m, int32_t col,
                                                  uint32_t evb, const uint8_t *__restrict__ tab) {
  const int32_t s = m.s, e = m.e;
  const int32_t lb = 8 * col;
  MarginRaw x{0, make_uint2(0x80808080u, 0x80808080u), 0, 0};
  if (m.info & kColEligible) {
    const int64_t a = m.p0 + lb;
    if (a >= 0 && a + 8 <= R.seq_cap) {  // one load; an edge word's loci outside the read masked
      const int32_t lo = min(max(s - lb, 0), 8), hi = min(max(e - lb, 0), 8);
      x.q = *reinterpret_cast<const gq_u64m *>(R.qual + a) & edge_mask(lo, hi);
      x.valid = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
    } else {
#pragma unroll
      for (int q8 = 0; q8 < 8; ++q8) {
        const int32_t l = lb + q8;
        if (l >= s && l < e) {
          x.q |= (uint64_t)R.qual[m.p0 + l] << (8 * q8);
          x.valid |= 1u << q8;
        }
      }
    }
    return x;
  }
  // general CIGAR: the count segments
  const int32_t nmd = (int32_t)(m.info & 0xFFFFu), nseg = (int32_t)((m.info >> 18) & 0xFFu);
  const uint32_t *sg = R.cev + R.caux_off[r] + nmd;
  const int64_t so = R.seq_off[r];
  uint64_t q = 0;
  uint32_t valid = 0;
#pragma unroll
  for (int q8 = 0; q8 < 8; ++q8) {
    const int32_t l = lb + q8;
    for (int32_t q2 = 0; q2 < nseg; ++q2) {
      const uint32_t a = sg[2 * q2], b = sg[2 * q2 + 1];
      const int32_t ra = s + (int32_t)(a & 0xFFFFu), rl = (int32_t)(a >> 16);
      if ((b >> 16) == 0 /* kSegCount */ && l >= ra && l < ra + rl) {
        q |= (uint64_t)R.qual[so + (int32_t)(b & 0xFFFFu) + (l - ra)] << (8 * q8);
        valid |= 1u << q8;
        break;
      }
    }
  }
  x.word = margin_terms8(m, q, valid, evb, tab);
  x.gen = 1;
  return x;
}

// The margin projection of the tumor reads, laid out as `proj` (a byte per projection nibble:
// word w of the row pool at mproj + 8 w), one wave per slice, a lane per word (the rows row_count
// assigned, stored); mnb marks slices holding a kMargin8None term.
template <int KU>
__global__ __launch_bounds__(256) void mproj_fill(DevReads R, int64_t n_slices, int min_mapq,
                                                  const uint8_t *__restrict__ tab, uint8_t *__restrict__ mproj,
                                                  uint8_t *__restrict__ mnb) {
  __shared__ PieceMeta s_meta[4][64];
  __shared__ uint32_t s_owner[4][KU * 64];
  __shared__ uint32_t s_row[4][64];  // the table row of the slice's first read's mapq (256 bytes)
  PieceMeta *meta = s_meta[threadIdx.x >> 6];
  uint32_t *owner = s_owner[threadIdx.x >> 6];
  uint32_t *row = s_row[threadIdx.x >> 6];
  const uint8_t *lrow = reinterpret_cast<const uint8_t *>(row);
  const int lane = threadIdx.x & 63;
  const int64_t w0 = wave_id();
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t slot = w0; slot < n_slices; slot += nw) {
    if (R.pbad[slot]) continue;  // uniform
    uint2 *out = reinterpret_cast<uint2 *>(mproj) + 16 * R.srow[slot];  // the slice's block rows
    const SliceWin W = slice_stored(R, slot);
    // most reads share one mapping quality: its table row in LDS saves the words' lookups a
    // round trip to the cache hierarchy
    const uint32_t lmq = W.rz > W.ra ? (uint32_t)R.mapq[W.ra] : 0u;
    row[lane] = reinterpret_cast<const uint32_t *>(tab + (lmq << 8))[lane];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    bool none = false;
    slice_fill<true, KU>(
        R, W, R.prow + R.soff[slot], meta, owner,
        [&](int64_t, PieceMeta &m, int64_t mdo) { return margin_setup(R, min_mapq, mdo, m); },
        [&](int64_t r, const PieceMeta &m, int32_t col, uint32_t evb) { return margin_fetch(R, r, m, col, evb, tab); },
        [&](bool act, const MarginRaw &x, int64_t, const PieceMeta &m, int32_t col, uint32_t evb) {
          if (act) {
            const uint2 w = x.gen ? x.word : margin_terms8(m, x.q, x.valid, evb, tab, lrow, lmq);
            out[16 * (int64_t)m.row + (col & 15)] = w;
            auto has = [](uint32_t v) {  // a zero byte
              return ((v - 0x01010101u) & ~v & 0x80808080u) != 0u;
            };
            none = none || has(w.x) || has(w.y);
          }
        });
    const bool any = __ballot(none) != 0;
    if ((threadIdx.x & 63) == 0) mnb[slot] = any ? 1 : 0;
  }
}

// The MD-event bits of read m's word at column col (bit k: locus 8 col + k): v holds up to four
// events loaded by the fetch (0xFFFFFFFF: none); a read with more has them in evb already.
__device__ __forceinline__ uint32_t word_event_bits(const ReadMeta &m, int32_t col, const uint32_t (&v)[4], uint32_t evb) {
  const int32_t i0 = 8 * col - m.s;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = (uint32_t)((int32_t)(v[k] >> 8) - i0);
    evb |= i < 8u ? 1u << i : 0u;
  }
  return evb;
}
struct MarginRW {
  MarginRaw x;
  uint32_t v[4];  // the read's events (up to four), for word_event_bits
  uint32_t evb;
};
__device__ __forceinline__ MarginRW margin_fetch_rw(const DevReads &R, int64_t r, const ReadMeta &m, int32_t col,
                                                    const uint8_t *__restrict__ tab, uint64_t pre = 0,
                                                    bool fast = false) {
  MarginRW o;
  const int32_t nmd = (int32_t)(m.info & 0xFFFFu);
  const uint32_t *ev = R.md_ev + m.md_off;
  o.evb = 0;
  if (m.evin) {  // the common read: its events came with its records (16-bit offsets; none: 0xFFFF)
    o.v[0] = (m.ev01 & 0xFFFFu) << 8;
    o.v[1] = (m.ev01 >> 16) << 8;
    o.v[2] = (m.ev23 & 0xFFFFu) << 8;
    o.v[3] = (m.ev23 >> 16) << 8;
  } else if (nmd <= 4) {  // its events in the same round of loads as the qualities
#pragma unroll
    for (int k = 0; k < 4; ++k) o.v[k] = k < nmd ? ev[k] : 0xFFFFFFFFu;
  } else {  // the first event at or past the word's first locus, then the word's events
#pragma unroll
    for (int k = 0; k < 4; ++k) o.v[k] = 0xFFFFFFFFu;
    const int32_t i0 = 8 * col - m.s;
    int k = 0, hi = nmd;
    while (k < hi) {
      const int mid = (k + hi) >> 1;
      if ((int32_t)(ev[mid] >> 8) < i0) k = mid + 1;
      else hi = mid;
    }
    for (; k < nmd; ++k) {
      const int32_t i = (int32_t)(ev[k] >> 8) - i0;
      if (i >= 8) break;
      o.evb |= 1u << i;
    }
  }
  const PieceMeta pm = piece_meta(m);
  if (fast) {  // (read_fill loaded the word's qualities: margin_fetch's one-load case)
    const int32_t lb = 8 * col;
    const int32_t lo = min(max(m.s - lb, 0), 8), hi = min(max(m.e - lb, 0), 8);
    o.x = MarginRaw{0, make_uint2(0x80808080u, 0x80808080u), 0, 0};
    o.x.q = pre & edge_mask(lo, hi);
    o.x.valid = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
  } else if (m.info & kColEligible) o.x = margin_fetch(R, r, pm, col, 0u, tab);  // (the terms come in the emit)
  else o.x = margin_fetch(R, r, pm, col, word_event_bits(m, col, o.v, o.evb), tab);
  return o;
}

// The margin projection, read-major (read_fill): a wave per 64 consecutive reads, a lane per
// word; mnb (zeroed by the caller) gets 1 on each slice holding a kMargin8None term.
template <int KU, int KW>
__global__ __launch_bounds__(256) void mproj_fill_rw(DevReads R, int min_mapq, const uint8_t *__restrict__ tab,
                                                     uint8_t *__restrict__ mproj, uint8_t *__restrict__ mnb, int dbg) {
  constexpr int kRows = 4;  // table rows staged per batch: its first kRows distinct mapping qualities
  __shared__ ReadMeta s_meta[4][64];
  __shared__ uint32_t s_owner[4][KU * 64];
  __shared__ uint32_t s_row[4][kRows * 64];
  uint32_t *row = s_row[threadIdx.x >> 6];
  const uint8_t *lrow = reinterpret_cast<const uint8_t *>(row);
  const int lane = threadIdx.x & 63;
  uint32_t lmq[kRows];  // (wave-uniform) the staged rows' mapping qualities; 0xFFFFFFFF: none
  uint2 *out = reinterpret_cast<uint2 *>(mproj);
  read_fill<KU, true, KW>(
      R, s_meta[threadIdx.x >> 6], s_owner[threadIdx.x >> 6], dbg, R.qual,
      [&](int64_t r0) {
        // a few mapping qualities cover a batch's reads (most share one): their table rows in LDS,
        // so a wave's words look their terms up there without a round trip to the cache hierarchy
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const int64_t rl = r0 + lane;
        const uint32_t mq = (uint32_t)R.mapq[rl < R.n_reads ? rl : r0];
        unsigned long long rem = __ballot(true);
#pragma unroll
        for (int k = 0; k < kRows; ++k) {
          lmq[k] = 0xFFFFFFFFu;
          if (rem) {  // (uniform)
            const uint32_t mk = (uint32_t)__builtin_amdgcn_readlane((int)mq, __ffsll((long long)rem) - 1);
            lmq[k] = mk;
            rem &= ~__ballot(mq == mk);
            row[64 * k + lane] = reinterpret_cast<const uint32_t *>(tab + (mk << 8))[lane];
          }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      },
      [&](const ReadMeta &m) { return !(min_mapq > 0 && (int)m.mq < min_mapq); },
      [&](int64_t r, const ReadMeta &m, int32_t col, uint64_t pre, bool fast) {
        return margin_fetch_rw(R, r, m, col, tab, pre, fast);
      },
      [&](bool act, const MarginRW &o, int64_t, const ReadMeta &m, int32_t col, int64_t grow, int64_t slot) {
        int k = -1;
#pragma unroll
        for (int j = kRows - 1; j >= 0; --j) k = m.mq == lmq[j] ? j : k;
        // (uniform: the wave's table lookups all in its LDS rows, or per lane)
        const bool all_lds = __ballot(act && !o.x.gen && k < 0) == 0;
        if (act) {
          const uint32_t evb = word_event_bits(m, col, o.v, o.evb);
          const uint8_t *lr = lrow + 256 * (k < 0 ? 0 : k);
          const uint2 w = o.x.gen ? o.x.word
                          : all_lds ? margin_terms8_lds(o.x.q, o.x.valid, evb, lr)
                                    : margin_terms8(piece_meta(m), o.x.q, o.x.valid, evb, tab, k < 0 ? nullptr : lr,
                                                    m.mq);
          out[16 * grow + (col & 15)] = w;
          auto has = [](uint32_t v) {  // a zero byte
            return ((v - 0x01010101u) & ~v & 0x80808080u) != 0u;
          };
          if (has(w.x) || has(w.y)) mnb[slot] = 1;
        }
      });
}

// ---- The margin projection by pieces (piece_fill in gq_host.h; A/B: GQ_FILL=pieces) ----
struct MarginCell {
  uint64_t q;       // the word's qualities (loci outside the read zero)
  uint32_t valid;   // byte mask of its loci inside the read (0: a read the mapq filter drops)
  uint16_t evb;     // its loci holding an MD event
  uint16_t mq;      // the read's mapping quality (its table row)
};
// The MD-event bits of read r's word at column col (bit k: locus 8 col + k), from its events.
__device__ __forceinline__ uint32_t word_events(const DevReads &R, int64_t md_off, uint32_t info, int32_t s,
                                                int32_t col) {
  const int32_t nmd = (int32_t)(info & 0xFFFFu);
  const uint32_t *ev = R.md_ev + md_off;
  const int32_t i0 = 8 * col - s;
  int k = 0, hi = nmd;
  while (k < hi) {
    const int mid = (k + hi) >> 1;
    if ((int32_t)(ev[mid] >> 8) < i0) k = mid + 1;
    else hi = mid;
  }
  uint32_t evb = 0;
  for (; k < nmd; ++k) {
    const int32_t i = (int32_t)(ev[k] >> 8) - i0;
    if (i >= 8) break;
    evb |= 1u << i;
  }
  return evb;
}

// ---- The margin projection by cells (the default; the projection's proj_fill_cells design) ----
// A wave per slice, a lane per cell: 32-byte window records in LDS (pool offset,
// [start, end), ColDesc info, mapping quality, up to four MD-event offsets), a u8 map cell ->
// window read, then per cell one 8-byte load of its qualities and eight table lookups in the
// LDS row of the wave's common mapping quality.  Every word written (kMargin8Zero where no kept
// element lies), 64 consecutive words per store; mnb[slot] = 1 where a word holds kMargin8None.
struct __attribute__((aligned(16))) MCellRec {
  uint32_t a;         // seq_off + leading clip - seq_off[window's first read]
  int32_t s, e;       // [start, end)
  uint32_t info;      // ColDesc info
  uint32_t mq;        // mapping quality; bit 8: dropped by the mapq filter; bit 9: events not below
  uint32_t ev01, ev23;  // up to four MD-event offsets from s, 16 bits each (0xFFFF: none)
  uint32_t pad;
};
__global__ __launch_bounds__(256) void mproj_fill_cells(DevReads R, int64_t n_slices, int min_mapq,
                                                        const uint8_t *__restrict__ tab, uint8_t *__restrict__ mproj,
                                                        uint8_t *__restrict__ mnb, int64_t *__restrict__ deep,
                                                        unsigned long long *__restrict__ n_deep) {
  constexpr int kWin = 255, kRows = 64;
  __shared__ MCellRec s_rec[4][kWin];
  __shared__ uint8_t s_map[4][kRows * 16];
  __shared__ uint32_t s_row[4][64];  // the table row of one mapping quality (256 bytes)
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  MCellRec *rec = s_rec[wv];
  uint8_t *map = s_map[wv];
  const uint8_t *lrow = reinterpret_cast<const uint8_t *>(s_row[wv]);
  uint32_t lmq = 0;  // most reads share one mapping quality: its row (the wave's first slice's first read)
  {
    const int64_t slot = wave_id();
    if (slot < n_slices) {
      const int64_t ra = R.sra[slot];
      lmq = ra < R.n_reads ? (uint32_t)R.mapq[ra] : 0u;
    }
    s_row[wv][lane] = reinterpret_cast<const uint32_t *>(tab + (lmq << 8))[lane];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  const uint2 zero = make_uint2(0x80808080u, 0x80808080u);
  auto has_none = [](uint2 w) {  // a kMargin8None (zero) byte
    auto z = [](uint32_t v) { return ((v - 0x01010101u) & ~v & 0x80808080u) != 0u; };
    return z(w.x) || z(w.y);
  };
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t slot = wave_id(); slot < n_slices; slot += nw) {
    const int64_t g0 = R.srow[slot];
    const int32_t nr = (int32_t)(R.srow[slot + 1] - g0);
    if (nr <= 0) continue;
    uint2 *out = reinterpret_cast<uint2 *>(mproj) + 16 * g0;
    const SliceWin W = slice_stored(R, slot);
    const int32_t nwin = (int32_t)(W.rz - W.ra);
    if (R.pbad[slot] || nwin > kWin || nwin <= 0) {
      for (int32_t c = lane; c < 16 * nr; c += 64) out[c] = zero;
      if (!R.pbad[slot] && nwin > kWin && lane == 0) deep[atomicAdd(n_deep, 1ull)] = slot;
      continue;
    }
    const int64_t base = R.seq_off[W.ra];
    const uint8_t *pool = R.qual + base;
    const int64_t span = R.seq_cap - base;
    const uint16_t *prw = R.prow + R.soff[slot];
    for (int32_t i = lane; i < nwin; i += 64) {
      const int64_t r = W.ra + i;
      const ColDesc d = R.cdesc[r];
      const int32_t ld = R.lead[r];
      const int64_t so = R.seq_off[r];
      const uint32_t mq = R.mapq[r];
      const int64_t mo = R.md_off[r];
      const int64_t av = so + (ld > 0 ? ld : 0) - base;  // (off the window's byte run: the slow path)
      MCellRec m;
      m.a = R.pool_ordered && av >= 0 && av < (int64_t)kCell3Far ? (uint32_t)av : kCell3Far;
      m.s = d.start;
      m.e = d.end;
      m.info = d.info;
      m.mq = mq | (min_mapq > 0 && (int)mq < min_mapq ? 0x100u : 0u);
      const int32_t nmd = (int32_t)(d.info & 0xFFFFu);
      uint32_t v[4];
      bool in = nmd <= 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = q < nmd && in ? R.md_ev[mo + q] >> 8 : 0xFFFFu;
        in = in && v[q] <= 0xFFFFu && (q >= nmd || v[q] < 0xFFFFu);
      }
      m.ev01 = (v[0] & 0xFFFFu) | (v[1] << 16);
      m.ev23 = (v[2] & 0xFFFFu) | (v[3] << 16);
      if (!in) m.mq |= 0x200u;
      m.pad = 0;
      rec[i] = m;
    }
    bool none = false;
    for (int32_t k0 = 0; k0 < nr; k0 += kRows) {
      const int32_t nk = nr - k0 < kRows ? nr - k0 : kRows;
      for (int32_t c = lane; c < 16 * nk; c += 64) map[c] = 0xFFu;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      for (int32_t i = lane; i < nwin; i += 64) {
        const int32_t row = prw[i];
        int32_t s0, sl;
        piece_of(R.prec[W.ra + i], W.qc0, s0, sl);
        if (row == 0xFFFF || sl <= 0 || row < k0 || row >= k0 + nk) continue;
        uint8_t *mp = map + 16 * (row - k0) + (s0 - W.qc0);
        for (int32_t j = 0; j < sl; ++j) mp[j] = (uint8_t)i;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      uint2 *o = out + 16 * k0;
      for (int32_t c00 = 0; c00 < 16 * nk; c00 += 256) {  // four cells per lane, their loads together
        uint64_t q[4];
        uint32_t valid[4], evb[4], mqs[4];
        uint32_t slow = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int32_t c = c00 + 64 * u + lane;
          const uint32_t p = c < 16 * nk ? map[c] : 0xFFu;
          q[u] = 0;
          valid[u] = 0;
          evb[u] = 0;
          mqs[u] = lmq;
          if (p == 0xFFu) continue;
          const MCellRec m = rec[p];
          if (m.mq & 0x100u) continue;  // dropped by the mapq filter: no element
          const int32_t lb = 8 * (W.qc0 + (c & 15));
          const int64_t v = (int64_t)m.a + lb - m.s;
          if (!(m.info & kColEligible) || (m.mq & 0x200u) || m.a == kCell3Far || v < 0 || v + 8 > span) {
            slow |= 1u << u;
            continue;
          }
          const int32_t lo = min(max(m.s - lb, 0), 8), hi = min(max(m.e - lb, 0), 8);
          q[u] = *reinterpret_cast<const gq_u64m *>(pool + (uint32_t)v);
          if (lo > 0 || hi < 8) q[u] &= edge_mask(lo, hi);
          valid[u] = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
          const int32_t i0 = lb - m.s;
          uint32_t eb = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t off = ((k < 2 ? m.ev01 : m.ev23) >> (16 * (k & 1))) & 0xFFFFu;
            const uint32_t ii = (uint32_t)((int32_t)off - i0);
            eb |= (off != 0xFFFFu && ii < 8u) ? 1u << ii : 0u;
          }
          evb[u] = eb;
          mqs[u] = m.mq & 0xFFu;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int32_t c = c00 + 64 * u + lane;
          if (c >= 16 * nk || ((slow >> u) & 1u)) continue;
          uint2 w = zero;
          if (valid[u])
            w = mqs[u] == lmq ? margin_terms8_lds(q[u], valid[u], evb[u], lrow)
                              : margin_terms8_lds(q[u], valid[u], evb[u], tab + (mqs[u] << 8));
          o[c] = w;
          none = none || has_none(w);
        }
        if (slow) {  // rare: a general CIGAR, more than four MD events, a word at the pool's end
#pragma unroll 1
          for (int u = 0; u < 4; ++u) {
            if (!((slow >> u) & 1u)) continue;
            const int32_t c = c00 + 64 * u + lane;
            const uint32_t p = map[c];
            const MCellRec m = rec[p];
            const int64_t r = W.ra + p;
            const int32_t ld = R.lead[r];
            PieceMeta pm;
            pm.p0 = R.seq_off[r] + (ld > 0 ? ld : 0) - m.s;  // (from the read itself: any pool order)
            pm.s = m.s;
            pm.e = m.e;
            pm.s0 = 0;
            pm.row = 0;
            pm.info = m.info;
            pm.mq = m.mq & 0xFFu;
            const int32_t col = W.qc0 + (c & 15);
            const uint32_t eb = word_events(R, R.md_off[r], m.info, m.s, col);
            const MarginRaw x = margin_fetch(R, r, pm, col, eb, tab);
            const uint2 w = x.gen ? x.word : margin_terms8(pm, x.q, x.valid, eb, tab);
            o[c] = w;
            none = none || has_none(w);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();  // (the next chunk rewrites the map)
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    const bool any = __ballot(none) != 0;
    if (lane == 0) mnb[slot] = any ? 1 : 0;
  }
}

// The listed (deep) slices' margin words, slice-major (their rows preset to kMargin8Zero by
// mproj_fill_cells).
__global__ __launch_bounds__(256) void mproj_fill_deep(DevReads R, const int64_t *__restrict__ deep,
                                                       const unsigned long long *__restrict__ n_deep, int min_mapq,
                                                       const uint8_t *__restrict__ tab, uint8_t *__restrict__ mproj,
                                                       uint8_t *__restrict__ mnb) {
  __shared__ PieceMeta s_meta[4][64];
  __shared__ uint32_t s_owner[4][64];
  PieceMeta *meta = s_meta[threadIdx.x >> 6];
  uint32_t *owner = s_owner[threadIdx.x >> 6];
  const int64_t nd = (int64_t)*n_deep;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave_id(); i < nd; i += nw) {
    const int64_t slot = deep[i];
    uint2 *out = reinterpret_cast<uint2 *>(mproj) + 16 * R.srow[slot];
    bool none = false;
    slice_fill<true, 1>(
        R, slice_stored(R, slot), R.prow + R.soff[slot], meta, owner,
        [&](int64_t, PieceMeta &m, int64_t mdo) { return margin_setup(R, min_mapq, mdo, m); },
        [&](int64_t r, const PieceMeta &m, int32_t col, uint32_t evb) { return margin_fetch(R, r, m, col, evb, tab); },
        [&](bool act, const MarginRaw &x, int64_t, const PieceMeta &m, int32_t col, uint32_t evb) {
          if (act) {
            const uint2 w = x.gen ? x.word : margin_terms8(m, x.q, x.valid, evb, tab);
            out[16 * (int64_t)m.row + (col & 15)] = w;
            auto has = [](uint32_t v) { return ((v - 0x01010101u) & ~v & 0x80808080u) != 0u; };
            none = none || has(w.x) || has(w.y);
          }
        });
    const bool any = __ballot(none) != 0;
    if ((threadIdx.x & 63) == 0) mnb[slot] = any ? 1 : 0;
  }
}

// The tumor's margin projection (a biased byte per locus-read, 128 B per row) slice by slice
// (piece_fill in gq_host.h): a wave per slice, a lane per piece, the rows built in LDS and written
// whole (kMargin8Zero where no element of a kept read lies: no preset).  mnb[slot] = 1 where a
// word holds a kMargin8None term.
__global__ __launch_bounds__(256) void mproj_fill_pieces(DevReads R, int64_t n_slices, int min_mapq,
                                                         const uint8_t *__restrict__ tab, uint8_t *__restrict__ mproj,
                                                         uint8_t *__restrict__ mnb) {
  __shared__ uint2 s_rows[4][kPieceRows * kPieceStride];
  __shared__ uint32_t s_row[4][64];  // the table row of one mapping quality (256 bytes)
  const int wv = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const uint8_t *lrow = reinterpret_cast<const uint8_t *>(s_row[wv]);
  uint32_t lmq = 0;  // most reads share one mapping quality: its row (the wave's first slice's first read)
  {
    const int64_t slot = wave_id();
    if (slot < n_slices) {
      const int64_t ra = R.sra[slot];
      lmq = ra < R.n_reads ? (uint32_t)R.mapq[ra] : 0u;
    }
    s_row[wv][lane] = reinterpret_cast<const uint32_t *>(tab + (lmq << 8))[lane];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  const uint2 zero = make_uint2(0x80808080u, 0x80808080u);
  piece_fill<uint2, MarginCell, true>(
      R, n_slices, s_rows[wv], reinterpret_cast<uint2 *>(mproj), zero,
      [&](const PieceRec &m) { return !(min_mapq > 0 && (int)m.mq < min_mapq); },
      [&](const PieceRec &m, int32_t col, MarginCell &x) {
        const int32_t nmd = (int32_t)(m.info & 0xFFFFu);
        if (!(m.info & kColEligible) || nmd > 4) return false;
        const int32_t lb = 8 * col;
        const int64_t a = m.p0 + lb;
        if (a < 0 || a + 8 > R.seq_cap) return false;
        const int32_t lo = min(max(m.s - lb, 0), 8), hi = min(max(m.e - lb, 0), 8);
        x.q = *reinterpret_cast<const gq_u64m *>(R.qual + a) & edge_mask(lo, hi);
        x.valid = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
        const int32_t i0 = lb - m.s;
        uint32_t evb = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // (the piece's events came with its record)
          const uint32_t i = (uint32_t)((int32_t)(m.ev[k] >> 8) - i0);
          evb |= (m.ev[k] != 0xFFFFFFFFu && i < 8u) ? 1u << i : 0u;
        }
        x.evb = (uint16_t)evb;
        x.mq = (uint16_t)m.mq;
        return true;
      },
      [&](const PieceRec &, int32_t, const MarginCell &x) {  // terms from the LDS row or the mapq's global row
        return x.mq == lmq ? margin_terms8_lds(x.q, x.valid, x.evb, lrow)
                           : margin_terms8_lds(x.q, x.valid, x.evb, tab + ((uint32_t)x.mq << 8));
      },
      [&](const PieceRec &m, int64_t r, int32_t col) {
        const PieceMeta pm = piece_rec_meta(m);
        const uint32_t evb = word_events(R, m.md_off, m.info, m.s, col);
        const MarginRaw x = margin_fetch(R, r, pm, col, evb, tab);
        return x.gen ? x.word : margin_terms8(pm, x.q, x.valid, evb, tab);
      },
      [](uint2 w) {  // a kMargin8None (zero) byte
        auto z = [](uint32_t v) { return ((v - 0x01010101u) & ~v & 0x80808080u) != 0u; };
        return z(w.x) || z(w.y);
      },
      [&](int64_t slot, bool none) {
        if (lane == 0) mnb[slot] = none ? 1 : 0;
      });
}

// The projection and the margin projection of one read set in one read-major pass (the
// projection derived for a caller that also reads the margin projection): one batch setup per 64
// reads, each word's bases and qualities loaded together; margin words only for reads the mapq
// filter keeps (the others keep the pool's kMargin8Zero fill).
struct PmRaw {
  ProjRaw p;
  MarginRW m;
};
__global__ __launch_bounds__(256) void pm_fill_rw(DevReads R, uint8_t *__restrict__ proj, int min_mapq,
                                                  const uint8_t *__restrict__ tab, uint8_t *__restrict__ mproj,
                                                  uint8_t *__restrict__ mnb, int dbg) {
  __shared__ ReadMeta s_meta[4][64];
  __shared__ uint32_t s_owner[4][64];
  __shared__ uint32_t s_row[4][64];  // the table row of the batch's first read's mapq (256 bytes)
  uint32_t *row = s_row[threadIdx.x >> 6];
  const uint8_t *lrow = reinterpret_cast<const uint8_t *>(row);
  const int lane = threadIdx.x & 63;
  uint32_t lmq = 0;
  uint32_t *pout = reinterpret_cast<uint32_t *>(proj);
  uint2 *mout = reinterpret_cast<uint2 *>(mproj);
  auto kept = [=](const ReadMeta &m) { return !(min_mapq > 0 && (int)m.mq < min_mapq); };
  read_fill<1, true, 1>(
      R, s_meta[threadIdx.x >> 6], s_owner[threadIdx.x >> 6], dbg, nullptr,
      [&](int64_t r0) {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        lmq = (uint32_t)R.mapq[r0];
        row[lane] = reinterpret_cast<const uint32_t *>(tab + (lmq << 8))[lane];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      },
      [](const ReadMeta &) { return true; },
      [&](int64_t r, const ReadMeta &m, int32_t col, uint64_t, bool) {
        return PmRaw{proj_fetch(R, r, piece_meta(m), col), margin_fetch_rw(R, r, m, col, tab)};
      },
      [&](bool act, const PmRaw &o, int64_t, const ReadMeta &m, int32_t col, int64_t grow, int64_t slot) {
        if (act)
          pout[16 * grow + (col & 15)] =
              o.p.gen ? o.p.word : proj_codes4((uint32_t)o.p.b) | (proj_codes4((uint32_t)(o.p.b >> 32)) << 4);
        const bool mact = act && kept(m);
        const bool all_lds = __ballot(mact && !o.m.x.gen && m.mq != lmq) == 0;  // uniform
        if (mact) {
          const uint32_t evb = word_event_bits(m, col, o.m.v, o.m.evb);
          const uint2 w = o.m.x.gen ? o.m.x.word
                          : all_lds ? margin_terms8_lds(o.m.x.q, o.m.x.valid, evb, lrow)
                                    : margin_terms8(piece_meta(m), o.m.x.q, o.m.x.valid, evb, tab, lrow, lmq);
          mout[16 * grow + (col & 15)] = w;
          auto has = [](uint32_t v) {  // a zero byte
            return ((v - 0x01010101u) & ~v & 0x80808080u) != 0u;
          };
          if (has(w.x) || has(w.y)) mnb[slot] = 1;
        }
      });
}

struct SomProjCfg {
  static constexpr int kT = 512;
  static constexpr int kWaves = 4;
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kU = 4;
  static constexpr int kMaxRows = kSliceRowsMax;  // rows per block (16-bit counts past 240 rows)
  static constexpr int kEnt = 6;
};

__device__ __forceinline__ unsigned som_reserve_lds(unsigned *ctr, unsigned n) {  // every lane active
  const uint32_t x = wave_incl_scan(n);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  unsigned base = 0;
  if ((threadIdx.x & 63) == 63 && total) base = atomicAdd(ctr, total);
  base = (unsigned)__builtin_amdgcn_readlane((int)base, 63);
  return base + x - n;
}

typedef short gq_short2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t add_sat2(uint32_t a, uint32_t b) {  // v_pk_add_i16 clamp
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(__builtin_bit_cast(gq_short2, a),
                                                                     __builtin_bit_cast(gq_short2, b)));
}

// A reference genome in HBM (gq_reference): contig c's base at locus l is b[off[c] + l]; each
// contig starts on a 512-byte boundary and is padded past its end to the next 512-locus block.
// b == nullptr: no reference, the pileup's base is the reads' MD-derived one.
struct RefView {
  const uint8_t *b;
  const int64_t *off;
};

// With a reference (DistributedUtil.scala:266-267) the MD-derived candidate test stands where the
// reference base is the one the reads' MD gives (the same pileup reference base); anywhere else
// the locus is a candidate and somatic_call decides it with the reference base.
__device__ __forceinline__ bool ref_agrees(uint32_t md_mask, uint32_t base) {
  const uint32_t bit = std_bit((uint8_t)base);
  return bit ? md_mask == bit : (md_mask == 0 && base == 'N');
}

template <bool kRef>
__global__ __launch_bounds__(SomProjCfg::kThreads) __attribute__((amdgpu_waves_per_eu(4))) void somatic_proj(
    const Tile *__restrict__ tiles_t, const Tile *__restrict__ tiles_n, int64_t n_tiles, DevReads RT,
    const uint8_t *__restrict__ mproj, const uint8_t *__restrict__ mnb, const int32_t *__restrict__ n_start,
    const int32_t *__restrict__ n_end,
    ComplexItem *__restrict__ cand, OutGeom og, Counters *ctr, int32_t *__restrict__ slow, RefView ref,
    int no_bound = 0) {
  using C = SomProjCfg;
  constexpr int T = C::kT, U = C::kU;
  // per locus: tumor event read bases (A | C << 16 at [i], T | G << 16 at [T + i]); MD bits
  // 0-3 | N << 4 | complex diff << 16
  __shared__ __attribute__((aligned(16))) uint32_t evw[C::kWaves][2 * T];
  __shared__ __attribute__((aligned(16))) uint32_t mkw[C::kWaves][T];
  __shared__ __attribute__((aligned(16))) uint32_t cvw[C::kWaves][T];  // normal coverage differences
  __shared__ unsigned outn[2];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint32_t *ev = evw[wave], *mk = mkw[wave], *cv = cvw[wave];
  {
    uint4 *e4 = reinterpret_cast<uint4 *>(ev + 8 * lane), *f4 = reinterpret_cast<uint4 *>(ev + T + 8 * lane), *m4 = reinterpret_cast<uint4 *>(mk + 8 * lane),
          *c4 = reinterpret_cast<uint4 *>(cv + 8 * lane);
    {  // separate stores (a chained assignment re-reads each word from LDS)
      const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
      e4[0] = z4; e4[1] = z4; f4[0] = z4; f4[1] = z4; m4[0] = z4; m4[1] = z4; c4[0] = z4; c4[1] = z4;
    }
  }
  if (threadIdx.x < 2) outn[threadIdx.x] = 0;
  __syncthreads();
  const int64_t per = n_tiles / gridDim.x, extra = n_tiles % gridDim.x;
  const int64_t i0 = blockIdx.x * per + min((int64_t)blockIdx.x, extra);
  const int64_t i1 = i0 + per + ((int64_t)blockIdx.x < extra ? 1 : 0);
  const unsigned long long cbase = og.slot(1, (int)blockIdx.x, 0), ccap = og.capA[1];
  unsigned visited = 0;
  for (int64_t i = i0 + wave; i < i1; i += C::kWaves) {
    const Tile tt = tiles_t[i], tn = tiles_n[i];
    const int32_t L0 = tt.L0, L1 = tt.L1;
    const int64_t rb = tt.rb, re = tt.re;
    const int32_t B0 = L0 & ~(T - 1), C0 = B0 >> 3;
    if ((tn.re - tn.rb) >= 65535) {
      if (lane == 0) slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)i;
      continue;
    }
    // ---- tumor: the block's projection rows (ProjRec) and the first sparse entries.  The
    // block exists only where tumor reads reach it (a tile may hold normal reads alone, past
    // the tumor's last read).  A pbad slice (a read the projection cannot take) or more than
    // kMaxRows rows (byte counters): somatic_tile.
    const bool tumor = re > rb;
    const int64_t qs = tumor ? tt.qs : 0;  // qoff[contig] + (B0 >> 7), from the plan
    const int64_t row0 = tumor ? RT.srow[qs] : 0;
    const int32_t g = lane >> 4;
    // this group's slice: its first row (from the block's first) and its rows; the loop runs to
    // the block's fullest slice
    const int32_t gbase = tumor ? (int32_t)(RT.srow[qs + g] - row0) : 0;
    const int32_t gn = tumor ? (int32_t)(RT.srow[qs + g + 1] - RT.srow[qs + g]) : 0;
    const int32_t ntot = tumor ? (int32_t)(RT.srow[qs + 4] - row0) : 0;
    int32_t nrows = gn;
#pragma unroll
    for (int d = 16; d < 64; d <<= 1) nrows = max(nrows, __shfl_xor(nrows, d, 64));
    const uint32_t bad4 = tumor ? *reinterpret_cast<const uint32_t *>(RT.pbad + qs) : 0u;
    const bool nb = tumor && *reinterpret_cast<const uint32_t *>(mnb + qs) != 0u;  // a slice without bounds
    const int64_t e0 = RT.pev_off[rb], e1 = RT.pev_off[re];
    constexpr int NE = C::kEnt;
    uint2 ent[NE];
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int64_t k = e0 + 64 * j + lane;
      ent[j] = make_uint2(0x80000000u, kPevNone);
      if (k < e1) ent[j] = RT.pev[k];
    }
    if (bad4 != 0 || nrows > C::kMaxRows) {
      if (lane == 0) slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)i;
      continue;
    }
    // ---- tumor column counts (bytes, widened into 16-bit pairs every 240 rows and at the end)
    //      and margin sums (the biased byte terms zero-extended into 16-bit pairs, loci 2k,
    //      2k + 1 in msum[k]: 240 rows of bytes fit, folded into 32 bits per locus with the
    //      counts): row k of each group's slice is one 64-byte load of base codes and one
    //      128-byte load of margin terms (past the slice's rows: out-of-range offsets, 0 — the
    //      bias is taken off for the group's own rows only)
    uint32_t ca[2] = {0, 0}, cc[2] = {0, 0}, ct[2] = {0, 0}, cg[2] = {0, 0};
    uint32_t wA[4] = {0, 0, 0, 0}, wC[4] = {0, 0, 0, 0}, wT[4] = {0, 0, 0, 0}, wG[4] = {0, 0, 0, 0};
    int32_t m32[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t msum[4] = {0, 0, 0, 0};
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(RT.proj + kProjRowBytes * row0), (short)0, kProjRowBytes * ntot, 0x00020000);
    const __amdgpu_buffer_rsrc_t msrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(mproj + 128 * row0), (short)0, 128 * ntot, 0x00020000);
    const uint32_t vl = 4u * (uint32_t)(lane & 15) + (uint32_t)kProjRowBytes * (uint32_t)gbase;
    uint32_t nac[2] = {0, 0}, ntg[2] = {0, 0};
    int nn = 0;
    auto fold = [&]() {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        ca[h] += nac[h] & 0x0F0F0F0Fu;
        cc[h] += (nac[h] >> 4) & 0x0F0F0F0Fu;
        ct[h] += ntg[h] & 0x0F0F0F0Fu;
        cg[h] += (ntg[h] >> 4) & 0x0F0F0F0Fu;
        nac[h] = ntg[h] = 0;
      }
      nn = 0;
    };
    auto widen = [&]() {
      auto w2 = [](uint32_t (&w)[4], uint32_t (&c)[2]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          w[2 * h] += __builtin_amdgcn_perm(0u, c[h], 0x0c010c00u);  // bytes 0, 1 -> halves
          w[2 * h + 1] += __builtin_amdgcn_perm(0u, c[h], 0x0c030c02u);
          c[h] = 0;
        }
      };
      w2(wA, ca);
      w2(wC, cc);
      w2(wT, ct);
      w2(wG, cg);
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // margin pairs into 32 bits per locus
        m32[2 * q] += (int32_t)(msum[q] & 0xFFFFu);
        m32[2 * q + 1] += (int32_t)(msum[q] >> 16);
        msum[q] = 0;
      }
    };
    auto issue = [&](int k0, uint32_t (&w)[U], uint2 (&m)[U]) {  // rows k0 .. k0 + U - 1
      const uint32_t va = vl + (uint32_t)kProjRowBytes * (uint32_t)k0;
      const int32_t rem = gn - k0;  // this group's rows left
      const uint32_t vm = 2u * va;  // 8 bytes of margin terms per 4-byte word of codes
#pragma unroll
      for (int u = 0; u < U; ++u) {  // past the slice's rows: out-of-range lane offsets
        const bool ok = u < rem;
        w[u] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)(ok ? va : 0x80000000u), kProjRowBytes * u, 0);
        const auto b = __builtin_amdgcn_raw_buffer_load_b64(msrc, (int)(ok ? vm : 0x80000000u), 128 * u, 0);
        m[u] = make_uint2(b[0], b[1]);
      }
    };
    auto count = [&](const uint32_t (&w)[U], const uint2 (&m)[U]) {
      if (nn + U > 15) fold();
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t lo = w[u] & 0x0F0F0F0Fu, hi = (w[u] >> 4) & 0x0F0F0F0Fu;  // loci 0-3, 4-7
        nac[0] += __builtin_amdgcn_perm(0u, 0x10000100u, lo);
        ntg[0] += __builtin_amdgcn_perm(0x10000001u, 0u, lo);
        nac[1] += __builtin_amdgcn_perm(0u, 0x10000100u, hi);
        ntg[1] += __builtin_amdgcn_perm(0x10000001u, 0u, hi);
        msum[0] += __builtin_amdgcn_perm(0u, m[u].x, 0x0c010c00u);  // loci 0, 1 (biased bytes -> halves)
        msum[1] += __builtin_amdgcn_perm(0u, m[u].x, 0x0c030c02u);  // loci 2, 3
        msum[2] += __builtin_amdgcn_perm(0u, m[u].y, 0x0c010c00u);
        msum[3] += __builtin_amdgcn_perm(0u, m[u].y, 0x0c030c02u);
      }
      nn += U;
    };
    uint32_t aw[U], bw[U];
    uint2 am[U], bm[U];
    issue(0, aw, am);
    // ---- tumor sparse entries, one lane per entry (germline_proj's encoding)
    auto apply = [&](uint2 p) {
      const int32_t l = (int32_t)p.x;
      if (p.y & kPevComplex) {
        const int64_t a = max((int64_t)l, (int64_t)B0);
        const int64_t b = min((int64_t)l + (int64_t)(p.y & kPevLenMask), (int64_t)B0 + T);  // mid-deletions too
        if (a < b) {
          atomicAdd(&mk[a - B0], 1u << 16);
          if (b < (int64_t)B0 + T) atomicAdd(&mk[b - B0], 0xFFFF0000u);
        }
      } else if (l >= B0 && l < B0 + T) {
        const uint32_t mm = p.y & 15u, c = (p.y >> 4) & 7u;
        if (mm) atomicOr(&mk[l - B0], mm);
        if (c < 4) atomicAdd(&ev[(c >> 1) * T + (l - B0)], 1u << (16 * (c & 1)));
        else if (c == 4) atomicAdd(&mk[l - B0], 1u << 4);
      }
    };
#pragma unroll
    for (int j = 0; j < NE; ++j) apply(ent[j]);
    for (int64_t q = e0 + 64 * NE; q < e1; q += 64) {
      const int64_t k = q + lane;
      if (k < e1) apply(RT.pev[k]);
    }
    // ---- normal depth: each read spans [start, end) (any element), as +1 / -1 differences
    for (int64_t q = tn.rb; q < tn.re; q += 64) {
      const int64_t r = q + lane;
      if (r < tn.re) {
        const int32_t a = max(n_start[r], B0), b = min(n_end[r], B0 + T);
        if (a < b) {
          atomicAdd(&cv[a - B0], 1u);
          if (b < B0 + T) atomicAdd(&cv[b - B0], 0xFFFFFFFFu);
        }
      }
    }
    for (int k0 = 0, since = 0;; k0 += 2 * U) {  // rows past the block's read 0 (out of the buffers' range)
      issue(k0 + U, bw, bm);
      count(aw, am);
      issue(k0 + 2 * U, aw, am);
      count(bw, bm);
      if (k0 + 2 * U >= nrows) break;
      since += 2 * U;
      if (since == 240) {  // uniform: bytes hold 240 rows at most
        fold();
        widen();
        since = 0;
      }
    }
    fold();
    widen();
#pragma unroll
    for (int j = 0; j < 8; ++j) m32[j] -= 128 * gn;  // the bias of the group's own rows
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ---- decision: candidate loci (somatic_tile's test)
    uint4 *e4 = reinterpret_cast<uint4 *>(ev + 8 * lane), *f4 = reinterpret_cast<uint4 *>(ev + T + 8 * lane), *m4 = reinterpret_cast<uint4 *>(mk + 8 * lane),
          *c4 = reinterpret_cast<uint4 *>(cv + 8 * lane);
    uint32_t e16[16], m8[8], v8[8];
    {
      const uint4 ea = e4[0], eb = e4[1], ec = f4[0], ed = f4[1], ma = m4[0], mb = m4[1], va = c4[0], vb = c4[1];
      e16[0] = ea.x, e16[1] = ea.y, e16[2] = ea.z, e16[3] = ea.w, e16[4] = eb.x, e16[5] = eb.y, e16[6] = eb.z;
      e16[7] = eb.w, e16[8] = ec.x, e16[9] = ec.y, e16[10] = ec.z, e16[11] = ec.w, e16[12] = ed.x, e16[13] = ed.y;
      e16[14] = ed.z, e16[15] = ed.w;
      m8[0] = ma.x, m8[1] = ma.y, m8[2] = ma.z, m8[3] = ma.w, m8[4] = mb.x, m8[5] = mb.y, m8[6] = mb.z, m8[7] = mb.w;
      v8[0] = va.x, v8[1] = va.y, v8[2] = va.z, v8[3] = va.w, v8[4] = vb.x, v8[5] = vb.y, v8[6] = vb.z, v8[7] = vb.w;
      {  // separate stores (a chained assignment re-reads each word from LDS)
        const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
        e4[0] = z4; e4[1] = z4; f4[0] = z4; f4[1] = z4; m4[0] = z4; m4[1] = z4; c4[0] = z4; c4[1] = z4;
      }
    }
    int32_t run_c = 0, run_n = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      run_c += (int32_t)m8[j] >> 16;
      run_n += (int32_t)v8[j];
    }
    int32_t ncx_run = (int32_t)wave_incl_scan((uint32_t)run_c) - run_c;
    int32_t dn_run = (int32_t)wave_incl_scan((uint32_t)run_n) - run_n;
    uint32_t qmask = 0, nq = 0;
    uint2 fb8 = make_uint2(0u, 0u);  // the reference bases of this lane's 8 loci
    if constexpr (kRef) fb8 = *reinterpret_cast<const uint2 *>(ref.b + ref.off[tt.contig] + B0 + 8 * lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int32_t l = B0 + 8 * lane + j;
      const bool in = l >= L0 && l < L1;
      const int q2 = j >> 1, sh = 16 * (j & 1);
      const uint32_t cA = (wA[q2] >> sh) & 0xFFFFu, cC = (wC[q2] >> sh) & 0xFFFFu;
      const uint32_t cT = (wT[q2] >> sh) & 0xFFFFu, cG = (wG[q2] >> sh) & 0xFFFFu;
      const uint32_t nN = (m8[j] >> 4) & 0xFFFu;
      ncx_run += (int32_t)m8[j] >> 16;
      dn_run += (int32_t)v8[j];
      const uint32_t ncx = ncx_run > 0 ? (uint32_t)ncx_run : 0u;
      const uint32_t depth = cA + cC + cT + cG + nN + ncx;
      const uint32_t eac = e16[j], etg = e16[8 + j];
      const uint32_t mask = (m8[j] & 15u) | (cA > (eac & 0xFFFFu) ? 1u : 0u) | (cC > (eac >> 16) ? 2u : 0u) |
                            (cT > (etg & 0xFFFFu) ? 4u : 0u) | (cG > (etg >> 16) ? 8u : 0u);
      const uint32_t low = mask & (0u - mask);
      const uint32_t c_ref = (cA & (0u - (low & 1u))) + (cC & (0u - ((low >> 1) & 1u))) +
                             (cT & (0u - ((low >> 2) & 1u))) + (cG & (0u - ((low >> 3) & 1u))) + (low == 0u ? nN : 0u);
      bool agree = true;
      if constexpr (kRef) agree = ref_agrees(mask, ((j < 4 ? fb8.x : fb8.y) >> (8 * (j & 3))) & 0xFFu);
      const bool single = mask != 0 && (mask & (mask - 1u)) == 0;
      const bool nonmatch = !agree || (mask & (mask - 1u)) != 0 || ncx > 0 || depth > c_ref;
      const bool bound = !no_bound && !nb && agree && single && ncx == 0 && nN == 0 &&
                         (float)m32[j] * 0.125f > 0.02f + 2e-4f * (float)depth;
      const bool tcand = depth > 0 && nonmatch && !bound;
      visited += (in && (depth > 0 || dn_run > 0)) ? 1u : 0u;
      const bool q = in && tcand && dn_run > 0;
      qmask |= q ? 1u << j : 0u;
      nq += q ? 1u : 0u;
    }
    if (__ballot(qmask != 0) != 0) {
      unsigned kq = som_reserve_lds(&outn[1], nq);
      for (int j = 0; j < 8; ++j)
        if ((qmask >> j) & 1u) {
          if (kq < ccap) cand[cbase + kq] = ComplexItem{(int32_t)i, B0 + 8 * lane + j, 0};
          ++kq;
        }
    }
  }
  // visited loci into the spread counters, this workgroup's candidate count
  __shared__ unsigned red;
  if (threadIdx.x == 0) red = 0;
  __syncthreads();
  if (visited) atomicAdd(&red, visited);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (red) atomicAdd(&ctr->spread[0][blockIdx.x & (kSpread - 1)], (unsigned long long)red);
    ctr->part[1][blockIdx.x] = outn[1];
  }
}
