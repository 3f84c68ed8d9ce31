// gq_kernels.h — device-side building blocks shared by the pileup kernels.
//
// Element semantics restate PileupElement.alignment / advanceToLocus
// (/root/reference/src/main/scala/org/hammerlab/guacamole/pileup/PileupElement.scala:68-248)
// and Pileup.referenceBaseAtLocus (pileup/Pileup.scala:157-165).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

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
  int64_t cigar_len, md_len;  // pool sizes (upload-time bounds checks)
  // derived at upload (read_shape):
  const int16_t *lead;   // leading soft clip of a [S|H]*(M|=|X)[S|H]* CIGAR, -1 otherwise
  const uint8_t *ev_rb;  // per MD event: the read's sequenced base at that position (0 for deletions)
  const uint8_t *clean;  // 1 if every sequenced byte of the read is one of A C G T N
  int32_t pool_ordered;  // reads' sequence bytes are disjoint and in read order in the pool
  // derived at upload for the germline column kernel (LDS-DMA'd per tile, see ColDesc)
  const struct ColDesc *cdesc;  // one per read
  const uint32_t *cev;          // per read: MD events (offset << 16 | MD base << 8 | read base), segments
  const int64_t *caux_off;      // n_reads + 1 offsets into cev
  // derived at upload for the projection kernels (germline_proj / somatic_proj, see ProjRec)
  const struct ProjRec *prec;   // n_reads + 1 (the last: a zero record)
  const uint8_t *proj;          // base codes, 8 loci (4 bits each) per word, in slice rows (see ProjRec)
  const int64_t *qoff;          // n_contigs + 1: each contig's first slice (slice = 128 loci)
  const int64_t *srow;          // qoff[n_contigs] + 1: each slice's first row in proj
  const uint2 *pev;             // per read: its sparse entries (MD events, N bases, complex ranges)
  const int64_t *pev_off;       // n_reads + 1 offsets into pev
  const uint8_t *pbad;          // per slice: 1 if a read the projection cannot take overlaps it
  const int64_t *sra;           // per slice: the first read of its window (slice_window)
  const int64_t *soff;          // per slice + 1: offsets of its window's reads' rows in prow
  const uint16_t *prow;         // per (slice, window read): the read's row there, 0xFFFF: no piece
  // derived at upload for plan_tiles: per 512-locus block g (qoff[c] / 4 + block in contig c),
  // the first read with pmax_end > the block's first locus and the first read starting at or
  // after it (a block index of the reads, so aligned tiles need no search over the contig)
  const int64_t *blk_rb, *blk_rs;
  // Scala String.hashCode of each sample slot's name (gq_reads.sample_hash; nullptr: slot order)
  const uint32_t *sample_hash;
};

// Per-read record of the projection kernels (8 bytes): the read spans the 8-locus columns
// [col0, col1).  Its projection holds four bits per locus, the read's base there as a code
// (A 1, C 3, T 4, G 7: ASCII & 7) where the element is a Match/Mismatch
// (PileupElement.scala:68-135), 0 elsewhere (outside the read, deleted / skipped loci,
// insertion and deletion anchors, N bases).  A column's word is 32 bits: byte j holds locus j
// in its low nibble and locus 4 + j in its high nibble.  A PIECE is one read's run of columns
// inside one 128-locus slice (16 columns).  The pool is in SLICE ROWS: slice q owns rows
// [srow[q], srow[q + 1]) of 16 words (kProjRowBytes = 64 bytes), word c of a row = column c of
// the slice.  The slice's
// pieces are packed into its rows by greedy interval partitioning in read order (a piece takes
// the first row that is free from its first column: as few rows as the slice's deepest column
// holds reads); the words no piece covers are zero.  So the 16 lanes that own a slice read row
// k with one 128-byte load (lane l16: word l16), and the rows are fewer than the pieces (a read
// ending in a slice shares a row with one starting there).  col1 =
// kProjNone marks a read the projection path cannot take (bases other than A C G T N, no MD
// tag, a P op ...); it has no words.
struct ProjRec {
  int32_t col0, col1;
};
static_assert(sizeof(ProjRec) == 8, "ProjRec layout");
constexpr int32_t kProjNone = (int32_t)0x80000000;
constexpr int kProjRowBytes = 64;  // a slice row: 16 columns x 8 loci x 4 bits
// A slice's rows are padded with zero rows to a multiple of kRowPad (row_count), so
// germline_proj bounds its row batches (kRowPad rows) once per batch, not once per row.
constexpr int kRowPad = 4;
// Sparse entries of a read (uint2 {x = locus, y}), in any order:
//   y bit 31 clear: MD event / N base at locus x: bits 0-3 the MD reference base's std_bit
//     (0 for an N base without an MD event), bits 4-6 the read base's category there (0-3 A C
//     T G: a Match/Mismatch element carrying an MD event; 4: an N base; 7: none, e.g. an event
//     on a deleted base);
//   y bit 31 set: loci [x, x + (y & kPevLenMask)) hold complex elements (insertion / deletion
//     anchors, mid-deletions, clipped N-skips): the exact kernel decides them;
//   y bits 31 and 30 set: loci [x, x + (y & kPevLenMask)) hold MidDeletion elements of one D
//     op whose MD deleted bases are all A/C/G/T (Alignment.scala:87-92: allele (MD base, "")).
//     germline_proj counts them as one more allele; the other kernels treat them as complex.
constexpr int32_t kSliceRowsMax = 2048;  // rows of one slice (its deepest column); deeper: pbad
constexpr uint32_t kPevComplex = 0x80000000u;
constexpr uint32_t kPevMidDel = 0x40000000u;
constexpr uint32_t kPevLenMask = 0x3FFFFFFFu;
constexpr uint32_t kPevNone = 7u << 4;  // a padding entry (no effect)

// Packed per-read record of the germline column kernel (24 bytes, DMA'd into LDS per tile).
struct ColDesc {
  int32_t start, end, pmax_end;
  uint32_t info;    // bits 0-15 n_md; bit 16 column-eligible: a single (M|=|X) block, A/C/G/T/N
                    // bases, MD present, span < 32768, n_md < 65536; bit 17 general: another CIGAR
                    // as segments (validated at upload), their number in bits 18-25
  uint32_t seq_lo;  // low 32 bits of the pool offset of the base at `start` (seq_off + leading clip;
                    // seq_off for a general read)
  uint32_t md_lo;   // low 32 bits of the read's offset in the auxiliary list (cev)
};
static_assert(sizeof(ColDesc) == 24, "ColDesc layout");
constexpr uint32_t kColEligible = 1u << 16;
constexpr uint32_t kColGeneral = 1u << 17;

// One locus tile: contiguous loci [L0, L1) of one contig, plus the index range
// [rb, re) of reads that can overlap it (pmax_end > L0, start < L1).
struct Tile {
  int64_t ordinal0;  // output ordinal of L0 (position in the concatenated loci ranges)
  int64_t rb, re;
  int32_t contig, L0, L1, range;
  int64_t sb0;     // germline column kernel: 16-aligned pool offset of the tile's sequence bytes
  int32_t sbytes;  // bytes to stage from sb0 when the whole read window fits one LDS stage, else 0
  int32_t mcnt;    // auxiliary-list words (MD events, segments) to stage from mb0
  union {
    int64_t mb0;  // germline column kernel: first auxiliary word to stage (a multiple of 4)
    int64_t qs;   // aligned (projection) tiles: the block's first slice, qoff[contig] + (block >> 7)
  };
};
static_assert(sizeof(Tile) == 64, "Tile layout");

// Setup record of an aligned projection tile (plan_tiles, beside its Tile): the row and
// sparse-entry offsets germline_proj would otherwise load in two dependent rounds per tile.
// germline_proj holds the next tile's Tile + TileX in one VGPR (a dword per lane 0-31) while it
// counts the current one.
struct TileX {
  int64_t row0;       // srow[qs]: the block's first projection row (its first slice's)
  int32_t nr[4];      // rows of slice qs + g
  uint32_t pbad4;     // byte g: pbad[qs + g]
  uint32_t pad0;
  int64_t e0, e1;     // pev_off[rb], pev_off[re]: the window's sparse entries
  int64_t pad[2];
};
static_assert(sizeof(TileX) == 64, "TileX layout");

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
// CallRec.flags of a germline variant candidate (counts in allele / ref_len, expanded by
// germline_expand) and of the second slot reserved with it
constexpr uint8_t kCandidate = 0xC0, kCandidateSlot = 0xC1;

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
  if (n <= 4) {  // the common read: its few events in one round of loads (no dependent search)
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = k < n ? ev[k] : 0xFFFFFFFFu;
    int r = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (r < 0 && k < n && (int32_t)(v[k] >> 8) == off) r = (int)(v[k] & 0xFFu);  // (the first, as the search)
    return r;
  }
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

// Match/Mismatch elements of one read over the loci [a, b) whose sequenced bytes start at
// global byte p0 (locus a): 16-byte aligned chunks, kChunkGroup loads issued before the
// first is used (one memory latency per group); each dword goes to
// sink.bases4(i, word, valid4) with no branch (bytes outside the run carry valid = 0 and
// add nothing; i may fall in the sink's guard band).
template <class Sink>
__device__ __forceinline__ void bases_run(const DevReads &R, int32_t a, int32_t b, int64_t p0, int32_t L0, uint8_t fl,
                                          Sink &sink, const StageView &sv, bool clean = false) {
  if (b <= a) return;
  const int64_t p1 = p0 + (b - a);
  const int64_t cb0 = p0 & ~(int64_t)15;
  const int nchunks = (int)((p1 - cb0 + 15) >> 4);
  const int32_t ioff = (a - L0) - (int32_t)(p0 - cb0);  // tile index of byte cb0
  const int64_t cend = cb0 + 16 * (int64_t)nchunks;
  constexpr int kChunkGroup = 6;
  auto run = [&](auto ld, auto clean_tag) {  // ld(q): chunk q, clamped to the last chunk (every load in bounds)
    constexpr bool CLEAN = decltype(clean_tag)::value;
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
          if (CLEAN) {  // A C G T N only (checked once per read at upload): no category checks
            sink.bases4_clean(ib, c[u].x, vm & 15u, fl);
            sink.bases4_clean(ib + 4, c[u].y, (vm >> 4) & 15u, fl);
            sink.bases4_clean(ib + 8, c[u].z, (vm >> 8) & 15u, fl);
            sink.bases4_clean(ib + 12, c[u].w, (vm >> 12) & 15u, fl);
          } else {
            sink.bases4(ib, c[u].x, vm & 15u, fl);
            sink.bases4(ib + 4, c[u].y, (vm >> 4) & 15u, fl);
            sink.bases4(ib + 8, c[u].z, (vm >> 8) & 15u, fl);
            sink.bases4(ib + 12, c[u].w, (vm >> 12) & 15u, fl);
          }
        }
      }
    }
  };
  // the clean / checked choice is per read (a wave pays for both only where its lanes' reads differ)
  auto run2 = [&](auto ld) {
    if (clean) run(ld, std::true_type{});
    else run(ld, std::false_type{});
  };
  if (cb0 >= sv.b0 && cend <= sv.b1) {  // staged in LDS
    const uint4 *base = sv.lds + ((cb0 - sv.b0) >> 4);
    run2([&](int q) -> uint4 { return base[q < nchunks ? q : nchunks - 1]; });
  } else if (cend > R.seq_cap) {  // last read of an unpadded pool: byte loads
    for (int64_t p = p0; p < p1; ++p) {
      const int32_t i = ioff + (int32_t)(p - cb0);
      const int32_t sh = (int32_t)((p - cb0) & 3) * 8;
      sink.bases4(i - (sh >> 3), (uint32_t)R.seq[p] << sh, 1u << (sh >> 3), fl);
    }
  } else {
    const uint4 *base = reinterpret_cast<const uint4 *>(R.seq + cb0);
    run2([&](int q) -> uint4 { return base[q < nchunks ? q : nchunks - 1]; });
  }
}

// MD events of a read (reference offsets relative to its start s) at loci [lo, hi) of one
// Match/Mismatch run: sink.event_i(i, read base, MD reference base).  The read base is the
// derived ev_rb where the read set has it (ensure_ev_bases), else the run's own sequenced base:
// seq[boff + l] for an event at locus l < rend (0 past the sequence, as ev_rb).  Events past the
// first four are loaded four at a time (all issued before use).
template <class Sink>
__device__ __forceinline__ void events_run(const uint32_t *ev, const uint8_t *evb, uint4 e4, uint4 b4, int32_t nmd,
                                           int32_t s, int32_t lo, int32_t hi, int32_t L0, uint8_t fl, Sink &sink,
                                           const uint8_t *seq, int64_t boff, int32_t rend) {
  bool done = false;
  for (int k0 = 0; k0 < nmd && !done; k0 += 4) {
    uint32_t v4[4], r4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u;
      const uint32_t ef = u == 0 ? e4.x : u == 1 ? e4.y : u == 2 ? e4.z : e4.w;
      const uint32_t bf = u == 0 ? b4.x : u == 1 ? b4.y : u == 2 ? b4.z : b4.w;
      v4[u] = k0 == 0 ? ef : (k < nmd ? ev[k] : 0xFFFFFFFFu);
      r4[u] = evb ? (k0 == 0 ? bf : (k < nmd ? evb[k] : 0u)) : 0u;
    }
    if (!evb) {  // the bases of this run's events, from the pool
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int32_t l = s + (int32_t)(v4[u] >> 8);
        if (k0 + u < nmd && l >= lo && l < hi && l < rend) r4[u] = seq[boff + l];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (done || k0 + u >= nmd) continue;
      const int32_t l = s + (int32_t)(v4[u] >> 8);
      if (l < lo) continue;
      if (l >= hi) {
        done = true;
        continue;
      }
      sink.event_i(l - L0, (uint8_t)r4[u], (uint8_t)(v4[u] & 0xFFu), fl);
    }
  }
}

// Per-lane walk of one read over the loci [L0, L1): every lane owns one read (64 reads in
// flight per wave).  Match/Mismatch runs go through bases_run + events_run; the other
// elements (PileupElement.scala:68-135) go to sink.elem(l, kind, base, mdb, ev, flags)
// with the read's MD-derived reference base mdb at l (MDTagUtils.getReference).
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
  const int64_t md_off = R.md_off[r];
  const int64_t seq_off = R.seq_off[r];
  const uint8_t fl = R.flags[r];
  const int32_t lead = R.lead[r];
  const bool clean = R.clean && R.clean[r] != 0;  // (no column records: the checked path)
  const uint32_t *ev = R.md_ev + md_off;
  // first four MD events and (ev_rb derived) the read bases under them, loaded with the metadata
  const uint8_t *evb = R.ev_rb ? R.ev_rb + md_off : nullptr;
  uint4 e4, b4 = make_uint4(0u, 0u, 0u, 0u);
  e4.x = 0 < nmd ? ev[0] : 0xFFFFFFFFu;
  e4.y = 1 < nmd ? ev[1] : 0xFFFFFFFFu;
  e4.z = 2 < nmd ? ev[2] : 0xFFFFFFFFu;
  e4.w = 3 < nmd ? ev[3] : 0xFFFFFFFFu;
  if (evb) {
    b4.x = 0 < nmd ? evb[0] : 0u;
    b4.y = 1 < nmd ? evb[1] : 0u;
    b4.z = 2 < nmd ? evb[2] : 0u;
    b4.w = 3 < nmd ? evb[3] : 0u;
  }
  const int32_t a = s > L0 ? s : L0;
  const int32_t b = e < L1 ? e : L1;
  if (lead >= 0) {  // [S|H]* (M|=|X) [S|H]*: every element is a Match/Mismatch
    bases_run(R, a, b, seq_off + lead + (a - s), L0, fl, sink, sv, clean);
    events_run(ev, evb, e4, b4, nmd, s, a, b, L0, fl, sink, R.seq, seq_off + lead - s, e);
    return;
  }
  // general CIGAR: operator by operator
  const int64_t cig_off = R.cigar_off[r];
  const int32_t ncig = R.n_cigar[r];
  const int32_t slen = R.seq_len[r];
  auto md_at = [&](int32_t l) -> int {  // MD event at locus l: base, or -1
    const int32_t off = l - s;
    for (int k = 0; k < nmd; ++k) {
      const uint32_t v = k < 4 ? (k == 0 ? e4.x : k == 1 ? e4.y : k == 2 ? e4.z : e4.w) : ev[k];
      const int32_t o = (int32_t)(v >> 8);
      if (o == off) return (int)(v & 0xFFu);
      if (o > off) break;
    }
    return -1;
  };
  int32_t ref = s, rpos = 0;
  bool lead_ins = false;  // I before any reference-consuming op on a read at locus 0 (PileupElement.scala:102-103, 240-245)
  bool seen_ref = false;
  uint32_t cc = ncig > 0 ? R.cigar[cig_off] : 0u;
  for (int k = 0; k < ncig; ++k) {
    const int op = (int)(cc & 15u);
    const int32_t len = (int32_t)(cc >> 4);
    const uint32_t cn = (k + 1 < ncig) ? R.cigar[cig_off + k + 1] : 0u;
    const int nextop = (k + 1 < ncig) ? (int)(cn & 15u) : -1;
    if (op == OP_I && !seen_ref && s == 0) lead_ins = true;
    if (op == OP_P) sink.error(1 /*GQ_E_ASSERT*/, (int64_t)ref);
    if (consumes_ref(op)) {
      seen_ref = true;
      const int32_t ra = ref, rb = ref + len;
      const int32_t xa = ra > L0 ? ra : L0, xb = rb < L1 ? rb : L1;
      if (xa < xb) {
        if (op == OP_M || op == OP_EQ || op == OP_X) {
          const bool first_ins = lead_ins && ra == 0;  // the element at locus 0 is an insertion
          const bool ins_anchor = (op == OP_M || op == OP_EQ) && nextop == OP_I;
          const bool del_anchor = nextop == OP_D;
          int32_t lo = first_ins ? ra + 1 : ra;
          int32_t hi = (ins_anchor || del_anchor) ? rb - 1 : rb;
          lo = lo > xa ? lo : xa;
          hi = hi < xb ? hi : xb;
          // bases past the end of the sequence: assertion in the reference (Seq index)
          const int32_t rend = ra + (slen - rpos);  // first locus without a sequenced base
          if (xb > rend) sink.error(1 /*GQ_E_ASSERT*/, (int64_t)rend);
          bases_run(R, lo, hi < rend ? hi : rend, seq_off + rpos + (lo - ra), L0, fl, sink, sv, clean);
          events_run(ev, evb, e4, b4, nmd, s, lo, hi, L0, fl, sink, R.seq, seq_off + rpos - ra, rend);
          auto special = [&](int32_t l, int kind) {  // an anchor element at l
            if (l < xa || l >= xb || rpos + (l - ra) >= slen) return;
            const uint8_t base = R.seq[seq_off + rpos + (l - ra)];
            const int v = md_at(l);
            sink.elem(l, kind, base, v >= 0 ? (uint8_t)v : base, v >= 0, fl);
          };
          if (first_ins) special(ra, K_INS);
          if ((ins_anchor || del_anchor) && !(first_ins && rb - 1 == ra)) special(rb - 1, ins_anchor ? K_INS : K_DEL);
        } else if (op == OP_D) {
          for (int32_t l = xa; l < xb; ++l) {  // mid-deletions
            const int v = md_at(l);
            if (v < 0) sink.error(3 /*GQ_E_MD*/, (int64_t)l);
            sink.elem(l, K_MID, (uint8_t)0, v >= 0 ? (uint8_t)v : (uint8_t)'N', true, fl);
          }
        } else {  // N: Clipped, MD-derived reference 'N'
          sink.clip_run(xa - L0, xb - L0, fl);
        }
      }
      ref += len;
    }
    if (consumes_read(op)) rpos += len;
    if (ref >= L1) break;
    cc = cn;
  }
}


// LDS histogram: six u32 words per locus (SoA: word * S + guard + i, so consecutive loci
// sit on consecutive banks), each holding two 16-bit counters.  A sequenced base b has
// code (b >> 1) & 7, distinct for A 0, C 1, T 2, G 3, N 7; a base whose code does not
// map back to it is "other" (slot 4).  slot = word * 2 + half:
//   W_AC = A | C << 16, W_TG = T | G << 16, W_OX = other | complex << 16,
//   W_NN = N << 16 | mask (bits 0-3: OR of the MD-derived standard reference bases of
//   event / complex elements; W_MASK aliases W_NN, read it with & 0xF),
//   W_EAC / W_ETG = A C / T G counts of Match/Mismatch elements carrying an MD mismatch event.
// Tiles whose read window could exceed 65535 reads never use this path (wide tiles).
enum : int { W_AC = 0, W_TG, W_OX, W_NN, W_EAC, W_ETG, W_N, W_MASK = W_NN };
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
  // four Match/Mismatch elements whose bytes are all A C G T N (checked once per read at
  // upload): counter word (b >> 2) & 3 (A C -> W_AC, T G -> W_TG, N -> W_NN), half (b >> 1) & 1;
  // the increment is valid << (16 * half)
  // one Match/Mismatch element with an A/C/G/T/N base b at tile index i (one atomic)
  __device__ __forceinline__ void base1_clean(int i, uint32_t b) {
    atomicAdd(cnt + ((b >> 2) & 3u) * S + kGuard + i, 1u << (((b >> 1) & 1u) << 4));
  }
  __device__ __forceinline__ void bases4_clean(int i, uint32_t w, uint32_t valid4, uint8_t) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t ws = (w >> (8 * j + 2)) & 3u, hb = (w >> (8 * j + 1)) & 1u;
      const uint32_t inc = ((valid4 >> j) & 1u) << (hb << 4);
      if (ABL & 4) {
        acc += inc;
        acc ^= ws;
      } else {
        atomicAdd(cnt + ws * S + kGuard + i + j, inc);
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
  // a complex element (insertion / deletion anchor, mid-deletion) at tile index i; its locus
  // is decided by the exact kernel, so no reference-base bit is needed
  __device__ __forceinline__ void complex_i(int i) { atomicAdd(at(W_OX, i), 1u << 16); }
  // Clipped elements (CIGAR N) at tile indices [i0, i1): complex, MD-derived reference 'N'
  __device__ __forceinline__ void clip_run(int i0, int i1, uint8_t) {
    for (int i = i0; i < i1; ++i) atomicAdd(at(W_OX, i), 1u << 16);
  }
  __device__ __forceinline__ void error(int code, int64_t where) { raise_error(err, (int64_t *)err_pos, code, where); }
};

}  // namespace gq
