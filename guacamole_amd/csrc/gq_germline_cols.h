// gq_germline_cols.h — germline_cols<T>: the germline-threshold pileup kernel.
//
// One workgroup per tile of T loci (XCD-aware tile order).  The tile's reads are
// start-sorted and their sequence bytes are one contiguous range of the pool, so the
// workgroup copies that range into LDS with LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave-instruction, fully coalesced) and then counts it COLUMN-MAJOR: lane j owns the
// four loci [4j, 4j + 4) of the tile and walks the reads covering them, reading one
// dword (4 bases) per read from LDS.  Counts live in registers as SWAR nibble fields
// (A|C and T|G per byte, one byte per locus) folded into byte counters every 15 reads,
// so the hot loop has no atomics and no histogram re-read:
//
//     w    = alignbyte(stage[a+1], stage[a], a)       4 bases at loci 4j..4j+3
//     sel  = w & 0x07070707                           A 1, C 3, T 4, N 6, G 7
//     n_ac += perm(0, 0x10000100, sel)                A -> 0x01, C -> 0x10 per byte
//     n_tg += perm(0x10000001, 0, sel)                T -> 0x01, G -> 0x10 per byte
//
// N = (reads fully covering the column) - A - C - T - G.  Everything the column pass does
// not cover goes through the LDS histogram (GermSink atomics) in a lane-per-read pass:
//   * the <= 3 + 3 loci of a read that only partially cover a column (its two ends),
//   * MD mismatch events (for the MD-derived reference base, Pileup.scala:157-165),
//   * reads that are not a single (M|=|X) block with A/C/G/T/N bases, or whose bytes are
//     not staged: the general per-read walker (walk_read_lane, PileupElement.scala:68-248).
// Tiles whose reads do not fit the stage are processed in several read chunks.  Then one
// thread per locus makes the GermlineThreshold decision (GermlineThresholdCaller.scala:90-179)
// for single-base pileups and queues the rest for germline_complex.
#pragma once

#include "gq_kernels.h"

// (included inside gq_pileup.hip's anonymous namespace, after `using namespace gq`)

// tile index of block b: blocks b, b + 8, b + 16, ... run on one XCD (round-robin
// dispatch), so give each XCD a contiguous run of tiles (reads straddling neighbouring
// tiles are then re-read from that XCD's L2).  A bijection on [0, n).
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t n) {
  const int64_t q = n >> 3, rem = n & 7;
  const int64_t x = b & 7, j = b >> 3;
  return x * q + (x < rem ? x : rem) + j;
}

// GermlineThresholdCaller.scala:100-177 for the loci of a tile whose histogram is complete
// in `cnt` (GermSink layout).  One thread per locus; loci needing exact alleles (indels,
// clips, other bases, several samples, ambiguous reference) are queued as ComplexItems.
// Output slots of germline_decide.  reserve(which, n) gives this lane's first slot for n
// records (which = 0) or complex items (1), wave-aggregated, relative to partition `part`
// of capacity cap[which]; slots >= cap are dropped (the host retries with more room).
struct LdsOut {  // germline_cols: one partition per workgroup, counters in LDS
  unsigned *lds;  // [2]
  unsigned long long base[2], cap[2];
  __device__ __forceinline__ unsigned long long reserve(int which, unsigned n) {
    return wave_reserve_lds(lds + which, n);
  }
};
struct GlobalOut {  // germline_walk: a partition per wave, counters in device memory
  Counters *ctr;
  int part;
  unsigned long long base[2], cap[2];
  __device__ __forceinline__ unsigned long long reserve(int which, unsigned n) {
    return wave_reserve(&ctr->part[which][part], n);
  }
};

template <int T, bool ZERO = false, class Out>
__device__ __forceinline__ void germline_decide(const uint32_t *cnt, const Tile &tl, int64_t tile_id, bool wide,
                                                int n_samples, int threshold, int emit_ref, int emit_no_call,
                                                CallRec *__restrict__ recs, ComplexItem *__restrict__ cplx,
                                                Out &out, unsigned &visited, unsigned &amb, unsigned &ties,
                                                const uint32_t *reg = nullptr) {
  // reg (germline_cols, one locus per thread): this thread's locus's A C T G N counts held in
  // registers, added to the LDS words
  constexpr int S = T + 2 * kGuard;
  const int32_t L0 = tl.L0;
  const bool multi_sample = n_samples > 1;
  const int nloci = tl.L1 - L0;
  // count * 100 / depth > threshold  <=>  count * 100 >= (threshold + 1) * depth  (integers, depth > 0);
  // 32-bit products when they cannot overflow (counts < 2^19, threshold <= 1000)
  const int64_t thr1 = (int64_t)threshold + 1;
  const bool narrow = thr1 >= 0 && thr1 <= 1001;
  const uint32_t thr1u = (uint32_t)thr1;
  auto passes = [=](uint32_t count, uint32_t depth) {
    return narrow ? count * 100u >= thr1u * depth : (int64_t)count * 100 >= thr1 * (int64_t)depth;
  };
  constexpr uint64_t kAltSym = ((uint64_t)'<' << 8) | ((uint64_t)'A' << 16) | ((uint64_t)'L' << 24) |
                               ((uint64_t)'T' << 32) | ((uint64_t)'>' << 40);
  // uniform trip count so every wave reaches the wave-level reservations together
  for (int i0 = 0; i0 < nloci; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    const bool in = i < nloci;
    // ---- summary of the locus, branch-free
    uint32_t wac = 0, wtg = 0, wox = 0, wnn = 0, eac = 0, etg = 0;
    if (in) {
      wac = cnt[W_AC * S + kGuard + i];
      wtg = cnt[W_TG * S + kGuard + i];
      wox = cnt[W_OX * S + kGuard + i];
      wnn = cnt[W_NN * S + kGuard + i];
      eac = cnt[W_EAC * S + kGuard + i];
      etg = cnt[W_ETG * S + kGuard + i];
    }
    if (ZERO && i < T) {  // ready for the next tile (one thread per locus: its own words)
      uint32_t *z = const_cast<uint32_t *>(cnt) + kGuard + i;
#pragma unroll
      for (int w = 0; w < W_N; ++w) z[w * S] = 0u;
    }
    uint32_t c[5] = {wac & 0xFFFFu, wac >> 16, wtg & 0xFFFFu, wtg >> 16, wnn >> 16};  // A C T G N
    if (reg) {
#pragma unroll
      for (int k = 0; k < 5; ++k) c[k] += in ? reg[k] : 0u;
    }
    const uint32_t cx = (wox & 0xFFFFu) + (wox >> 16);  // other bases + complex elements
    const uint32_t depth = c[0] + c[1] + c[2] + c[3] + c[4] + cx;
    // MD-derived reference bases present: event / complex bits, plus every base with more
    // reads than reads carrying a mismatch event there (those read the base as reference)
    const uint32_t mask = (wnn & 0xFu) | (c[0] > (eac & 0xFFFFu) ? 1u : 0u) | (c[1] > (eac >> 16) ? 2u : 0u) |
                          (c[2] > (etg & 0xFFFFu) ? 4u : 0u) | (c[3] > (etg >> 16) ? 8u : 0u);
    const bool live = in && depth > 0;
    const bool ambiguous = (mask & (mask - 1)) != 0;
    const uint32_t low = mask & (0u - mask);  // the first standard reference base, as a bit
    const uint32_t c_ref = low == 1u ? c[0] : low == 2u ? c[1] : low == 4u ? c[2] : low == 8u ? c[3] : c[4];
    const bool to_complex = (wide && in) || (live && (ambiguous || cx > 0 || multi_sample));
    // every non-reference allele has count <= depth - c_ref: if that does not pass, no
    // alternate allele does (HomRef if the reference passes, else NoCall)
    const bool homref = live && !to_complex && !passes(depth - c_ref, depth);
    const bool ref_pass = c_ref > 0 && passes(c_ref, depth);
    const bool emit_hr = homref && (ref_pass ? emit_ref : emit_no_call);
    const bool general = live && !to_complex && !homref;
    visited += (live && !(wide && in)) ? 1u : 0u;
    amb += (live && ambiguous && !wide) ? 1u : 0u;
    if (__ballot(to_complex || emit_hr || general) == 0) continue;  // the common case: nothing to write
    // ---- records
    CallRec out0, out1;  // named (not an array): no scratch
    unsigned nout = 0;
    const uint8_t ref = mask ? bit_base(mask) : (uint8_t)'N';
    const int32_t pos = L0 + i;
    const uint64_t ord = (uint64_t)(tl.ordinal0 + i);
    auto push = [&](const CallRec &rr) {
      if (nout == 0) out0 = rr;
      else out1 = rr;
      ++nout;
    };
    if (emit_hr) {
      CallRec rr;
      rr.key = ord << 12;
      rr.contig = tl.contig;
      rr.pos = pos;
      rr.sample = 0;
      rr.gt0 = rr.gt1 = ref_pass ? GQ_GT_REF : GQ_GT_NOCALL;
      rr.flags = 0;
      rr.ref_len = 1;
      rr.alt_len = 5;
      rr.allele = (uint64_t)ref | kAltSym;
      push(rr);
    }
    if (general) {
      // a variant candidate: its counts travel in a placeholder record pair (two slots), which
      // germline_expand turns into the 0-2 Genotype records (GermlineThresholdCaller.scala:100-177)
      // after the kernel: the long case split stays out of this loop
      CallRec rr;
      rr.key = ord << 12;
      rr.contig = tl.contig;
      rr.pos = pos;
      rr.sample = 0;
      rr.gt0 = ref;
      rr.gt1 = 0;
      rr.flags = kCandidate;
      rr.ref_len = (uint16_t)c[4];
      rr.alt_len = 0;
      rr.allele = (uint64_t)c[0] | ((uint64_t)c[1] << 16) | ((uint64_t)c[2] << 32) | ((uint64_t)c[3] << 48);
      push(rr);
      rr.flags = kCandidateSlot;
      push(rr);
    }
    // reserve + write records (wave-aggregated, in the writer's partition)
    const unsigned long long base = out.reserve(0, nout);
    CallRec *prec = recs + out.base[0];
    if (nout > 0 && base < out.cap[0]) prec[base] = out0;
    if (nout > 1 && base + 1 < out.cap[0]) prec[base + 1] = out1;
    const unsigned long long cb = out.reserve(1, to_complex ? 1u : 0u);
    if (to_complex && cb < out.cap[1])
      cplx[out.base[1] + cb] = ComplexItem{(int32_t)tile_id, L0 + i, wide ? 1 : 0};
  }
}

// The variant candidates of germline_decide -> Genotype records, one thread per record slot
// (GermlineThresholdCaller.scala:100-177 for a pileup of single-base alleles; counts < 2^16).
// Allele (ref, b) keys: count << 8 | (255 - canonical rank); canonical order of Allele(ref, alt)
// for one ref is the alt byte order A < C < G < N < T, i.e. the categories 0, 1, 3, 4, 2.
// Sorting keys descending = sortBy(-count), ties canonical.  Unused slots get a key past
// every ordinal (dead_key) and are counted in n_dead; they sort behind the live records.
__global__ void germline_expand(CallRec *__restrict__ recs, Counters *ctr, OutGeom og, int threshold,
                                int emit_ref, int emit_no_call, uint64_t dead_key) {
  const unsigned long long n = ctr->n_rec;
  const int64_t thr1 = (int64_t)threshold + 1;
  auto passes = [=](uint32_t count, uint32_t depth) { return (int64_t)count * 100 >= thr1 * (int64_t)depth; };
  constexpr uint64_t kAltSym = ((uint64_t)'<' << 8) | ((uint64_t)'A' << 16) | ((uint64_t)'L' << 24) |
                               ((uint64_t)'T' << 32) | ((uint64_t)'>' << 40);
  unsigned dead = 0, ties = 0;
  (void)n;
  // partition by partition (block per partition): its slots [0, kept count)
  for (int p = blockIdx.x; p < kParts; p += gridDim.x) {
   const unsigned long long cnt = ctr->part_off[0][p + 1] - ctr->part_off[0][p];
   for (unsigned long long k = threadIdx.x; k < cnt; k += blockDim.x) {
    const unsigned long long slot = og.slot(0, p, k);
    const CallRec cand = recs[slot];
    if (cand.flags != kCandidate) continue;  // an ordinary record, or the second slot of a pair
    const uint32_t c[5] = {(uint32_t)(cand.allele & 0xFFFFu), (uint32_t)((cand.allele >> 16) & 0xFFFFu),
                           (uint32_t)((cand.allele >> 32) & 0xFFFFu), (uint32_t)(cand.allele >> 48), cand.ref_len};
    const uint32_t depth = c[0] + c[1] + c[2] + c[3] + c[4];
    const uint8_t ref = cand.gt0;
    uint32_t k0 = 0, k1 = 0, k2 = 0;  // top three passing keys
    int npass = 0;
#pragma unroll
    for (int rank = 0; rank < 5; ++rank) {
      const int cat = (0x24310 >> (4 * rank)) & 0xF;
      const uint32_t cc = c[cat];
      if (cc == 0 || !passes(cc, depth)) continue;
      ++npass;
      uint32_t key = (cc << 8) | (uint32_t)(255 - rank);
      if (key > k0) { const uint32_t t = k0; k0 = key; key = t; }
      if (key > k1) { const uint32_t t = k1; k1 = key; key = t; }
      if (key > k2) { k2 = key; }
    }
    auto key_base = [](uint32_t key) -> uint8_t {
      const int rank = 255 - (int)(key & 0xFFu);
      return cat_base((0x24310 >> (4 * rank)) & 0xF);
    };
    const bool tie = npass >= 2 && ((k0 >> 8) == (k1 >> 8) || (npass >= 3 && (k1 >> 8) == (k2 >> 8)));
    if (tie) ++ties;
    const uint8_t fl = tie ? GQ_FLAG_TIE : 0;
    // the case split -> up to two records (g0, g1, alt base or the symbolic <ALT>)
    const uint8_t b0 = key_base(k0), b1 = key_base(k1);
    int nout = 0;
    uint8_t ga0 = 0, ga1 = 0, aa = 0, gb0 = 0, gb1 = 0, ab = 0;
    bool syma = false;
    if (npass == 0) {
      if (emit_no_call) nout = 1, ga0 = ga1 = GQ_GT_NOCALL, syma = true;
    } else if (npass == 1 && b0 == ref) {
      if (emit_ref) nout = 1, ga0 = ga1 = GQ_GT_REF, syma = true;
    } else if (npass == 1) {
      nout = 1, ga0 = ga1 = GQ_GT_ALT, aa = b0;
    } else {
      const bool v1 = b0 != ref, v2 = b1 != ref;
      if (v1 != v2) {
        nout = 1, ga0 = GQ_GT_REF, ga1 = GQ_GT_ALT, aa = v1 ? b0 : b1;
      } else if (v1 && v2) {
        nout = 2, ga0 = gb0 = GQ_GT_ALT, ga1 = gb1 = GQ_GT_OTHERALT, aa = b0, ab = b1;
      }
      // two non-variant single-base alleles cannot occur (all Match alleles share ref)
    }
    // the pair's two slots are consecutive in the partition (reserved together); an unused
    // slot gets the dead key.  Records are written as two 16-byte halves (CallRec layout).
    auto put = [&](unsigned long long at, bool live, int sub, uint8_t g0, uint8_t g1, uint8_t alt, bool sym) {
      const uint64_t key = live ? (cand.key | (uint64_t)sub) : dead_key;
      const uint64_t allele = sym ? ((uint64_t)ref | kAltSym) : ((uint64_t)ref | ((uint64_t)alt << 8));
      const uint32_t w3 = (uint32_t)cand.sample | ((uint32_t)g0 << 8) | ((uint32_t)g1 << 16) |
                          ((uint32_t)(live ? fl : 0) << 24);
      const uint32_t w4 = 1u | ((uint32_t)(sym ? 5 : 1) << 16);  // ref_len 1, alt_len
      uint4 *d = reinterpret_cast<uint4 *>(recs + at);
      d[0] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), (uint32_t)cand.contig, (uint32_t)cand.pos);
      d[1] = make_uint4(w3, w4, (uint32_t)allele, (uint32_t)(allele >> 32));
    };
    put(slot, nout > 0, 0, ga0, ga1, aa, syma);
    put(slot + 1, nout > 1, 1, gb0, gb1, ab, false);
    dead += nout > 1 ? 0u : nout > 0 ? 1u : 2u;
   }
  }
  // one atomic per wave (a per-thread add on one word serialises ~10^5 threads at the L2)
  for (int d = 32; d >= 1; d >>= 1) {
    dead += __shfl_xor(dead, d, 64);
    ties += __shfl_xor(ties, d, 64);
  }
  if ((threadIdx.x & 63) == 0) {  // spread over kSpread words (one word serialises ~10 ns per add)
    const int sl = (int)((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kSpread - 1));
    if (dead) atomicAdd(&ctr->spread[3][sl], (unsigned long long)dead);
    if (ties) atomicAdd(&ctr->spread[2][sl], (unsigned long long)ties);
  }
}

// Run counters (visited / ambiguous / tie loci) of a workgroup, added once at its end.
__device__ __forceinline__ void add_run_counters(Counters *ctr, unsigned visited, unsigned amb, unsigned ties,
                                                 int slot) {
  __shared__ unsigned red[3];
  if (threadIdx.x < 3) red[threadIdx.x] = 0;
  __syncthreads();
  if (visited) atomicAdd(&red[0], visited);
  if (amb) atomicAdd(&red[1], amb);
  if (ties) atomicAdd(&red[2], ties);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int sl = slot & (kSpread - 1);
    if (red[0]) atomicAdd(&ctr->spread[0][sl], (unsigned long long)red[0]);
    if (red[1]) atomicAdd(&ctr->spread[1][sl], (unsigned long long)red[1]);
    if (red[2]) atomicAdd(&ctr->spread[2][sl], (unsigned long long)red[2]);
  }
}

// Geometry of the column kernel (T = 512 loci per tile, two lanes per 4-locus column).
// Per workgroup: two LDS buffers of {sequence stage, ColDesc rows, MD events} (the next
// tile's are DMA'd while this one is counted), the histogram words, the column buckets:
// about 80 KiB, two workgroups per CU.  plan_tiles marks tiles whose window fits.
#ifndef GQ_DMA_W0
#define GQ_DMA_W0 5   // waves GQ_DMA_W0 .. 7 issue the DMA (measured: 5 beats 4 and 6)
#endif
#ifndef GQ_B_T0
#define GQ_B_T0 0     // thread GQ_B_T0 + k builds the row of read k
#endif
#ifndef GQ_EV_T0
#define GQ_EV_T0 96   // thread GQ_EV_T0 + k takes the MD events of read k (waves 1-4)
#endif
struct ColsCfg {
  static constexpr int kT = 512;
  static constexpr int kThreads = 512;
  static constexpr int kLanesPerCol = kThreads / (kT / 4);  // rows of a column split over 4 lanes
  static constexpr int kStage = 24 * 1024;  // sequence bytes (1 KiB DMA pieces)
#ifndef GQ_COLS_BATCH
#define GQ_COLS_BATCH 5
#endif
  static constexpr int kBatch = GQ_COLS_BATCH;  // rows per lane per column-pass batch (8 lanes per column)
  static constexpr int kMeta = 208;         // reads per tile (ColDesc rows); the row buffer holds
                                            // kRowCap rows: 8 * kBatch zero rows pad the batches
  static constexpr int kRowCap = 256;
  static_assert(kMeta + 8 * kBatch <= kRowCap, "row padding");
  static constexpr int kEv = 512;           // auxiliary words (MD events, segments of general reads)
  static constexpr int kExtra = 64;         // column rows of general reads' count segments
  // one buffer: stage | rows (+16 B alignment, +256 B dword-DMA tail) | events (same)
  static constexpr int kRowsOff = kStage + 16;  // + 16 zero bytes after the stage (kZero)
  static constexpr int kEvOff = kRowsOff + kRowCap * 24 + 16 + 256;
  static constexpr int kBuf = kEvOff + kEv * 4 + 16 + 256;
};

// Byte counters of one lane's 8-locus column: c_x[0] for loci c..c+3, c_x[1] for c+4..c+7,
// one byte per locus (A C T G and cv = reads with a base there); nrow = rows added since the
// last flush (bounds every byte, <= 255).  Flushed into the LDS words with atomics only when a
// column is deeper than 255 reads.
struct ColCounts {
  uint32_t ca[2] = {0, 0}, cc[2] = {0, 0}, ct[2] = {0, 0}, cg[2] = {0, 0}, cv[2] = {0, 0}, nrow = 0;
  __device__ __forceinline__ void flush(uint32_t *cnt, int S, int c) {
    if (nrow == 0) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t cn = cv[h] - (ca[h] + cc[h] + ct[h] + cg[h]);  // bytewise, no borrow
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t sel = 0x0C000C00u | ((uint32_t)(4 + b) << 16) | (uint32_t)b;  // [x_b, 0, y_b, 0]
        const uint32_t ac = __builtin_amdgcn_perm(cc[h], ca[h], sel), tg = __builtin_amdgcn_perm(cg[h], ct[h], sel);
        const uint32_t nn = ((cn >> (8 * b)) & 0xFFu) << 16;
        const int i = kGuard + c + 4 * h + b;
        if (ac) atomicAdd(cnt + W_AC * S + i, ac);
        if (tg) atomicAdd(cnt + W_TG * S + i, tg);
        if (nn) atomicAdd(cnt + W_NN * S + i, nn);
      }
    }
    ca[0] = ca[1] = cc[0] = cc[1] = ct[0] = ct[1] = cg[0] = cg[1] = cv[0] = cv[1] = nrow = 0;
  }
};

// LDS-DMA of the global byte range [g, g + n) into LDS at `l` (16-B aligned g), by wave
// `wave` of NW, as 1 KiB (dwordx4) or 256 B (dword) pieces.
template <int NW, int WIDTH>
__device__ __forceinline__ void dma_range(const uint8_t *g, uint8_t *l, int n, int wave, int lane) {
  constexpr int P = 64 * WIDTH;
  const int np = (n + P - 1) / P;
  for (int q = wave; q < np; q += NW) {
    const void *src = (const void *)(g + q * P + lane * WIDTH);
    __attribute__((address_space(3))) void *dst = (__attribute__((address_space(3))) void *)(l + q * P);
    if constexpr (WIDTH == 16) __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
    else __builtin_amdgcn_global_load_lds(src, dst, 4, 0, 0);
  }
}

constexpr uint32_t kSegCountK = 0;

// Column row of tile loci [a, b) (clamped to 16 bits) and base = LDS address of tile locus 0
// in the row's bytes.
__device__ __forceinline__ uint2 col_row(int32_t a, int32_t b, uint32_t base, int T) {
  const int32_t sc = a > -8 ? a : -8, ec = b < T + 8 ? b : T + 8;
  return make_uint2((uint32_t)((sc & 0xFFFF) | (ec << 16)), base);
}

// germline_cols: persistent workgroups, each over a contiguous run of tiles (XCD-local
// neighbours: reads straddling two tiles are re-read from L2).  Per tile:
//   A  wait for this tile's DMA (issued one tile earlier), then DMA the next tile
//   B  thread per read: the column row (clamped s | e << 16, LDS address of tile locus 0,
//      written over the ColDesc's pmax_end / seq_lo words) and the column-bucket histogram
//   C  scan of the buckets -> each lane's row range [lo, hi)
//   D  column pass (lanes t and t + 128 take alternate rows of column t % 128)
//   E  per-read pass: column ends and MD events into the LDS histogram (GermSink)
//   F  flush, decision (germline_decide), histogram zeroed for the next tile
// Tiles that do not fit (plan_tiles: sbytes == 0) or hold a read the column path cannot
// count are listed in `slow` for germline_walk.
__global__ __launch_bounds__(ColsCfg::kThreads) void germline_cols(
    const Tile *__restrict__ tiles, int64_t n_tiles, const uint8_t *__restrict__ seq,
    const ColDesc *__restrict__ cdesc, const uint32_t *__restrict__ cev, int n_samples, int threshold, int emit_ref,
    int emit_no_call, CallRec *__restrict__ recs, ComplexItem *__restrict__ cplx, OutGeom og, Counters *ctr,
    int32_t *__restrict__ slow, int dbg) {
  // dbg (diagnostics, env GQ_DBG; results are wrong when bits 0-3, 5, 6 are set): 1 skip the
  // column pass, 2 skip the per-read pass, 4 skip the decision, 8 skip the DMA; 16 phase
  // clocks; 32 skip the column ends, 64 skip the MD events
  using C = ColsCfg;
  constexpr int T = C::kT, NT = C::kThreads, NW = NT / 64, W = 8, NCOL = T / W;
  static_assert(NCOL == 64 && NT == 8 * NCOL, "one wave scans the columns; eight lanes per column");
  constexpr int S = T + 2 * kGuard;
  constexpr int kNever = (int)(0x7FFFu | 0x80000000u);  // s = 32767, e = -32768: covers no column
  __shared__ __attribute__((aligned(16))) uint32_t cnt[W_N * S];
  __shared__ __attribute__((aligned(16))) uint8_t buf[2][C::kBuf];
  // per buffer parity: column buckets (rows starting (lo 16) / prefix-max end reaching (hi 16))
  // and the count of extra rows; the extra rows (general reads' count segments) themselves are
  // written by B(i + 1) only after D(i) has read them (barrier 1), so one array serves
  __shared__ uint32_t hist[2][NCOL];
  __shared__ __attribute__((aligned(8))) uint2 xrow[C::kExtra];
  // byte masks of the bases [lo, hi) of an 8-locus column, lo, hi in 0..8: 0x07 per base
  __shared__ __attribute__((aligned(8))) uint2 bmask[81];
  __shared__ unsigned n_xrow[2];
  __shared__ unsigned outn[2];  // records / complex items of this workgroup's partition

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // this workgroup's tiles [i0, i1)
  const int64_t per = n_tiles / gridDim.x, extra = n_tiles % gridDim.x;
  const int64_t i0 = blockIdx.x * per + min((int64_t)blockIdx.x, extra);
  const int64_t i1 = i0 + per + ((int64_t)blockIdx.x < extra ? 1 : 0);
  uint64_t clk[7] = {0, 0, 0, 0, 0, 0, 0};

  // DMA of a tile's window into buffer b, by waves GQ_DMA_W0 .. 7 (waves 0-2 build rows meanwhile)
  auto issue = [&](const Tile &tn, int b) {
    if (tn.sbytes <= 0 || (dbg & 8) || wave < GQ_DMA_W0) return;
    uint8_t *L = buf[b];
    const int w4 = wave - GQ_DMA_W0;
    dma_range<NW - GQ_DMA_W0, 16>(seq + tn.sb0, L, tn.sbytes, w4, lane);
    const int64_t d0 = (tn.rb * 24) & ~(int64_t)15;
    dma_range<NW - GQ_DMA_W0, 4>(reinterpret_cast<const uint8_t *>(cdesc) + d0, L + C::kRowsOff, (int)(tn.re * 24 - d0), w4,
                    lane);
    if (tn.mcnt > 0)
      dma_range<NW - GQ_DMA_W0, 4>(reinterpret_cast<const uint8_t *>(cev + tn.mb0), L + C::kEvOff, tn.mcnt * 4, w4, lane);
  };
  {  // zero the histogram words, the buckets and the 16 zero bytes after each stage
    uint4 *c4 = reinterpret_cast<uint4 *>(cnt);
    for (int i = t; i < W_N * S / 4; i += NT) c4[i] = make_uint4(0u, 0u, 0u, 0u);
    if (t < 2 * NCOL) hist[t >> 6][t & (NCOL - 1)] = 0;
    if (t < 2) *reinterpret_cast<uint4 *>(buf[t] + C::kStage) = make_uint4(0u, 0u, 0u, 0u);
    if (t < 2) outn[t] = 0;
    if (t < 2) n_xrow[t] = 0;
    if (t < 81) {
      const int lo = t / 9, hi = t % 9;
      uint32_t m0 = 0, m1 = 0;
      for (int j = 0; j < 8; ++j)
        if (j >= lo && j < hi) {
          if (j < 4) m0 |= 0x07u << (8 * j);
          else m1 |= 0x07u << (8 * (j - 4));
        }
      bmask[t] = make_uint2(m0, m1);
    }
  }
  LdsOut out{outn, {og.slot(0, (int)blockIdx.x, 0), og.slot(1, (int)blockIdx.x, 0)}, {og.capA[0], og.capA[1]}};
  unsigned visited = 0, amb = 0, ties = 0;
  // tile descriptors travel as one dword per lane (lanes 0-15) loaded two tiles ahead with a
  // vector load: a scalar load would share lgkmcnt with the LDS traffic and stall it
  auto load_desc = [&](int64_t k) -> uint32_t {
    return (k < i1 && lane < 16) ? reinterpret_cast<const uint32_t *>(tiles + k)[lane] : 0u;
  };
  auto unpack = [](uint32_t v) {
    Tile x;
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = (uint32_t)__builtin_amdgcn_readlane((int)v, k);
    x.ordinal0 = (int64_t)((uint64_t)w[0] | ((uint64_t)w[1] << 32));
    x.rb = (int64_t)((uint64_t)w[2] | ((uint64_t)w[3] << 32));
    x.re = (int64_t)((uint64_t)w[4] | ((uint64_t)w[5] << 32));
    x.contig = (int32_t)w[6];
    x.L0 = (int32_t)w[7];
    x.L1 = (int32_t)w[8];
    x.range = (int32_t)w[9];
    x.sb0 = (int64_t)((uint64_t)w[10] | ((uint64_t)w[11] << 32));
    x.sbytes = (int32_t)w[12];
    x.mcnt = (int32_t)w[13];
    x.mb0 = (int64_t)((uint64_t)w[14] | ((uint64_t)w[15] << 32));
    return x;
  };
  // Row state a thread keeps from building a tile's rows (B) to its per-read pass (E)
  struct RowState {
    int32_t s = 0, base = 0, seg = 0, nseg = 0;
    bool general = false;
  };
  // ---- B: rows of tile tb in buffer bb (thread per read) and its column buckets; threads
  //      nch .. nch + 8 * kBatch - 1 write the zero rows that pad the column pass's batches.
  //      Returns this thread's "the tile cannot take the column path" vote.
  auto build = [&](const Tile &tb, int bb, RowState &rs) -> int {
    rs = RowState{};
    int not_col = tb.sbytes <= 0;
    if (not_col) return 1;
    const int32_t L0 = tb.L0, L1 = tb.L1;
    uint8_t *L = buf[bb];
    const int64_t d0 = (tb.rb * 24) & ~(int64_t)15;
    uint32_t *rows = reinterpret_cast<uint32_t *>(L + C::kRowsOff + (tb.rb * 24 - d0));  // 6 words per read
    const uint32_t *evs = reinterpret_cast<const uint32_t *>(L + C::kEvOff);
    const int nch = (int)(tb.re - tb.rb);
    const uint32_t sb_lo = (uint32_t)(uint64_t)tb.sb0, mb_lo = (uint32_t)(uint64_t)tb.mb0;
    uint32_t *hb = hist[bb];
    const int k = t - GQ_B_T0;  // thread per read
    if (k >= 0 && k < nch) {
      uint32_t *d = rows + 6 * k;
      const int32_t s = (int32_t)d[0], e = (int32_t)d[1], pe = (int32_t)d[2];
      const uint32_t info = d[3];
      const int32_t srel = s - L0, erel = e - L0, perel = pe - L0;
      const uint32_t sa = d[4] - sb_lo;  // stage address of the base at `start`
      const uint32_t ea = d[5] - mb_lo;  // staged index of the first MD event
      const int32_t nmd = (int32_t)(info & 0xFFFFu);
      uint2 row = make_uint2(0u, 0u);  // empty: s = e = 0
      bool mine = false;
      if (e > L0 && s < L1) {
        const uint32_t nseg = (info >> 18) & 0xFFu;
        const bool evs_in = ea + (uint32_t)nmd + 2u * nseg <= (uint32_t)tb.mcnt;
        const bool ok = (info & kColEligible) && sa + (uint32_t)(e - s) <= (uint32_t)tb.sbytes && evs_in;
        const bool gen = (info & kColGeneral) && evs_in;
        if (gen) {  // its count segments become extra column rows
          rs.general = true;
          mine = true;
          rs.s = srel;
          rs.base = (int32_t)sa;
          rs.seg = (int32_t)(ea + (uint32_t)nmd);
          rs.nseg = (int32_t)nseg;
          for (uint32_t q = 0; q < nseg; ++q) {
            const uint32_t w0 = evs[ea + nmd + 2 * q], w1 = evs[ea + nmd + 2 * q + 1];
            if ((w1 >> 16) != kSegCountK) continue;
            const int32_t a = srel + (int32_t)(w0 & 0xFFFFu), b = a + (int32_t)(w0 >> 16);
            const uint32_t so = sa + (w1 & 0xFFFFu);  // stage address of the segment's first base
            if (so + (uint32_t)(b - a) > (uint32_t)tb.sbytes) not_col = 1;
            if (b <= 0 || a >= L1 - L0) continue;
            const unsigned x = atomicAdd(&n_xrow[bb], 1u);
            if (x >= (unsigned)C::kExtra) {
              not_col = 1;
              continue;
            }
            xrow[x] = col_row(a, b, so - (uint32_t)a, T);
          }
        } else if (!ok) {
          not_col = 1;
        } else {
          row = col_row(srel, erel, sa - (uint32_t)srel, T);
          mine = true;
        }
      }
      // rows [0, hi(col)) start at or before the column's last locus; rows [0, lo(col))
      // have prefix-max end at or before its first locus (so cover none of it)
      const int bs = srel < 0 ? 0 : srel >> 3, bp = perel < 0 ? 0 : (perel + 7) >> 3;
      if (bs < NCOL) atomicAdd(&hb[bs], 1u);
      if (bp < NCOL) atomicAdd(&hb[bp], 1u << 16);
      // the row's words become: d0 d1 the column row, d4 = n_md | first event << 16 | mine << 31,
      // d5 = tile-relative start (for the MD-event pass)
      *reinterpret_cast<uint2 *>(d) = row;
      *reinterpret_cast<uint2 *>(d + 4) =
          make_uint2((uint32_t)nmd | (ea << 16) | (mine ? 0x80000000u : 0u), (uint32_t)srel);
    } else if (k >= 0 && k < nch + 8 * C::kBatch && k < C::kRowCap) {
      uint32_t *d = rows + 6 * k;
      *reinterpret_cast<uint2 *>(d) = make_uint2(0u, 0u);
    }
    return not_col;
  };

  // Software pipeline over this workgroup's tiles, two barriers per tile.  Iteration i:
  //   C/D/E(i)   bucket scan, column pass, per-read pass of tile i (buffer i & 1)
  //   barrier 1  tile i's histogram complete; DMA(i + 1) landed (issued one iteration ago)
  //   DMA(i + 2) into buffer i & 1 (free now); B(i + 1) on buffer (i + 1) & 1; decide(i)
  //   barrier 2  tile i + 1's rows / buckets complete (its column-path vote); tile i's
  //              histogram words zeroed by its decision
  // Buckets (hist) and extra rows (xrow, n_xrow) are kept per buffer parity.
  Tile tc{}, tn{};  // tile i (rows built) and tile i + 1
  uint32_t d2 = 0;  // raw descriptor of tile i + 2 (one dword per lane, loaded ahead)
  RowState rs_c, rs_n;
  int slow_c = 1;
  if (i0 < i1) {
    tc = unpack(load_desc(i0));
    issue(tc, 0);
    if (i0 + 1 < i1) {
      tn = unpack(load_desc(i0 + 1));
      issue(tn, 1);
    }
    d2 = load_desc(i0 + 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // the zeroing above, and tile i0's DMA
    slow_c = __syncthreads_or(build(tc, 0, rs_c));
    if (slow_c && t == 0) slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)i0;
  }
  int it = 0;
  for (int64_t i = i0; i < i1; ++i, ++it) {
    const int b = it & 1;
    const uint64_t ta = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    uint32_t regc[5] = {0, 0, 0, 0, 0};  // A C T G N of locus t from the column pass
    if (!slow_c) {
      const Tile &tl = tc;
      const int32_t L0 = tl.L0, L1 = tl.L1;
      uint8_t *L = buf[b];
      const uint32_t *st32 = reinterpret_cast<const uint32_t *>(L);
      const int64_t d0 = (tl.rb * 24) & ~(int64_t)15;
      uint32_t *rows = reinterpret_cast<uint32_t *>(L + C::kRowsOff + (tl.rb * 24 - d0));
      const uint32_t *evs = reinterpret_cast<const uint32_t *>(L + C::kEvOff);
      const int nch = (int)(tl.re - tl.rb);
      // ---- C: inclusive scan of the packed buckets over the 64 columns, by every wave (no
      //      barrier): lane l scans column l, then each lane fetches its own column's value
      const int col = t >> 3, par = t & 7;  // lanes 8q .. 8q + 7 share column q, every eighth row
      const uint32_t v = (uint32_t)__shfl((int)wave_incl_scan(hist[b][lane]), col, 64);
      const int lo = (int)(v >> 16), hi = (int)(v & 0xFFFFu);
      // ---- D: column pass: lanes par, par + P, ... of the column's rows, U rows per batch, all
      //      loads of a batch issued before use.  Per row: 3 LDS dwords -> 8 bases (2 dwords),
      //      code = byte & 7 (A 1, C 3, T 4, N 6, G 7), two v_perm tables per dword into
      //      A|C / T|G nibble fields, folded into byte counters before they can overflow.
      constexpr int P = 8, U = C::kBatch;  // lanes per column, rows per batch (a column has ~31 rows at 30x)
      const int c = W * col;
      ColCounts cc;
      uint32_t nac[2] = {0, 0}, ntg[2] = {0, 0}, nv[2] = {0, 0}, nnib = 0;  // nibble / byte fields, rows in them
      auto fold = [&]() {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          cc.ca[h] += nac[h] & 0x0F0F0F0Fu;
          cc.cc[h] += (nac[h] >> 4) & 0x0F0F0F0Fu;
          cc.ct[h] += ntg[h] & 0x0F0F0F0Fu;
          cc.cg[h] += (ntg[h] >> 4) & 0x0F0F0F0Fu;
          cc.cv[h] += nv[h];
          nac[h] = ntg[h] = nv[h] = 0;
        }
        nnib = 0;
      };
      // rows k0, k0 + P, ... of a row table at byte stride bs (rows past the range are empty
      //   rows): the bases of [max(s, c), min(e, c + 8)) via a byte-mask lookup, so rows that
      //   cover the column only partly (read ends) are counted here too
      auto batch = [&](const uint8_t *tab, int bs, int k0, auto uu) {
        constexpr int U = decltype(uu)::value;
        const uint8_t *rp = tab + bs * k0;
        uint2 m[U];
#pragma unroll
        for (int u = 0; u < U; ++u) m[u] = *reinterpret_cast<const uint2 *>(rp + bs * P * u);
        uint32_t a[U];
        uint2 bm[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int32_t s = (int32_t)(int16_t)(m[u].x & 0xFFFFu) - c, e = ((int32_t)m[u].x >> 16) - c;
          const int32_t l = s < 0 ? 0 : (s > 8 ? 8 : s), h = e < 0 ? 0 : (e > 8 ? 8 : e);
          const bool ov = h > l;
          a[u] = ov ? m[u].y + (uint32_t)c : (uint32_t)C::kStage;  // 12 zero bytes
          bm[u] = bmask[ov ? 9 * l + h : 0];
        }
        uint32_t w0[U], w1[U], w2[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t *q = st32 + (a[u] >> 2);
          w0[u] = q[0];
          w1[u] = q[1];
          w2[u] = q[2];
        }
        if (nnib + U > 15) fold();
        if (cc.nrow + U > 255) {
          fold();
          cc.flush(cnt, S, c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t s0 = __builtin_amdgcn_alignbyte(w1[u], w0[u], a[u]) & bm[u].x;
          const uint32_t s1 = __builtin_amdgcn_alignbyte(w2[u], w1[u], a[u]) & bm[u].y;
          nac[0] += __builtin_amdgcn_perm(0u, 0x10000100u, s0);
          ntg[0] += __builtin_amdgcn_perm(0x10000001u, 0u, s0);
          nac[1] += __builtin_amdgcn_perm(0u, 0x10000100u, s1);
          ntg[1] += __builtin_amdgcn_perm(0x10000001u, 0u, s1);
          nv[0] += bm[u].x & 0x01010101u;
          nv[1] += bm[u].y & 0x01010101u;
        }
        nnib += U;
        cc.nrow += U;
      };
      if (!(dbg & 1)) {
        for (int k0 = lo + par; k0 < hi; k0 += P * U)
          batch(reinterpret_cast<const uint8_t *>(rows), 24, k0, std::integral_constant<int, U>{});
        // extra rows (rare): one at a time, no padding
        const int nx = (int)min(n_xrow[b], (unsigned)C::kExtra);
        for (int k0 = par; k0 < nx; k0 += P)
          batch(reinterpret_cast<const uint8_t *>(xrow), 8, k0, std::integral_constant<int, 1>{});
      }
      fold();
      // the column's totals in all eight of its lanes (quad sums, then + the half-row mirror:
      // lane i <-> 7 - i); lane par keeps locus c + par (= t) for the decision.  Bytes cannot
      // overflow while the column's reads sum to <= 255; otherwise (deep pileups) each lane
      // flushes its own counts into the LDS words.
      {
        auto csum = [](uint32_t x) {
          x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm 1 0 3 2
          x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // quad_perm 2 3 0 1
          x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
          return x;
        };
        // a column deeper than 255 rows: each lane flushes its own counts instead
        const uint32_t nq = csum(cc.nrow);
        if (nq > 255) {
          cc.flush(cnt, S, c);
        } else {
          const int h = par >> 2, sh = 8 * (par & 3);
          const uint32_t a0 = csum(cc.ca[0]), a1 = csum(cc.ca[1]), c0 = csum(cc.cc[0]), c1 = csum(cc.cc[1]);
          const uint32_t t0 = csum(cc.ct[0]), t1 = csum(cc.ct[1]), g0 = csum(cc.cg[0]), g1 = csum(cc.cg[1]);
          const uint32_t v0 = csum(cc.cv[0]), v1 = csum(cc.cv[1]);
          regc[0] = ((h ? a1 : a0) >> sh) & 0xFFu;
          regc[1] = ((h ? c1 : c0) >> sh) & 0xFFu;
          regc[2] = ((h ? t1 : t0) >> sh) & 0xFFu;
          regc[3] = ((h ? g1 : g0) >> sh) & 0xFFu;
          regc[4] = (((h ? v1 : v0) >> sh) & 0xFFu) - regc[0] - regc[1] - regc[2] - regc[3];
        }
      }
      // ---- E: thread GQ_EV_T0 + k: the MD events of read k; the builders of general
      //      reads: their complex segment loci (into the LDS histogram, GermSink)
      if (!(dbg & 2)) {
        GermSink<T, 0> sink{cnt, L0, &ctr->err, &ctr->err_pos};
        if (rs_c.general) {  // segments: the complex loci (count segments are column rows)
          for (int32_t q = 0; q < rs_c.nseg; ++q) {
            const uint32_t w0 = evs[rs_c.seg + 2 * q], w1 = evs[rs_c.seg + 2 * q + 1];
            const int32_t a = rs_c.s + (int32_t)(w0 & 0xFFFFu), bq = a + (int32_t)(w0 >> 16);
            if (bq <= 0 || a >= T || (w1 >> 16) == kSegCountK) continue;
            for (int32_t l = a > 0 ? a : 0; l < (bq < T ? bq : T); ++l) sink.complex_i(l);
          }
        }
        const int k = t - GQ_EV_T0;
        if (k >= 0 && k < nch && !(dbg & 64)) {
          const uint32_t *d = rows + 6 * k;
          const uint32_t d4 = d[4];
          const int32_t nmd = (int32_t)(d4 & 0xFFFFu);
          if ((d4 & 0x80000000u) && nmd > 0) {
            const int32_t s = (int32_t)d[5], x1 = L1 - L0;
            const int32_t e0 = (int32_t)((d4 >> 16) & 0x7FFFu);
            for (int32_t k0 = 0; k0 < nmd; k0 += 4) {  // events are sorted by offset; 4 loads in flight
              uint32_t w4[4];
#pragma unroll
              for (int u = 0; u < 4; ++u) w4[u] = evs[e0 + min(k0 + u, nmd - 1)];
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const int32_t l = s + (int32_t)(w4[u] >> 16);
                if (k0 + u < nmd && l >= 0 && l < x1) sink.event_i(l, (uint8_t)w4[u], (uint8_t)(w4[u] >> 8), 0);
              }
            }
          }
        }
      }
    }
    const uint64_t te = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // DMA(i + 1) has landed (this wave's part)
    __syncthreads();                                   // 1: histogram of tile i complete
    const uint64_t tb = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    if (t < NCOL) hist[b][t] = 0;  // buffer parity b is next built for tile i + 2
    if (t == 0) n_xrow[b] = 0;
    Tile t2{};
    const bool has2 = i + 2 < i1, has1 = i + 1 < i1;
    if (has2) {
      t2 = unpack(d2);
      d2 = load_desc(i + 3);
      issue(t2, b);
    }
    const int vote = has1 ? build(tn, b ^ 1, rs_n) : 0;
    // ---- F: decision of tile i, then its histogram words are zeroed for tile i + 1
    // (each thread zeroes the words of its own locus after reading them)
    if (!slow_c)
      germline_decide<T, true>(cnt, tc, i, false, n_samples, threshold, emit_ref, emit_no_call, recs, cplx, out,
                               visited, amb, ties, regc);
    const uint64_t tf = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    const int slow_n = __syncthreads_or(vote);  // 2: rows of tile i + 1 complete
    if (has1 && slow_n && t == 0) slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)(i + 1);
    if (dbg & 16) {
      const uint64_t now = __builtin_readcyclecounter();
      clk[0] += now - ta;  // tile total
      clk[1] += te - ta;   // scan + column pass + per-read pass
      clk[2] += tb - te;   // vmcnt + barrier 1
      clk[3] += tf - tb;   // DMA issue + next tile's rows + decision
      clk[4] += 1;
      clk[5] += now - tf;  // barrier 2
    }
    tc = tn;
    tn = t2;
    rs_c = rs_n;
    slow_c = has1 ? slow_n : 1;
  }
  add_run_counters(ctr, visited, amb, ties, (int)blockIdx.x);
  if (t == 0) {  // this workgroup's partition counts (may exceed the capacity: host retry)
    ctr->part[0][blockIdx.x] = outn[0];
    ctr->part[1][blockIdx.x] = outn[1];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((dbg & 16) && lane == 0 && clk[4]) {
    atomicAdd(&ctr->prof[0], (unsigned long long)clk[0]);
    atomicAdd(&ctr->prof[1], (unsigned long long)clk[1]);
    atomicAdd(&ctr->prof[2], (unsigned long long)clk[2]);
    atomicAdd(&ctr->prof[3], (unsigned long long)clk[3]);
    atomicAdd(&ctr->prof[7], (unsigned long long)clk[4]);
    atomicAdd(&ctr->prof[4], (unsigned long long)clk[5]);
    atomicAdd(&ctr->prof[5], (unsigned long long)clk[6]);
  }
}

// The tiles germline_cols handed over: every read walked lane-per-read (walk_read_lane,
// PileupElement.scala:68-248) into the LDS histogram, bases from HBM.  A grid-stride loop
// over the list ctr->n_slow long.
template <int T>
// four waves per SIMD (<= 128 VGPRs, 163 unconstrained): 0.092 -> 0.080 ms on the bench shard
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void germline_walk(const Tile *__restrict__ tiles, const int32_t *__restrict__ slow,
                                                        DevReads R, int threshold, int emit_ref, int emit_no_call,
                                                        CallRec *__restrict__ recs, ComplexItem *__restrict__ cplx,
                                                        OutGeom og,
                                                        Counters *ctr) {
  constexpr int S = T + 2 * kGuard;
  __shared__ __attribute__((aligned(16))) uint32_t cnt[W_N * S];
  const int64_t n = (int64_t)ctr->n_slow;
  const int part = kPartsCols + (int)((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kPartsWalk - 1));
  GlobalOut out{ctr, part, {og.slot(0, part, 0), og.slot(1, part, 0)}, {og.capB[0], og.capB[1]}};
  unsigned visited = 0, amb = 0, ties = 0;
  for (int64_t q = blockIdx.x; q < n; q += gridDim.x) {
    const int64_t tid_tile = slow[q];
    const Tile tl = tiles[tid_tile];
    const bool wide = (tl.re - tl.rb) >= 65535;
    uint4 *c4 = reinterpret_cast<uint4 *>(cnt);
    for (int i = threadIdx.x; i < W_N * S / 4; i += blockDim.x) c4[i] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    if (!wide) {
      GermSink<T, 0> sink{cnt, tl.L0, &ctr->err, &ctr->err_pos};
      for (int64_t r = tl.rb + threadIdx.x; r < tl.re; r += blockDim.x) walk_read_lane(R, r, tl.L0, tl.L1, sink);
    }
    __syncthreads();
    germline_decide<T>(cnt, tl, tid_tile, wide, R.n_samples, threshold, emit_ref, emit_no_call, recs, cplx, out,
                       visited, amb, ties);
    __syncthreads();
  }
  add_run_counters(ctr, visited, amb, ties, (int)blockIdx.x);
}
