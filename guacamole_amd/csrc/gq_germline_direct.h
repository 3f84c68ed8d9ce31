// gq_germline_direct.h — germline_direct: the germline-threshold pileup kernel straight from the
// resident reads, with no projection.  Its inputs are the SoA arrays plus the upload-time
// derivation every caller needs (read_prep: each read's shape and the read bases under its MD
// events; block_index: each 512-locus block's read window), so one germline call over freshly
// derived reads streams the sequence pool once: there is no 4-bit projection to write and read
// back, no row assignment, and no separate A/C/G/T/N scan of the pool (pool_clean).
//
// One WAVE per 512-locus tile (aligned to a 512-locus block B0), four waves per workgroup, each
// on its own tiles, as germline_proj.  Lane l owns the 8-locus column [B0 + 8l, B0 + 8l + 8).
// The tile's read window (SlidingWindow.scala:83-128: every read overlapping the block, in start
// order) goes through in chunks of up to kSlots runs:
//
//   runs     lane = read, 64 reads a round: the read's fields in one round of coalesced loads;
//            each run of its Match/Mismatch elements in the block (one for a [S|H]* M [S|H]*
//            read, a general CIGAR's count segments from general_segments: PileupElement.scala:
//            68-248) becomes an 8-byte slot in LDS (first / end locus relative to B0, the pool
//            offset of the column's bytes relative to the tile's base); a slot marks the columns
//            it spans in two per-column words (the last slot starting at or before the column,
//            the first slot ending in or after it: LDS max / min).  A general CIGAR's complex
//            ranges (insertion / deletion anchors, clipped N-skips) and MidDeletion ranges go
//            into LDS difference words; MD events (PileupElement.scala:108-118, Pileup.scala:
//            157-165) into the reference-base mask and the event read-base counts, as
//            germline_proj's sparse entries do.
//   counts   lane l walks only the slots that can cover its column: [first slot ending past the
//            column's first locus, last slot starting before its end] — a prefix maximum and a
//            suffix minimum of the per-column words.  One unaligned 8-byte buffer load per slot
//            (three batches of four in flight), the loci outside the run masked, the bases
//            counted in SWAR registers through v_perm tables (A C T G in nibbles folded into
//            bytes every 12 slots, N in bytes; the DEEP instantiation widens into 16-bit pairs
//            every 240).  The same v_perm checks every counted byte is one of A C G T N; a block
//            with any other byte (an "other" base allele), a read without MD, a CIGAR the
//            segments cannot express, a round of more than kSlots runs, or more than 65535 window
//            reads goes to germline_walk, which is exact for every read.
//
// Then each lane makes the GermlineThreshold decision (GermlineThresholdCaller.scala:90-179) for
// its eight loci exactly as germline_proj does (variant candidates, Ref / NoCall records and
// complex items leave the same way), with its N count from the SWAR registers.
#pragma once

#include "gq_kernels.h"

// (included inside gq_pileup.hip's anonymous namespace, after gq_germline_proj.h)

#ifndef GQ_DIR_WPE
#define GQ_DIR_WPE 4  // waves per SIMD the register budget must allow
#endif
#ifndef GQ_DIR_MASKED
#define GQ_DIR_MASKED 0
#endif
#ifndef GQ_DIR_EVPF
#define GQ_DIR_EVPF 0
#endif
#ifndef GQ_DIR_U
#define GQ_DIR_U 4
#endif
struct DirCfg {
  static constexpr int kT = 512;       // loci per tile: 64 lanes x 8 loci
  static constexpr int kWaves = 4;     // waves per workgroup, each on its own tiles
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kU = GQ_DIR_U;  // slots per batch (their loads issued before use; 240 % kU == 0)
  static constexpr int kRound = 64;    // window reads per round (a lane each)
  static constexpr int kSlots = 256;   // runs per chunk (LDS slots)
  static constexpr int64_t kMaxWin = 65535;  // window reads (16-bit counts); more: germline_walk
  static constexpr int64_t kShallow = 255;   // window reads of the byte-count instantiation
};

// (byte_range_mask, wave_incl_max_i, wave_suffix_min_i: gq_direct_common.h)

// DEEP = false: every tile whose window holds at most kShallow reads (per-locus counts fit bytes:
// no 16-bit widening; event counts in bytes); deeper tiles are listed (deep, ctr->n_deep) for the
// DEEP instantiation, whose waves take them from the list, widen the counts into 16-bit pairs
// every 240 slots, and write into the walker's output partitions.
template <bool DEEP>
__global__ __launch_bounds__(DirCfg::kThreads) __attribute__((amdgpu_waves_per_eu(GQ_DIR_WPE))) void germline_direct(
    const Tile *__restrict__ tiles, int64_t n_tiles, DevReads R, int threshold, int emit_ref, int emit_no_call,
    CallRec *__restrict__ recs, ComplexItem *__restrict__ cplx, OutGeom og, Counters *ctr, int32_t *__restrict__ slow,
    int32_t *__restrict__ deep, int dbg) {
  // dbg (diagnostics, env GQ_DBG; results are wrong when set): 1 skip the base loads, 4 skip the
  // decision, 16 phase clocks, 32 skip the counting, 64 skip the MD events, 128 skip the events'
  // read-base loads
  using C = DirCfg;
  constexpr int T = C::kT, U = C::kU;
  constexpr int EW = DEEP ? 2 * T : T;  // event words: 16-bit pairs (DEEP) or four bytes per locus
  // per locus, locus x of the block at word ix(x) = (x & 7) * 64 + (x >> 3) (a lane's eight loci
  // on 64 consecutive words each): event read bases (DEEP: A | C << 16 at [x], T | G << 16 at
  // [T + x]; else A | C << 8 | T << 16 | G << 24 at [x]), MD bits 0-3 | complex diff << 16,
  // MidDeletion diffs
  __shared__ __attribute__((aligned(16))) uint32_t evw[C::kWaves][EW];
  __shared__ __attribute__((aligned(16))) uint32_t mkw[C::kWaves][T];
  __shared__ __attribute__((aligned(16))) uint32_t dlw[C::kWaves][T];
  // the chunk's slots (first locus - B0 | end locus - B0 << 16 as int16s, pool offset of B0's
  // column relative to the tile's base) and per column the last slot starting at or before it /
  // the first slot ending in or after it
  __shared__ __attribute__((aligned(16))) uint2 rcw[C::kWaves][C::kSlots];
  __shared__ int32_t hxw[C::kWaves][64], hnw[C::kWaves][64];
  __shared__ unsigned outn[2];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint32_t *ev = evw[wave], *mk = mkw[wave], *dl = dlw[wave];
  uint2 *rc = rcw[wave];
  int32_t *hx = hxw[wave], *hn = hnw[wave];
  auto ix = [](int32_t x) { return ((x & 7) << 6) | (x >> 3); };
  auto zero_words = [&]() {  // 16-byte stores, lane l at 16 l (no conflicts)
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    uint4 *e4 = reinterpret_cast<uint4 *>(ev), *m4 = reinterpret_cast<uint4 *>(mk), *d4 = reinterpret_cast<uint4 *>(dl);
#pragma unroll
    for (int q = 0; q < EW / 256; ++q) e4[64 * q + lane] = z4;
    m4[lane] = z4; m4[64 + lane] = z4; d4[lane] = z4; d4[64 + lane] = z4;
  };
  zero_words();
  if (threadIdx.x < 2) outn[threadIdx.x] = 0;
  __syncthreads();
  const int64_t per = n_tiles / gridDim.x, extra = n_tiles % gridDim.x;
  const int64_t i0 = blockIdx.x * per + min((int64_t)blockIdx.x, extra);
  const int64_t i1 = i0 + per + ((int64_t)blockIdx.x < extra ? 1 : 0);
  // output partitions: the workgroup's own (LDS counters), or the DEEP waves' walker partitions
  const int part = DEEP ? kPartsCols + (int)((blockIdx.x * C::kWaves + wave) & (kPartsWalk - 1)) : (int)blockIdx.x;
  const unsigned long long obase[2] = {og.slot(0, part, 0), og.slot(1, part, 0)};
  const unsigned long long ocap[2] = {og.cap(0, part), og.cap(1, part)};
  auto reserve = [&](int which, unsigned n) -> unsigned long long {
    return DEEP ? wave_reserve(&ctr->part[which][part], n) : (unsigned long long)wave_reserve_lds_n(outn + which, n);
  };
  unsigned visited = 0, amb = 0, ties = 0;
  uint64_t clk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool multi_sample = R.n_samples > 1;
  const int64_t thr1 = (int64_t)threshold + 1;
  const uint32_t thr1u = (uint32_t)(thr1 < 0 ? 0 : thr1 > 101 ? 101 : thr1);
  const uint32_t thr1b = thr1u & 0xFFu;
  auto passes = [=](uint32_t count, uint32_t depth) { return (count & 0xFFFFu) * 100u >= thr1b * (depth & 0xFFFFu); };
  // a tile's record: dword d on lane d < 16, every field read into scalars at once (a VGPR read
  // lane by lane later must not live across the tile: the register allocator may spill it under a
  // partial exec mask, which keeps only the active lanes' values)
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc((void *)tiles, (short)0, (int)(64 * n_tiles), 0x00020000);
  const uint32_t tvo = lane < 16 ? 4u * (uint32_t)lane : 0x80000000u;
  auto fetch = [&](int64_t t) -> uint32_t { return __builtin_amdgcn_raw_buffer_load_b32(trs, (int)tvo, (int)(64 * t), 0); };
  auto f32 = [](uint32_t rec, int d) { return (uint32_t)__builtin_amdgcn_readlane((int)rec, d); };
  auto f64 = [&](uint32_t rec, int d) { return (int64_t)((uint64_t)f32(rec, d) | ((uint64_t)f32(rec, d + 1) << 32)); };
  const int32_t colr = 8 * lane;  // this lane's column, relative to the block: loci [B0 + colr, B0 + colr + 8)
  // DEEP: the listed tiles, a wave at a time over the grid; else this workgroup's run of tiles
  const int64_t n_deep = DEEP ? (int64_t)min(ctr->n_deep, (unsigned long long)n_tiles) : 0;
  const int64_t iend = DEEP ? n_deep : i1, istep = DEEP ? (int64_t)gridDim.x * C::kWaves : C::kWaves;
  int64_t i = DEEP ? (int64_t)blockIdx.x * C::kWaves + wave : i0 + wave;
  for (; i < iend; i += istep) {
    const uint64_t t_a = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    const int64_t tid = DEEP ? (int64_t)__builtin_amdgcn_readfirstlane(deep[i]) : i;  // the tile
    // Tile: ordinal0 dw 0-1, rb 2-3, re 4-5, contig 6, L0 7, L1 8
    const uint32_t rec = fetch(tid);
    const int64_t ord0 = f64(rec, 0);
    const int32_t tcontig = (int32_t)f32(rec, 6);
    const int32_t L0 = (int32_t)f32(rec, 7), L1 = (int32_t)f32(rec, 8);
    const int64_t rb = f64(rec, 2), re = f64(rec, 4);
    const int32_t B0 = L0 & ~(T - 1);
    const int32_t col = B0 + colr;
    if (re <= rb) continue;  // no reads: nothing visited
    if (re - rb > C::kMaxWin) {
      if (lane == 0) slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)tid;
      continue;
    }
    if (!DEEP && re - rb > C::kShallow) {  // counts past a byte: the DEEP instantiation
      if (lane == 0) deep[atomicAdd(&ctr->n_deep, 1ull)] = (int32_t)tid;
      continue;
    }
    // ---- counters: nibbles (A | C << 4 per byte in nac, T | G << 4 in ntg; loci 0-3 of the
    //      column in [0], 4-7 in [1]) folded into byte counters every 12 slots, N straight into
    //      bytes; DEEP: widened into 16-bit pairs (loci 2q, 2q + 1 in w?[q]) every 240 slots
    uint32_t ca[2] = {0, 0}, cc[2] = {0, 0}, ct[2] = {0, 0}, cg[2] = {0, 0}, cn[2] = {0, 0};
    uint32_t wA[4] = {0, 0, 0, 0}, wC[4] = {0, 0, 0, 0}, wT[4] = {0, 0, 0, 0}, wG[4] = {0, 0, 0, 0},
             wN[4] = {0, 0, 0, 0};
    uint32_t nac[2] = {0, 0}, ntg[2] = {0, 0};
    int nn = 0, since = 0;
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
      if (!DEEP) return;
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
      w2(wN, cn);
    };
    bool bad = false;   // this lane saw a read the kernel cannot take (the block goes to the walker)
    uint32_t badb = 0;  // counted bytes other than A C G T N
    const uint64_t t_b = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    // the round's fields (lane = read), loaded one round ahead
    struct Fields {
      int32_t s, e, nmd, ld;
      int64_t so, mo;
    };
    auto load_fields = [&](int64_t c0) {
      Fields f{0, 0, 0, 0, 0, 0};
      const int64_t r = c0 + lane;
      if (r < re) {
        f.s = R.start[r];
        f.e = R.end[r];
        f.so = R.seq_off[r];
        f.ld = R.lead[r];
        f.nmd = R.n_md[r];
        f.mo = R.md_off[r];
      }
      return f;
    };
    // the tile's pool base: the lowest pool offset of its first round's reads, less 8 (a column
    // may start up to 7 loci before its run); a run whose bytes lie below it or 2^31 past it
    // sends the block to the walker.  A load of a dead (slot, column) pair takes an offset past
    // the buffer's range and reads 0 without touching memory.
    int64_t tbase = 0;
    bool defer = false;
    __amdgpu_buffer_rsrc_t srs;
    Fields nf = load_fields(rb);
    int64_t c0 = rb;
    bool first_round = true;
    // GQ_DIR_EVPF: the next round's first four MD events, issued at the end of a round (its
    // fields have arrived by then), so a round does not start with a dependent load
    uint32_t pv4[4] = {0u, 0u, 0u, 0u};
    int64_t pv_c0 = -1;  // the round pv4 belongs to
    while (c0 < re) {  // ---- a chunk: rounds while their runs fit kSlots slots, then the counting
      const uint64_t t_round = (dbg & 16) ? __builtin_readcyclecounter() : 0;
      hx[lane] = -1;
      hn[lane] = 0x7FFFFFFF;
      int32_t nslot = 0;
      while (c0 < re) {
        const uint64_t t_rd = (dbg & 16) ? __builtin_readcyclecounter() : 0;
        const int64_t r = c0 + lane;
        const bool valid = r < re;
        const Fields f = nf;
        const int32_t s = f.s, e = f.e, nmd = f.nmd, ld = f.ld;
        const int64_t so = f.so, mo = f.mo;
        const bool nomd = valid && nmd < 0;  // MappedRead.scala:57-60: the walker raises it where it applies
        const bool gen = valid && !nomd && ld < 0;
        // runs of this read in the block: one for a simple read, the count segments of a general one
        uint32_t nrun = valid && !nomd && !gen && e > B0 && s < B0 + T ? 1u : 0u;
        // the read's first four MD events, in flight while its runs are placed
        const bool evr = valid && !nomd && nmd > 0 && s < B0 + T && !(dbg & 64);
        uint32_t v4[4] = {0u, 0u, 0u, 0u};
        auto load_ev = [&](int32_t k0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v4[j] = R.md_ev[mo + (k0 + j < nmd ? k0 + j : nmd - 1)];
        };
        // an event's read base where it is A C T G (an N there is counted with the bases)
        auto ev_add = [&](int32_t l, uint8_t base) {
          const int cat = base_cat(base);
          if (cat < 4) {
            const int32_t x = ix(l - B0);
            if (DEEP) atomicAdd(&ev[(cat >> 1) * T + x], 1u << (16 * (cat & 1)));
            else atomicAdd(&ev[x], 1u << (8 * cat));
          }
        };
        if (evr) {
          if (GQ_DIR_EVPF && pv_c0 == c0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v4[j] = pv4[j];
          } else {
            load_ev(0);
          }
        }
        // (a general read: slots for its (M|=|X) operations, read_prep's bound on its count
        // segments; those outside the block stay empty)
        if (gen && e > B0 && s < B0 + T) nrun = (uint32_t)min(-1 - ld, C::kSlots);
        const uint32_t incl = wave_incl_scan(nrun);
        const int32_t total = (int32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint64_t t_f = (dbg & 16) ? __builtin_readcyclecounter() : 0;
        if (nslot > 0 && nslot + total > C::kSlots) break;  // (the round opens the next chunk)
        if (total > C::kSlots) {  // (one round's runs past the slots: the walker)
          bad = true;
          c0 = re;
          break;
        }
        if (c0 + C::kRound < re) nf = load_fields(c0 + C::kRound);  // the next round's, in flight
        if (first_round) {  // the tile's pool base, from the first round's reads
          int64_t so_min = valid ? so : INT64_MAX;
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_xor(so_min, d, 64);
            so_min = o < so_min ? o : so_min;
          }
          defer = !DEEP && so_min < 8;  // the pool's head: the DEEP instantiation (shifted loads)
          tbase = so_min >= 8 ? so_min - 8 : 0;  // (uniform: the buffer descriptor in scalar registers)
          tbase = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)tbase >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)tbase));
          const int64_t span = R.seq_cap - tbase;
          srs = __builtin_amdgcn_make_buffer_rsrc((void *)(R.seq + tbase), (short)0,
                                                  (int)(span < 0x7FFFFFFF ? span : 0x7FFFFFFF), 0x00020000);
          first_round = false;
        }
        bad = bad || nomd ||
              (valid && (so < tbase || so + (ld > 0 ? ld : 0) + (e > s ? e - s : 0) + 16384 + 1024 - tbase >= 0x7FFFFFF0ll));
        // the runs into their slots, each marking the columns it spans
        int32_t slot = nslot + (int32_t)(incl - nrun);
        auto put = [&](int32_t a, int32_t b, int64_t p) {  // loci [a, b) whose bases start at pool offset p
          const int32_t s16 = min(max(a - B0, -32768), 32767), e16 = min(max(b - B0, -32768), 32767);
          const int32_t K = (int32_t)(p - tbase - (int64_t)(a - B0));  // pool offset of locus B0 (a virtual one), from the base
          rc[slot] = make_uint2((uint32_t)(uint16_t)s16 | ((uint32_t)(uint16_t)e16 << 16), (uint32_t)K);
          atomicMax(&hx[min(max(s16, 0), T - 1) >> 3], slot);
          atomicMin(&hn[min(max(e16 - 1, 0), T - 1) >> 3], slot);
          ++slot;
        };
        if (nrun && !gen) put(s, e, so + (ld > 0 ? ld : 0));
        if (gen && e > B0 && s < B0 + T) {  // count segments into slots; complex / MidDeletion ranges as differences over the block
          const int32_t slot_end = slot + (int32_t)nrun;
          const bool ok = general_segments(R, r, [&](uint32_t kind, int32_t ro, int32_t len, int32_t sp, int32_t) {
            const int32_t a = s + ro, b = a + len;
            if (b <= B0 || a >= B0 + T) return;
            if (kind == kSegCount) {
              if (slot < slot_end) put(a, b, so + sp);
              else bad = true;  // (more count segments than read_prep's bound: not expected)
              if (evr) {  // the segment's events in the block: their read bases
                const int32_t x0 = a > B0 ? a : B0, x1 = b < B0 + T ? b : B0 + T;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                  const int32_t l = s + (int32_t)(v4[j] >> 8);
                  if (j < nmd && l >= x0 && l < x1) ev_add(l, R.seq[so + sp + (l - a)]);
                }
                for (int32_t k = 4; k < nmd; ++k) {
                  const int32_t l = s + (int32_t)(R.md_ev[mo + k] >> 8);
                  if (l >= x1) break;
                  if (l >= x0) ev_add(l, R.seq[so + sp + (l - a)]);
                }
              }
            } else {
              const bool mid = kind == kSegMidDel;  // MidDeletion elements: their own count
              uint32_t *dw = mid ? dl : mk;
              const int32_t x0 = a > B0 ? a : B0, x1 = b < B0 + T ? b : B0 + T;
              atomicAdd(&dw[ix(x0 - B0)], mid ? 1u : 1u << 16);
              if (x1 < B0 + T) atomicAdd(&dw[ix(x1 - B0)], mid ? 0xFFFFFFFFu : 0xFFFF0000u);
            }
          });
          bad = bad || !ok;
          for (; slot < slot_end; ++slot) rc[slot] = make_uint2(0u, 0u);  // empty: no column reads it live
        }
        if (dbg & 16) {  // round phase clocks: to the fields and run counts | slots and segments
          const uint64_t t_g = __builtin_readcyclecounter();
          clk[6] += t_f - t_rd;
          clk[7] += t_g - t_f;
        }
        // MD events in the block: the MD reference base's bit, and (a simple read; a general
        // one's went with its count segments) the read base's count: the base at lead + offset
        // of the (M|=|X) run (lead + run <= sequence: read_prep's shape test)
        if (evr) {
          for (int32_t k0 = 0;;) {
            bool past = false;
            uint8_t b4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int32_t o = (int32_t)(v4[j] >> 8);
              b4[j] = !gen && o < e - s ? ((dbg & 128) ? (uint8_t)'A' : R.seq[so + ld + o]) : (uint8_t)0;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int32_t l = s + (int32_t)(v4[j] >> 8);
              past = past || l >= B0 + T;
              if (k0 + j >= nmd || l < B0 || l >= B0 + T) continue;
              const uint32_t m = std_bit((uint8_t)(v4[j] & 0xFFu));
              if (m) atomicOr(&mk[ix(l - B0)], m);
              if (b4[j]) ev_add(l, b4[j]);
            }
            k0 += 4;
            if (past || k0 >= nmd) break;
            load_ev(k0);
          }
        }
        if (GQ_DIR_EVPF && c0 + C::kRound < re) {  // the next round's first events (nf arrived)
          const bool nv = c0 + C::kRound + lane < re && nf.nmd > 0 && nf.s < B0 + T;
#pragma unroll
          for (int j = 0; j < 4; ++j) pv4[j] = nv ? R.md_ev[nf.mo + (j < nf.nmd ? j : nf.nmd - 1)] : 0u;
          pv_c0 = c0 + C::kRound;
        }
        nslot += total;
        c0 += C::kRound;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const uint64_t t_r = (dbg & 16) ? __builtin_readcyclecounter() : 0;
      // ---- this lane's slots: [first slot ending past its column's first locus, last slot
      //      starting before its column's end]
      int32_t last = wave_incl_max_i(hx[lane]);
      int32_t first = wave_suffix_min_i(hn[lane]);
      if (GQ_DIR_GROUP > 1) {  // a group's lanes walk the group's slots together (first / last are
                               // monotone in the column): one slot per step and group, so a load
                               // instruction touches one read's bytes per group, not one per lane
        first = __shfl(first, lane & ~(GQ_DIR_GROUP - 1), 64);
        last = __shfl(last, lane | (GQ_DIR_GROUP - 1), 64);
      }
      const int32_t nl = last >= first ? last - first + 1 : 0;
      int32_t kmax = nl;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) kmax = max(kmax, __shfl_xor(kmax, d, 64));
      kmax = (dbg & 32) ? 0 : __builtin_amdgcn_readfirstlane(kmax);  // (dbg & 32: no counting)
      // the slot schedule: iteration k takes the slot s of [first, first + kmax) with s = k (mod
      // kmax), so every group reaches a slot at the same iteration (k = s mod kmax) and one load
      // instruction reads a read's bytes for all the groups its run covers (the lines it touches
      // are fetched once, while they are hot); t0 = the offset of iteration 0
      const int32_t t0 = (GQ_GDIR_ROT && kmax > 0 && nl > 0) ? (kmax - first % kmax) % kmax : 0;
      // a batch: U slots' 8-byte loads, all issued before any is used; mt = the column's loci
      // inside the run [a, b)
      auto issue = [&](int32_t k0, uint2 (&x)[U], uint32_t (&mt)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int32_t k = k0 + u;
          int32_t t = t0 + k;  // (GQ_GDIR_ROT) the lane's slot offset at iteration k
          t = t >= kmax ? t - kmax : t;
          const bool mine = GQ_GDIR_ROT ? (k < kmax && t < nl) : k < nl;
          const uint2 d = rc[mine ? first + (GQ_GDIR_ROT ? t : k) : 0];
          const int32_t s16 = (int32_t)(int16_t)(d.x & 0xFFFFu), e16 = (int32_t)(int16_t)(d.x >> 16);
          const int32_t a = min(max(s16 - colr, 0), 8), b = min(max(e16 - colr, 0), 8);
          const bool live = mine && b > a && !(dbg & 1);
          // (vi >= -7 for a live pair, byte a being the run's; < 0 only at the pool's head, whose
          // tiles the DEEP instantiation takes: its load clamped to the base and shifted back)
          const int32_t vi = (int32_t)d.y + colr;
          const uint32_t vo = live ? (uint32_t)(DEEP ? max(vi, 0) : vi) : 0x80000000u;
          if (GQ_DIR_MASKED) {  // dead lanes off the load (exec-masked) instead of out of range
            x[u] = make_uint2(0u, 0u);
            if (live) {
              const auto w = __builtin_amdgcn_raw_buffer_load_b64(srs, (int)vo, 0, 0);
              x[u] = make_uint2(w[0], w[1]);
            }
          } else {
            const auto w = __builtin_amdgcn_raw_buffer_load_b64(srs, (int)vo, 0, 0);
            x[u] = make_uint2(w[0], w[1]);
          }
          mt[u] = live ? (uint32_t)a | ((uint32_t)b << 4) | (DEEP ? (uint32_t)max(-vi, 0) << 8 : 0u) : 0u;
        }
      };
      auto count = [&](const uint2 (&x)[U], const uint32_t (&mt)[U]) {
        if (nn + U > 15) fold();
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint64_t m = byte_range_mask((int32_t)(mt[u] & 15u), (int32_t)((mt[u] >> 4) & 15u));
          uint64_t w64 = (uint64_t)x[u].x | ((uint64_t)x[u].y << 32);
          if (DEEP) w64 <<= (mt[u] >> 5) & 56u;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t wh = (uint32_t)(w64 >> (32 * h)), mh = (uint32_t)(m >> (32 * h));
            const uint32_t xc = wh & 0x07070707u;
            // the byte a code stands for: A 1, C 3, T 4, N 6, G 7 (codes 0 2 5: none)
            const uint32_t ex = __builtin_amdgcn_perm(0x474EFF54u, 0x43FF41FFu, xc);
            badb |= (dbg & 1) ? 0u : (wh ^ ex) & mh;
            const uint32_t cd = xc & mh;
            nac[h] += __builtin_amdgcn_perm(0u, 0x10000100u, cd);  // A -> 0x01, C -> 0x10
            ntg[h] += __builtin_amdgcn_perm(0x10000001u, 0u, cd);  // T -> 0x01, G -> 0x10
            cn[h] += __builtin_amdgcn_perm(0x00010000u, 0u, cd);   // N -> 0x01
          }
        }
        nn += U;
        since += U;
        if (DEEP && since == 240) {  // uniform: bytes hold 240 slots at most
          fold();
          widen();
          since = 0;
        }
      };
      if (kmax > 0) {  // two batches in flight while one is counted
        uint2 xa[U], xb2[U], xc2[U];
        uint32_t ma[U], mb[U], mc[U];
        issue(0, xa, ma);
        issue(U, xb2, mb);
        for (int32_t k0 = 0;; k0 += 3 * U) {
          issue(k0 + 2 * U, xc2, mc);
          count(xa, ma);
          if (k0 + U >= kmax) break;
          issue(k0 + 3 * U, xa, ma);
          count(xb2, mb);
          if (k0 + 2 * U >= kmax) break;
          issue(k0 + 4 * U, xb2, mb);
          count(xc2, mc);
          if (k0 + 3 * U >= kmax) break;
        }
      }
      if (dbg & 16) {  // phase clocks: the chunk's runs (fields, slots, events) | its counting
        const uint64_t t_s = __builtin_readcyclecounter();
        clk[2] += t_r - t_round;
        clk[3] += t_s - t_r;
      }
    }
    fold();
    widen();
    const uint64_t t_c = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    if (__ballot(bad || badb != 0) != 0) {  // the walker takes the block (exact for every read)
      zero_words();
      if (lane == 0) {
        if (defer) deep[atomicAdd(&ctr->n_deep, 1ull)] = (int32_t)tid;
        else slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)tid;
      }
      continue;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t kinds = 0, nrec = 0, ncpx = 0, livem = 0, ambm = 0;
    int32_t mid0 = 0;  // MidDeletion elements entering this lane's first locus
    // locus j's count: a 16-bit half of w (DEEP), else a byte of c
    auto cnt = [](const uint32_t (&w)[4], const uint32_t (&c)[2], int j) {
      if (DEEP) {
        const int q = j >> 1;
        const uint32_t x = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
        return (x >> (16 * (j & 1))) & 0xFFFFu;
      }
      return (c[j >> 2] >> (8 * (j & 3))) & 0xFFu;
    };
    // the reference-base mask of a locus: MD bits, plus each base with more Match/Mismatch
    // elements than events (an element without an event reads the reference)
    auto ref_mask = [](uint32_t mw, uint32_t eac, uint32_t etg, uint32_t cA, uint32_t cC, uint32_t cT, uint32_t cG) {
      return (mw & 15u) | (cA > (eac & 0xFFFFu) ? 1u : 0u) | (cC > (eac >> 16) ? 2u : 0u) |
             (cT > (etg & 0xFFFFu) ? 4u : 0u) | (cG > (etg >> 16) ? 8u : 0u);
    };
    if (!(dbg & 4)) {
      // complex elements per locus: prefix of the range differences over the block
      int32_t run = 0, mrun0 = 0;
      uint32_t m8[8], d8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        m8[j] = mk[64 * j + lane];
        d8[j] = dl[64 * j + lane];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        run += (int32_t)m8[j] >> 16;
        mrun0 += (int32_t)d8[j];
      }
      int32_t ncx_run = (int32_t)wave_incl_scan((uint32_t)run) - run;  // before this lane's loci
      mid0 = (int32_t)wave_incl_scan((uint32_t)mrun0) - mrun0;
      int32_t mid_run = mid0;
      const int32_t ilo = min(max(L0 - col, 0), 8), ihi = min(max(L1 - col, 0), 8);
      const uint32_t inm = ((1u << ihi) - 1u) & ~((1u << ilo) - 1u);
      // ---- decision (GermlineThresholdCaller.scala:97-177 for pileups of single-base and
      //      MidDeletion alleles): kind 0 nothing, 1 a Ref/NoCall record, 2 a variant candidate
      //      (record pair), 3 complex
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t e0 = ev[64 * j + lane], e1 = DEEP ? ev[T + 64 * j + lane] : 0u;
        const uint32_t eacj = DEEP ? e0 : (e0 & 0xFFu) | ((e0 & 0xFF00u) << 8);
        const uint32_t etgj = DEEP ? e1 : ((e0 >> 16) & 0xFFu) | ((e0 >> 8) & 0xFF0000u);
        const uint32_t m8j = m8[j];
        const int32_t ddj = (int32_t)d8[j];
        const uint32_t cA = cnt(wA, ca, j), cC = cnt(wC, cc, j), cT = cnt(wT, ct, j), cG = cnt(wG, cg, j);
        const uint32_t nN = cnt(wN, cn, j);
        ncx_run += (int32_t)m8j >> 16;
        const uint32_t ncx = ncx_run > 0 ? (uint32_t)ncx_run : 0u;
        mid_run += ddj;
        const uint32_t nmid = mid_run > 0 ? (uint32_t)mid_run : 0u;  // MidDeletion elements (allele (ref, ""))
        const uint32_t depth = cA + cC + cT + cG + nN + ncx + nmid;
        const uint32_t mask = ref_mask(m8j, eacj, etgj, cA, cC, cT, cG);
        const bool live = ((inm >> j) & 1u) != 0 && depth > 0;
        const bool ambiguous = (mask & (mask - 1u)) != 0;
        const uint32_t low = mask & (0u - mask);  // the first standard reference base, as a bit (or 0: N)
        const uint32_t c_ref = (cA & (0u - (low & 1u))) + (cC & (0u - ((low >> 1) & 1u))) +
                               (cT & (0u - ((low >> 2) & 1u))) + (cG & (0u - ((low >> 3) & 1u))) +
                               (low == 0u ? nN : 0u);
        // two alleles in one mutable.HashMap bucket (Scala map order by first occurrence:
        // germline_complex): ref C with two of G, N and (C, ""); ref G with T and (G, "")
        const bool g0 = cG > 0, n0 = nN > 0, d0 = nmid > 0;
        const bool cgn = low == 2u && ((g0 && n0) || (g0 && d0) || (n0 && d0));
        const bool gtm = low == 8u && cT > 0 && d0;
        const bool to_complex = live && (ambiguous || ncx > 0 || multi_sample || cgn || gtm);
        const bool alt_pass = passes(depth - c_ref, depth);  // some other allele may pass
        const bool general = live && !to_complex && alt_pass;
        const bool ref_pass = c_ref > 0 && passes(c_ref, depth);
        const bool emit_hr = live && !to_complex && !alt_pass && (ref_pass ? emit_ref != 0 : emit_no_call != 0);
        livem |= (live ? 1u : 0u) << j;
        ambm |= (live && ambiguous ? 1u : 0u) << j;
        kinds |= (to_complex ? 3u : general ? 2u : emit_hr ? 1u : 0u) << (2 * j);
      }
    }
    {  // counts from the per-locus fields: kind 1 one record, 2 a record pair, 3 a complex item
      const uint32_t hi = (kinds >> 1) & 0x5555u, lo = kinds & 0x5555u;
      nrec = (uint32_t)__popc(lo & ~hi) + 2u * (uint32_t)__popc(hi & ~lo);
      ncpx = (uint32_t)__popc(lo & hi);
      visited += (uint32_t)__popc(livem);
      amb += (uint32_t)__popc(ambm);
    }
    if (__ballot(kinds != 0) != 0) {  // rare: records / complex items to write
      const unsigned long long rbase = reserve(0, nrec);
      const unsigned long long cbase = reserve(1, ncpx);
      CallRec *prec_out = recs + obase[0];
      unsigned long long kr = rbase, kc = cbase;
      constexpr uint64_t kAltSym = ((uint64_t)'<' << 8) | ((uint64_t)'A' << 16) | ((uint64_t)'L' << 24) |
                                   ((uint64_t)'T' << 32) | ((uint64_t)'>' << 40);
      int32_t mrun = mid0;
      for (int j = 0; j < 8; ++j) {
        mrun += (int32_t)dl[64 * j + lane];
        const uint32_t nmid = mrun > 0 ? (uint32_t)mrun : 0u;
        const uint32_t kind = (kinds >> (2 * j)) & 3u;
        if (__ballot(kind != 0) == 0) continue;  // no lane writes for locus j (uniform skip)
        if (kind == 0) continue;
        const int32_t pos = col + j;
        if (kind == 3) {
          if (kc < ocap[1]) cplx[obase[1] + kc] = ComplexItem{(int32_t)tid, pos, 0};
          ++kc;
          continue;
        }
        const uint32_t cA = cnt(wA, ca, j), cC = cnt(wC, cc, j), cT = cnt(wT, ct, j), cG = cnt(wG, cg, j);
        const uint32_t mw = mk[64 * j + lane];
        const uint32_t nN = cnt(wN, cn, j);
        const uint32_t e0 = ev[64 * j + lane], e1 = DEEP ? ev[T + 64 * j + lane] : 0u;
        const uint32_t mask = ref_mask(mw, DEEP ? e0 : (e0 & 0xFFu) | ((e0 & 0xFF00u) << 8),
                                       DEEP ? e1 : ((e0 >> 16) & 0xFFu) | ((e0 >> 8) & 0xFF0000u), cA, cC, cT, cG);
        const uint8_t ref = mask ? bit_base(mask) : (uint8_t)'N';
        const uint64_t ord = (uint64_t)(ord0 + (pos - L0));
        CallRec rr;
        rr.key = ord << 12;
        rr.contig = tcontig;
        rr.pos = pos;
        rr.sample = 0;
        if (kind == 1) {
          const uint32_t depth = cA + cC + cT + cG + nN + nmid;
          const uint32_t low = mask & (0u - mask);
          const uint32_t c_ref = low == 1u ? cA : low == 2u ? cC : low == 4u ? cT : low == 8u ? cG : nN;
          const bool ref_pass = c_ref > 0 && passes(c_ref, depth);
          rr.gt0 = rr.gt1 = ref_pass ? GQ_GT_REF : GQ_GT_NOCALL;
          rr.flags = 0;
          rr.ref_len = 1;
          rr.alt_len = 5;
          rr.allele = (uint64_t)ref | kAltSym;
          if (kr < ocap[0]) prec_out[kr] = rr;
          ++kr;
        } else {
          // a variant candidate: counts in a placeholder record pair, expanded by germline_expand
          rr.gt0 = ref;
          rr.gt1 = 0;
          rr.flags = kCandidate;
          rr.ref_len = (uint16_t)nN;
          rr.alt_len = (uint16_t)nmid;
          rr.allele = (uint64_t)cA | ((uint64_t)cC << 16) | ((uint64_t)cT << 32) | ((uint64_t)cG << 48);
          if (kr < ocap[0]) prec_out[kr] = rr;
          rr.flags = kCandidateSlot;
          if (kr + 1 < ocap[0]) prec_out[kr + 1] = rr;
          kr += 2;
        }
      }
    }
    zero_words();  // for the next tile (the wave's own words: no barrier)
    if (dbg & 16) {  // phase clocks (cycles per tile and wave): setup, records + counting, -, -, decision
      const uint64_t t_f = __builtin_readcyclecounter();
      clk[0] += t_b - t_a;
      clk[1] += t_c - t_b;
      clk[4] += t_f - t_c;
      clk[5] += 1;
    }
  }
  if ((dbg & 16) && lane == 0 && clk[5])
    for (int k = 0; k < 8; ++k) atomicAdd(&ctr->prof[k], (unsigned long long)clk[k]);
  add_run_counters(ctr, visited, amb, ties, (int)blockIdx.x);
  if (!DEEP && threadIdx.x == 0) {  // this workgroup's partition counts (may exceed the capacity: host retry)
    ctr->part[0][blockIdx.x] = outn[0];
    ctr->part[1][blockIdx.x] = outn[1];
  }
}
