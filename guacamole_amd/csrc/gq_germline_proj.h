// gq_germline_proj.h — germline_proj: the germline-threshold pileup kernel over the read
// projections derived at upload (proj rows, pev: gq_pileup.hip row_count / proj_fill /
// pev_fill).
//
// One WAVE per 512-locus tile, no workgroup barriers: tiles are aligned to 512-locus blocks
// (plan(..., aligned)), so lane l owns the 8-locus column [B0 + 8l, B0 + 8l + 8) of its tile's
// block B0, and lanes 16g .. 16g + 15 own slice g's projection rows (ProjRec: 16 words each,
// word c = column c of the slice as eight 4-bit codes, the reads packed into rows by interval
// partitioning), one 64-byte row per group and load, no per-row address arithmetic beyond the
// slice's bound:
//
//     w    = buffer_load_b32(row k of slice g, lane l16)          (rows past the slice's: 0)
//     lo, hi = w & 0x0F0F0F0F, (w >> 4) & 0x0F0F0F0F      loci 0-3, 4-7 as byte codes
//     nac += perm(0, 0x10000100, lo | hi)                 A -> 0x01, C -> 0x10 per byte
//     ntg += perm(0x10000001, 0, lo | hi)                 T -> 0x01, G -> 0x10 per byte
//
// (the projection holds base codes A 1, C 3, T 4, G 7 and 0 where the read has no
// Match/Mismatch element, so neither the read's ends nor its deletions need a mask).  Counts
// are SWAR nibbles folded into byte counters every 12 rows and into 16-bit pairs every 240, in
// registers (so 500x blocks stay here).  The sparse rest —
// MD mismatch events (PileupElement.scala:108-118, Pileup.scala:157-165: the MD-derived
// reference base), N bases, complex ranges (insertion / deletion anchors, mid-deletions,
// N-skips) — comes from the tile's pev entries, one lane per entry, into three LDS words per
// locus.  Then each lane makes the GermlineThreshold decision (GermlineThresholdCaller.scala:
// 90-179) for its eight loci; variant candidates, Ref/NoCall records and complex items leave
// as in germline_decide.  Blocks a read the projection cannot take overlaps (pbad: also slices
// past kSliceRowsMax rows) go to germline_walk.
#pragma once

#include "gq_kernels.h"

// (included inside gq_pileup.hip's anonymous namespace, after gq_germline_common.h)

#ifndef GQ_PROJ_WPE
#define GQ_PROJ_WPE 4  // waves per SIMD the register budget must allow (5: 72 B/lane of spills, 4 % slower)
#endif
#ifndef GQ_PROJ_WAVES
#define GQ_PROJ_WAVES 4
#endif
#ifndef GQ_PROJ_ENT
#define GQ_PROJ_ENT 6
#endif
#ifndef GQ_PROJ_NB
#define GQ_PROJ_NB 4  // row batches per round (NB - 1 in flight while one is counted)
#endif
#ifndef GQ_PROJ_LAZY
#define GQ_PROJ_LAZY 0  // A/B: 1 reads each locus's complex / MidDeletion words twice instead of holding them
#endif
#ifndef GQ_PROJ_GMIN
#define GQ_PROJ_GMIN 0  // A/B: 1 skips the per-group row bound below the block's fewest rows (measured slower)
#endif
struct ProjCfg {
  static constexpr int kT = 512;       // loci per tile: 64 lanes x 8 loci
  static constexpr int kWaves = GQ_PROJ_WAVES;  // waves per workgroup, each on its own tiles
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kU = 4;  // rows per batch (all loads issued before use); 3 batches in flight
  static constexpr int kMaxRows = kSliceRowsMax;  // rows per block (16-bit counts past 240 rows)
  static constexpr int kEnt = GQ_PROJ_ENT;  // sparse entries per lane loaded with the records (the rest: a loop)
};

// Wave-aggregated reservation of n slots per lane on an LDS counter (every lane active).
__device__ __forceinline__ unsigned wave_reserve_lds_n(unsigned *ctr, unsigned n) {
  const uint32_t x = wave_incl_scan(n);
  const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  unsigned base = 0;
  if ((threadIdx.x & 63) == 63 && total) base = atomicAdd(ctr, total);
  base = (unsigned)__builtin_amdgcn_readlane((int)base, 63);
  return base + x - n;
}

__global__ __launch_bounds__(ProjCfg::kThreads) __attribute__((amdgpu_waves_per_eu(GQ_PROJ_WPE))) void germline_proj(
    const Tile *__restrict__ tiles, const TileX *__restrict__ tilex, int64_t n_tiles, const uint8_t *__restrict__ proj, const uint2 *__restrict__ pev, int n_samples, int threshold, int emit_ref,
    int emit_no_call,
    CallRec *__restrict__ recs, ComplexItem *__restrict__ cplx, OutGeom og, Counters *ctr,
    int32_t *__restrict__ slow, int dbg) {
  // dbg (diagnostics, env GQ_DBG; results are wrong when set): 1 skip the projection loads,
  // 2 skip the sparse entries, 4 skip the decision, 8 skip writing its records
  using C = ProjCfg;
  constexpr int T = C::kT, U = C::kU;
  // per locus: event read bases (A | C << 16 at [i], T | G << 16 at [T + i]); MD bits 0-3 |
  // N << 4 | complex diff << 16.  Locus x of the block is word ix(x) = (x & 7) * 64 + (x >> 3):
  // lane l's eight loci (8 l + j) sit at j * 64 + l, so the decision's reads (every lane, one j)
  // are 64 consecutive words — no bank conflicts (8 l + j put every lane of a read on four banks).
  __shared__ __attribute__((aligned(16))) uint32_t evw[C::kWaves][2 * T];
  __shared__ __attribute__((aligned(16))) uint32_t mkw[C::kWaves][T];
  __shared__ __attribute__((aligned(16))) uint32_t dlw[C::kWaves][T];  // MidDeletion range differences
  __shared__ unsigned outn[2];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint32_t *ev = evw[wave], *mk = mkw[wave], *dl = dlw[wave];
  auto ix = [](int32_t x) { return ((x & 7) << 6) | (x >> 3); };
  // the tile's LDS words back to 0: 16-byte stores, lane l at 16 l (consecutive: no conflicts)
  auto zero_words = [&]() {  // separate stores (a chained assignment re-reads each word from LDS)
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    uint4 *e4 = reinterpret_cast<uint4 *>(ev), *m4 = reinterpret_cast<uint4 *>(mk), *d4 = reinterpret_cast<uint4 *>(dl);
    e4[lane] = z4; e4[64 + lane] = z4; e4[128 + lane] = z4; e4[192 + lane] = z4;
    m4[lane] = z4; m4[64 + lane] = z4; d4[lane] = z4; d4[64 + lane] = z4;
  };
  zero_words();
  if (threadIdx.x < 2) outn[threadIdx.x] = 0;
  __syncthreads();
  const int64_t per = n_tiles / gridDim.x, extra = n_tiles % gridDim.x;
  const int64_t i0 = blockIdx.x * per + min((int64_t)blockIdx.x, extra);
  const int64_t i1 = i0 + per + ((int64_t)blockIdx.x < extra ? 1 : 0);
  LdsOut out{outn, {og.slot(0, (int)blockIdx.x, 0), og.slot(1, (int)blockIdx.x, 0)}, {og.capA[0], og.capA[1]}};
  unsigned visited = 0, amb = 0, ties = 0;
  uint64_t clk[6] = {0, 0, 0, 0, 0, 0};
  const int g = lane >> 4;
  const bool multi_sample = n_samples > 1;
  // count * 100 / depth > threshold <=> count * 100 >= (threshold + 1) * depth (integers, depth > 0);
  // with count <= depth < 2^16 the factor clamps to [0, 101] (101: never; 0: always) in 32 bits
  const int64_t thr1 = (int64_t)threshold + 1;
  const uint32_t thr1u = (uint32_t)(thr1 < 0 ? 0 : thr1 > 101 ? 101 : thr1);
  // (16-bit operands, so the products take full-rate 24-bit multiplies: a locus has at most
  // kSliceRowsMax elements, one per row of its slice)
  const uint32_t thr1b = thr1u & 0xFFu;
  auto passes = [=](uint32_t count, uint32_t depth) { return (count & 0xFFFFu) * 100u >= thr1b * (depth & 0xFFFFu); };
  // the tile record (Tile + TileX: dword d on lane d < 32) of the wave's next tile, loaded one
  // tile ahead: its fields are in a register when the tile starts (no dependent setup rounds)
  // (TileX array follows the Tiles: one buffer over both, lane d < 16 reads Tile dword d,
  // lanes 16-31 TileX dword d - 16, the rest an out-of-range offset; the tile in the scalar
  // offset.  plan sizes the arrays below 2^31 bytes.)
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc((void *)tiles, (short)0, (int)(128 * n_tiles), 0x00020000);
  const uint32_t tvo = lane < 16 ? 4u * (uint32_t)lane
                       : lane < 32 ? (uint32_t)(64 * n_tiles) + 4u * (uint32_t)(lane - 16)
                                   : 0x80000000u;
  auto fetch = [&](int64_t t) -> uint32_t {
    return __builtin_amdgcn_raw_buffer_load_b32(trs, (int)tvo, (int)(64 * t), 0);
  };
  auto f32 = [](uint32_t rec, int d) { return (uint32_t)__builtin_amdgcn_readlane((int)rec, d); };
  auto f64 = [&](uint32_t rec, int d) { return (int64_t)((uint64_t)f32(rec, d) | ((uint64_t)f32(rec, d + 1) << 32)); };
  // A tile's row context: the buffer over its block's rows, this lane's offset in its slice's
  // first row, and its slice's rows (gn = 0: every load of the tile reads 0).  Rows past the
  // slice's, and (dbg & 1, diagnostics) every row, fall out of the buffer's range and read 0.
  struct RowCtx {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t vl;
    int32_t gn;
    int32_t gmin;  // the fewest rows of the block's four slices (wave-uniform): batches below it need no bound
  };
  auto row_ctx = [&](uint32_t rec) -> RowCtx {
    const int64_t row0 = f64(rec, 16);
    const int32_t nr0 = (int32_t)f32(rec, 18), nr1 = (int32_t)f32(rec, 19), nr2 = (int32_t)f32(rec, 20),
                  nr3 = (int32_t)f32(rec, 21);
    // (masks, not selects: nested selects on the lane's group compile to divergent branches)
    const int32_t gbase = (nr0 & -(int32_t)(g >= 1)) + (nr1 & -(int32_t)(g >= 2)) + (nr2 & -(int32_t)(g >= 3));
    RowCtx x;
    x.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)(proj + kProjRowBytes * row0), (short)0,
                                               (dbg & 1) ? 0 : kProjRowBytes * (nr0 + nr1 + nr2 + nr3), 0x00020000);
    x.vl = 4u * (uint32_t)(lane & 15) + (uint32_t)kProjRowBytes * (uint32_t)gbase;
    x.gn = (nr0 & -(int32_t)(g == 0)) | (nr1 & -(int32_t)(g == 1)) | (nr2 & -(int32_t)(g == 2)) |
           (nr3 & -(int32_t)(g == 3));
    x.gmin = (dbg & 1) ? 0 : min(min(nr0, nr1), min(nr2, nr3));
    return x;
  };
  // the block's fullest slice, and whether the tile runs here (reads, no pbad slice, rows in range)
  auto rec_rows = [&](uint32_t rec) {
    return max(max((int32_t)f32(rec, 18), (int32_t)f32(rec, 19)), max((int32_t)f32(rec, 20), (int32_t)f32(rec, 21)));
  };
  auto rec_runs = [&](uint32_t rec) {
    return f64(rec, 4) > f64(rec, 2) && f32(rec, 22) == 0u && rec_rows(rec) <= C::kMaxRows;
  };
  // rows k0 .. k0 + U - 1 of each group's slice: the lane offset, or an out-of-range one past
  // the slice's rows; + 64 u in the scalar offset (in range whenever the lane offset is).  One
  // 32-bit word per lane and row: the column's eight 4-bit codes.
  auto issue = [&](const RowCtx &x, int32_t k0, uint32_t (&w)[U]) {
    const uint32_t vb = x.vl + (uint32_t)kProjRowBytes * (uint32_t)k0;
    if (GQ_PROJ_GMIN && k0 + U <= x.gmin) {  // uniform: every group's slice has these rows (most batches)
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = __builtin_amdgcn_raw_buffer_load_b32(x.rsrc, (int)vb, kProjRowBytes * u, 0);
      return;
    }
    // (slices hold a multiple of kRowPad = U rows: a batch lies wholly inside its group's slice or
    // wholly past it, one bound per batch)
    const uint32_t v = k0 < x.gn ? vb : 0x80000000u;
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = __builtin_amdgcn_raw_buffer_load_b32(x.rsrc, (int)v, kProjRowBytes * u, 0);
  };
  static_assert(U == kRowPad, "row batches are the slices' row padding");
  // Tiles are software-pipelined: the Tile + TileX records arrive two tiles ahead, and a tile's
  // last counting round issues the NEXT tile's first three row batches, so those loads are in
  // flight while this tile's sparse entries and decision run (no loads past the rows are
  // issued, and nothing waits for them).  primed: rows 0 .. 3U - 1 of the tile starting now are
  // already in a, b, c.
  constexpr int NB = GQ_PROJ_NB;
  static_assert(240 % (NB * U) == 0, "the 16-bit widening runs on a round boundary");
  uint32_t bf[NB][U];
  // the first kEnt sparse entries per lane of a tile's reads (the rest: a loop), applied before
  // its counting (the entry loads' latency overlaps the primed row batches')
  constexpr int NE = C::kEnt;
  auto load_ent = [&](uint2 (&ent)[NE], int64_t e0, int64_t e1) {
    // a buffer over the window's first entries (32-bit lane offsets).  Past them the load
    // reads 0 and the locus becomes INT_MIN, outside every block: no effect.
    const uint32_t nb = (dbg & 2) ? 0u : 8u * (uint32_t)min(e1 - e0, (int64_t)NE * 64);
    const __amdgpu_buffer_rsrc_t ers =
        __builtin_amdgcn_make_buffer_rsrc((void *)(pev + e0), (short)0, (int)nb, 0x00020000);
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const uint32_t o = 8u * (uint32_t)lane + 512u * j;
      const auto w = __builtin_amdgcn_raw_buffer_load_b64(ers, (int)o, 0, 0);
      ent[j] = make_uint2(w[0] | (o < nb ? 0u : 0x80000000u), w[1]);
    }
  };
  bool primed = false;
  int64_t i = i0 + wave;
  uint32_t rec_c = i < i1 ? fetch(i) : 0u;
  uint32_t rec_n = i + C::kWaves < i1 ? fetch(i + C::kWaves) : 0u;
  for (; i < i1; i += C::kWaves) {
    const uint64_t t_a = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    const uint32_t rec = rec_c;
    rec_c = rec_n;
    if (i + 2 * C::kWaves < i1) rec_n = fetch(i + 2 * C::kWaves);
    const bool was_primed = primed;
    primed = false;
    // Tile: ordinal0 dw 0-1, rb 2-3, re 4-5, contig 6, L0 7, L1 8; TileX from dw 16: row0 16-17,
    // nr[4] 18-21, pbad4 22, e0 24-25, e1 26-27
    const int32_t L0 = (int32_t)f32(rec, 7), L1 = (int32_t)f32(rec, 8);
    const int64_t rb = f64(rec, 2), re = f64(rec, 4);
    const int32_t B0 = L0 & ~(T - 1);
    if (re <= rb) continue;  // no reads: nothing visited
    // A pbad slice (a read the projection cannot take) or more than kMaxRows rows: the walker.
    const int32_t nrows = rec_rows(rec);
    if (f32(rec, 22) != 0u || nrows > C::kMaxRows) {
      if (lane == 0) slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)i;
      continue;
    }
    const RowCtx cur = row_ctx(rec);
    if (!was_primed) {
#pragma unroll
      for (int q = 0; q + 1 < NB; ++q) issue(cur, q * U, bf[q]);
    }
    const int64_t e0 = f64(rec, 24), e1 = f64(rec, 26);
    uint2 ent[NE];
    load_ent(ent, e0, e1);
    const uint64_t t_b = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    // ---- sparse entries of the tile's reads, one lane per entry, into the LDS words
    auto apply = [&](uint2 p) {
      const int32_t l = (int32_t)p.x;
      if (p.y & kPevComplex) {  // a range: +1 at its first locus, -1 past its last
        const int64_t a = max((int64_t)l, (int64_t)B0);
        const int64_t b = min((int64_t)l + (int64_t)(p.y & kPevLenMask), (int64_t)B0 + T);
        const bool mid = (p.y & kPevMidDel) != 0;  // MidDeletion elements: their own count
        uint32_t *dw = mid ? dl : mk;
        if (a < b) {
          atomicAdd(&dw[ix((int32_t)(a - B0))], mid ? 1u : 1u << 16);
          if (b < (int64_t)B0 + T) atomicAdd(&dw[ix((int32_t)(b - B0))], mid ? 0xFFFFFFFFu : 0xFFFF0000u);
        }
      } else if (l >= B0 && l < B0 + T) {
        const uint32_t m = p.y & 15u, c = (p.y >> 4) & 7u;
        const int32_t x = ix(l - B0);
        if (m) atomicOr(&mk[x], m);
        if (c < 4) atomicAdd(&ev[(c >> 1) * T + x], 1u << (16 * (c & 1)));
        else if (c == 4) atomicAdd(&mk[x], 1u << 4);
      }
    };
#pragma unroll
    for (int j = 0; j < NE; ++j) apply(ent[j]);
    if (!(dbg & 2))
      for (int64_t q = e0 + 64 * NE; q < e1; q += 64) {  // the rest (rare)
        const int64_t k = q + lane;
        if (k < e1) apply(pev[k]);
      }
    // the next tile of this wave: its first batches leave with this tile's last round
    const bool next_ok = i + C::kWaves < i1 && rec_runs(rec_c);
    RowCtx nxt = cur;
    nxt.gn = 0;
    nxt.gmin = 0;
    if (next_ok) nxt = row_ctx(rec_c);
    // ---- column counts: byte counters per base (loci 0-3 of the column in [0], 4-7 in [1]),
    //      widened into 16-bit pairs (loci 2q, 2q + 1 in w?[q]) every 240 rows and at the end.
    //      Row k of each group's slice: one 64-byte load per group.  Three batches of loads
    //      stay in flight while a fourth is counted.
    uint32_t ca[2] = {0, 0}, cc[2] = {0, 0}, ct[2] = {0, 0}, cg[2] = {0, 0};
    uint32_t wA[4] = {0, 0, 0, 0}, wC[4] = {0, 0, 0, 0}, wT[4] = {0, 0, 0, 0}, wG[4] = {0, 0, 0, 0};
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
    };
    // a row word holds loci 0-3 of the column in its low nibbles (byte j: locus j) and loci 4-7
    // in its high nibbles; split, each half is four byte codes for the perm tables
    auto count = [&](const uint32_t (&w)[U]) {
      if (nn + U > 15) fold();
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t lo = w[u] & 0x0F0F0F0Fu, hi = (w[u] >> 4) & 0x0F0F0F0Fu;
        nac[0] += __builtin_amdgcn_perm(0u, 0x10000100u, lo);
        ntg[0] += __builtin_amdgcn_perm(0x10000001u, 0u, lo);
        nac[1] += __builtin_amdgcn_perm(0u, 0x10000100u, hi);
        ntg[1] += __builtin_amdgcn_perm(0x10000001u, 0u, hi);
      }
      nn += U;
    };
    // rows k0 .. k0 + NB U - 1 per round; the last round (uniform) issues the next tile's rows
    // 0 .. (NB - 1) U - 1 instead of this tile's past its end
    for (int32_t k0 = 0, since = 0;; k0 += NB * U) {
      const bool last = k0 + NB * U >= nrows;
      issue(cur, k0 + (NB - 1) * U, bf[NB - 1]);
#pragma unroll
      for (int q = 0; q + 1 < NB; ++q) {
        count(bf[q]);
        issue(last ? nxt : cur, last ? q * U : k0 + (NB + q) * U, bf[q]);
      }
      count(bf[NB - 1]);
      if (last) break;
      since += NB * U;
      if (since == 240) {  // uniform: bytes hold 240 rows at most
        fold();
        widen();
        since = 0;
      }
    }
    primed = next_ok;
    const uint64_t t_c = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    const uint64_t t_d = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    fold();
    widen();
    const uint64_t t_e = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t kinds = 0, nrec = 0, ncpx = 0, livem = 0, ambm = 0;
    int32_t mid0 = 0;  // MidDeletion elements entering this lane's first locus
    // locus j's 16-bit count of base w (a dynamic j selects among four registers)
    auto cnt16 = [](const uint32_t (&w)[4], int j) {
      const int q = j >> 1;
      const uint32_t x = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
      return (x >> (16 * (j & 1))) & 0xFFFFu;
    };
    // the reference-base mask of a locus: MD bits, plus each base with more Match/Mismatch
    // elements than events (an element without an event reads the reference)
    auto ref_mask = [](uint32_t mw, uint32_t eac, uint32_t etg, uint32_t cA, uint32_t cC, uint32_t cT, uint32_t cG) {
      return (mw & 15u) | (cA > (eac & 0xFFFFu) ? 1u : 0u) | (cC > (eac >> 16) ? 2u : 0u) |
             (cT > (etg & 0xFFFFu) ? 4u : 0u) | (cG > (etg >> 16) ? 8u : 0u);
    };
    if (!(dbg & 4)) {
      // complex elements per locus: prefix of the range differences over the block
      // this lane's eight words of each array, read once (conflict-free rows of 64 words)
      // (GQ_PROJ_LAZY: summed here, read again per locus below — fewer live registers)
      int32_t run = 0, mrun0 = 0;
#if GQ_PROJ_LAZY
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        run += (int32_t)mk[64 * j + lane] >> 16;
        mrun0 += (int32_t)dl[64 * j + lane];
      }
#else
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
#endif
      int32_t ncx_run = (int32_t)wave_incl_scan((uint32_t)run) - run;  // before this lane's loci
      mid0 = (int32_t)wave_incl_scan((uint32_t)mrun0) - mrun0;  // the same for the MidDeletion ranges
      int32_t mid_run = mid0;
      // the lane's loci inside [L0, L1) as bits (most lanes: all eight)
      const int32_t lb0 = B0 + 8 * lane;
      const int32_t ilo = min(max(L0 - lb0, 0), 8), ihi = min(max(L1 - lb0, 0), 8);
      const uint32_t inm = ((1u << ihi) - 1u) & ~((1u << ilo) - 1u);
      // ---- decision (GermlineThresholdCaller.scala:97-177 for pileups of single-base and
      //      MidDeletion alleles), eight loci, four unrolled at a time with their LDS words read
      //      in the loop (the next tile's row batches are in flight in registers meanwhile):
      //      kind 0 nothing, 1 a Ref/NoCall record, 2 a variant candidate (record pair), 3 complex
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#if GQ_PROJ_LAZY
        const uint32_t eacj = ev[64 * j + lane], etgj = ev[T + 64 * j + lane], m8j = mk[64 * j + lane];
        const int32_t ddj = (int32_t)dl[64 * j + lane];
#else
        const uint32_t eacj = ev[64 * j + lane], etgj = ev[T + 64 * j + lane], m8j = m8[j];
        const int32_t ddj = (int32_t)d8[j];
#endif
        {
        const bool in = (inm >> j) & 1u;
        const uint32_t cA = cnt16(wA, j), cC = cnt16(wC, j), cT = cnt16(wT, j), cG = cnt16(wG, j);
        const uint32_t nN = (m8j >> 4) & 0xFFFu;
        ncx_run += (int32_t)m8j >> 16;
        const uint32_t ncx = ncx_run > 0 ? (uint32_t)ncx_run : 0u;
        mid_run += ddj;
        const uint32_t nmid = mid_run > 0 ? (uint32_t)mid_run : 0u;  // MidDeletion elements (allele (ref, ""))
        const uint32_t depth = cA + cC + cT + cG + nN + ncx + nmid;
        const uint32_t mask = ref_mask(m8j, eacj, etgj, cA, cC, cT, cG);
        // lane predicates (the common hom-ref locus writes nothing); kinds carries the result
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
    }
    {  // counts from the per-locus fields: kind 1 one record, 2 a record pair, 3 a complex item
      const uint32_t hi = (kinds >> 1) & 0x5555u, lo = kinds & 0x5555u;
      nrec = (uint32_t)__popc(lo & ~hi) + 2u * (uint32_t)__popc(hi & ~lo);
      ncpx = (uint32_t)__popc(lo & hi);
      visited += (uint32_t)__popc(livem);
      amb += (uint32_t)__popc(ambm);
    }
    if (!(dbg & 8) && __ballot(kinds != 0) != 0) {  // rare: records / complex items to write
      const unsigned rbase = wave_reserve_lds_n(out.lds + 0, nrec);
      const unsigned cbase = wave_reserve_lds_n(out.lds + 1, ncpx);
      CallRec *prec_out = recs + out.base[0];
      unsigned kr = rbase, kc = cbase;
      constexpr uint64_t kAltSym = ((uint64_t)'<' << 8) | ((uint64_t)'A' << 16) | ((uint64_t)'L' << 24) |
                                   ((uint64_t)'T' << 32) | ((uint64_t)'>' << 40);
      int32_t mrun = mid0;
      for (int j = 0; j < 8; ++j) {
        mrun += (int32_t)dl[64 * j + lane];
        const uint32_t nmid = mrun > 0 ? (uint32_t)mrun : 0u;
        const uint32_t kind = (kinds >> (2 * j)) & 3u;
        if (__ballot(kind != 0) == 0) continue;  // no lane writes for locus j (uniform skip)
        if (kind == 0) continue;
        const int32_t pos = B0 + 8 * lane + j;
        if (kind == 3) {
          if (kc < out.cap[1]) cplx[out.base[1] + kc] = ComplexItem{(int32_t)i, pos, 0};
          ++kc;
          continue;
        }
        const uint32_t cA = cnt16(wA, j), cC = cnt16(wC, j), cT = cnt16(wT, j), cG = cnt16(wG, j);
        const uint32_t mw = mk[64 * j + lane];
        const uint32_t nN = (mw >> 4) & 0xFFFu;
        const uint32_t mask = ref_mask(mw, ev[64 * j + lane], ev[T + 64 * j + lane], cA, cC, cT, cG);
        const uint8_t ref = mask ? bit_base(mask) : (uint8_t)'N';
        const uint64_t ord = (uint64_t)(f64(rec, 0) + (pos - L0));
        CallRec rr;
        rr.key = ord << 12;
        rr.contig = (int32_t)f32(rec, 6);
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
          if (kr < out.cap[0]) prec_out[kr] = rr;
          ++kr;
        } else {
          // a variant candidate: counts in a placeholder record pair, expanded by germline_expand
          rr.gt0 = ref;
          rr.gt1 = 0;
          rr.flags = kCandidate;
          rr.ref_len = (uint16_t)nN;
          rr.alt_len = (uint16_t)nmid;
          rr.allele = (uint64_t)cA | ((uint64_t)cC << 16) | ((uint64_t)cT << 32) | ((uint64_t)cG << 48);
          if (kr < out.cap[0]) prec_out[kr] = rr;
          rr.flags = kCandidateSlot;
          if (kr + 1 < out.cap[0]) prec_out[kr + 1] = rr;
          kr += 2;
        }
      }
    }
    zero_words();  // for the next tile (the wave's own words: no barrier)
    if (dbg & 16) {  // phase clocks (cycles per tile and wave): setup + entries, counting, -, widen, decision
      const uint64_t t_f = __builtin_readcyclecounter();
      clk[0] += t_b - t_a;
      clk[1] += t_c - t_b;
      clk[2] += t_d - t_c;
      clk[3] += t_e - t_d;
      clk[4] += t_f - t_e;
      clk[5] += 1;
    }
  }
  if ((dbg & 16) && lane == 0 && clk[5])
    for (int k = 0; k < 6; ++k) atomicAdd(&ctr->prof[k], (unsigned long long)clk[k]);
  add_run_counters(ctr, visited, amb, ties, (int)blockIdx.x);
  if (threadIdx.x == 0) {  // this workgroup's partition counts (may exceed the capacity: host retry)
    ctr->part[0][blockIdx.x] = outn[0];
    ctr->part[1][blockIdx.x] = outn[1];
  }
}
