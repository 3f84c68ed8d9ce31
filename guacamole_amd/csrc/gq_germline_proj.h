// gq_germline_proj.h — germline_proj: the germline-threshold pileup kernel over the read
// projections derived at upload (proj, pieces, pev: gq_pileup.hip proj_fill / piece_fill /
// pev_fill).
//
// One WAVE per 512-locus tile, no workgroup barriers: tiles are aligned to 512-locus blocks
// (plan(..., aligned)), so lane l owns the 8-locus column [B0 + 8l, B0 + 8l + 8) of its tile's
// block B0.  Lanes 16g .. 16g + 15 (group g) own the 128-locus slice [B0 + 128g, B0 + 128g +
// 128), whose projection words are one contiguous run in the slice-major pool (ProjRec), and
// walk the slice's pieces (the reads with words there, in read order; PieceRec), one piece per
// group per step:
//
//     rec = piece k's record (16 per stage, one per lane, shared in the group by ds_bpermute)
//     d   = l16 - s0(rec)
//     w   = buffer_load_b64(block's words, d < len(rec) ? 8 (base(rec) + d) : out of range -> 0)
//     nac += perm(0, 0x10000100, w.x | w.y)               A -> 0x01, C -> 0x10 per byte
//     ntg += perm(0x10000001, 0, w.x | w.y)               T -> 0x01, G -> 0x10 per byte
//
// (the projection holds base codes A 1, C 3, T 4, G 7 and 0 where the read has no
// Match/Mismatch element, so neither the read's ends nor its deletions need a mask).  Counts
// are SWAR nibbles folded into byte counters every 15 reads, in registers.  The sparse rest —
// MD mismatch events (PileupElement.scala:108-118, Pileup.scala:157-165: the MD-derived
// reference base), N bases, complex ranges (insertion / deletion anchors, mid-deletions,
// N-skips) — comes from the tile's pev entries, one lane per entry, into two LDS words per
// locus.  Then each lane makes the GermlineThreshold decision (GermlineThresholdCaller.scala:
// 90-179) for its eight loci; variant candidates, Ref/NoCall records and complex items leave
// as in germline_decide.  Blocks a read the projection cannot take overlaps (pbad), or with
// more than 255 pieces in one slice, go to germline_walk.
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
struct ProjCfg {
  static constexpr int kT = 512;       // loci per tile: 64 lanes x 8 loci
  static constexpr int kWaves = GQ_PROJ_WAVES;  // waves per workgroup, each on its own tiles
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kU = 4;  // pieces per group per batch (all loads issued before use); 4 batches per stage
  static constexpr int kMaxRows = 255;  // pieces per slice (byte counters); deeper blocks: walker
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
    const Tile *__restrict__ tiles, const TileX *__restrict__ tilex, int64_t n_tiles, const uint32_t *__restrict__ pcs,
    const uint8_t *__restrict__ proj, const uint2 *__restrict__ pev, int n_samples, int threshold, int emit_ref,
    int emit_no_call,
    CallRec *__restrict__ recs, ComplexItem *__restrict__ cplx, OutGeom og, Counters *ctr,
    int32_t *__restrict__ slow, int dbg) {
  // dbg (diagnostics, env GQ_DBG; results are wrong when set): 1 skip the projection loads,
  // 2 skip the sparse entries, 4 skip the decision
  using C = ProjCfg;
  constexpr int T = C::kT, U = C::kU;
  __shared__ __attribute__((aligned(16))) uint32_t evw[C::kWaves][T];  // event read bases: A C T G bytes
  __shared__ __attribute__((aligned(16))) uint32_t mkw[C::kWaves][T];  // MD bits 0-3 | N << 8 | complex diff << 16
  __shared__ unsigned outn[2];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint32_t *ev = evw[wave], *mk = mkw[wave];
  {
    uint4 *e4 = reinterpret_cast<uint4 *>(ev + 8 * lane), *m4 = reinterpret_cast<uint4 *>(mk + 8 * lane);
    e4[0] = e4[1] = m4[0] = m4[1] = make_uint4(0u, 0u, 0u, 0u);
  }
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
  auto passes = [=](uint32_t count, uint32_t depth) { return count * 100u >= thr1u * depth; };
  // the tile record (Tile + TileX: dword d on lane d < 32) of the wave's next tile, loaded one
  // tile ahead: its fields are in a register when the tile starts (no dependent setup rounds)
  auto fetch = [&](int64_t t) -> uint32_t {
    const uint32_t *t32 = reinterpret_cast<const uint32_t *>(tiles + t);
    const uint32_t *x32 = reinterpret_cast<const uint32_t *>(tilex + t);
    return lane < 16 ? t32[lane] : lane < 32 ? x32[lane - 16] : 0u;
  };
  auto f32 = [](uint32_t rec, int d) { return (uint32_t)__builtin_amdgcn_readlane((int)rec, d); };
  auto f64 = [&](uint32_t rec, int d) { return (int64_t)((uint64_t)f32(rec, d) | ((uint64_t)f32(rec, d + 1) << 32)); };
  uint32_t next_rec = i0 + wave < i1 ? fetch(i0 + wave) : 0u;
  for (int64_t i = i0 + wave; i < i1; i += C::kWaves) {
    const uint64_t t_a = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    const uint32_t rec = next_rec;
    if (i + C::kWaves < i1) next_rec = fetch(i + C::kWaves);
    // Tile: ordinal0 dw 0-1, rb 2-3, re 4-5, contig 6, L0 7, L1 8; TileX from dw 16: sb0, sb4,
    // e0, e1, pb0 (16-25), pbd[4] (26-29), pbad4 (30)
    const int32_t L0 = (int32_t)f32(rec, 7), L1 = (int32_t)f32(rec, 8);
    const int64_t rb = f64(rec, 2), re = f64(rec, 4);
    const int32_t B0 = L0 & ~(T - 1);
    if (re <= rb) continue;  // no reads: nothing visited
    // ---- the block's slices (one per group): their piece ranges and pbad flags (from the
    //      record), the first kEnt sparse entries per lane of the window's reads and the first
    //      three 16-piece stages of each group's piece records, loaded together.  A pbad slice
    //      (a read the projection cannot take) or more than kMaxRows pieces in a slice: the walker.
    const int64_t sb0 = f64(rec, 16), sb4 = f64(rec, 18);
    const int32_t pd0 = (int32_t)f32(rec, 26), pd1 = (int32_t)f32(rec, 27), pd2 = (int32_t)f32(rec, 28),
                  pd3 = (int32_t)f32(rec, 29);
    const int32_t plo = g == 0 ? 0 : g == 1 ? pd0 : g == 2 ? pd1 : pd2;
    const int32_t phi = g == 0 ? pd0 : g == 1 ? pd1 : g == 2 ? pd2 : pd3;
    const int64_t pbg = f64(rec, 24) + plo;
    const int32_t ng = phi - plo;
    const uint32_t badg = (f32(rec, 30) >> (8 * g)) & 0xFFu;
    const int64_t e0 = f64(rec, 20), e1 = f64(rec, 22);
    constexpr int NE = C::kEnt;
    uint2 ent[NE];
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const int64_t k = e0 + 64 * j + lane;
      ent[j] = make_uint2(0x80000000u, kPevNone);
      if (!(dbg & 2) && k < e1) ent[j] = pev[k];
    }
    const int32_t l16 = lane & 15;
    auto stage = [&](int32_t k) -> uint32_t {  // piece record of row k + l16 of this group
      return k + l16 < ng ? pcs[pbg + k + l16] : kPieceNone;
    };
    uint32_t P0 = stage(0), P1 = stage(16), P2 = stage(32);
    const int32_t nmax = max(max(pd0, pd1 - pd0), max(pd2 - pd1, pd3 - pd2));
    if (__ballot(badg != 0) != 0 || nmax > C::kMaxRows) {
      if (lane == 0) slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)i;
      continue;
    }
    const uint64_t t_b = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    // ---- column counts: byte counters per base (loci 0-3 of the column in [0], 4-7 in [1]).
    //      Row k of group g is piece k of its slice: record from the 16-piece stage in a
    //      register (ds_bpermute within the group), word (rec >> 9) + l16 - s0 when this
    //      lane's column is inside the piece, else an out-of-range offset (the load returns
    //      0).  Three batches of loads stay in flight while a fourth is counted.
    uint32_t ca[2] = {0, 0}, cc[2] = {0, 0}, ct[2] = {0, 0}, cg[2] = {0, 0};
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(proj + 8 * sb0), (short)0, (int)(8 * (sb4 - sb0)), 0x00020000);
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
    const int32_t bp = (lane & 48) << 2;  // ds_bpermute address of the group's lane 0
    // lane offset B + l16 - 16 (dbg & 1, diagnostics: every load out of range)
    const uint32_t lm16 = (dbg & 1) ? 0x10000000u : (uint32_t)l16 - 16u, ibit = 16u + (uint32_t)l16;
    auto issue = [&](uint32_t P, int u0, uint32_t (&w0)[U], uint32_t (&w1)[U]) {
      uint32_t rv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) rv[u] = (uint32_t)__builtin_amdgcn_ds_bpermute(bp + 4 * (u0 + u), (int)P);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t rr = rv[u];
        // (B + l16 - 16) * 8 | (lane invalid) << 31 (PieceRec)
        const uint32_t inv = (rr >> ibit) & 1u;
        const uint32_t voff = (((rr & 0xFFFFu) + lm16) << 3) | (inv << 31);
        const auto w = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)voff, 0, 0);
        w0[u] = w[0];
        w1[u] = w[1];
      }
    };
    auto count = [&](const uint32_t (&w0)[U], const uint32_t (&w1)[U]) {
      if (nn + U > 15) fold();
#pragma unroll
      for (int u = 0; u < U; ++u) {
        nac[0] += __builtin_amdgcn_perm(0u, 0x10000100u, w0[u]);
        ntg[0] += __builtin_amdgcn_perm(0x10000001u, 0u, w0[u]);
        nac[1] += __builtin_amdgcn_perm(0u, 0x10000100u, w1[u]);
        ntg[1] += __builtin_amdgcn_perm(0x10000001u, 0u, w1[u]);
      }
      nn += U;
    };
    uint32_t a0[U], a1[U], b0[U], b1[U], c0[U], c1[U], d0[U], d1[U];
    issue(P0, 0, a0, a1);
    issue(P0, U, b0, b1);
    issue(P0, 2 * U, c0, c1);
    // ---- sparse entries of the tile's reads, one lane per entry, into the LDS words
    auto apply = [&](uint2 p) {
      const int32_t l = (int32_t)p.x;
      if (p.y & kPevComplex) {
        const int64_t a = max((int64_t)l, (int64_t)B0);
        const int64_t b = min((int64_t)l + (int64_t)(p.y & ~kPevComplex), (int64_t)B0 + T);
        if (a < b) {
          atomicAdd(&mk[a - B0], 1u << 16);
          if (b < (int64_t)B0 + T) atomicAdd(&mk[b - B0], 0xFFFF0000u);
        }
      } else if (l >= B0 && l < B0 + T) {
        const uint32_t m = p.y & 15u, c = (p.y >> 4) & 7u;
        if (m) atomicOr(&mk[l - B0], m);
        if (c < 4) atomicAdd(&ev[l - B0], 1u << (8 * c));
        else if (c == 4) atomicAdd(&mk[l - B0], 1u << 8);
      }
    };
    const uint64_t t_c = (dbg & 16) ? __builtin_readcyclecounter() : 0;
#pragma unroll
    for (int j = 0; j < NE; ++j) apply(ent[j]);
    if (!(dbg & 2))
      for (int64_t q = e0 + 64 * NE; q < e1; q += 64) {  // the rest (rare)
        const int64_t k = q + lane;
        if (k < e1) apply(pev[k]);
      }
    const uint64_t t_d = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    static_assert(4 * U == 16, "a loop iteration is one 16-piece stage");
    for (int32_t k0 = 0;; k0 += 16) {  // P0: rows k0 .. k0 + 15, P1: the next 16, P2: the 16 after
      issue(P0, 3 * U, d0, d1);
      const bool more = k0 + 16 < nmax;  // wave-uniform
      count(a0, a1);  // past the last stage P1 is all kPieceNone: the loads fall out of range
      issue(P1, 0, a0, a1);
      count(b0, b1);
      issue(P1, U, b0, b1);
      count(c0, c1);
      issue(P1, 2 * U, c0, c1);
      count(d0, d1);
      if (!more) break;
      P0 = P1;
      P1 = P2;
      P2 = stage(k0 + 48);
    }
    fold();
    const uint64_t t_e = (dbg & 16) ? __builtin_readcyclecounter() : 0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint4 *e4 = reinterpret_cast<uint4 *>(ev + 8 * lane), *m4 = reinterpret_cast<uint4 *>(mk + 8 * lane);
    uint32_t kinds = 0, nrec = 0, ncpx = 0;
    if (!(dbg & 4)) {
      uint32_t e8[8], m8[8];
      {
        const uint4 ea = e4[0], eb = e4[1], ma = m4[0], mb = m4[1];
        e8[0] = ea.x, e8[1] = ea.y, e8[2] = ea.z, e8[3] = ea.w, e8[4] = eb.x, e8[5] = eb.y, e8[6] = eb.z, e8[7] = eb.w;
        m8[0] = ma.x, m8[1] = ma.y, m8[2] = ma.z, m8[3] = ma.w, m8[4] = mb.x, m8[5] = mb.y, m8[6] = mb.z, m8[7] = mb.w;
      }
      // complex elements per locus: prefix of the range differences over the block
      int32_t run = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) run += (int32_t)m8[j] >> 16;
      int32_t ncx_run = (int32_t)wave_incl_scan((uint32_t)run) - run;  // before this lane's loci
      // ---- decision (GermlineThresholdCaller.scala:97-177 for single-base pileups), eight loci:
      //      kind 0 nothing, 1 a Ref/NoCall record, 2 a variant candidate (record pair), 3 complex
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int32_t l = B0 + 8 * lane + j;
        const bool in = l >= L0 && l < L1;
        const int h = j >> 2, sh = 8 * (j & 3);
        const uint32_t cA = (ca[h] >> sh) & 0xFFu, cC = (cc[h] >> sh) & 0xFFu;
        const uint32_t cT = (ct[h] >> sh) & 0xFFu, cG = (cg[h] >> sh) & 0xFFu;
        const uint32_t nN = (m8[j] >> 8) & 0xFFu;
        ncx_run += (int32_t)m8[j] >> 16;
        const uint32_t ncx = ncx_run > 0 ? (uint32_t)ncx_run : 0u;
        const uint32_t depth = cA + cC + cT + cG + nN + ncx;
        const uint32_t ew = e8[j];
        const uint32_t mask = (m8[j] & 15u) | (cA > (ew & 0xFFu) ? 1u : 0u) | (cC > ((ew >> 8) & 0xFFu) ? 2u : 0u) |
                              (cT > ((ew >> 16) & 0xFFu) ? 4u : 0u) | (cG > (ew >> 24) ? 8u : 0u);
        // branch-free (0/1 integers): the common hom-ref locus writes nothing
        const uint32_t live = (in ? 1u : 0u) & (depth > 0 ? 1u : 0u);
        const uint32_t ambiguous = (mask & (mask - 1u)) != 0 ? 1u : 0u;
        const uint32_t low = mask & (0u - mask);  // the first standard reference base, as a bit (or 0: N)
        const uint32_t c_ref = cA * (low & 1u) + cC * ((low >> 1) & 1u) + cT * ((low >> 2) & 1u) + cG * (low >> 3) +
                               nN * (low == 0u ? 1u : 0u);
        // ref C with G and N present: Scala map order by first occurrence (germline_complex)
        const uint32_t cgn = (low == 2u ? 1u : 0u) & (cG > 0 ? 1u : 0u) & (nN > 0 ? 1u : 0u);
        const uint32_t to_complex = live & (ambiguous | (ncx > 0 ? 1u : 0u) | (multi_sample ? 1u : 0u) | cgn);
        const uint32_t simple = live & (to_complex ^ 1u);
        const uint32_t alt_pass = passes(depth - c_ref, depth) ? 1u : 0u;  // some other allele may pass
        const uint32_t homref = simple & (alt_pass ^ 1u);
        const uint32_t ref_pass = (c_ref > 0 && passes(c_ref, depth)) ? 1u : 0u;
        const uint32_t emit_hr = homref & (ref_pass ? (uint32_t)(emit_ref != 0) : (uint32_t)(emit_no_call != 0));
        const uint32_t general = simple & alt_pass;
        visited += live;
        amb += live & ambiguous;
        const uint32_t kind = to_complex * 3u + general * 2u + emit_hr;  // at most one is set
        kinds |= kind << (2 * j);
        nrec += emit_hr + 2u * general;
        ncpx += to_complex;
      }
    }
    if (__ballot(kinds != 0) != 0) {  // rare: records / complex items to write
      const unsigned rbase = wave_reserve_lds_n(out.lds + 0, nrec);
      const unsigned cbase = wave_reserve_lds_n(out.lds + 1, ncpx);
      CallRec *prec_out = recs + out.base[0];
      unsigned kr = rbase, kc = cbase;
      constexpr uint64_t kAltSym = ((uint64_t)'<' << 8) | ((uint64_t)'A' << 16) | ((uint64_t)'L' << 24) |
                                   ((uint64_t)'T' << 32) | ((uint64_t)'>' << 40);
      for (int j = 0; j < 8; ++j) {
        const uint32_t kind = (kinds >> (2 * j)) & 3u;
        if (__ballot(kind != 0) == 0) continue;  // no lane writes for locus j (uniform skip)
        if (kind == 0) continue;
        const int32_t pos = B0 + 8 * lane + j;
        if (kind == 3) {
          if (kc < out.cap[1]) cplx[out.base[1] + kc] = ComplexItem{(int32_t)i, pos, 0};
          ++kc;
          continue;
        }
        const int sh = 8 * (j & 3);
        const bool hi = j >= 4;
        const uint32_t cA = ((hi ? ca[1] : ca[0]) >> sh) & 0xFFu, cC = ((hi ? cc[1] : cc[0]) >> sh) & 0xFFu;
        const uint32_t cT = ((hi ? ct[1] : ct[0]) >> sh) & 0xFFu, cG = ((hi ? cg[1] : cg[0]) >> sh) & 0xFFu;
        const uint32_t mw = mk[8 * lane + j], ew = ev[8 * lane + j];
        const uint32_t nN = (mw >> 8) & 0xFFu;
        const uint32_t mask = (mw & 15u) | (cA > (ew & 0xFFu) ? 1u : 0u) | (cC > ((ew >> 8) & 0xFFu) ? 2u : 0u) |
                              (cT > ((ew >> 16) & 0xFFu) ? 4u : 0u) | (cG > (ew >> 24) ? 8u : 0u);
        const uint8_t ref = mask ? bit_base(mask) : (uint8_t)'N';
        const uint64_t ord = (uint64_t)(f64(rec, 0) + (pos - L0));
        CallRec rr;
        rr.key = ord << 12;
        rr.contig = (int32_t)f32(rec, 6);
        rr.pos = pos;
        rr.sample = 0;
        if (kind == 1) {
          const uint32_t depth = cA + cC + cT + cG + nN;
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
          rr.alt_len = 0;
          rr.allele = (uint64_t)cA | ((uint64_t)cC << 16) | ((uint64_t)cT << 32) | ((uint64_t)cG << 48);
          if (kr < out.cap[0]) prec_out[kr] = rr;
          rr.flags = kCandidateSlot;
          if (kr + 1 < out.cap[0]) prec_out[kr + 1] = rr;
          kr += 2;
        }
      }
    }
    e4[0] = e4[1] = m4[0] = m4[1] = make_uint4(0u, 0u, 0u, 0u);  // this lane's words, for the next tile
    if (dbg & 16) {  // phase clocks (cycles per tile and wave): setup, first loads, entries, counting, decision
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
