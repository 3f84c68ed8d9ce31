// gq_somatic_direct.h — somatic_direct: the somatic-standard candidate test straight from the
// resident reads, with no projection and no margin projection.  Included inside gq_somatic.hip's
// anonymous namespace, after gq_somatic_proj.h (margin_table, RefView, ref_agrees).
//
// It restates somatic_proj's per-locus test (SomaticStandardCaller.scala:184-206: the tumor
// pileup must hold a non-Match element, the normal's must be non-empty; loci whose tumor pileup
// provably has the hom-ref genotype as its maximum-likelihood genotype are dropped) on
// germline_direct's machinery (gq_germline_direct.h): one WAVE per 512-locus tile, lane l owns
// the 8-locus column [B0 + 8l, B0 + 8l + 8), the tile's tumor read window goes through in chunks
// of up to kSlots runs, each run of Match/Mismatch elements an 8-byte LDS slot; lanes walk their
// column's slots in groups of four columns (GQ_DIR_GROUP) with one unaligned 8-byte load of
// bases AND one of qualities per (slot, column):
//   counts   base codes in SWAR registers as germline_direct's DEEP instantiation (16-bit pairs);
//   margins  each element's hom-ref margin term (margin_table: the mproj bytes, biased by 128,
//            1/8 units) looked up for a Match element (the read's mapping-quality row of the
//            table, staged in LDS for the tile's first read's mapq) and added per locus; at an
//            MD event the element is a Mismatch: the runs phase adds term(mismatch) -
//            term(match) for that element (its quality loaded with its read base), so each
//            locus sums exactly the terms the margin projection held.  A kMargin8None term
//            anywhere in the tile drops the tile's bound (somatic_proj: the block's slices);
//            reads below min_mapq add no term (QualityAlignedReadsFilter).
// MD events, N bases and complex ranges (insertion / deletion anchors, mid-deletions, clipped
// N-skips) are handled as germline_direct does (mid-deletions count as complex here), and the
// normal's depth comes from its reads' [start, end) as a difference array (somatic_proj).  A tile
// the kernel cannot take (a byte other than A C G T N, a read without MD, a CIGAR the segments
// cannot express, a round of more than kSlots runs, a window past 65535 reads) goes to
// somatic_tile, as somatic_proj's pbad tiles do.  The candidates leave through the same
// per-workgroup partitions, so cand_prep and the callers see somatic_proj's list (the bound
// is the same sum of the same bytes, so the same loci).
#pragma once

#ifndef GQ_SOMD_PAIR
#define GQ_SOMD_PAIR 0
#endif
#ifndef GQ_SDIR_GROUP
#define GQ_SDIR_GROUP 1  // lanes walking their slots together (under the rotated schedule every lane
                         // covering a slot reads it at the same iteration: groups of 1 / 2 / 4 / 8
                         // measured 6.25 / 6.36 / 6.61 / 7.02 ms at chr20 60x)
#endif

struct SomDirCfg {
  static constexpr int kT = 512;
  static constexpr int kWaves = 4;
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kU = 4;         // slots per batch
  static constexpr int kRound = 64;    // window reads per round
  static constexpr int kSlots = 256;   // runs per chunk
  static constexpr int64_t kMaxWin = 65535;
};

template <bool kRef>
__global__ __launch_bounds__(SomDirCfg::kThreads) void somatic_direct(
    const Tile *__restrict__ tiles_t, const Tile *__restrict__ tiles_n, int64_t n_tiles, DevReads R,
    const int32_t *__restrict__ n_start, const int32_t *__restrict__ n_end, const uint8_t *__restrict__ tab,
    int min_mapq, ComplexItem *__restrict__ cand, OutGeom og, Counters *ctr, int32_t *__restrict__ slow, RefView ref,
    int no_bound, int dbg) {
  // dbg (diagnostics: env GQ_DBG >> 16, clear of the callers' bits; results are wrong when set):
  // 1 no margin lookups, 2 no normal depth, 32 no counting, 64 no MD events
  using C = SomDirCfg;
  constexpr int T = C::kT, U = C::kU;
  // per locus x of the block at word ix(x) = (x & 7) * 64 + (x >> 3): event read bases (A | C << 16
  // at [x], T | G << 16 at [T + x]); MD bits 0-3 | complex diff << 16; normal coverage
  // differences; margin corrections (signed, 1/8 units)
  __shared__ __attribute__((aligned(16))) uint32_t evw[C::kWaves][2 * T];
  __shared__ __attribute__((aligned(16))) uint32_t mkw[C::kWaves][T];
  __shared__ __attribute__((aligned(16))) uint32_t cvw[C::kWaves][T];
  __shared__ __attribute__((aligned(16))) int32_t mcw[C::kWaves][T];
  __shared__ __attribute__((aligned(16))) uint2 rcw[C::kWaves][C::kSlots];
  __shared__ uint16_t rqw[C::kWaves][C::kSlots];  // each slot's read: mapq | kept << 8 (0: no margin terms)
  __shared__ int32_t hxw[C::kWaves][64], hnw[C::kWaves][64];
  // per workgroup: the margin_table rows of mapping qualities 0-63 (the aligners' range), byte
  // mq << 8 | q << 1 | match as in the global table (16 KiB; a read of higher mapq looks its
  // terms up there)
  __shared__ __attribute__((aligned(16))) uint32_t mterm_w[64 * 256 / 4];
  // GQ_SOMD_PAIR: the Match terms of a quality pair (q0, q1 < 64) of the workgroup's first
  // tumor read's mapq, t(q0) | t(q1) << 8 at q0 | q1 << 6: one LDS read per two elements
  __shared__ uint16_t ptab[GQ_SOMD_PAIR ? 4096 : 1];
  __shared__ unsigned outn[2];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint32_t *ev = evw[wave], *mk = mkw[wave], *cv = cvw[wave];
  int32_t *mc = mcw[wave];
  uint2 *rc = rcw[wave];
  uint16_t *rq = rqw[wave];
  int32_t *hx = hxw[wave], *hn = hnw[wave];
  auto ix = [](int32_t x) { return ((x & 7) << 6) | (x >> 3); };
  auto zero_words = [&]() {
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    uint4 *e4 = reinterpret_cast<uint4 *>(ev), *m4 = reinterpret_cast<uint4 *>(mk), *c4 = reinterpret_cast<uint4 *>(cv),
          *g4 = reinterpret_cast<uint4 *>(mc);
#pragma unroll
    for (int q = 0; q < 2 * T / 256; ++q) e4[64 * q + lane] = z4;
    m4[lane] = z4; m4[64 + lane] = z4; c4[lane] = z4; c4[64 + lane] = z4; g4[lane] = z4; g4[64 + lane] = z4;
  };
  zero_words();
  if (threadIdx.x < 2) outn[threadIdx.x] = 0;
  const int64_t per = n_tiles / gridDim.x, extra = n_tiles % gridDim.x;
  const int64_t i0 = blockIdx.x * per + min((int64_t)blockIdx.x, extra);
  const int64_t i1 = i0 + per + ((int64_t)blockIdx.x < extra ? 1 : 0);
  for (int w = threadIdx.x; w < 64 * 256 / 4; w += C::kThreads) mterm_w[w] = reinterpret_cast<const uint32_t *>(tab)[w];
  uint32_t pmq = 0x100u;  // (none)
  if (GQ_SOMD_PAIR && i0 < i1) {
    const Tile t0 = tiles_t[i0];
    pmq = t0.re > t0.rb ? (uint32_t)R.mapq[t0.rb] : 0x100u;
    if (pmq < 0x100u) {
      const uint8_t *row = tab + (pmq << 8);
      for (int e = threadIdx.x; e < 4096; e += C::kThreads)
        ptab[e] = (uint16_t)((uint32_t)row[((e & 63) << 1) | 1] | ((uint32_t)row[(((e >> 6) & 63) << 1) | 1] << 8));
    }
  }
  __syncthreads();
  const uint8_t *mterm = reinterpret_cast<const uint8_t *>(mterm_w);
  const unsigned long long cbase = og.slot(1, (int)blockIdx.x, 0), ccap = og.capA[1];
  unsigned visited = 0;
  const int32_t colr = 8 * lane;
  // the margin term byte of a Match (match = 1) or Mismatch element of quality q from row p
  auto term = [](const uint8_t *p, uint32_t q, uint32_t match) -> uint32_t {
    return (q & 0x80u) ? (uint32_t)kMargin8None : (uint32_t)p[((q & 0x7Fu) << 1) | match];
  };
  for (int64_t i = i0 + wave; i < i1; i += C::kWaves) {
    const Tile tt = tiles_t[i], tn = tiles_n[i];
    const int32_t L0 = tt.L0, L1 = tt.L1;
    const int64_t rb = tt.rb, re = tt.re;
    const int32_t B0 = L0 & ~(T - 1);
    const int32_t col = B0 + colr;
    if (tn.re - tn.rb >= C::kMaxWin || re - rb > C::kMaxWin) {
      if (lane == 0) slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)i;
      continue;
    }
    // ---- normal depth: each read spans [start, end) (any element), as +1 / -1 differences
    for (int64_t q = tn.rb; q < ((dbg & 2) ? tn.rb : tn.re); q += 64) {
      const int64_t r = q + lane;
      if (r < tn.re) {
        const int32_t a = max(n_start[r], B0), b = min(n_end[r], B0 + T);
        if (a < b) {
          atomicAdd(&cv[ix(a - B0)], 1u);
          if (b < B0 + T) atomicAdd(&cv[ix(b - B0)], 0xFFFFFFFFu);
        }
      }
    }
    // counters: nibbles folded into bytes every 12 slots, widened into 16-bit pairs every 240
    uint32_t ca[2] = {0, 0}, cc[2] = {0, 0}, ct[2] = {0, 0}, cg[2] = {0, 0}, cn[2] = {0, 0};
    uint32_t wA[4] = {0, 0, 0, 0}, wC[4] = {0, 0, 0, 0}, wT[4] = {0, 0, 0, 0}, wG[4] = {0, 0, 0, 0},
             wN[4] = {0, 0, 0, 0};
    uint32_t nac[2] = {0, 0}, ntg[2] = {0, 0};
    uint32_t msum[4] = {0, 0, 0, 0};  // biased margin bytes, loci 2k, 2k + 1 as 16-bit pairs
    int32_t m32[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int32_t iters = 0;  // slot iterations (each adds 8 biased bytes: 128 each where nothing counts)
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
      auto w2 = [](uint32_t (&w)[4], uint32_t (&c)[2]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          w[2 * h] += __builtin_amdgcn_perm(0u, c[h], 0x0c010c00u);
          w[2 * h + 1] += __builtin_amdgcn_perm(0u, c[h], 0x0c030c02u);
          c[h] = 0;
        }
      };
      w2(wA, ca);
      w2(wC, cc);
      w2(wT, ct);
      w2(wG, cg);
      w2(wN, cn);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        m32[2 * q] += (int32_t)(msum[q] & 0xFFFFu);
        m32[2 * q + 1] += (int32_t)(msum[q] >> 16);
        msum[q] = 0;
      }
    };
    bool bad = false, none = false;
    uint32_t badb = 0;
    struct Fields {
      int32_t s, e, nmd, ld;
      int64_t so, mo;
      uint32_t mq;
    };
    auto load_fields = [&](int64_t c0) {
      Fields f{0, 0, 0, 0, 0, 0, 0};
      const int64_t r = c0 + lane;
      if (r < re) {
        f.s = R.start[r];
        f.e = R.end[r];
        f.so = R.seq_off[r];
        f.ld = R.lead[r];
        f.nmd = R.n_md[r];
        f.mo = R.md_off[r];
        f.mq = R.mapq[r];
      }
      return f;
    };
    int64_t tbase = 0;
    __amdgpu_buffer_rsrc_t srs, qrs;
    Fields nf = load_fields(rb);
    int64_t c0 = rb;
    bool first_round = true;
    while (c0 < re) {  // ---- a chunk: rounds while their runs fit kSlots slots, then the counting
      hx[lane] = -1;
      hn[lane] = 0x7FFFFFFF;
      int32_t nslot = 0;
      while (c0 < re) {
        const int64_t r = c0 + lane;
        const bool valid = r < re;
        const Fields f = nf;
        const int32_t s = f.s, e = f.e, nmd = f.nmd, ld = f.ld;
        const int64_t so = f.so, mo = f.mo;
        const uint32_t mq = f.mq;
        const bool kept = min_mapq <= 0 || (int)mq >= min_mapq;
        const bool nomd = valid && nmd < 0;
        const bool gen = valid && !nomd && ld < 0;
        uint32_t nrun = valid && !nomd && !gen && e > B0 && s < B0 + T ? 1u : 0u;
        const bool evr = valid && !nomd && nmd > 0 && s < B0 + T && !(dbg & 64);
        uint32_t v4[4] = {0u, 0u, 0u, 0u};
        auto load_ev = [&](int32_t k0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v4[j] = R.md_ev[mo + (k0 + j < nmd ? k0 + j : nmd - 1)];
        };
        // an event's element at locus l: its read base's count (A C T G; an N there is counted
        // with the bases), and its margin term as a Mismatch in place of the Match term the
        // counting adds (a term outside the table drops the tile's bound)
        auto ev_add = [&](int32_t l, uint8_t base, uint8_t qv) {
          const int32_t x = ix(l - B0);
          const int cat = base_cat(base);
          if (cat < 4) atomicAdd(&ev[(cat >> 1) * T + x], 1u << (16 * (cat & 1)));
          if (kept) {
            uint32_t t0, t1;
            if (mq < 64u) {  // (the workgroup's LDS rows)
              t0 = term(mterm + (mq << 8), qv, 0u);
              t1 = term(mterm + (mq << 8), qv, 1u);
            } else {
              t0 = term(tab + (mq << 8), qv, 0u);
              t1 = term(tab + (mq << 8), qv, 1u);
            }
            none = none || t0 == kMargin8None || t1 == kMargin8None;
            if (t0 != t1) atomicAdd(&mc[x], (int32_t)t0 - (int32_t)t1);
          }
        };
        if (evr) load_ev(0);
        if (gen && e > B0 && s < B0 + T) nrun = (uint32_t)min(-1 - ld, C::kSlots);
        const uint32_t incl = wave_incl_scan(nrun);
        const int32_t total = (int32_t)__builtin_amdgcn_readlane((int)incl, 63);
        if (nslot > 0 && nslot + total > C::kSlots) break;  // (the round opens the next chunk)
        if (total > C::kSlots) {
          bad = true;
          c0 = re;
          break;
        }
        if (c0 + C::kRound < re) nf = load_fields(c0 + C::kRound);
        if (first_round) {  // the tile's pool base, from the first round's reads
          int64_t so_min = valid ? so : INT64_MAX;
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_xor(so_min, d, 64);
            so_min = o < so_min ? o : so_min;
          }
          tbase = so_min >= 8 ? so_min - 8 : 0;
          tbase = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)tbase >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)tbase));
          const int64_t span = R.seq_cap - tbase;
          const int sp32 = (int)(span < 0x7FFFFFFF ? span : 0x7FFFFFFF);
          srs = __builtin_amdgcn_make_buffer_rsrc((void *)(R.seq + tbase), (short)0, sp32, 0x00020000);
          qrs = __builtin_amdgcn_make_buffer_rsrc((void *)(R.qual + tbase), (short)0, sp32, 0x00020000);
          first_round = false;
        }
        bad = bad || nomd ||
              (valid && (so < tbase || so + (ld > 0 ? ld : 0) + (e > s ? e - s : 0) + 16384 + 1024 - tbase >= 0x7FFFFFF0ll));
        int32_t slot = nslot + (int32_t)(incl - nrun);
        auto put = [&](int32_t a, int32_t b, int64_t p) {
          const int32_t s16 = min(max(a - B0, -32768), 32767), e16 = min(max(b - B0, -32768), 32767);
          const int32_t K = (int32_t)(p - tbase - (int64_t)(a - B0));
          rc[slot] = make_uint2((uint32_t)(uint16_t)s16 | ((uint32_t)(uint16_t)e16 << 16), (uint32_t)K);
          rq[slot] = kept ? (uint16_t)(mq | 0x100u) : (uint16_t)0;  // (a read the mapq filter drops: no terms)
          atomicMax(&hx[min(max(s16, 0), T - 1) >> 3], slot);
          atomicMin(&hn[min(max(e16 - 1, 0), T - 1) >> 3], slot);
          ++slot;
        };
        if (nrun && !gen) put(s, e, so + (ld > 0 ? ld : 0));
        if (gen && e > B0 && s < B0 + T) {
          const int32_t slot_end = slot + (int32_t)nrun;
          const bool ok = general_segments(R, r, [&](uint32_t kind, int32_t ro, int32_t len, int32_t sp, int32_t) {
            const int32_t a = s + ro, b = a + len;
            if (b <= B0 || a >= B0 + T) return;
            if (kind == kSegCount) {
              if (slot < slot_end) put(a, b, so + sp);
              else bad = true;
              if (evr) {
                const int32_t x0 = a > B0 ? a : B0, x1 = b < B0 + T ? b : B0 + T;
                for (int32_t k = 0; k < nmd; ++k) {
                  const int32_t l = s + (int32_t)(R.md_ev[mo + k] >> 8);
                  if (l >= x1) break;
                  if (l >= x0) ev_add(l, R.seq[so + sp + (l - a)], R.qual[so + sp + (l - a)]);
                }
              }
            } else {  // complex ranges and mid-deletions: complex here (somatic_proj's kPevComplex)
              const int32_t x0 = a > B0 ? a : B0, x1 = b < B0 + T ? b : B0 + T;
              atomicAdd(&mk[ix(x0 - B0)], 1u << 16);
              if (x1 < B0 + T) atomicAdd(&mk[ix(x1 - B0)], 0xFFFF0000u);
            }
          });
          bad = bad || !ok;
          for (; slot < slot_end; ++slot) {
            rc[slot] = make_uint2(0u, 0u);
            rq[slot] = 0;
          }
        }
        // MD events in the block: the MD reference base's bit; for a simple read its element's
        // read base and margin correction (a general read's went with its count segments)
        if (evr) {
          for (int32_t k0 = 0;;) {
            bool past = false;
            uint8_t b4[4], q4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int32_t o = (int32_t)(v4[j] >> 8);
              const bool in = !gen && o < e - s;
              b4[j] = in ? R.seq[so + ld + o] : (uint8_t)0;
              q4[j] = in ? R.qual[so + ld + o] : (uint8_t)0;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int32_t l = s + (int32_t)(v4[j] >> 8);
              past = past || l >= B0 + T;
              if (k0 + j >= nmd || l < B0 || l >= B0 + T) continue;
              const uint32_t m = std_bit((uint8_t)(v4[j] & 0xFFu));
              if (m) atomicOr(&mk[ix(l - B0)], m);
              if (!gen && (int32_t)(v4[j] >> 8) < e - s) ev_add(l, b4[j], q4[j]);
            }
            k0 += 4;
            if (past || k0 >= nmd) break;
            load_ev(k0);
          }
        }
        nslot += total;
        c0 += C::kRound;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // ---- this lane's group's slots
      int32_t last = wave_incl_max_i(hx[lane]);
      int32_t first = wave_suffix_min_i(hn[lane]);
      if (GQ_SDIR_GROUP > 1) {
        first = __shfl(first, lane & ~(GQ_SDIR_GROUP - 1), 64);
        last = __shfl(last, lane | (GQ_SDIR_GROUP - 1), 64);
      }
      const int32_t nl = last >= first ? last - first + 1 : 0;
      int32_t kmax = nl;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) kmax = max(kmax, __shfl_xor(kmax, d, 64));
      kmax = (dbg & 32) ? 0 : __builtin_amdgcn_readfirstlane(kmax);
      // the slot schedule: iteration k takes the slot s of [first, first + kmax) with s = k (mod
      // kmax), so every group reaches a slot at the same iteration (k = s mod kmax) and one load
      // instruction reads a read's bytes for all the groups its run covers (the lines it touches
      // are fetched once, while they are hot); t0 = the offset of iteration 0
      const int32_t t0 = (GQ_DIR_ROT && kmax > 0 && nl > 0) ? (kmax - first % kmax) % kmax : 0;
      // a batch: U slots' base and quality loads, all issued before any is used
      auto issue = [&](int32_t k0, uint2 (&x)[U], uint2 (&y)[U], uint32_t (&mt)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int32_t k = k0 + u;
          int32_t t = t0 + k;  // (GQ_DIR_ROT) the lane's slot offset at iteration k
          t = t >= kmax ? t - kmax : t;
          const bool mine = GQ_DIR_ROT ? (k < kmax && t < nl) : k < nl;
          const int32_t sl = mine ? first + (GQ_DIR_ROT ? t : k) : 0;
          const uint2 d = rc[sl];
          const uint32_t mqs = rq[sl];  // mapq | kept << 8
          const int32_t s16 = (int32_t)(int16_t)(d.x & 0xFFFFu), e16 = (int32_t)(int16_t)(d.x >> 16);
          const int32_t a = min(max(s16 - colr, 0), 8), b = min(max(e16 - colr, 0), 8);
          const bool live = mine && b > a;
          const int32_t vi = (int32_t)d.y + colr;
          const uint32_t vo = live ? (uint32_t)max(vi, 0) : 0x80000000u;
          const auto w = __builtin_amdgcn_raw_buffer_load_b64(srs, (int)vo, 0, 0);
          const auto q = __builtin_amdgcn_raw_buffer_load_b64(qrs, (int)vo, 0, 0);
          x[u] = make_uint2(w[0], w[1]);
          y[u] = make_uint2(q[0], q[1]);
          mt[u] = live ? (uint32_t)a | ((uint32_t)b << 4) | ((uint32_t)max(-vi, 0) << 8) | (mqs << 16) : 0u;
        }
      };
      auto count = [&](const uint2 (&x)[U], const uint2 (&y)[U], const uint32_t (&mt)[U]) {
        if (nn + U > 15) fold();
        bool low_mq = true;  // (uniform) every slot of the batch with terms has its row in LDS
#pragma unroll
        for (int u = 0; u < U; ++u) low_mq = low_mq && (!((mt[u] >> 24) & 1u) || ((mt[u] >> 16) & 0xFFu) < 64u);
        const bool lds_terms = __ballot(!low_mq) == 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t la = mt[u] & 15u, lb = (mt[u] >> 4) & 15u, sh = (mt[u] >> 5) & 56u;
          const uint32_t mqs = (mt[u] >> 16) & 0xFFu;
          const bool kept_s = ((mt[u] >> 24) & 1u) != 0u;
          const uint64_t m = byte_range_mask((int32_t)la, (int32_t)lb);
          const uint64_t w64 = ((uint64_t)x[u].x | ((uint64_t)x[u].y << 32)) << sh;
          const uint64_t q64 = ((uint64_t)y[u].x | ((uint64_t)y[u].y << 32)) << sh;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t wh = (uint32_t)(w64 >> (32 * h)), mh = (uint32_t)(m >> (32 * h));
            const uint32_t xc = wh & 0x07070707u;
            const uint32_t ex = __builtin_amdgcn_perm(0x474EFF54u, 0x43FF41FFu, xc);
            badb |= (wh ^ ex) & mh;
            const uint32_t cd = xc & mh;
            nac[h] += __builtin_amdgcn_perm(0u, 0x10000100u, cd);
            ntg[h] += __builtin_amdgcn_perm(0x10000001u, 0u, cd);
            cn[h] += __builtin_amdgcn_perm(0x00010000u, 0u, cd);
          }
          // margin terms of the Match elements (bytes outside the run or of a dropped read: 128):
          // branch-free lookups (a quality past the table reads its byte and is replaced by
          // kMargin8None), packed into two words, then masked
          uint32_t tv[2];
          const uint64_t live = kept_s ? m : 0ull;
          const bool pu = !kept_s || (mqs == pmq && (q64 & live & 0xC0C0C0C0C0C0C0C0ull) == 0ull);
          if (dbg & 1) {
            tv[0] = tv[1] = 0x80808080u;  // (diagnostics: no lookups)
          } else if (GQ_SOMD_PAIR && __ballot(!pu) == 0) {  // (uniform) every slot on the pair table
            uint32_t pr[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const uint32_t c2 = (uint32_t)(q64 >> (16 * j)) & 0xFFFFu;
              pr[j] = ptab[(c2 & 63u) | ((c2 >> 2) & 0xFC0u)];
            }
            const uint32_t lo = (uint32_t)live, hi = (uint32_t)(live >> 32);
            tv[0] = ((pr[0] | (pr[1] << 16)) & lo) | (0x80808080u & ~lo);
            tv[1] = ((pr[2] | (pr[3] << 16)) & hi) | (0x80808080u & ~hi);
            auto zb = [](uint32_t v) { return ((v - 0x01010101u) & ~v & 0x80808080u) != 0u; };
            none = none || zb(tv[0]) || zb(tv[1]);
          } else {
            uint32_t t8[8];
            if (lds_terms) {
              const uint8_t *rowl = mterm + ((mqs & 63u) << 8);
#pragma unroll
              for (int k = 0; k < 8; ++k) t8[k] = rowl[((((uint32_t)(q64 >> (8 * k))) & 0x7Fu) << 1) | 1u];
            } else {
              const uint8_t *rowg = tab + (mqs << 8);
#pragma unroll
              for (int k = 0; k < 8; ++k) t8[k] = rowg[(((uint32_t)(q64 >> (8 * k)) & 0x7Fu) << 1) | 1u];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) t8[k] = ((q64 >> (8 * k + 7)) & 1u) ? (uint32_t)kMargin8None : t8[k];
            const uint32_t lo = (uint32_t)live, hi = (uint32_t)(live >> 32);
            tv[0] = ((t8[0] | (t8[1] << 8) | (t8[2] << 16) | (t8[3] << 24)) & lo) | (0x80808080u & ~lo);
            tv[1] = ((t8[4] | (t8[5] << 8) | (t8[6] << 16) | (t8[7] << 24)) & hi) | (0x80808080u & ~hi);
            auto zb = [](uint32_t v) { return ((v - 0x01010101u) & ~v & 0x80808080u) != 0u; };
            none = none || zb(tv[0]) || zb(tv[1]);
          }
          msum[0] += __builtin_amdgcn_perm(0u, tv[0], 0x0c010c00u);
          msum[1] += __builtin_amdgcn_perm(0u, tv[0], 0x0c030c02u);
          msum[2] += __builtin_amdgcn_perm(0u, tv[1], 0x0c010c00u);
          msum[3] += __builtin_amdgcn_perm(0u, tv[1], 0x0c030c02u);
        }
        nn += U;
        since += U;
        iters += U;
        if (since == 240) {  // uniform: bytes and 16-bit margin pairs hold 240 slots at most
          fold();
          widen();
          since = 0;
        }
      };
      if (kmax > 0) {  // one batch in flight while one is counted
        uint2 xa[U], xb[U], ya[U], yb[U];
        uint32_t ma[U], mb[U];
        issue(0, xa, ya, ma);
        for (int32_t k0 = 0;; k0 += 2 * U) {
          issue(k0 + U, xb, yb, mb);
          count(xa, ya, ma);
          if (k0 + U >= kmax) break;
          issue(k0 + 2 * U, xa, ya, ma);
          count(xb, yb, mb);
          if (k0 + 2 * U >= kmax) break;
        }
      }
    }
    fold();
    widen();
    if (__ballot(bad || badb != 0) != 0) {  // somatic_tile takes the tile (exact for every read)
      zero_words();
      if (lane == 0) slow[atomicAdd(&ctr->n_slow, 1ull)] = (int32_t)i;
      continue;
    }
    const bool nb = __ballot(none) != 0;  // a term outside the table: no bound in this tile
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ---- decision: candidate loci (somatic_proj's test)
    uint32_t m8[8], v8[8], e8a[8], e8b[8];
    int32_t g8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m8[j] = mk[64 * j + lane];
      v8[j] = cv[64 * j + lane];
      e8a[j] = ev[64 * j + lane];
      e8b[j] = ev[T + 64 * j + lane];
      g8[j] = mc[64 * j + lane];
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
    uint2 fb8 = make_uint2(0u, 0u);
    if constexpr (kRef) fb8 = *reinterpret_cast<const uint2 *>(ref.b + ref.off[tt.contig] + B0 + 8 * lane);
    const int32_t bias = 128 * iters;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int32_t l = col + j;
      const bool in = l >= L0 && l < L1;
      const int q2 = j >> 1, sh = 16 * (j & 1);
      const uint32_t cA = (wA[q2] >> sh) & 0xFFFFu, cC = (wC[q2] >> sh) & 0xFFFFu;
      const uint32_t cT = (wT[q2] >> sh) & 0xFFFFu, cG = (wG[q2] >> sh) & 0xFFFFu;
      const uint32_t nN = (wN[q2] >> sh) & 0xFFFFu;
      ncx_run += (int32_t)m8[j] >> 16;
      dn_run += (int32_t)v8[j];
      const uint32_t ncx = ncx_run > 0 ? (uint32_t)ncx_run : 0u;
      const uint32_t depth = cA + cC + cT + cG + nN + ncx;
      const uint32_t eac = e8a[j], etg = e8b[j];
      const uint32_t mask = (m8[j] & 15u) | (cA > (eac & 0xFFFFu) ? 1u : 0u) | (cC > (eac >> 16) ? 2u : 0u) |
                            (cT > (etg & 0xFFFFu) ? 4u : 0u) | (cG > (etg >> 16) ? 8u : 0u);
      const uint32_t low = mask & (0u - mask);
      const uint32_t c_ref = (cA & (0u - (low & 1u))) + (cC & (0u - ((low >> 1) & 1u))) +
                             (cT & (0u - ((low >> 2) & 1u))) + (cG & (0u - ((low >> 3) & 1u))) + (low == 0u ? nN : 0u);
      bool agree = true;
      if constexpr (kRef) agree = ref_agrees(mask, ((j < 4 ? fb8.x : fb8.y) >> (8 * (j & 3))) & 0xFFu);
      const bool single = mask != 0 && (mask & (mask - 1u)) == 0;
      const bool nonmatch = !agree || (mask & (mask - 1u)) != 0 || ncx > 0 || depth > c_ref;
      const int32_t msj = m32[j] - bias + g8[j];  // the locus's margin, 1/8 units
      const bool bound = !no_bound && !nb && agree && single && ncx == 0 && nN == 0 &&
                         (float)msj * 0.125f > 0.02f + 2e-4f * (float)depth;
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
          if (kq < ccap) cand[cbase + kq] = ComplexItem{(int32_t)i, col + j, 0};
          ++kq;
        }
    }
    zero_words();  // for the next tile (the wave's own words: no barrier)
  }
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
