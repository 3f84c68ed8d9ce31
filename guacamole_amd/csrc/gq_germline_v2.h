// gq_germline_v2.h — germline-threshold tile kernel, locus-major form (the default).
//
// One workgroup of W waves owns a tile of T = 256 * W loci; lane l of wave w owns the four
// consecutive loci 256 w + 4 l .. + 3.  Per batch of up to 64 W reads:
//   1. the batch's contiguous sequence bytes are copied HBM -> LDS by LDS-DMA
//      (global_load_lds_dwordx4: 1 KiB per wave-instruction, fully coalesced) while every
//      thread loads one read's metadata (coalesced) into an LDS table;
//   2. each wave walks the reads overlapping its 256 loci in start order (wave-uniform
//      loop: the read's fields are broadcast from LDS); every lane reads its 4 bases with
//      two aligned ds_read_b32 + v_alignbyte and counts them into byte-lane registers (one
//      byte per locus per category, SWAR: (b >> 1) & 7 -> v_perm table lookups) — no LDS
//      atomics, no histogram in LDS; MD events and CIGAR anchors are wave-uniform and touch
//      one lane each;
//   3. byte counters are folded into 16-bit pair accumulators every <= 250 reads.
// Then each lane decides its four loci exactly as germline_tile (v1) does.
//
// Element semantics: PileupElement.scala:68-248 (restated in gq_kernels.h walk_read_lane);
// decision: GermlineThresholdCaller.scala:100-177.
#pragma once

namespace {

constexpr int kV2Stage = 40 * 1024;  // sequence bytes staged per batch
constexpr int kV2Pad = 16;           // LDS slack before / after the staged bytes
constexpr int kEvBias = 1 << 20;     // pooled simple-read events hold tile locus + kEvBias

struct ByteCounters {  // byte j = locus i0 + j
  uint32_t A, C, T, G;  // Match/Mismatch elements by sequenced base
  uint32_t V, E;        // all Match/Mismatch elements / those whose base is one of A C G T N
  uint32_t X;           // non-SNV elements (insertion / deletion anchors, mid-deletions, clipped)
  uint32_t eA, eC, eT, eG;  // SNV elements carrying an MD mismatch event, by sequenced base
};

struct PairAcc {  // 16-bit pair accumulators for one locus
  uint32_t AC, TG, VE, X, eAC, eTG;
};

// 0x01 in byte j for lo <= j < hi (clamped to [0, 4))
__device__ __forceinline__ uint32_t range_mask4(int lo, int hi) {
  lo = lo < 0 ? 0 : lo;
  hi = hi > 4 ? 4 : hi;
  if (hi <= lo) return 0u;
  const uint32_t up = 0x01010101u >> (8 * (4 - hi));
  return up & (0x01010101u << (8 * lo));
}

// four sequenced bases (bytes of w, valid where vm has 0x01) into the byte counters
__device__ __forceinline__ void count_word(ByteCounters &bc, uint32_t w, uint32_t vm) {
  const uint32_t code4 = (w >> 1) & 0x07070707u;
  const uint32_t exp4 = __builtin_amdgcn_perm(0x4E000000u, 0x47544341u, code4);  // A C T G . . . N
  const uint32_t x = w ^ exp4;
  const uint32_t nz = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;  // bit 7 set in non-zero bytes
  const uint32_t eq = ((nz >> 7) ^ 0x01010101u) & vm;           // valid bytes that are A C G T N
  const uint32_t oh = __builtin_amdgcn_perm(0x10000000u, 0x08040201u, code4);  // one-hot A C T G . . . N
  bc.A += oh & eq;
  bc.C += (oh >> 1) & eq;
  bc.T += (oh >> 2) & eq;
  bc.G += (oh >> 3) & eq;
  bc.V += vm;
  bc.E += eq;
}

__device__ __forceinline__ void fold_counters(ByteCounters &bc, PairAcc *acc) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int sh = 8 * j;
    auto b = [&](uint32_t v) { return (v >> sh) & 0xFFu; };
    acc[j].AC += b(bc.A) | (b(bc.C) << 16);
    acc[j].TG += b(bc.T) | (b(bc.G) << 16);
    acc[j].VE += b(bc.V) | (b(bc.E) << 16);
    acc[j].X += b(bc.X);
    acc[j].eAC += b(bc.eA) | (b(bc.eC) << 16);
    acc[j].eTG += b(bc.eT) | (b(bc.eG) << 16);
  }
  bc.A = bc.C = bc.T = bc.G = bc.V = bc.E = bc.X = bc.eA = bc.eC = bc.eT = bc.eG = 0u;
}

#define UNI(x) __builtin_amdgcn_readfirstlane(x)

template <int W, int ABL = 0>
__global__ __launch_bounds__(64 * W) void germline_tile_v2(const Tile *__restrict__ tiles, DevReads R, int threshold,
                                                           int emit_ref, int emit_no_call, CallRec *__restrict__ recs,
                                                           unsigned long long rec_cap,
                                                           ComplexItem *__restrict__ cplx,
                                                           unsigned long long cplx_cap, Counters *ctr) {
  constexpr int NT = 64 * W;   // threads = reads per batch
  constexpr int TL = 256 * W;  // loci per tile
  constexpr int EVP = 4 * NT;  // LDS pool of MD events (offset << 8 | base) + the read base under each
  constexpr int CGP = 2 * NT;  // LDS pool of CIGAR operators of general reads
  __shared__ __attribute__((aligned(16))) uint32_t stage32[(kV2Stage + 2 * kV2Pad) / 4];
  __shared__ int32_t m_s[NT], m_boff[NT];
  __shared__ int16_t m_e[NT], m_pm[NT];  // clamped to [-16, T + 16]
  __shared__ uint32_t m_w0[NT];  // bit0 simple CIGAR, bit1 staged, bit2 events pooled, bit3 CIGAR pooled,
                                 // bits 8-15 n_cigar (pooled only), bits 16-31 event pool offset
  __shared__ uint32_t m_w1[NT];  // bits 0-15 n_md (0 if none), bits 16-31 CIGAR pool offset
  __shared__ uint32_t ev_pool[EVP], cg_pool[CGP];
  __shared__ uint8_t rb_pool[EVP];
  const Tile tl = tiles[blockIdx.x];
  const int32_t L0 = tl.L0;
  const int nloci = tl.L1 - L0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int a = wave * 256;  // this wave's loci [a, a + 256) (tile-relative)
  const int i0 = a + 4 * lane;
  const int bnd = min(a + 256, nloci);
  const bool wide = (tl.re - tl.rb) >= 65535;

  ByteCounters bc{};
  PairAcc acc[4] = {};
  uint32_t mask4 = 0;  // MD-derived standard reference bases: 4 bits per byte
  int since_fold = 0;

  auto fail = [&](int code, int64_t where) { raise_error(&ctr->err, (int64_t *)&ctr->err_pos, code, where); };
  auto clamp16 = [](int32_t v) -> int16_t { return (int16_t)(v < -16 ? -16 : v > TL + 16 ? TL + 16 : v); };

  // count the SNV run [lo, hi) (tile-relative) of a read whose byte for locus i is at LDS
  // byte offset boff + i (staged) or at global byte gbase + i (unstaged)
  auto snv_run = [&](int lo, int hi, int boff, bool staged, int64_t gbase) {
    const uint32_t vm = range_mask4(lo - i0, hi - i0);
    if (vm == 0u) return;
    uint32_t w;
    if (staged) {
      const int addr = boff + i0;
      const uint32_t x0 = stage32[addr >> 2], x1 = stage32[(addr >> 2) + 1];
      w = __builtin_amdgcn_alignbyte(x1, x0, (uint32_t)(addr & 3));
    } else {
      w = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((vm >> (8 * j)) & 1u) w |= (uint32_t)R.seq[gbase + i0 + j] << (8 * j);
    }
    count_word(bc, w, vm);
  };
  auto stage_byte = [&](int boff, bool staged, int64_t gbase, int i) -> uint8_t {
    if (staged) {
      const int addr = boff + i;
      return (uint8_t)(stage32[addr >> 2] >> (8 * (addr & 3)));
    }
    return R.seq[gbase + i];
  };
  auto owner_of = [&](int t) { return (t - a) >> 2; };
  // an SNV element at locus t carries an MD event: read base rb, MD reference base mdb
  auto snv_event = [&](int t, uint8_t rb, uint8_t mdb) {
    const int c = base_cat(rb);
    const uint32_t bit = std_bit(mdb);
    if (lane == owner_of(t)) {
      const uint32_t sh = 8u * (uint32_t)((t - a) & 3), inc = 1u << sh;
      // selects, not an if-chain: the compiler would turn the chain into an indexed (scratch) access
      bc.eA += c == 0 ? inc : 0u;
      bc.eC += c == 1 ? inc : 0u;
      bc.eT += c == 2 ? inc : 0u;
      bc.eG += c == 3 ? inc : 0u;
      mask4 |= bit << sh;
    }
  };
  // a non-SNV element at locus t whose MD-derived reference base is mdb (< 0: none)
  auto complex_one = [&](int t, int mdb) {
    if (t < a || t >= bnd) return;
    if (lane == owner_of(t)) {
      const uint32_t sh = 8u * (uint32_t)((t - a) & 3);
      bc.X += 1u << sh;
      if (mdb >= 0) mask4 |= std_bit((uint8_t)mdb) << sh;
    }
  };

  if (!wide) {
    int nb = 0;
    for (int64_t r0 = tl.rb; r0 < tl.re; r0 += nb) {
      // ---- batch: up to NT reads whose sequence bytes fit the stage
      nb = (int)min((int64_t)NT, tl.re - r0);
      const int64_t B0 = R.seq_off[r0] & ~(int64_t)15;
      int64_t n1k = 0;
      for (;;) {
        const int64_t B1 = R.seq_off[r0 + nb - 1] + R.seq_len[r0 + nb - 1];
        n1k = B1 > B0 ? (B1 - B0 + 1023) >> 10 : 0;
        if (n1k * 1024 <= kV2Stage && B0 + n1k * 1024 <= R.seq_cap) break;
        if (nb == 1) {
          n1k = 0;  // a read larger than the stage (or the pool end): read it from HBM
          break;
        }
        nb = (nb + 1) >> 1;
      }
      // the batch's MD events and CIGAR operators are contiguous in their pools (reads are
      // stored in order): copied to LDS with coalesced loads, like the bases
      const int64_t last = r0 + nb - 1;
      const int64_t ev_lo = R.md_off[r0], ev_hi = R.md_off[last] + max(R.n_md[last], 0);
      const int64_t cg_lo = R.cigar_off[r0], cg_hi = R.cigar_off[last] + R.n_cigar[last];
      const bool ev_fit = ev_hi >= ev_lo && ev_hi - ev_lo <= EVP;
      const bool cg_fit = cg_hi >= cg_lo && cg_hi - cg_lo <= CGP;
      __syncthreads();  // previous batch finished with the stage and the tables
      for (int64_t q = wave; q < n1k; q += W)
        __builtin_amdgcn_global_load_lds((const void *)(R.seq + B0 + q * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void *)(stage32 + (kV2Pad + q * 1024) / 4),
                                         16, 0, 0);
      if (ev_fit) {
        const int n_ev = (int)(ev_hi - ev_lo);
        uint32_t ev[EVP / NT];
        uint8_t rb[EVP / NT];
#pragma unroll
        for (int u = 0; u < EVP / NT; ++u) {
          const int q = (int)threadIdx.x + u * NT;
          ev[u] = q < n_ev ? R.md_ev[ev_lo + q] : 0u;
          rb[u] = q < n_ev ? R.ev_rb[ev_lo + q] : (uint8_t)0;
        }
#pragma unroll
        for (int u = 0; u < EVP / NT; ++u) {
          const int q = (int)threadIdx.x + u * NT;
          if (q < n_ev) {
            ev_pool[q] = ev[u];
            rb_pool[q] = rb[u];
          }
        }
      }
      if (cg_fit) {
        const int n_cg = (int)(cg_hi - cg_lo);
        uint32_t cg[CGP / NT];
#pragma unroll
        for (int u = 0; u < CGP / NT; ++u) {
          const int q = (int)threadIdx.x + u * NT;
          cg[u] = q < n_cg ? R.cigar[cg_lo + q] : 0u;
        }
#pragma unroll
        for (int u = 0; u < CGP / NT; ++u) {
          const int q = (int)threadIdx.x + u * NT;
          if (q < n_cg) cg_pool[q] = cg[u];
        }
      }
      // ---- read table: one thread per read (coalesced metadata loads)
      int my_s = 0;
      uint32_t my_w0 = 0, my_nm = 0;
      if ((int)threadIdx.x < nb) {
        const int t = threadIdx.x;
        const int64_t r = r0 + t;
        const int32_t s = R.start[r] - L0, e = R.end[r] - L0;
        const int64_t so = R.seq_off[r];
        const int32_t sl = R.seq_len[r];
        const int32_t nmd = R.n_md[r];
        const int16_t ld = R.lead[r];
        const int32_t ncig = R.n_cigar[r];
        const int64_t mo = R.md_off[r], co = R.cigar_off[r];
        const bool staged = n1k > 0 && so >= B0 && so + sl <= B0 + n1k * 1024;
        if (nmd < 0 && e > 0 && s < nloci) fail(GQ_E_NO_MD, (int64_t)s + L0);
        const int nm = nmd > 0 ? min(nmd, 65535) : 0;
        uint32_t w0 = (ld >= 0 ? 1u : 0u) | (staged ? 2u : 0u);
        uint32_t w1 = (uint32_t)nm;
        if (nm > 0 && nm == nmd && ev_fit && mo >= ev_lo && mo + nm <= ev_hi)
          w0 |= 4u | ((uint32_t)(mo - ev_lo) << 16);
        if (ld < 0 && ncig <= 255 && cg_fit && co >= cg_lo && co + ncig <= cg_hi) {
          w0 |= 8u | ((uint32_t)ncig << 8);
          w1 |= (uint32_t)(co - cg_lo) << 16;
        }
        m_s[t] = s;
        m_e[t] = clamp16(e);
        m_pm[t] = clamp16(R.pmax_end[r] - L0);
        const int32_t base = staged ? (int32_t)(so - B0) + kV2Pad : 0;
        m_boff[t] = ld >= 0 ? base + ld - s : base;
        m_w0[t] = w0;
        m_w1[t] = w1;
        my_s = s;
        my_w0 = w0;
        my_nm = (uint32_t)nm;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      // events of simple reads -> (tile locus + bias) << 8 | MD base, read base | 0x80, so the
      // event pass below needs no per-read lookup
      if ((my_w0 & 5u) == 5u) {
        const int evo = (int)(my_w0 >> 16);
        for (int q = 0; q < (int)my_nm; ++q) {
          const uint32_t ev = ev_pool[evo + q];
          ev_pool[evo + q] = ((uint32_t)(my_s + (int)(ev >> 8) + kEvBias) << 8) | (ev & 0xFFu);
          rb_pool[evo + q] = (uint8_t)(rb_pool[evo + q] | 0x80u);
        }
      }
      __syncthreads();
      if (a < nloci) {
        // ---- first read of the batch that can reach this wave's loci (prefix-max end > a)
        int first = nb;
        for (int c0 = 0; c0 < nb; c0 += 64) {
          const bool v = c0 + lane < nb && (int)m_pm[c0 + lane] > a;
          const unsigned long long bl = __ballot(v);
          if (bl) {
            first = c0 + __ffsll((long long)bl) - 1;
            break;
          }
        }
        for (int c0 = first; c0 < nb; c0 += 64) {
          // 64 reads' table rows, one per lane; broadcast per read with v_readlane
          const int kk = min(c0 + lane, nb - 1);
          const int vs = m_s[kk], ve = m_e[kk], vboff = m_boff[kk];
          const uint32_t vw0 = m_w0[kk], vw1 = m_w1[kk];
          const bool in_chunk = c0 + lane < nb;
          if (__ballot(in_chunk && vs < bnd) == 0ull) break;  // reads are start-sorted: nothing further
          const bool ov = in_chunk && vs < bnd && ve > a;
          // -- simple reads, four at a time (independent LDS loads in flight together)
          unsigned long long sb = (ABL & 1) ? 0ull : __ballot(ov && (vw0 & 3u) == 3u);  // simple and staged
          while (sb) {
            int jj[4];
            int nj = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              jj[u] = sb ? __ffsll((long long)sb) - 1 : -1;
              if (sb) {
                sb &= sb - 1;
                ++nj;
              }
            }
            uint32_t x0[4], x1[4], vm[4], sh[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              vm[u] = 0u;
              x0[u] = x1[u] = sh[u] = 0u;
              if (u < nj) {
                const int rs = __builtin_amdgcn_readlane(vs, jj[u]);
                const int re = __builtin_amdgcn_readlane(ve, jj[u]);
                const int bo = __builtin_amdgcn_readlane(vboff, jj[u]);
                vm[u] = range_mask4(rs - i0, re - i0);
                const int addr = bo + i0;
                sh[u] = (uint32_t)(addr & 3);
                if (vm[u]) {
                  x0[u] = stage32[addr >> 2];
                  x1[u] = stage32[(addr >> 2) + 1];
                }
              }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (u < nj) count_word(bc, __builtin_amdgcn_alignbyte(x1[u], x0[u], sh[u]), vm[u]);
            since_fold += nj;
            if (since_fold >= 250) {
              fold_counters(bc, acc);
              since_fold = 0;
            }
          }
          // -- everything else, one read at a time: unstaged simple reads, simple reads whose
          //    events are not pooled, general CIGARs
          unsigned long long ob = (ABL & 4) ? 0ull : (__ballot(ov && (vw0 & 3u) != 3u) | __ballot(ov && (vw0 & 5u) == 1u && (vw1 & 0xFFFFu)));
          while (ob) {
            const int j = __ffsll((long long)ob) - 1;
            ob &= ob - 1;
            const int s = __builtin_amdgcn_readlane(vs, j);
            const int e = __builtin_amdgcn_readlane(ve, j);
            const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)vw0, j);
            const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)vw1, j);
            const int boff = __builtin_amdgcn_readlane(vboff, j);
            const bool staged = (w0 & 2u) != 0;
            const int64_t r = r0 + c0 + j;
            const int nmd = (int)(w1 & 0xFFFFu);
            const bool ev_lds = (w0 & 4u) != 0;
            const int evo = (int)(w0 >> 16);
            if (w0 & 1u) {
              if (!staged) snv_run(s, e, boff, false, R.seq_off[r] + R.lead[r] - s);
              if (!ev_lds) {  // events not pooled: read them from HBM
                const int64_t mo = R.md_off[r];
                for (int q = 0; q < nmd; ++q) {
                  const uint32_t ev = R.md_ev[mo + q];
                  const int t = s + (int)(ev >> 8);
                  if (t >= bnd) break;
                  if (t < a) continue;
                  snv_event(t, R.ev_rb[mo + q], (uint8_t)(ev & 0xFFu));
                }
              }
            } else {
              // general CIGAR: operators and MD events held one per lane, walked wave-uniformly
              const bool cg_lds = (w0 & 8u) != 0;
              const int cgo = (int)(w1 >> 16);
              const int ncig = cg_lds ? (int)((w0 >> 8) & 0xFFu) : R.n_cigar[r];
              const int64_t cgb = R.cigar_off[r], mob = R.md_off[r];
              // first 64 operators / events in registers; beyond that from memory
              const uint32_t vcig = lane < ncig ? (cg_lds ? cg_pool[cgo + lane] : R.cigar[cgb + lane]) : 0u;
              const uint32_t vev = lane < nmd ? (ev_lds ? ev_pool[evo + lane] : R.md_ev[mob + lane]) : 0xFFFFFFFFu;
              const uint32_t vrb = lane < nmd ? (ev_lds ? rb_pool[evo + lane] : R.ev_rb[mob + lane]) : 0u;
              auto cig_at = [&](int c) -> uint32_t {
                return c < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)vcig, c)
                              : (cg_lds ? cg_pool[cgo + c] : R.cigar[cgb + c]);
              };
              auto md_at = [&](int t) -> int {  // MD event at locus t of this read: base or -1
                const unsigned long long hb = __ballot(lane < nmd && (int)(vev >> 8) == t - s);
                if (hb) return (int)((uint32_t)__builtin_amdgcn_readlane((int)vev, __ffsll((long long)hb) - 1) & 0xFFu);
                for (int q = 64; q < nmd; ++q) {
                  const uint32_t ev = ev_lds ? ev_pool[evo + q] : R.md_ev[mob + q];
                  if ((int)(ev >> 8) == t - s) return (int)(ev & 0xFFu);
                }
                return -1;
              };
              const int slen = R.seq_len[r];
              const int64_t gread = staged ? 0 : R.seq_off[r];
              const bool at_zero = (int64_t)s + L0 == 0;
              int ref = s, rp = 0;
              bool seen_ref = false, lead_ins = false;
              for (int c = 0; c < ncig; ++c) {
                const uint32_t cc = cig_at(c);
                const int op = (int)(cc & 15u);
                const int len = (int)(cc >> 4);
                const int nextop = c + 1 < ncig ? (int)(cig_at(c + 1) & 15u) : -1;
                if (op == OP_I && !seen_ref && at_zero) lead_ins = true;
                if (op == OP_P) fail(GQ_E_ASSERT, (int64_t)ref + L0);
                if (consumes_ref(op)) {
                  seen_ref = true;
                  const int ra = ref, rb2 = ref + len;
                  if (rb2 > a && ra < bnd) {
                    if (op == OP_M || op == OP_EQ || op == OP_X) {
                      const bool first_ins = lead_ins && (int64_t)ra + L0 == 0;
                      const bool last_anchor = ((op == OP_M || op == OP_EQ) && nextop == OP_I) || nextop == OP_D;
                      const int lo = first_ins ? ra + 1 : ra;
                      const int hi = last_anchor ? rb2 - 1 : rb2;
                      if (rp + len > slen) fail(GQ_E_ASSERT, (int64_t)ra + L0 + (slen - rp));
                      const int sboff = boff + rp - ra;
                      const int64_t sgb = gread + rp - ra;
                      snv_run(lo, min(hi, ra + (slen - rp)), sboff, staged, sgb);
                      // MD events on the SNV run
                      const int elo = max(lo, a), ehi = min(hi, bnd);
                      unsigned long long eb = __ballot(lane < nmd && s + (int)(vev >> 8) >= elo &&
                                                       s + (int)(vev >> 8) < ehi);
                      while (eb) {
                        const int q = __ffsll((long long)eb) - 1;
                        eb &= eb - 1;
                        const uint32_t ev = (uint32_t)__builtin_amdgcn_readlane((int)vev, q);
                        snv_event(s + (int)(ev >> 8), (uint8_t)__builtin_amdgcn_readlane((int)vrb, q),
                                  (uint8_t)(ev & 0xFFu));
                      }
                      for (int q = 64; q < nmd; ++q) {
                        const uint32_t ev = ev_lds ? ev_pool[evo + q] : R.md_ev[mob + q];
                        const int t = s + (int)(ev >> 8);
                        if (t >= elo && t < ehi) snv_event(t, ev_lds ? rb_pool[evo + q] : R.ev_rb[mob + q],
                                                           (uint8_t)(ev & 0xFFu));
                      }
                      auto anchor = [&](int t) {  // insertion / deletion anchor: a non-SNV element
                        if (t < a || t >= bnd || rp + (t - ra) >= slen) return;
                        const int v = md_at(t);
                        complex_one(t, v >= 0 ? v : (int)stage_byte(sboff, staged, sgb, t));
                      };
                      if (first_ins) anchor(ra);
                      if (last_anchor && rb2 - 1 > (first_ins ? ra : ra - 1)) anchor(rb2 - 1);
                    } else if (op == OP_D) {
                      for (int t = max(ra, a); t < min(rb2, bnd); ++t) {  // mid-deletions
                        const int v = md_at(t);
                        if (v < 0) fail(GQ_E_MD, (int64_t)t + L0);
                        complex_one(t, v < 0 ? 'N' : v);
                      }
                    } else {  // N: clipped, MD-derived reference 'N'
                      bc.X += range_mask4(max(ra, a) - i0, min(rb2, bnd) - i0);
                    }
                  }
                  ref += len;
                }
                if (consumes_read(op)) rp += len;
                if (ref >= bnd) break;
              }
            }
            if (++since_fold >= 250) {
              fold_counters(bc, acc);
              since_fold = 0;
            }
          }
        }
        // ---- MD events of simple reads: 64 per step, each lane one event; the events on
        //      this wave's loci are then applied by their owner lanes
        const int n_ev = (ev_fit && !(ABL & 2)) ? (int)(ev_hi - ev_lo) : 0;
        for (int q0 = 0; q0 < n_ev; q0 += 64) {
          const int q = q0 + lane;
          const uint32_t ev = q < n_ev ? ev_pool[q] : 0u;
          const uint32_t rb = q < n_ev ? rb_pool[q] : 0u;
          const int t = (int)(ev >> 8) - kEvBias;
          unsigned long long hb = __ballot(q < n_ev && (rb & 0x80u) && t >= a && t < bnd);
          while (hb) {
            const int j = __ffsll((long long)hb) - 1;
            hb &= hb - 1;
            const uint32_t evj = (uint32_t)__builtin_amdgcn_readlane((int)ev, j);
            snv_event((int)(evj >> 8) - kEvBias, (uint8_t)(__builtin_amdgcn_readlane((int)rb, j) & 0x7F),
                      (uint8_t)(evj & 0xFFu));
          }
        }
      }
    }
    fold_counters(bc, acc);
  }

  // ---- decision for the lane's four loci (GermlineThresholdCaller.scala:100-177)
  const bool multi_sample = R.n_samples > 1;
  unsigned visited = 0, amb = 0, ties = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = i0 + j;
    CallRec out0, out1;
    unsigned nout = 0;
    bool to_complex = false;
    if (i < nloci && wide) {
      to_complex = true;
    } else if (i < nloci) {
      const uint32_t cA = acc[j].AC & 0xFFFFu, cC = acc[j].AC >> 16, cT = acc[j].TG & 0xFFFFu, cG = acc[j].TG >> 16;
      const uint32_t V = acc[j].VE & 0xFFFFu, E = acc[j].VE >> 16;
      const uint32_t cN = E - (cA + cC + cT + cG);
      const uint32_t cx = (V - E) + acc[j].X;  // other bases + non-SNV elements
      const uint32_t depth = V + acc[j].X;
      if (depth > 0) {
        ++visited;
        uint32_t mask = (mask4 >> (8 * j)) & 0xFu;
        if (cA > (acc[j].eAC & 0xFFFFu)) mask |= 1u;
        if (cC > (acc[j].eAC >> 16)) mask |= 2u;
        if (cT > (acc[j].eTG & 0xFFFFu)) mask |= 4u;
        if (cG > (acc[j].eTG >> 16)) mask |= 8u;
        const bool ambiguous = __popc(mask) > 1;
        if (ambiguous) ++amb;
        if (ambiguous || cx > 0 || multi_sample) {
          to_complex = true;
        } else {
          const uint8_t ref = mask ? bit_base(mask) : (uint8_t)'N';
          const int rc = mask ? (__ffs((int)mask) - 1) : 4;
          const uint32_t c_ref = rc == 0 ? cA : rc == 1 ? cC : rc == 2 ? cT : rc == 3 ? cG : cN;
          const int32_t pos = L0 + i;
          const uint64_t ord = (uint64_t)(tl.ordinal0 + i);
          auto mk = [&](uint8_t g0, uint8_t g1, uint8_t alt1, bool alt_sym, int sub, uint8_t fl) {
            CallRec rr;
            rr.key = (ord << 12) | (uint64_t)sub;
            rr.contig = tl.contig;
            rr.pos = pos;
            rr.sample = 0;
            rr.gt0 = g0;
            rr.gt1 = g1;
            rr.flags = fl;
            rr.ref_len = 1;
            if (alt_sym) {  // (ref, "<ALT>")
              rr.alt_len = 5;
              rr.allele = (uint64_t)ref | ((uint64_t)'<' << 8) | ((uint64_t)'A' << 16) | ((uint64_t)'L' << 24) |
                          ((uint64_t)'T' << 32) | ((uint64_t)'>' << 40);
            } else {
              rr.alt_len = 1;
              rr.allele = (uint64_t)ref | ((uint64_t)alt1 << 8);
            }
            return rr;
          };
          if ((long long)(depth - c_ref) * 100 / (long long)depth <= threshold) {
            // no non-reference allele can pass: HomRef if the reference allele passes, else NoCall
            const bool ref_pass = c_ref > 0 && (long long)c_ref * 100 / (long long)depth > threshold;
            if (ref_pass ? emit_ref : emit_no_call)
              PUSH_OUT(mk(ref_pass ? GQ_GT_REF : GQ_GT_NOCALL, ref_pass ? GQ_GT_REF : GQ_GT_NOCALL, 0, true, 0, 0));
          } else {
            const uint32_t cnt5[5] = {cA, cC, cT, cG, cN};
            uint32_t k0 = 0, k1 = 0, k2 = 0;  // top three passing keys: count << 8 | (255 - canonical rank)
            int npass = 0;
#pragma unroll
            for (int rank = 0; rank < 5; ++rank) {
              const int cat = (0x24310 >> (4 * rank)) & 0xF;  // alt byte order A < C < G < N < T
              const uint32_t cc = cnt5[cat];
              if (cc == 0 || (long long)cc * 100 / (long long)depth <= threshold) continue;
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
            const uint8_t b0 = key_base(k0), b1 = key_base(k1);
            if (npass == 0) {
              if (emit_no_call) PUSH_OUT(mk(GQ_GT_NOCALL, GQ_GT_NOCALL, 0, true, 0, fl));
            } else if (npass == 1 && b0 == ref) {
              if (emit_ref) PUSH_OUT(mk(GQ_GT_REF, GQ_GT_REF, 0, true, 0, fl));
            } else if (npass == 1) {
              PUSH_OUT(mk(GQ_GT_ALT, GQ_GT_ALT, b0, false, 0, fl));
            } else {
              const bool v1 = b0 != ref, v2 = b1 != ref;
              if (v1 != v2) {
                PUSH_OUT(mk(GQ_GT_REF, GQ_GT_ALT, v1 ? b0 : b1, false, 0, fl));
              } else if (v1 && v2) {
                PUSH_OUT(mk(GQ_GT_ALT, GQ_GT_OTHERALT, b0, false, 0, fl));
                PUSH_OUT(mk(GQ_GT_ALT, GQ_GT_OTHERALT, b1, false, 1, fl));
              }
            }
          }
        }
      }
    }
    const unsigned long long base = wave_reserve(&ctr->n_rec, nout);
    if (nout > 0 && base < rec_cap) recs[base] = out0;
    if (nout > 1 && base + 1 < rec_cap) recs[base + 1] = out1;
    const unsigned long long cb = wave_reserve(&ctr->n_complex, to_complex ? 1u : 0u);
    if (to_complex && cb < cplx_cap) cplx[cb] = ComplexItem{(int32_t)blockIdx.x, L0 + i, wide ? 1 : 0};
  }
  __shared__ unsigned red[3];
  __syncthreads();
  if (threadIdx.x < 3) red[threadIdx.x] = 0;
  __syncthreads();
  if (visited) atomicAdd(&red[0], visited);
  if (amb) atomicAdd(&red[1], amb);
  if (ties) atomicAdd(&red[2], ties);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int sl = blockIdx.x & (kSpread - 1);
    if (red[0]) atomicAdd(&ctr->spread[0][sl], (unsigned long long)red[0]);
    if (red[1]) atomicAdd(&ctr->spread[1][sl], (unsigned long long)red[1]);
    if (red[2]) atomicAdd(&ctr->spread[2][sl], (unsigned long long)red[2]);
  }
}

#undef UNI

}  // namespace
