// gq_somatic_call.h — somatic_call: the exact per-candidate caller of somatic-standard
// (SomaticStandard.Caller.findPotentialVariantAtLocus + the driver's filters,
// commands/SomaticStandardCaller.scala:124-245; Likelihood.scala:99-201; AlleleEvidence.scala:
// 58-101), one wave per candidate locus.  Included by gq_somatic.hip inside its anonymous
// namespace, after the helpers it uses (WinInit, SomWin, phred_success, success_to_phred).
//
// Each covering read is classified ONCE: the wave walks both samples' covering reads together
// (the two samples' searches, scans and per-read loads in the same latency rounds), stores one
// 16-byte element record per read in pileup element order, and every later step — the
// pileup reference base, the allele table, the filters, both likelihood folds, the evidence —
// reads those records instead of re-walking CIGARs and MD tags.
//
// Two instantiations:
//   DEEP = false  records in LDS, kFastCap elements per sample; a candidate whose pileup is
//                 deeper is appended to the deep list (counted visit and all, it is wholly the
//                 deep kernel's);
//   DEEP = true   records in a global scratch slice per wave sized on the host from the deepest
//                 listed pileup: no depth limit.  Also runs the heap-order loci (amb_in).
#pragma once

constexpr int kFastCap = 128;      // elements per sample held in LDS by the fast kernel
constexpr int kRankScanMaxG = 256 * 257 / 2;  // normal genotypes ranked in HashTrieMap order (256 eligible alleles)
constexpr int kWideNS = 16;        // the wide kernel's allele-table slots: 1024 distinct alleles per sample
constexpr int kDeepTermCap = 256;  // deep kernel: elements per LDS chunk of the likelihood fold

// Element record (16 bytes), one per covering read in pileup element order:
//   x  rp    read position of the element (SNV / DEL: its base; INS: its first alt byte)
//   y  aux   INS: alt bytes; DEL: deleted length
//   z  base | kind << 8 | quality (as a signed byte) << 16 | mapq << 24
//   w  n_mismatch | flags (3 bits) << 16 | allele-table index (13 bits) << 19
constexpr uint32_t kElAct = 1u, kElPass = 2u, kElFwd = 4u;
__device__ __forceinline__ int el_q(const uint4 &e) { return (int)(int8_t)(uint8_t)(e.z >> 16); }
__device__ __forceinline__ int el_mq(const uint4 &e) { return (int)(e.z >> 24); }
__device__ __forceinline__ uint32_t el_flags(const uint4 &e) { return (e.w >> 16) & 0x7u; }
__device__ __forceinline__ int el_tidx(const uint4 &e) { return (int)(e.w >> 19); }

// One element's three possible log terms (log(2(1 - pc)), log(pc + (1 - pc)), log(2 pc); 0 when
// the mapq filter drops it) and its allele-table index: one 32-byte LDS record per element.
struct TermRec {
  double t0, th, t2;
  int32_t tj, pad;
};

// Per-wave working memory (LDS for the fast kernel, a global scratch slice for the deep one).
struct CallMem {
  int32_t *cov[2];  // [cap] covering reads (offset from the tile's rb), pileup element order
  uint4 *el[2];     // [cap] element records
  uint32_t *tmp;    // [2 cap] heap-order reorder / evidence values
  int16_t *order;   // [64 kSlots]
  uint8_t *is_var;  // [64 kSlots]
  double *ll;       // [maxG]
  uint32_t *gkey;   // deep kernels: [2 maxG] the genotypes' map keys (the variant mass past 128 genotypes)
  double *gsum;     // deep kernels: [maxG] the variant likelihoods in map order
  struct TermRec *terms;  // [tcap] LDS: a chunk of elements' log terms + table indexes (the fold)
  int tcap;
  const double *succ;     // PhredUtils.phredToSuccessProbability table (g_succ) copied to LDS
  int cap, maxG;
};

// Deep-kernel scratch geometry: bytes per wave for `cap` elements per sample, maxG genotypes and
// ns allele-table slots.
__host__ __device__ __forceinline__ size_t deep_wave_bytes(int cap, int maxG, int ns = kSlots) {
  return (size_t)cap * (2 * 4 + 2 * 16 + 2 * 4) + 64 * (size_t)ns * 3 + (size_t)maxG * 24 + 64;
}
__device__ __forceinline__ CallMem deep_mem(uint8_t *base, int cap, int maxG, int ns = kSlots) {
  CallMem m;
  uint8_t *p = base;
  m.el[0] = (uint4 *)p;
  p += (size_t)cap * 16;
  m.el[1] = (uint4 *)p;
  p += (size_t)cap * 16;
  m.ll = (double *)p;
  p += (size_t)maxG * 8;
  m.gsum = (double *)p;
  p += (size_t)maxG * 8;
  m.gkey = (uint32_t *)p;
  p += (size_t)maxG * 8;
  m.cov[0] = (int32_t *)p;
  p += (size_t)cap * 4;
  m.cov[1] = (int32_t *)p;
  p += (size_t)cap * 4;
  m.tmp = (uint32_t *)p;
  p += (size_t)cap * 8;
  m.order = (int16_t *)p;
  p += 64 * (size_t)ns * 2;
  m.is_var = p;
  m.terms = nullptr;  // (the kernel points it at its LDS)
  m.tcap = 0;
  m.cap = cap;
  m.maxG = maxG;
  return m;
}

// The pileup's allele table (a sample's distinct alleles; entry j on lane j & 63, register
// slot j >> 6) and its totals.
template <int NS>
struct Pile {
  static constexpr int kNS = NS;
  uint64_t klo[NS], khi[NS];
  AlleleDesc desc[NS];
  uint32_t n_all[NS], n_f[NS];
  int nt;
  uint32_t depth_all, depth_f, fwd_f;
  uint8_t refbase;
  bool ambiguous, overflow;
};

template <int NS>
__device__ __forceinline__ AlleleDesc pile_entry(const Pile<NS> &P, int j) {
  AlleleDesc d{};
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (s == (j >> 6)) {
      const int o = j & 63;
      d.read = __shfl(P.desc[s].read, o, 64);
      d.aux = __shfl(P.desc[s].aux, o, 64);
      d.rp = __shfl(P.desc[s].rp, o, 64);
      d.kind = (uint8_t)__shfl((int)P.desc[s].kind, o, 64);
      d.rb = (uint8_t)__shfl((int)P.desc[s].rb, o, 64);
      d.base = (uint8_t)__shfl((int)P.desc[s].base, o, 64);
    }
  return d;
}

// Table index of `key` in P (-1: absent).
template <int NS>
__device__ __forceinline__ int pile_find(const Pile<NS> &P, Key128 key) {
  const int lane = threadIdx.x & 63;
  int found = -1;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const unsigned long long hb = __ballot((s * 64 + lane) < P.nt && P.klo[s] == key.lo && P.khi[s] == key.hi);
    if (found < 0 && hb) found = s * 64 + (__ffsll((long long)hb) - 1);
  }
  return found;
}


struct GenoOut {
  int n, G, best_g, bi, bj;
  double best_l, var_sum;
  bool order_tie;    // two variant genotypes with equal immutable-map keys (insertion order used)
  uint64_t cyc_fold; // (diagnostics) cycles from entry to the end of the row fold
};

// Likelihood.likelihoodsOfAllPossibleGenotypesFromPileup (normalised, not log space) over the
// sample's filtered elements (records in `el`, n of them).  Eligible alleles (filtered count
// > 0, standard alt bases, Likelihood.scala:106) ranked by Allele order; genotype g <-> (i <= j)
// in the reference's enumeration order; the per-genotype row fold is Colt's aggregate (the LAST
// element first, Likelihood.scala:185) with StrictMath log; normalisation in the reference's
// order (:190-199); maxBy = the first maximum.  The normal's variant mass (with_var_sum) adds
// the variant genotypes' likelihoods in the iteration order of the immutable Map `toMap`
// builds (SomaticStandardCaller.scala:206-217): generation order up to four genotypes, the
// HashTrieMap's beyond (gq_scala_order.h).
template <int NS>
__device__ __forceinline__ GenoOut genotypes_el(const DevReads &R, const Pile<NS> &P, const uint4 *el, int n_el, int32_t pos,
                                                bool include_alignment, bool with_var_sum, CallMem &m, Counters *ctr) {
  const int lane = threadIdx.x & 63;
  GenoOut res{};
  const uint64_t cyc0 = __builtin_readcyclecounter();
  bool elig[NS], var[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int j = s * 64 + lane;
    elig[s] = j < P.nt && P.n_f[s] > 0 && allele_std_alt(R, P.desc[s], pos);
    var[s] = j < P.nt && allele_is_variant(R, P.desc[s], pos);
  }
  int n = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) n += __popcll(__ballot(elig[s]));
  res.n = n;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int rank = 0;
    for (int k = 0; k < P.nt; ++k) {
      bool ek = false;
#pragma unroll
      for (int t = 0; t < NS; ++t)
        if (t == (k >> 6)) ek = __shfl((int)elig[t], k & 63, 64);
      if (!ek) continue;  // uniform
      const AlleleDesc dk = pile_entry(P, k);
      if (elig[s] && k != s * 64 + lane && allele_cmp(R, dk, P.desc[s], pos) < 0) ++rank;
    }
    if (elig[s]) m.order[rank] = (int16_t)(s * 64 + lane);
    if (s * 64 + lane < 64 * NS) m.is_var[s * 64 + lane] = var[s] ? 1 : 0;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const int G = n * (n + 1) / 2;
  res.G = G;
  if (G == 0) return res;
  if (G > m.maxG) {
    raise_at(ctr, GQ_E_CAPACITY, pos);
    res.G = 0;
    return res;
  }
  const double ln2d = sm::log(2.0) * (double)P.depth_f;
  // the three possible log terms of an element (0 for an element the mapq filter drops: starting
  // the fold at +0.0 and adding 0.0 for those is bit-identical to Colt's fold over the filtered
  // elements; no term is -0.0)
  auto elem_terms = [&](int k, int &tj, double &t0, double &th, double &t2) {
    const uint4 e = el[k];
    const uint32_t fl = el_flags(e);
    tj = el_tidx(e);
    t0 = th = t2 = 0.0;
    if ((fl & kElAct) && (fl & kElPass)) {
      const int q = el_q(e);
      if (q < 0) raise_at(ctr, GQ_E_ASSERT, pos);  // PhredUtils: negative phred
      auto succ = [&](int x) { return m.succ[x > 255 ? 255 : (x < 0 ? 0 : x)]; };  // phred_success from LDS
      double pc = succ(q);
      if (include_alignment) pc = pc * succ(el_mq(e));  // probabilityCorrectIncludingAlignment
      const double pw = 1.0 - pc;
      t2 = sm::log(pc + pc);
      th = sm::log(pc + pw);
      t0 = sm::log(pw + pw);
    }
  };
  // the row fold, lanes = genotypes: Colt's aggregate starts from the LAST element.  The terms
  // go to LDS records (lanes = elements) m.tcap elements at a time, last chunk first, and each
  // genotype lane folds a chunk four records per batch, the batch's loads issued before its adds.
  for (int g0 = 0; g0 < G; g0 += 64) {
    const int g = g0 + lane;
    int i = 0, j = 0;
    if (g < G) genotype_index(g, n, i, j);
    const int ei = g < G ? m.order[i] : -1, ej = g < G ? m.order[j] : -1;
    auto pick = [&](const TermRec &t) {
      const int sel = (ei == t.tj ? 1 : 0) + (ej == t.tj ? 1 : 0);
      return sel == 0 ? t.t0 : sel == 1 ? t.th : t.t2;
    };
    double agg = 0.0;
    for (int cend = n_el; cend > 0; cend -= m.tcap) {
      const int cbeg = cend > m.tcap ? cend - m.tcap : 0;
      for (int c0 = cbeg; c0 < cend; c0 += 64) {
        const int k = c0 + lane;
        if (k >= cend) continue;
        TermRec t;
        elem_terms(k, t.tj, t.t0, t.th, t.t2);
        t.pad = 0;
        m.terms[k - cbeg] = t;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const TermRec *tr = m.terms - cbeg;  // tr[k] = element k's record
      int k = cend - 1;
      for (; k >= cbeg + 3; k -= 4) {
        const TermRec a = tr[k], b = tr[k - 1], c = tr[k - 2], d = tr[k - 3];
        const double pa = pick(a), pb = pick(b), pc = pick(c), pd = pick(d);
        agg = agg + pa;
        agg = agg + pb;
        agg = agg + pc;
        agg = agg + pd;
      }
      for (; k >= cbeg; --k) agg = agg + pick(tr[k]);
      __builtin_amdgcn_wave_barrier();  // (the next chunk rewrites the records)
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (g < G) m.ll[g] = agg + sm::log(1.0) - ln2d;
  }
  res.cyc_fold = __builtin_readcyclecounter() - cyc0;
  double tot = 0.0;
  for (int g0 = 0; g0 < G; g0 += 64) {
    const double e = (g0 + lane < G) ? sm::exp(m.ll[g0 + lane]) : 0.0;
    for (int j = 0; j < 64 && g0 + j < G; ++j) tot = tot + lane_f64(e, j);
  }
  const double lt = sm::log(tot);
  double best = 0.0;
  int bestg = -1;
  for (int g0 = 0; g0 < G; g0 += 64) {
    const int g = g0 + lane;
    double L = 0.0;
    if (g < G) {
      L = sm::exp(m.ll[g] - lt);
      m.ll[g] = L;  // the normalised likelihood, for the variant mass below
    }
    for (int j = 0; j < 64 && g0 + j < G; ++j) {
      const double Lj = lane_f64(L, j);
      if (bestg < 0 || Lj > best) {
        best = Lj;
        bestg = g0 + j;
      }
    }
  }
  res.best_g = bestg;
  res.best_l = best;
  int i, j;
  genotype_index(bestg, n, i, j);
  res.bi = m.order[i];
  res.bj = m.order[j];
  if (!with_var_sum) return res;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // the variant genotypes' mass in the immutable Map's order
  double vsum = 0.0;
  if (G <= 4) {  // Map1..Map4: insertion (= generation) order
    for (int g = 0; g < G; ++g) {
      int a, b;
      genotype_index(g, n, a, b);
      if (m.is_var[m.order[a]] || m.is_var[m.order[b]]) vsum = vsum + m.ll[g];
    }
  } else if (G > kRankScanMaxG) {  // (the rank scan below is quadratic in G)
    raise_at(ctr, GQ_E_CAPACITY, pos);
  } else if (G > 128) {
    // (the deep kernels' scratch, past 128 genotypes) the same map order: every genotype's key
    // in m.gkey, each variant genotype's rank by a scan over them, its likelihood to m.gsum[rank]
    for (int a0 = 0; a0 < n; a0 += 64) {
      const int a = a0 + lane;
      const uint32_t h = allele_scala_hash(R, pile_entry(P, m.order[a < n ? a : 0]), pos);  // (every lane: shuffles)
      if (a < n) m.tmp[a] = h;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int g0 = 0; g0 < G; g0 += 64) {
      const int g = g0 + lane;
      if (g < G) {
        int a = 0, b = 0;
        genotype_index(g, n, a, b);
        const bool v = m.is_var[m.order[a]] || m.is_var[m.order[b]];
        const uint64_t key = scala::trie_key(scala::genotype_hash(m.tmp[a], m.tmp[b]));
        m.gkey[2 * g] = (uint32_t)key;
        m.gkey[2 * g + 1] = (uint32_t)(key >> 32) | (v ? 0x80000000u : 0u);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    bool tie = false;
    int nvar = 0;
    for (int g0 = 0; g0 < G; g0 += 64) {
      const int g = g0 + lane;
      const bool vg = g < G && (m.gkey[2 * g + 1] & 0x80000000u);
      if (vg) {
        const uint64_t kg = (uint64_t)m.gkey[2 * g] | ((uint64_t)(m.gkey[2 * g + 1] & 0x7FFFFFFFu) << 32);
        int r = 0;
        for (int h = 0; h < G; ++h) {
          const uint32_t hi = m.gkey[2 * h + 1];
          if (!(hi & 0x80000000u)) continue;
          const uint64_t kh = (uint64_t)m.gkey[2 * h] | ((uint64_t)(hi & 0x7FFFFFFFu) << 32);
          if (kh < kg || (kh == kg && h < g)) ++r;
          if (kh == kg && h != g) tie = true;
        }
        m.gsum[r] = m.ll[g];
      }
      nvar += __popcll(__ballot(vg));
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int r = 0; r < nvar; ++r) vsum = vsum + m.gsum[r];
    res.order_tie = __ballot(tie) != 0;
  } else {
    // HashTrieMap: ascending trie key of each genotype's Scala hash; equal keys (a full 32-bit
    // hash collision, a ListMap there) keep insertion order and are flagged.  G <= kMaxG = 128:
    // two genotype chunks, the keys in tmp (2 words per genotype: 2 * kFastCap >= 2 * 128).
    static_assert(kMaxG <= 128 && 2 * kFastCap >= 2 * kMaxG, "genotype key scratch");
    const uint32_t ah = lane < n ? allele_scala_hash(R, pile_entry(P, m.order[lane < n ? lane : 0]), pos) : 0u;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int g = 64 * c + lane;
      int a = 0, b = 0;
      if (g < G) genotype_index(g, n, a, b);
      const uint32_t ha = (uint32_t)__shfl((int)ah, a & 63, 64), hb = (uint32_t)__shfl((int)ah, b & 63, 64);
      if (g < G) {
        const bool v = m.is_var[m.order[a]] || m.is_var[m.order[b]];
        const uint64_t key = scala::trie_key(scala::genotype_hash(ha, hb));
        m.tmp[2 * g] = (uint32_t)key;
        m.tmp[2 * g + 1] = (uint32_t)(key >> 32) | (v ? 0x80000000u : 0u);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    int rank[2];
    double Lr[2];
    bool tie = false;
    int nvar = 0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int g = 64 * c + lane;
      rank[c] = -1;
      Lr[c] = 0.0;
      const bool vg = g < G && (m.tmp[2 * g + 1] & 0x80000000u);
      if (vg) {
        const uint64_t kg = (uint64_t)m.tmp[2 * g] | ((uint64_t)(m.tmp[2 * g + 1] & 0x7FFFFFFFu) << 32);
        int r = 0;
        for (int h = 0; h < G; ++h) {
          const uint32_t hi = m.tmp[2 * h + 1];
          if (!(hi & 0x80000000u)) continue;
          const uint64_t kh = (uint64_t)m.tmp[2 * h] | ((uint64_t)(hi & 0x7FFFFFFFu) << 32);
          if (kh < kg || (kh == kg && h < g)) ++r;
          if (kh == kg && h != g) tie = true;
        }
        rank[c] = r;
        Lr[c] = m.ll[g];
      }
      nvar += __popcll(__ballot(vg));
    }
    for (int r = 0; r < nvar; ++r) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const unsigned long long b = __ballot(rank[c] == r);
        if (b) vsum = vsum + lane_f64(Lr[c], __ffsll((long long)b) - 1);
      }
    }
    res.order_tie = __ballot(tie) != 0;
  }
  res.var_sum = vsum;
  return res;
}

// k-th smallest (0-based) of the n values val(tmp[base + e]) by bisection over the value range
// [lo, hi]: each round counts the values <= mid with ballots (n <= 64: one ballot).
template <class V>
__device__ __forceinline__ int kth_bisect(const uint32_t *tmp, int base, uint32_t n, uint32_t k, int lo, int hi, V val) {
  const int lane = threadIdx.x & 63;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;  // floor (arithmetic shift)
    uint32_t c = 0;
    for (uint32_t e0 = 0; e0 < n; e0 += 64) {
      const uint32_t e = e0 + lane;
      c += (uint32_t)__popcll(__ballot(e < n && val(tmp[base + e]) <= mid));
    }
    if (c > k) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// Evidence of the called allele in both samples (AlleleEvidence.apply, AlleleEvidence.scala:
// 58-101): per sample the filtered elements whose table index is its target (-1: none), their
// (mapq, quality, mismatches) gathered in element order into tmp (sample s at s * cap); the
// four running means (Breeze, element order) on lanes 0-3 together; medians by bisection.
template <int NS>
__device__ __forceinline__ void evidence_pair(const Pile<NS> &PT, const Pile<NS> &PN, const uint4 *elT, int nT,
                                              const uint4 *elN, int nN, int tgtT, int tgtN, double likT, double likN,
                                              int32_t pos, CallMem &m, gq_evidence &evT, gq_evidence &evN) {
  const int lane = threadIdx.x & 63;
  uint32_t n[2] = {0, 0}, fwd[2] = {0, 0};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const uint4 *el = s ? elN : elT;
    const int ne = s ? nN : nT, target = s ? tgtN : tgtT;
    for (int c0 = 0; c0 < ne; c0 += 64) {
      const int k = c0 + lane;
      bool hit = false;
      uint32_t packed = 0, fl = 0;
      if (k < ne && target >= 0) {
        const uint4 e = el[k];
        fl = el_flags(e);
        hit = (fl & kElAct) && (fl & kElPass) && el_tidx(e) == target;
        packed = (uint32_t)el_mq(e) | (((e.z >> 16) & 0xFFu) << 8) | ((e.w & 0xFFFFu) << 16);
      }
      const unsigned long long hb = __ballot(hit);
      const uint32_t before = (uint32_t)__popcll(hb & ((1ull << lane) - 1ull));
      if (hit) m.tmp[s * m.cap + n[s] + before] = packed;
      fwd[s] += (uint32_t)__popcll(__ballot(hit && (fl & kElFwd)));
      n[s] += (uint32_t)__popcll(hb);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // breeze.stats.mean, running mean in element order: lane 2 s + f = sample s, field f (0 mapq, 1 quality)
  double mu = 0.0;
  {
    const int s = (lane >> 1) & 1, f = lane & 1;
    const uint32_t ns = s ? n[1] : n[0];
    const uint32_t nmax = n[0] > n[1] ? n[0] : n[1];
    for (uint32_t k0 = 0; k0 < nmax; k0 += 64) {
      // 64 values of each sample in one round of loads (lane j: value k0 + j), then the running
      // means by readlane (no memory on the loop's dependence chain)
      const uint32_t v0 = k0 + lane < n[0] ? m.tmp[k0 + lane] : 0u;
      const uint32_t v1 = k0 + lane < n[1] ? m.tmp[m.cap + k0 + lane] : 0u;
      const uint32_t top = nmax - k0 < 64u ? nmax - k0 : 64u;
      for (uint32_t kk = 0; kk < top; ++kk) {
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)v0, (int)kk);
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)v1, (int)kk);
        const uint32_t k = k0 + kk;
        if (lane < 4 && k < ns) {
          const uint32_t v = s ? a1 : a0;
          const double x = f ? (double)(int8_t)((v >> 8) & 0xFFu) : (double)(v & 0xFFu);
          mu += (x - mu) / (double)(k + 1);
        }
      }
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    gq_evidence &ev = s ? evN : evT;
    const Pile<NS> &P = s ? PN : PT;
    ev.likelihood = s ? likN : likT;
    ev.read_depth = (int32_t)P.depth_f;
    ev.forward_depth = (int32_t)P.fwd_f;
    ev.allele_read_depth = (int32_t)n[s];
    ev.allele_forward_depth = (int32_t)fwd[s];
    if (n[s] == 0) {
      ev.mean_mq = ev.median_mq = ev.mean_bq = ev.median_bq = ev.median_mismatches = __builtin_nan("");
      continue;
    }
    ev.mean_mq = lane_f64(mu, 2 * s);
    ev.mean_bq = lane_f64(mu, 2 * s + 1);
    const int base = s * m.cap;
    const uint32_t ns = n[s];
    auto f_mq = [](uint32_t v) { return (int)(v & 0xFFu); };
    auto f_bq = [](uint32_t v) { return (int)(int8_t)((v >> 8) & 0xFFu); };
    auto f_mm = [](uint32_t v) { return (int)(v >> 16); };
    const uint32_t k = (ns & 1) ? (ns - 1) / 2 : ns / 2 - 1;
    if (ns <= 64) {
      // one value per lane: bisection over [min, max] with ballots only (no memory in the
      // rounds), and for an even count the next order statistic from one more count
      const bool valid = (uint32_t)lane < ns;
      const uint32_t v = valid ? m.tmp[base + lane] : 0u;
      auto med = [&](int x, bool half_int, double *outd) {
        int lo = wave_min_i32(valid ? x : INT32_MAX), hi = wave_max_i32(valid ? x : INT32_MIN);
        while (lo < hi) {
          const int mid = (int)(((int64_t)lo + (int64_t)hi) >> 1);
          if ((uint32_t)__popcll(__ballot(valid && x <= mid)) > k) hi = mid;
          else lo = mid + 1;
        }
        const int a = lo;
        if (ns & 1) {
          *outd = (double)a;
          return;
        }
        const bool more = (uint32_t)__popcll(__ballot(valid && x <= a)) > k + 1;
        const int b = more ? a : wave_min_i32(valid && x > a ? x : INT32_MAX);
        *outd = half_int ? (double)((a + b) / 2) : ((double)a + (double)b) / 2.0;  // Int median (parity unpinned)
      };
      med(f_mq(v), false, &ev.median_mq);
      med(f_bq(v), false, &ev.median_bq);
      med(f_mm(v), true, &ev.median_mismatches);
    } else if (ns & 1) {
      ev.median_mq = (double)kth_bisect(m.tmp, base, ns, k, 0, 255, f_mq);
      ev.median_bq = (double)kth_bisect(m.tmp, base, ns, k, -128, 127, f_bq);
      ev.median_mismatches = (double)kth_bisect(m.tmp, base, ns, k, 0, 65535, f_mm);
    } else {
      ev.median_mq = ((double)kth_bisect(m.tmp, base, ns, k, 0, 255, f_mq) +
                      (double)kth_bisect(m.tmp, base, ns, k + 1, 0, 255, f_mq)) / 2.0;
      ev.median_bq = ((double)kth_bisect(m.tmp, base, ns, k, -128, 127, f_bq) +
                      (double)kth_bisect(m.tmp, base, ns, k + 1, -128, 127, f_bq)) / 2.0;
      ev.median_mismatches = (double)((kth_bisect(m.tmp, base, ns, k, 0, 65535, f_mm) +
                                       kth_bisect(m.tmp, base, ns, k + 1, 0, 65535, f_mm)) / 2);  // Int median (parity unpinned)
    }
  }
}

// The deep list: candidates the fast kernel hands over (their item index), and the deepest
// pileup among them and the heap-order loci (sizes the deep kernel's scratch).
struct DeepIO {
  int64_t *list;             // fast kernel: out; deep kernel: in
  unsigned long long cap;    // list capacity (fast kernel)
  int64_t n_in;              // deep kernel: list length
  uint8_t *scratch;          // deep kernel: per-wave slices
  int scap, maxG;            // deep kernel: elements per sample per wave, genotypes
  int64_t *wide;             // deep kernel: out, the candidates past its allele table (the wide kernel's)
  unsigned long long wcap;   // its capacity
};

// One candidate with what its wave needs before the first search, gathered by cand_prep in list
// order, so the caller loads one record (one candidate ahead) instead of walking the item ->
// tile -> window -> initial group chain of dependent loads on its critical path.
struct CandRec {
  int64_t rb[2];         // the tile's first read (tumor, normal): element read offsets are relative to it
  int64_t ra[2], rz[2];  // the reads that can cover pos: [first pmax_end > pos, first start > pos) of the tile window
  int64_t ord0;          // output ordinal of the tile's first locus
  int32_t pos, contig, L0, flags;
  int32_t win, tile;
  int32_t E[2];  // per sample: end of its window's initial group (reorder where pos < E); INT32_MIN: none
};

// The candidates' records, a wave per output partition (lanes over its items: no search for
// the partition of a flat index), each with the binary searches for its covering-read range
// done here, a thread per candidate, where half a million of them overlap.
__global__ void cand_prep(const Tile *__restrict__ tiles_t, const Tile *__restrict__ tiles_n,
                          const ComplexItem *__restrict__ items, OutGeom og, const Counters *__restrict__ ctr, SomWin sw,
                          DevReads RT, DevReads RN, CandRec *__restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = wave_id();
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t q = w0; q < kParts; q += nw) {
    const unsigned long long o0 = ctr->part_off[1][q], o1 = ctr->part_off[1][q + 1];
    for (unsigned long long k = lane; k < o1 - o0; k += 64) {
      const ComplexItem item = items[og.slot(1, (int)q, k)];
      const Tile &tt = tiles_t[item.tile], &tn = tiles_n[item.tile];
      CandRec c;
      c.rb[0] = tt.rb;
      c.rb[1] = tn.rb;
      {  // the four binary searches in one loop (independent dependence chains)
        const int32_t pos = item.pos;
        int64_t lo[4] = {tt.rb, tt.rb, tn.rb, tn.rb}, hi[4] = {tt.re, tt.re, tn.re, tn.re};
        for (;;) {
          bool any = false;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if (lo[q] >= hi[q]) continue;
            any = true;
            const int64_t mid = (lo[q] + hi[q]) >> 1;
            const DevReads &R = q < 2 ? RT : RN;
            const bool past = (q & 1) ? R.start[mid] > pos : R.pmax_end[mid] > pos;
            if (past) hi[q] = mid;
            else lo[q] = mid + 1;
          }
          if (!any) break;
        }
        c.ra[0] = lo[0];
        c.rz[0] = lo[1];
        c.ra[1] = lo[2];
        c.rz[1] = lo[3];
      }
      c.ord0 = tt.ordinal0;
      c.pos = item.pos;
      c.contig = tt.contig;
      c.L0 = tt.L0;
      c.flags = item.flags;
      c.win = sw.range_win[tt.range];
      c.tile = item.tile;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const WinInit wi = sw.wi[2 * c.win + s];
        c.E[s] = wi.n > 0 ? wi.E : INT32_MIN;
      }
      out[o0 + k] = c;
    }
  }
}

// The caller's front: the covering reads of both samples (pileup element order) and one element
// record per covering read (m.el, m.cov), and per lane the std-bit mask of the MD-derived
// reference bases it saw (mask; OR over the wave = the pileup's reference-base set).  Latency-bound
// (dependent searches and per-read loads).  Returns false when the candidate leaves this kernel:
// deeper than m.cap (the fast kernels list it for the deep one).
template <bool DEEP>
__device__ __forceinline__ bool call_front(const CandRec &cr, int64_t it, const DevReads &RT, const DevReads &RN,
                                           const gq_somatic_params &prm, Counters *ctr, const SomWin &sw, CallMem &m,
                                           int dbg, const DeepIO &dio, uint32_t (&nc)[2], uint32_t (&mask)[2]) {
  const int lane = threadIdx.x & 63;
  const int32_t pos = cr.pos;
  const int64_t rb[2] = {cr.rb[0], cr.rb[1]};
  // ---- covering reads of both samples: in [first pmax_end > pos, first start > pos) of each
  //      tile window (cand_prep's searches)
  const int64_t ra[2] = {cr.ra[0], cr.ra[1]}, rz[2] = {cr.rz[0], cr.rz[1]};
  // the element record of covering read r (its scalars given), and its MD-derived reference
  // base's std bit into mk
  auto elem = [&](const DevReads &R, int64_t r, int32_t st, int ld, int64_t so, int mq, uint8_t rfl, int32_t nmd,
                  int64_t mdo, uint32_t nmm, uint32_t &mk) -> uint4 {
    uint32_t fl = 0;
    int32_t rp = 0, aux = 0;
    uint32_t base = 0, kind = K_SNV;
    int q = 0;
    if (ld >= 0) {
      const int32_t off = pos - st;
      rp = ld + off;
      base = R.seq[so + rp];
      q = (int)(int8_t)R.qual[so + rp];
      if (nmd < 0) {
        raise_at(ctr, GQ_E_NO_MD, pos);
      } else {
        const int v = nmd > 0 ? md_find(R.md_ev + mdo, nmd, off) : -1;
        mk |= std_bit((uint8_t)(v >= 0 ? v : (int)base));
        fl = kElAct;
      }
    } else {
      const int v = md_ref_at(R, r, pos);
      if (v < 0) {
        raise_at(ctr, v == -4 ? GQ_E_NO_MD : v == -3 ? GQ_E_MD : GQ_E_ASSERT, pos);
      } else {
        mk |= std_bit((uint8_t)v);
        AlleleDesc d;
        int errc = 0;
        if (!classify(R, r, pos, 0, d, &errc)) {
          raise_at(ctr, errc, pos);
        } else {
          fl = kElAct;
          kind = d.kind;
          base = d.base;
          rp = d.rp;
          aux = d.aux;
          q = elem_quality(R, d, so, mq);
        }
      }
    }
    if (prm.min_mapq <= 0 || mq >= prm.min_mapq) fl |= kElPass;  // QualityAlignedReadsFilter
    if (!(rfl & 1)) fl |= kElFwd;
    return make_uint4((uint32_t)rp, (uint32_t)aux,
                      base | (kind << 8) | ((uint32_t)(uint8_t)(int8_t)q << 16) | ((uint32_t)mq << 24),
                      (nmm & 0xFFFFu) | (fl << 16));
  };
  if (!DEEP && !(dbg & 64) && rz[0] - ra[0] <= 64 && rz[1] - ra[1] <= 64 && !(pos < cr.E[0]) && !(pos < cr.E[1])) {
    // the common candidate: each window fits one chunk and no initial group reorders it, so the
    // covers and the element records come in one pass, a lane per window read: its interval
    // and scalars in one round of loads, then its base / quality / MD event
    mask[0] = mask[1] = 0;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const DevReads &R = s ? RN : RT;
      const int64_t r = ra[s] + lane;
      const bool in = r < rz[s];
      const int64_t rr = in ? r : ra[s];
      int32_t st = 0, en = 0, nmd = 0;
      int ld = 0, mq = 0;
      int64_t so = 0, mdo = 0;
      uint8_t rfl = 0;
      uint32_t nmm = 0;
      if (rz[s] > ra[s]) {
        st = R.start[rr];
        en = R.end[rr];
        ld = (int)R.lead[rr];
        so = R.seq_off[rr];
        mq = (int)R.mapq[rr];
        rfl = R.flags[rr];
        nmd = R.n_md[rr];
        mdo = R.md_off[rr];
        nmm = (uint32_t)R.n_mismatch[rr];
      }
      const bool c = in && st <= pos && pos < en;
      const unsigned long long b = __ballot(c);
      const uint32_t at = (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
      nc[s] = (uint32_t)__popcll(b);
      if (c) {
        m.cov[s][at] = (int32_t)(r - rb[s]);
        m.el[s][at] = elem(R, r, st, ld, so, mq, rfl, nmd, mdo, nmm, mask[s]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    return true;
  }
  nc[0] = nc[1] = 0;
  {
    const int64_t span = max(rz[0] - ra[0], rz[1] - ra[1]);
    for (int64_t c0 = 0; c0 < span; c0 += 64) {
      bool c[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const DevReads &R = s ? RN : RT;
        const int64_t r = ra[s] + c0 + lane;
        c[s] = r < rz[s] && R.start[r] <= pos && pos < R.end[r];
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const unsigned long long b = __ballot(c[s]);
        const uint32_t at = nc[s] + (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
        if (c[s] && at < (uint32_t)m.cap) m.cov[s][at] = (int32_t)(ra[s] + c0 + lane - rb[s]);
        nc[s] += (uint32_t)__popcll(b);
      }
    }
  }
  if (nc[0] > (uint32_t)m.cap || nc[1] > (uint32_t)m.cap || (!DEEP && (dbg & 64))) {
    if constexpr (!DEEP) {  // deeper than the LDS records (or GQ_DBG & 64, tests): the deep kernel's, whole
      if (lane == 0) {
        const unsigned long long k = atomicAdd(&ctr->n_deep, 1ull);
        if (k < dio.cap) dio.list[k] = it;
        atomicMax(&ctr->deep_max, (unsigned long long)max(nc[0], nc[1]));
      }
    } else {
      raise_at(ctr, GQ_E_CAPACITY, pos);  // the host sized the scratch from deep_max
    }
    return false;
  }
  // ---- pileup element order: where the window's initial (heap-ordered) group still covers
  //      pos, its reads are a prefix of the list, reordered by heap rank (SlidingWindow
  //      currentRegions(), DistributedUtil.scala:260-274; Pile.atGreaterLocus keeps them first)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (!(pos < cr.E[s])) continue;  // uniform
    const WinInit w = sw.wi[2 * cr.win + s];
    const DevReads &R = s ? RN : RT;
    int p = 0;
    for (int k0 = 0; k0 < (int)nc[s]; k0 += 64) {
      const int k = k0 + lane;
      p += (int)__popcll(__ballot(k < (int)nc[s] && R.start[rb[s] + m.cov[s][k]] <= w.F));
    }
    for (int k = lane; k < p; k += 64) {
      const int64_t r = rb[s] + m.cov[s][k];
      int lo = 0, hi = w.n;
      while (lo < hi) {
        const int md = (lo + hi) >> 1;
        if (sw.init_reads[w.off + md] < r) lo = md + 1;
        else hi = md;
      }
      m.tmp[k] = (uint32_t)sw.init_rank[w.off + lo];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int k = lane; k < p; k += 64) {
      int before = 0;
      for (int j = 0; j < p; ++j) before += m.tmp[j] < m.tmp[k] ? 1 : 0;
      m.tmp[m.cap + before] = (uint32_t)m.cov[s][k];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int k = lane; k < p; k += 64) m.cov[s][k] = (int32_t)m.tmp[m.cap + k];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  // ---- elements, both samples' chunks together: each covering read's scalars in one round,
  //      then (a single aligned block, the common read) its base, quality and MD event at
  //      pos; other reads take the general CIGAR walk (classify) and md_ref_at
  mask[0] = mask[1] = 0;
  {
    const uint32_t span = max(nc[0], nc[1]);
    for (uint32_t c0 = 0; c0 < span; c0 += 64) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const DevReads &R = s ? RN : RT;
        const uint32_t k = c0 + lane;
        if (k >= nc[s]) continue;
        const int64_t r = rb[s] + m.cov[s][k];
        m.el[s][k] = elem(R, r, R.start[r], (int)R.lead[r], R.seq_off[r], (int)R.mapq[r], R.flags[r], R.n_md[r],
                          R.md_off[r], (uint32_t)R.n_mismatch[r], mask[s]);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  return true;
}

// The element store between the split caller's kernels (somatic_front -> somatic_call_k<false,
// true>), for the candidates [b0, b1) of the list: per candidate a header {nc tumor, nc normal,
// reference-base mask tumor, normal} (nc tumor = kElSkip: the front listed it for the deep
// kernel) and kFastCap element records and covering-read offsets per sample.
constexpr uint32_t kElSkip = 0xFFFFFFFFu;
struct ElemStore {
  uint4 *hdr;
  uint4 *el;
  int32_t *cov;
  int64_t b0, b1;
};

// WPE: waves per SIMD the fast kernel's register budget must allow (3: 168 VGPRs and some
// spills; 2: no spills; GQ_CALL_WPE picks, see gq_somatic_standard).  The deep kernel: 2.
template <bool DEEP, bool BACK = false, int WPE = 3, int NSD = kSlots>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DEEP ? 2 : WPE))) void somatic_call_k(
    const CandRec *__restrict__ cands, DevReads RT, DevReads RN, gq_somatic_params prm, SomRec *__restrict__ recs,
    unsigned long long rec_cap,
    uint8_t *__restrict__ pool, unsigned long long pool_cap, OutGeom og, Counters *ctr, SomWin sw,
    AmbItem *__restrict__ amb_out, unsigned long long amb_cap, const AmbItem *__restrict__ amb_in,
    const uint8_t *__restrict__ amb_ref, int64_t n_amb_in, RefView ref, int dbg, DeepIO dio, ElemStore es) {
  // BACK: the candidates [es.b0, es.b1) whose covers and element records somatic_front stored.
  // amb_in == nullptr: the candidates (fast kernel) or the deep list (deep kernel); loci where a
  // sample's MD-derived reference bases disagree are listed (amb_out) for the heap-order replay.
  // amb_in != nullptr (deep kernel only): the listed loci with both samples' bases resolved
  // (amb_ref[2 i + set]).  ref.b != nullptr: every pileup's base is the reference genome's.
  constexpr int FW = kSomWaves;
  constexpr int NS = DEEP ? NSD : 1;  // allele-table slots: 64 NS distinct alleles per sample
  __shared__ int32_t s_cov[DEEP ? 1 : FW][2][kFastCap];
  __shared__ uint4 s_el[DEEP ? 1 : FW][2][kFastCap];
  __shared__ uint32_t s_tmp[DEEP ? 1 : FW][2 * kFastCap];
  __shared__ int16_t s_order[DEEP ? 1 : FW][64 * NS];
  __shared__ uint8_t s_var[DEEP ? 1 : FW][64 * NS];
  __shared__ double s_ll[DEEP ? 1 : FW][kMaxG];
  __shared__ TermRec s_terms[FW][DEEP ? kDeepTermCap : kFastCap];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // (wave-uniform, and known to be: the candidate records then load into scalar registers)
  const int64_t gwave = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t nwaves_total = ((int64_t)gridDim.x * blockDim.x) >> 6;
  CallMem m;
  if constexpr (DEEP) {
    m = deep_mem(dio.scratch + (size_t)gwave * deep_wave_bytes(dio.scap, dio.maxG, NS), dio.scap, dio.maxG, NS);
    m.terms = s_terms[wv];
    m.tcap = kDeepTermCap;
  } else {
    m.cov[0] = s_cov[wv][0];
    m.cov[1] = s_cov[wv][1];
    m.el[0] = s_el[wv][0];
    m.el[1] = s_el[wv][1];
    m.tmp = s_tmp[wv];
    m.order = s_order[wv];
    m.is_var = s_var[wv];
    m.ll = s_ll[wv];
    m.gkey = nullptr;
    m.gsum = nullptr;
    m.terms = s_terms[wv];
    m.tcap = kFastCap;
    m.cap = kFastCap;
    m.maxG = kMaxG;
  }
  static_assert(!(DEEP && BACK), "the deep kernel runs its own front");
  // amb_sel: a heap-order replay over the amb_in positions listed in dio.list (the wide kernel
  // over the replayed loci the deep kernel's table could not hold), not over all of amb_in
  const bool amb_sel = DEEP && amb_in != nullptr && dio.n_in > 0;
  const unsigned long long n_items = amb_sel  ? (unsigned long long)dio.n_in
                                     : amb_in ? (unsigned long long)n_amb_in
                                     : DEEP ? (unsigned long long)dio.n_in
                                     : BACK ? (unsigned long long)es.b1
                                            : ctr->part_off[1][kParts];
  const int64_t li0 = BACK ? es.b0 + gwave : gwave;
  // dbg & 16: phase clocks per candidate and wave (front or the stored records' load, -, tables,
  // tumor genotypes, normal genotypes + evidence + record, candidates), summed per workgroup in LDS (a global
  // atomic per phase would queue every wave on one address) and added to ctr->prof at the end
  __shared__ unsigned long long s_clk[6];
  __shared__ double s_succ[256];
  if (threadIdx.x < 6) s_clk[threadIdx.x] = 0;
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_succ[i] = g_succ[i];
  __syncthreads();
  m.succ = s_succ;
  uint64_t tk = 0;
  auto tick = [&](int k) {
    if (dbg & 16) {
      const uint64_t t = __builtin_readcyclecounter();
      if (k >= 0 && lane == 0) atomicAdd(&s_clk[k], (unsigned long long)(t - tk));
      tk = t;
    }
  };
  // the next candidate's record is loaded one candidate ahead (it lands while this one runs)
  // (la: the item's position in amb_in, whose resolved reference bases it reads)
  auto fetch_item = [&](int64_t li, int64_t &it, int64_t &la) -> CandRec {
    la = amb_sel ? dio.list[li] : li;
    it = amb_in ? amb_in[la].item : DEEP ? dio.list[li] : li;
    return cands[it];
  };
  int64_t it_next = 0, la_next = 0;
  CandRec item_next{};
  if (li0 < (int64_t)n_items) item_next = fetch_item(li0, it_next, la_next);
  for (int64_t li = li0; li < (int64_t)n_items; li += nwaves_total) {
    tick(-1);
    if ((dbg & 16) && lane == 0) atomicAdd(&s_clk[5], 1ull);
    const int64_t it = it_next, la = la_next;
    const CandRec item = item_next;
    if (li + nwaves_total < (int64_t)n_items) item_next = fetch_item(li + nwaves_total, it_next, la_next);
    const int32_t pos = item.pos;
    const int32_t t_contig = item.contig, t_L0 = item.L0;
    const int64_t t_ord0 = item.ord0;
    const int64_t rb[2] = {item.rb[0], item.rb[1]};
    uint32_t nc[2], mask[2];
    if constexpr (BACK) {
      // the front's records -> LDS (the tables, folds and evidence read them across lanes)
      const uint4 h = es.hdr[li - es.b0];
      if (h.x == kElSkip) continue;
      nc[0] = h.x;
      nc[1] = h.y;
      mask[0] = h.z;
      mask[1] = h.w;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const size_t o = ((size_t)(li - es.b0) * 2 + s) * kFastCap;
        for (uint32_t k = lane; k < nc[s]; k += 64) {
          m.el[s][k] = es.el[o + k];
          m.cov[s][k] = es.cov[o + k];
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    } else {
      if (!call_front<DEEP>(item, it, RT, RN, prm, ctr, sw, m, dbg, dio, nc, mask)) continue;
    }
    Pile<NS> PS[2];
    const int fb = ref.b ? (int)ref.b[ref.off[t_contig] + pos] : -1;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint32_t mk = mask[s];
      for (int d = 1; d < 64; d <<= 1) mk |= __shfl_xor(mk, d, 64);
      PS[s].ambiguous = fb < 0 && __popc(mk) > 1;
      PS[s].refbase = amb_in ? amb_ref[2 * la + s] : fb >= 0 ? (uint8_t)fb : mk ? bit_base(mk) : (uint8_t)'N';
    }
    tick(0);
    if (dbg & 2048) continue;  // ablation: covers + elements
    // ---- allele tables (the records now get their pileup reference base: SNV / DEL keys)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const DevReads &R = s ? RN : RT;
      Pile<NS> &P = PS[s];
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        P.klo[t] = P.khi[t] = 0;
        P.n_all[t] = P.n_f[t] = 0;
      }
      P.nt = 0;
      P.depth_all = P.depth_f = P.fwd_f = 0;
      P.overflow = false;
      for (uint32_t c0 = 0; c0 < nc[s]; c0 += 64) {
        const uint32_t k = c0 + lane;
        uint4 e = make_uint4(0, 0, 0, 0);
        if (k < nc[s]) e = m.el[s][k];
        const uint32_t fl = el_flags(e);
        const bool act = k < nc[s] && (fl & kElAct);
        const bool pass = act && (fl & kElPass);
        AlleleDesc d;
        d.read = rb[s] + (k < nc[s] ? m.cov[s][k] : 0);
        d.rp = (int32_t)e.x;
        d.aux = (int32_t)e.y;
        d.base = (uint8_t)(e.z & 0xFFu);
        d.kind = (uint8_t)((e.z >> 8) & 0xFFu);
        d.rb = P.refbase;
        d.pad = 0;
        Key128 key{0, 0};
        if (act) key = allele_key(R, d, pos, 0);
        const unsigned long long actb = __ballot(act), passb = __ballot(pass);
        P.depth_all += (uint32_t)__popcll(actb);
        P.depth_f += (uint32_t)__popcll(passb);
        P.fwd_f += (uint32_t)__popcll(__ballot(pass && (fl & kElFwd)));
        int mine = -1;
        unsigned long long pending = actb;
        while (pending) {
          const int leader = __ffsll((long long)pending) - 1;
          const uint64_t klo = __shfl(key.lo, leader, 64), khi = __shfl(key.hi, leader, 64);
          const bool match = act && key.lo == klo && key.hi == khi;
          const unsigned long long mb = __ballot(match);
          const uint32_t na = (uint32_t)__popcll(mb), nf = (uint32_t)__popcll(mb & passb);
          int found = -1;
#pragma unroll
          for (int t = 0; t < NS; ++t) {
            const unsigned long long hb = __ballot((t * 64 + lane) < P.nt && P.klo[t] == klo && P.khi[t] == khi);
            if (found < 0 && hb) found = t * 64 + (__ffsll((long long)hb) - 1);
          }
          if (found < 0) {
            if (P.nt >= 64 * NS) {
              P.overflow = true;
            } else {
              found = P.nt++;
              const int owner = found & 63, sl = found >> 6;
              AlleleDesc ldsc;
              ldsc.read = __shfl(d.read, leader, 64);
              ldsc.aux = __shfl(d.aux, leader, 64);
              ldsc.rp = __shfl(d.rp, leader, 64);
              ldsc.kind = (uint8_t)__shfl((int)d.kind, leader, 64);
              ldsc.rb = P.refbase;
              ldsc.base = (uint8_t)__shfl((int)d.base, leader, 64);
              ldsc.pad = 0;
#pragma unroll
              for (int t = 0; t < NS; ++t)
                if (t == sl && lane == owner) {
                  P.klo[t] = klo;
                  P.khi[t] = khi;
                  P.desc[t] = ldsc;
                }
            }
          }
          if (found >= 0) {
            const int owner = found & 63, sl = found >> 6;
#pragma unroll
            for (int t = 0; t < NS; ++t)
              if (t == sl && lane == owner) {
                P.n_all[t] += na;
                P.n_f[t] += nf;
              }
            if (match) mine = found;
          }
          pending &= ~mb;
        }
        if (act && mine >= 0) m.el[s][k].w = (e.w & 0x0007FFFFu) | ((uint32_t)mine << 19);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    Pile<NS> &PT = PS[0], &PN = PS[1];
    // more genotypes than this kernel's likelihood scratch holds (n eligible alleles: n (n + 1) / 2)
    // also leave for the next kernel up
    auto too_many_g = [&](const DevReads &R, const Pile<NS> &P) {
      int n = 0;
#pragma unroll
      for (int t = 0; t < NS; ++t)
        n += __popcll(__ballot((t * 64 + lane) < P.nt && P.n_f[t] > 0 && allele_std_alt(R, P.desc[t], pos)));
      return n * (n + 1) / 2 > m.maxG;
    };
    if (PT.overflow || PN.overflow || too_many_g(RT, PT) || too_many_g(RN, PN)) {
      if constexpr (!DEEP) {  // more distinct alleles than the fast table: the deep kernel's
        if (lane == 0) {
          const unsigned long long k = atomicAdd(&ctr->n_deep, 1ull);
          if (k < dio.cap) dio.list[k] = it;
          atomicMax(&ctr->deep_max, (unsigned long long)max(nc[0], nc[1]));
        }
      } else if (NS < kWideNS) {  // more than the deep table: the wide kernel's (a replayed
        if (lane == 0) {          // locus by its position in amb_in, with its resolved bases)
          const unsigned long long k = atomicAdd(&ctr->n_wide, 1ull);
          if (k < dio.wcap) dio.wide[k] = amb_in ? la : it;
        }
      } else {
        raise_at(ctr, GQ_E_CAPACITY, pos);
      }
      continue;
    }
    if ((item.flags & 1) && !amb_in && (PT.depth_all + PN.depth_all) > 0 && lane == 0)
      atomicAdd(&ctr->spread[0][it & (kSpread - 1)], 1ull);
    if (!amb_in && (PT.ambiguous || PN.ambiguous)) {  // heap order decides a reference base: list it
      if (lane == 0) {
        const unsigned long long k = atomicAdd(&ctr->n_amb, 1ull);
        if (k < amb_cap) amb_out[k] = AmbItem{item.tile, pos, it};
        atomicMax(&ctr->deep_max, (unsigned long long)max(nc[0], nc[1]));
      }
      continue;
    }
    tick(2);
    if (dbg & 4096) continue;  // ablation: up to the tables
    if (prm.filter_multi_allelic) {  // MultiAllelicPileupFilter (PileupFilter.scala:29-44)
      if (PT.nt > 2) PT.depth_f = 0;
      if (PN.nt > 2) PN.depth_f = 0;
    }
    // SomaticStandardCaller.scala:184-190
    if (PT.depth_f == 0 || PN.depth_f == 0 || (int64_t)PT.depth_f > (int64_t)prm.max_read_depth ||
        (int64_t)PN.depth_f > (int64_t)prm.max_read_depth)
      continue;
    {  // the tumor pileup must hold a non-Match element: Match = allele (ref, ref) of one byte
      uint32_t ref_match = 0;
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        const bool mt = (t * 64 + lane) < PT.nt && PT.desc[t].kind == K_SNV && PT.desc[t].base == PT.refbase;
        ref_match += (uint32_t)wave_sum(mt ? (double)PT.n_f[t] : 0.0);
      }
      if (ref_match == PT.depth_f) continue;
    }
    // the multi-allelic filter empties a pileup: no element passes then
    const int nT = PT.depth_f ? (int)nc[0] : 0, nN = PN.depth_f ? (int)nc[1] : 0;
    const GenoOut tg = genotypes_el(RT, PT, m.el[0], nT, pos, true, false, m, ctr);
    tick(3);
    if ((dbg & 16) && lane == 0) atomicAdd(&s_clk[1], (unsigned long long)tg.cyc_fold);  // (inside phase 3)
    if (dbg & 8192) continue;  // ablation: up to the tumor genotypes
    if (tg.G == 0) continue;
    const bool t_var = m.is_var[tg.bi] || m.is_var[tg.bj];
    if (!t_var) continue;
    const AlleleDesc a1 = pile_entry(PT, tg.bi), a2 = pile_entry(PT, tg.bj);
    const GenoOut ng = genotypes_el(RN, PN, m.el[1], nN, pos, false, true, m, ctr);
    const double nvs = ng.G == 0 ? 0.0 : ng.var_sum;
    const double odds = tg.best_l / nvs;
    if (!(odds * 100.0 >= (double)prm.odds)) continue;
    uint8_t knife = near_edge(odds * 100.0, (double)prm.odds) ? GQ_FLAG_KNIFE_EDGE : 0;
    // first variant allele of the ML genotype with a non-empty alt (SomaticStandardCaller.scala:227)
    const bool v1 = allele_is_variant(RT, a1, pos) && allele_alt_len(a1) > 0;
    const bool v2 = allele_is_variant(RT, a2, pos) && allele_alt_len(a2) > 0;
    if (!v1 && !v2) continue;
    const AlleleDesc al = v1 ? a1 : a2;
    const int t_idx = v1 ? tg.bi : tg.bj;
    const int rl = allele_ref_len(al), alt_l = allele_alt_len(al);
    const Key128 nkey = key_from(rl, rl, 0, [&](int, int i) { return allele_byte(RT, al, pos, 0, i); });
    const int n_idx = PN.depth_f ? pile_find(PN, nkey) : -1;
    // log-odds and the phred likelihood need no evidence (its likelihoods are tg.best_l and
    // 1 - nvs): a candidate the driver's filters drop on them skips the evidence pass
    const double log_odds = sm::log(odds);
    const double lik = tg.best_l * (1.0 - nvs) - 1e-10;
    const int gqv = success_to_phred(lik);
    if (prm.apply_filters == 1 && (!(log_odds > (double)prm.min_lod) || !(gqv >= prm.min_likelihood))) continue;
    gq_evidence tev, nev;
    evidence_pair(PT, PN, m.el[0], nT, m.el[1], nN, t_idx, n_idx, tg.best_l, 1.0 - nvs, pos, m, tev, nev);
    if (phred_rounding_edge(lik)) knife |= GQ_FLAG_KNIFE_EDGE;
    const float vaf = (float)tev.allele_read_depth / (float)tev.read_depth;
    if (prm.apply_filters == 1) {  // SomaticStandardCaller.scala:124-137 then SomaticGenotypeFilter.apply (:285-307)
      const bool depth_ok = tev.read_depth >= prm.min_tumor_read_depth && tev.read_depth < prm.max_tumor_read_depth &&
                            nev.read_depth >= prm.min_normal_read_depth && nev.read_depth < 0x7FFFFFFF;
      if (!depth_ok) continue;
      if (!(tev.allele_read_depth >= prm.min_tumor_alternate_read_depth)) continue;
      if (!(log_odds > (double)prm.min_lod)) continue;
      if (near_edge(log_odds, (double)prm.min_lod)) knife |= GQ_FLAG_KNIFE_EDGE;
      if (!(gqv >= prm.min_likelihood)) continue;
      if (!((double)vaf * 100.0 > (double)prm.min_vaf)) continue;
      if (!(tev.mean_mq >= prm.min_average_mapping_quality && nev.mean_mq >= prm.min_average_mapping_quality)) continue;
      if (near_edge(tev.mean_mq, prm.min_average_mapping_quality) || near_edge(nev.mean_mq, prm.min_average_mapping_quality) ||
          near_edge(tev.mean_mq, prm.min_average_base_quality) || near_edge(nev.mean_mq, prm.min_average_base_quality))
        knife |= GQ_FLAG_KNIFE_EDGE;
      // the "average base quality" filter tests mean mapping quality (SomaticGenotypeFilter.scala:194-195)
      if (!(tev.mean_mq >= prm.min_average_base_quality && nev.mean_mq >= prm.min_average_base_quality)) continue;
      if (!(tev.median_mismatches <= (double)prm.max_median_mismatches)) continue;
    } else if (prm.apply_filters == 2) {  // SomaticGenotypeFilter(Seq, ...) as the caller suite uses it
      if (!(tev.read_depth >= prm.min_tumor_read_depth && tev.read_depth < prm.max_tumor_read_depth &&
            nev.read_depth >= prm.min_normal_read_depth && nev.read_depth < 0x7FFFFFFF))
        continue;
      if (!((double)vaf * 100.0 > (double)prm.min_vaf)) continue;
      if (!(gqv >= prm.min_likelihood)) continue;
      if (prm.min_tumor_alternate_read_depth > 0 && !(tev.allele_read_depth >= prm.min_tumor_alternate_read_depth))
        continue;
    }
    SomRec rr;
    rr.key = (uint64_t)(t_ord0 + (pos - t_L0)) << 12;
    rr.contig = t_contig;
    rr.pos = pos;
    rr.ref_len = (uint16_t)rl;
    rr.alt_len = (uint16_t)alt_l;
    rr.flags = (PT.ambiguous ? 1 : 0) | (PN.ambiguous ? 2 : 0) | knife;
    rr.pad[0] = rr.pad[1] = rr.pad[2] = 0;
    rr.log_odds = log_odds;
    rr.gq = gqv;
    rr.pad2 = 0;
    rr.tumor = tev;
    rr.normal = nev;
    if (rl + alt_l <= 8) {
      uint64_t v = 0;
      int j = 0;
      for (int i = 0; i < rl; ++i) v |= (uint64_t)allele_byte(RT, al, pos, 0, i) << (8 * j++);
      for (int i = 0; i < alt_l; ++i) v |= (uint64_t)allele_byte(RT, al, pos, 1, i) << (8 * j++);
      rr.allele = v;
    } else {
      unsigned long long off = 0;
      if (lane == 0) off = atomicAdd(&ctr->pool_used, (unsigned long long)(rl + alt_l));
      off = __shfl(off, 0, 64);
      if (off + rl + alt_l <= pool_cap)
        for (int i = lane; i < rl + alt_l; i += 64)
          pool[off + i] = i < rl ? allele_byte(RT, al, pos, 0, i) : allele_byte(RT, al, pos, 1, i - rl);
      rr.allele = off;
    }
    if (lane == 0) {
      const unsigned long long k = atomicAdd(&ctr->n_rec, 1ull);
      if (k < rec_cap) recs[k] = rr;
    }
    tick(4);
  }
  if (dbg & 16) {
    __syncthreads();
    if (threadIdx.x < 6 && s_clk[threadIdx.x]) atomicAdd(&ctr->prof[threadIdx.x], s_clk[threadIdx.x]);
  }
}

// The split caller's front (GQ_CALL_SPLIT=1; off by default, see gq_somatic_standard): covers
// and element records of the candidates [es.b0, es.b1) into the element store, one wave per
// candidate.  It holds only the front's registers (4 waves per SIMD against the one kernel's 3);
// measured, that did not pay for the store's traffic and the second pass over the candidates.
#ifndef GQ_FRONT_WPE
#define GQ_FRONT_WPE 4
#endif
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GQ_FRONT_WPE))) void somatic_front(
    const CandRec *__restrict__ cands, DevReads RT, DevReads RN, gq_somatic_params prm, Counters *ctr, SomWin sw,
    int dbg, DeepIO dio, ElemStore es) {
  constexpr int FW = kSomWaves;
  __shared__ int32_t s_cov[FW][2][kFastCap];
  __shared__ uint32_t s_tmp[FW][2 * kFastCap];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // (wave-uniform, and known to be: the candidate records then load into scalar registers)
  const int64_t gwave = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t nwaves_total = ((int64_t)gridDim.x * blockDim.x) >> 6;
  CallMem m{};
  m.cov[0] = s_cov[wv][0];
  m.cov[1] = s_cov[wv][1];
  m.tmp = s_tmp[wv];
  m.cap = kFastCap;
  m.maxG = kMaxG;
  CandRec item_next{};
  if (es.b0 + gwave < es.b1) item_next = cands[es.b0 + gwave];
  for (int64_t li = es.b0 + gwave; li < es.b1; li += nwaves_total) {
    const CandRec item = item_next;
    if (li + nwaves_total < es.b1) item_next = cands[li + nwaves_total];
    const size_t o = (size_t)(li - es.b0) * 2 * kFastCap;
    m.el[0] = es.el + o;  // the element records go straight to the store
    m.el[1] = es.el + o + kFastCap;
    uint32_t nc[2], mask[2];
    const bool go = call_front<false>(item, li, RT, RN, prm, ctr, sw, m, dbg, dio, nc, mask);
    uint4 h = make_uint4(kElSkip, 0, 0, 0);
    if (go) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        for (int d = 1; d < 64; d <<= 1) mask[s] |= __shfl_xor(mask[s], d, 64);
        for (uint32_t k = lane; k < nc[s]; k += 64) es.cov[o + (size_t)s * kFastCap + k] = m.cov[s][k];
      }
      h = make_uint4(nc[0], nc[1], mask[0], mask[1]);
    }
    if (lane == 0) es.hdr[li - es.b0] = h;
    __builtin_amdgcn_wave_barrier();  // (the next candidate rewrites this wave's LDS)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}
