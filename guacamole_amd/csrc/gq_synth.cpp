// gq_synth.cpp — deterministic, multithreaded synthetic read generator.
//
// Produces the gq_reads SoA (include/gqpileup.h) directly, MD already parsed into
// events, for configurations up to whole-genome scale.  Every random draw comes
// from a counter-based generator keyed by (seed, stream, index), so the output is
// independent of the thread count.
//
// Model: reference i.i.d. with GC 0.41; germline het SNVs (rate het, VAF 0.5),
// hom-alt SNVs (rate hom), indels (rate indel, 1-10 bp, 2/3 het, 1/2 insertions);
// optional somatic SNVs (rate somatic) at VAF U(0.1, 0.5) present only in a
// "tumor" draw; reads of length L start at Poisson(depth/L) per position,
// haplotype and strand 50/50, mapq 60 (2 % uniform 0..59), base qualities from a
// mixture on 2..41 (mean ~33.5) and substitution errors with probability
// 10^(-q/10).  Reads crossing an indel carry the corresponding I/D CIGAR op
// (reads are error-free through an indel to keep the alignment canonical).
#include <stdint.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
inline uint64_t rnd(uint64_t seed, uint64_t stream, uint64_t i) { return mix64(mix64(seed ^ (stream * 0x632be59bd9b4e019ull)) ^ i); }
inline double u01(uint64_t x) { return (double)(x >> 11) * (1.0 / 9007199254740992.0); }

const uint8_t kBases[4] = {'A', 'C', 'G', 'T'};
inline int base_idx(uint8_t b) { return b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : 3; }

enum Stream : uint64_t {
  S_REF = 1, S_SNV = 2, S_SNV_ALT = 3, S_SNV_HAP = 4, S_INDEL = 5, S_INDEL_P = 6, S_START = 7, S_READ = 8,
  S_BASE = 9, S_SOM = 10, S_SOM_P = 11
};

struct Indel {
  int64_t pos;
  int32_t del;
  int32_t ins_len;
  uint8_t haps;
  uint8_t ins[10];
};

int nthreads() {
  const char *e = getenv("GQ_SYNTH_THREADS");
  int n = e ? atoi(e) : (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(n, 32));
}

template <class F>
void parallel_for(int64_t n, F &&f) {
  const int T = nthreads();
  const int64_t chunk = (n + T - 1) / T;
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    int64_t a = t * chunk, b = std::min(n, a + chunk);
    if (a >= b) break;
    th.emplace_back([=, &f]() { f(t, a, b); });
  }
  for (auto &x : th) x.join();
}

}  // namespace

extern "C" {

typedef struct {
  int64_t length;
  double depth;
  int32_t read_len;
  uint64_t seed;          // variant / reference seed (shared by tumor and normal)
  uint64_t read_seed;     // read sampling seed (differs between tumor and normal)
  double het, hom, indel, somatic;
  int32_t with_somatic;   // 1 => reads carry somatic alleles (tumor)
} gq_synth_params;

typedef struct {
  int64_t n_reads;
  int32_t *start, *end, *pmax_end;
  uint8_t *mapq, *flags, *sample;
  int64_t *seq_off;
  int32_t *seq_len;
  int64_t *cigar_off;
  int32_t *n_cigar;
  int64_t *md_off;
  int32_t *n_md;
  uint16_t *n_mismatch;
  int64_t seq_bytes, cigar_len, md_len;
  uint8_t *seq, *qual;
  uint32_t *cigar, *md_ev;
  uint8_t *ref;           // reference bases [length]
  int64_t n_snv, n_indel, n_somatic;
} gq_synth_out;

void gq_synth_free(gq_synth_out *o) {
  if (!o) return;
  void *ps[] = {o->start, o->end, o->pmax_end, o->mapq, o->flags, o->sample, o->seq_off, o->seq_len, o->cigar_off,
                o->n_cigar, o->md_off, o->n_md, o->n_mismatch, o->seq, o->qual, o->cigar, o->md_ev, o->ref};
  for (void *p : ps) free(p);
  memset(o, 0, sizeof(*o));
}

int gq_synth_generate(const gq_synth_params *P, gq_synth_out *o) {
  memset(o, 0, sizeof(*o));
  const int64_t G = P->length;
  const int L = P->read_len;
  if (G <= 2 * L + 64 || L <= 0 || L > 4096) return 1;
  // ---- reference
  uint8_t *ref = (uint8_t *)malloc((size_t)G);
  parallel_for(G, [&](int, int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      double u = u01(rnd(P->seed, S_REF, (uint64_t)i));
      ref[i] = u < 0.295 ? 'A' : u < 0.5 ? 'C' : u < 0.705 ? 'G' : 'T';
    }
  });
  // ---- germline SNVs: per-position Bernoulli, 2 haplotype copies
  uint8_t *hap0 = (uint8_t *)malloc((size_t)G), *hap1 = (uint8_t *)malloc((size_t)G);
  std::atomic<int64_t> nsnv{0};
  parallel_for(G, [&](int, int64_t a, int64_t b) {
    int64_t k = 0;
    for (int64_t i = a; i < b; ++i) {
      hap0[i] = hap1[i] = ref[i];
      double u = u01(rnd(P->seed, S_SNV, (uint64_t)i));
      if (u < P->het + P->hom) {
        uint8_t alt = kBases[(base_idx(ref[i]) + 1 + (int)(rnd(P->seed, S_SNV_ALT, (uint64_t)i) % 3)) & 3];
        uint8_t haps = u < P->hom ? 3 : (uint8_t)(1 + (rnd(P->seed, S_SNV_HAP, (uint64_t)i) & 1));
        if (haps & 1) hap0[i] = alt;
        if (haps & 2) hap1[i] = alt;
        ++k;
      }
    }
    nsnv += k;
  });
  // ---- indels (sequential scan, sparse); SNVs next to an indel are removed
  std::vector<Indel> indels;
  {
    int64_t last_end = -100;
    for (int64_t i = L; i < G - L - 16; ++i) {
      if (u01(rnd(P->seed, S_INDEL, (uint64_t)i)) >= P->indel) continue;
      if (i <= last_end + 2) continue;
      uint64_t r = rnd(P->seed, S_INDEL_P, (uint64_t)i);
      Indel d{};
      d.pos = i;
      int len = 1 + (int)(r % 10);
      d.haps = ((r >> 8) % 3 == 0) ? 3 : (uint8_t)(1 + ((r >> 12) & 1));
      if ((r >> 16) & 1) {
        d.del = len;
      } else {
        d.ins_len = len;
        for (int j = 0; j < len; ++j) d.ins[j] = kBases[(r >> (20 + 2 * j)) & 3];
      }
      for (int64_t j = std::max<int64_t>(0, i - 1); j <= std::min<int64_t>(G - 1, i + d.del + 1); ++j) {
        hap0[j] = ref[j];
        hap1[j] = ref[j];
      }
      last_end = i + d.del + 1;
      indels.push_back(d);
    }
  }
  // ---- somatic SNVs (tumor only): positions + alt + VAF
  std::vector<int64_t> som_pos;
  std::vector<uint8_t> som_alt;
  std::vector<double> som_vaf;
  if (P->somatic > 0) {
    for (int64_t i = L; i < G - L; ++i) {
      double u = u01(rnd(P->seed, S_SOM, (uint64_t)i));
      if (u >= P->somatic) continue;
      uint64_t r = rnd(P->seed, S_SOM_P, (uint64_t)i);
      som_pos.push_back(i);
      som_alt.push_back(kBases[(base_idx(hap0[i]) + 1 + (int)(r % 3)) & 3]);
      som_vaf.push_back(0.1 + 0.4 * u01(mix64(r)));
    }
  }
  // ---- read starts: Poisson(lambda) reads per start position in [0, G - L - 16)
  const int64_t span = G - L - 16;
  const double lam = P->depth / (double)L;
  const double e0 = std::exp(-lam);
  const int T = nthreads();
  std::vector<int64_t> per(T + 1, 0);
  auto count_at = [&](int64_t i) -> int {
    double u = u01(rnd(P->read_seed, S_START, (uint64_t)i));
    int k = 0;
    double p = e0, c = e0;
    while (u > c && k < 64) {
      ++k;
      p *= lam / k;
      c += p;
    }
    return k;
  };
  const int64_t chunk = (span + T - 1) / T;
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        int64_t a = t * chunk, b = std::min(span, a + chunk), n = 0;
        for (int64_t i = a; i < b; ++i) n += count_at(i);
        per[t + 1] = n;
      });
    for (auto &x : th) x.join();
  }
  for (int t = 0; t < T; ++t) per[t + 1] += per[t];
  const int64_t N = per[T];
  o->n_reads = N;
  o->start = (int32_t *)malloc(sizeof(int32_t) * (size_t)std::max<int64_t>(N, 1));
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        int64_t a = t * chunk, b = std::min(span, a + chunk), w = per[t];
        for (int64_t i = a; i < b; ++i) {
          int k = count_at(i);
          for (int j = 0; j < k; ++j) o->start[w++] = (int32_t)i;
        }
      });
    for (auto &x : th) x.join();
  }
  // ---- per-read fields and bases
  o->end = (int32_t *)malloc(sizeof(int32_t) * (size_t)std::max<int64_t>(N, 1));
  o->mapq = (uint8_t *)malloc((size_t)std::max<int64_t>(N, 1));
  o->flags = (uint8_t *)malloc((size_t)std::max<int64_t>(N, 1));
  o->sample = (uint8_t *)calloc((size_t)std::max<int64_t>(N, 1), 1);
  o->seq_off = (int64_t *)malloc(sizeof(int64_t) * (size_t)std::max<int64_t>(N, 1));
  o->seq_len = (int32_t *)malloc(sizeof(int32_t) * (size_t)std::max<int64_t>(N, 1));
  o->n_cigar = (int32_t *)malloc(sizeof(int32_t) * (size_t)std::max<int64_t>(N, 1));
  o->n_md = (int32_t *)malloc(sizeof(int32_t) * (size_t)std::max<int64_t>(N, 1));
  o->n_mismatch = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)std::max<int64_t>(N, 1));
  o->seq_bytes = N * (int64_t)L;
  o->seq = (uint8_t *)malloc((size_t)std::max<int64_t>(o->seq_bytes, 1));
  o->qual = (uint8_t *)malloc((size_t)std::max<int64_t>(o->seq_bytes, 1));
  // per-thread variable-length outputs (cigar ops, md events), concatenated afterwards
  std::vector<std::vector<uint32_t>> tcig(T), tev(T);
  std::vector<int64_t> rb(T + 1, 0);
  const int64_t rchunk = (N + T - 1) / T;
  double err_p[256];
  for (int q = 0; q < 256; ++q) err_p[q] = std::pow(10.0, -q / 10.0);
  std::vector<int64_t> ind_pos(indels.size());
  for (size_t i = 0; i < indels.size(); ++i) ind_pos[i] = indels[i].pos;
  {
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t]() {
        const int64_t a = t * rchunk, b = std::min(N, a + rchunk);
        std::vector<uint32_t> &cig = tcig[t];
        std::vector<uint32_t> &ev = tev[t];
        std::vector<uint8_t> tmp(L);
        for (int64_t r = a; r < b; ++r) {
          const uint64_t rr = rnd(P->read_seed, S_READ, (uint64_t)r);
          const int h = (int)(rr & 1);
          const bool rev = (rr >> 1) & 1;
          int mq = 60;
          if (u01(mix64(rr)) < 0.02) mq = (int)((rr >> 40) % 60);
          o->mapq[r] = (uint8_t)mq;
          o->flags[r] = rev ? 1 : 0;
          o->seq_off[r] = r * (int64_t)L;
          o->seq_len[r] = L;
          const uint8_t *hap = h ? hap1 : hap0;
          int64_t s = o->start[r];
          uint8_t *sq = o->seq + r * (int64_t)L;
          uint8_t *qq = o->qual + r * (int64_t)L;
          // indel on this haplotype within the read's reach?
          auto it = std::lower_bound(ind_pos.begin(), ind_pos.end(), s - 12);
          bool special = false;
          for (auto jt = it; jt != ind_pos.end() && *jt < s + L; ++jt) {
            const Indel &d = indels[(size_t)(jt - ind_pos.begin())];
            if (((d.haps >> h) & 1) && d.pos + d.del >= s) special = true;
          }
          // qualities
          for (int i = 0; i < L; ++i) {
            uint64_t x = rnd(P->read_seed, S_BASE, (uint64_t)(r * L + i));
            double u = u01(x);
            int q;
            if (u < 0.75) q = 33 + (int)((x >> 8) % 9);
            else if (u < 0.95) q = 20 + (int)((x >> 8) % 13);
            else q = 2 + (int)((x >> 8) % 18);
            qq[i] = (uint8_t)q;
          }
          const size_t ev0 = ev.size(), cig0 = cig.size();
          int nmm = 0;
          if (!special) {
            for (int i = 0; i < L; ++i) sq[i] = hap[s + i];
            if (!som_pos.empty()) {
              auto lo = std::lower_bound(som_pos.begin(), som_pos.end(), s);
              for (auto jt = lo; jt != som_pos.end() && *jt < s + L; ++jt) {
                size_t k = (size_t)(jt - som_pos.begin());
                if (P->with_somatic && u01(rnd(P->read_seed, S_SOM_P, (uint64_t)(r * 131 + k))) < som_vaf[k])
                  sq[*jt - s] = som_alt[k];
              }
            }
            for (int i = 0; i < L; ++i) {  // substitution errors, p = 10^(-q/10)
              uint64_t x = rnd(P->read_seed ^ 0x5555, S_BASE, (uint64_t)(r * L + i));
              if (u01(x) < err_p[qq[i]])
                sq[i] = kBases[(base_idx(sq[i]) + 1 + (int)((x >> 3) % 3)) & 3];
            }
            cig.push_back(((uint32_t)L << 4) | 0u);
            for (int i = 0; i < L; ++i)
              if (sq[i] != ref[s + i]) {
                ev.push_back(((uint32_t)i << 8) | ref[s + i]);
                ++nmm;
              }
            o->end[r] = (int32_t)(s + L);
          } else {
            // a start inside a deleted run moves past it
            {
              auto jt = std::upper_bound(ind_pos.begin(), ind_pos.end(), s);
              if (jt != ind_pos.begin()) {
                const Indel &d = indels[(size_t)(jt - ind_pos.begin() - 1)];
                if (((d.haps >> h) & 1) && d.del && d.pos < s && s <= d.pos + d.del) s = d.pos + d.del + 1;
              }
            }
            o->start[r] = (int32_t)s;
            int i = 0;
            int64_t p = s;
            auto push = [&](int op, int n) {
              if (cig.size() > cig0 && (int)(cig.back() & 15u) == op) cig.back() += (uint32_t)n << 4;
              else cig.push_back(((uint32_t)n << 4) | (uint32_t)op);
            };
            auto nxt = std::lower_bound(ind_pos.begin(), ind_pos.end(), p);
            while (i < L) {
              sq[i] = hap[p];
              push(0, 1);
              if (sq[i] != ref[p]) {
                ev.push_back(((uint32_t)(p - s) << 8) | ref[p]);
                ++nmm;
              }
              ++i;
              while (nxt != ind_pos.end() && *nxt < p) ++nxt;
              if (nxt != ind_pos.end() && *nxt == p && i < L) {
                const Indel &d = indels[(size_t)(nxt - ind_pos.begin())];
                if ((d.haps >> h) & 1) {
                  if (d.del) {
                    push(2, d.del);
                    for (int j = 1; j <= d.del; ++j) ev.push_back(((uint32_t)(p + j - s) << 8) | ref[p + j]);
                    p += d.del;
                  } else if (i + d.ins_len < L) {
                    push(1, d.ins_len);
                    for (int j = 0; j < d.ins_len; ++j) sq[i++] = d.ins[j];
                  }
                }
              }
              ++p;
            }
            o->end[r] = (int32_t)p;
          }
          o->n_cigar[r] = (int32_t)(cig.size() - cig0);
          o->n_md[r] = (int32_t)(ev.size() - ev0);
          o->n_mismatch[r] = (uint16_t)std::min(nmm, 65535);
        }
      });
    for (auto &x : th) x.join();
  }
  // ---- concatenate variable-length pools
  o->cigar_off = (int64_t *)malloc(sizeof(int64_t) * (size_t)std::max<int64_t>(N, 1));
  o->md_off = (int64_t *)malloc(sizeof(int64_t) * (size_t)std::max<int64_t>(N, 1));
  int64_t nc = 0, ne = 0;
  for (int t = 0; t < T; ++t) {
    nc += (int64_t)tcig[t].size();
    ne += (int64_t)tev[t].size();
  }
  o->cigar_len = nc;
  o->md_len = ne;
  o->cigar = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)std::max<int64_t>(nc, 1));
  o->md_ev = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)std::max<int64_t>(ne, 1));
  {
    int64_t co = 0, eo = 0;
    for (int t = 0; t < T; ++t) {
      memcpy(o->cigar + co, tcig[t].data(), tcig[t].size() * 4);
      memcpy(o->md_ev + eo, tev[t].data(), tev[t].size() * 4);
      co += (int64_t)tcig[t].size();
      eo += (int64_t)tev[t].size();
    }
    co = eo = 0;
    for (int64_t r = 0; r < N; ++r) {
      o->cigar_off[r] = co;
      o->md_off[r] = eo;
      co += o->n_cigar[r];
      eo += o->n_md[r];
    }
  }
  // ---- restore (contig, start) order if a shifted start broke it (stable), prefix-max end
  bool sorted = true;
  for (int64_t r = 1; r < N && sorted; ++r) sorted = o->start[r - 1] <= o->start[r];
  if (!sorted) {
    std::vector<int64_t> ord((size_t)N);
    for (int64_t r = 0; r < N; ++r) ord[(size_t)r] = r;
    std::stable_sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) { return o->start[x] < o->start[y]; });
    auto perm = [&](auto *arr) {
      using E = std::remove_pointer_t<decltype(arr)>;
      std::vector<E> tmp((size_t)N);
      for (int64_t r = 0; r < N; ++r) tmp[(size_t)r] = arr[ord[(size_t)r]];
      memcpy(arr, tmp.data(), sizeof(E) * (size_t)N);
    };
    perm(o->start); perm(o->end); perm(o->mapq); perm(o->flags); perm(o->seq_off); perm(o->seq_len);
    perm(o->cigar_off); perm(o->n_cigar); perm(o->md_off); perm(o->n_md); perm(o->n_mismatch);
  }
  o->pmax_end = (int32_t *)malloc(sizeof(int32_t) * (size_t)std::max<int64_t>(N, 1));
  int32_t m = INT32_MIN;
  for (int64_t r = 0; r < N; ++r) {
    m = std::max(m, o->end[r]);
    o->pmax_end[r] = m;
  }
  o->ref = ref;
  o->n_snv = nsnv;
  o->n_indel = (int64_t)indels.size();
  o->n_somatic = (int64_t)som_pos.size();
  free(hap0);
  free(hap1);
  return 0;
}

// One BAM record per read of [a, e) appended to `b` (ref_id from the read's local contig, read
// name "r<name_base + index>"); MD strings are rebuilt from the MD events the way
// synthetic.md_string does (a deleted base without an event is written as N).
static void bam_records(const gq_synth_out *o, int64_t a, int64_t e, const int64_t *crb, int32_t n_local,
                        const int32_t *ref_id, int64_t name_base, std::string &b) {
  auto put32 = [](std::string &s, uint32_t v) { s.append((const char *)&v, 4); };
  std::string md;
  static const char kNib[] = "=ACMGRSVTWYHKDBN";
  uint8_t code[256];
  memset(code, 15, sizeof(code));
  for (int k = 0; k < 16; ++k) code[(uint8_t)kNib[k]] = (uint8_t)k;
  int32_t lc = 0;
  while (lc + 1 < n_local && crb[lc + 1] <= a) ++lc;
  for (int64_t r = a; r < e; ++r) {
    while (lc + 1 < n_local && crb[lc + 1] <= r) ++lc;
    const uint32_t *cg = o->cigar + o->cigar_off[r];
    const int32_t nc = o->n_cigar[r], ls = o->seq_len[r];
    const uint32_t *ev = o->md_ev + o->md_off[r];
    const int32_t ne = std::max(o->n_md[r], 0);
    md.clear();
    int64_t run = 0, ref = 0;
    int32_t k = 0;
    for (int32_t c = 0; c < nc; ++c) {
      const uint32_t op = cg[c] & 15, ln = cg[c] >> 4;
      if (op == 0 || op == 7 || op == 8) {
        const int64_t end = ref + ln;
        while (k < ne && (int64_t)(ev[k] >> 8) < end) {
          const int64_t off = ev[k] >> 8;
          run += off - ref;
          md += std::to_string(run);
          md += (char)(ev[k] & 0xFF);
          run = 0;
          ref = off + 1;
          ++k;
        }
        run += end - ref;
        ref = end;
      } else if (op == 2) {
        md += std::to_string(run);
        md += '^';
        for (uint32_t j = 0; j < ln; ++j) {
          if (k < ne && (int64_t)(ev[k] >> 8) == ref + j) md += (char)(ev[k++] & 0xFF);
          else md += 'N';
        }
        run = 0;
        ref += ln;
      } else if (op == 3) {
        ref += ln;
      }
    }
    md += std::to_string(run);
    const std::string name = "r" + std::to_string(name_base + r);
    const uint32_t l_name = (uint32_t)name.size() + 1;
    const uint32_t block = 32 + l_name + 4 * (uint32_t)nc + (uint32_t)(ls + 1) / 2 + (uint32_t)ls + 3 +
                           (uint32_t)md.size() + 1;
    put32(b, block);
    put32(b, (uint32_t)ref_id[lc]);
    put32(b, (uint32_t)o->start[r]);
    b += (char)l_name;
    b += (char)o->mapq[r];
    b.append("\0\0", 2);  // bin (unused by readers here)
    const uint16_t ncig = (uint16_t)nc, flag = (o->flags[r] & 1) ? 16 : 0;
    b.append((const char *)&ncig, 2);
    b.append((const char *)&flag, 2);
    put32(b, (uint32_t)ls);
    put32(b, 0xFFFFFFFFu);
    put32(b, 0xFFFFFFFFu);
    put32(b, 0);
    b.append(name.c_str(), l_name);
    b.append((const char *)cg, 4 * (size_t)nc);
    const uint8_t *sq = o->seq + o->seq_off[r];
    for (int32_t j = 0; j < ls; j += 2) {
      const uint8_t hi = code[sq[j]], lo = j + 1 < ls ? code[sq[j + 1]] : 0;
      b += (char)((hi << 4) | lo);
    }
    b.append((const char *)(o->qual + o->seq_off[r]), (size_t)ls);
    b.append("MDZ", 3);
    b.append(md.c_str(), md.size() + 1);
  }
}

// One BGZF block of src[0, len) (len <= 65280; len 0: the EOF marker).
static void bgzf_block(const uint8_t *src, int64_t len, int level, std::string &out) {
  z_stream z;
  memset(&z, 0, sizeof(z));
  deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
  std::string buf(deflateBound(&z, (uLong)len) + 64, '\0');
  z.next_in = const_cast<uint8_t *>(src);
  z.avail_in = (uInt)len;
  z.next_out = (Bytef *)&buf[18];
  z.avail_out = (uInt)(buf.size() - 26);
  deflate(&z, Z_FINISH);
  const size_t clen = z.total_out;
  deflateEnd(&z);
  const uint32_t bsize = (uint32_t)(18 + clen + 8);
  const uint8_t hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0,
                           (uint8_t)((bsize - 1) & 0xFF), (uint8_t)((bsize - 1) >> 8)};
  memcpy(&buf[0], hdr, 18);
  const uint32_t crc = (uint32_t)crc32(0L, src, (uInt)len), isz = (uint32_t)len;
  memcpy(&buf[18 + clen], &crc, 4);
  memcpy(&buf[18 + clen + 4], &isz, 4);
  buf.resize(bsize);
  out.swap(buf);
}

// A coordinate-sorted BAM (or a piece of one) of the read set, streamed in chunks of reads:
// each chunk's records are serialised and BGZF-compressed (level `level`) on every thread and
// appended, so memory stays bounded by the chunk whatever the read count.
//   n_ref / ref_names / ref_lens: the header's dictionary (written when flags & 1);
//   crb[n_local + 1], ref_id[n_local]: the reads' local contigs and their header ids;
//   flags: 1 = header first, 2 = the EOF block last, 4 = append to the file;
//   name_base: read names are "r<name_base + index>" (unique across the pieces of one file).
// A piece written without header / EOF is a run of whole BGZF blocks: pieces concatenate.
int gq_synth_write_bam_ex(const gq_synth_out *o, const char *path, int32_t n_ref, const char **ref_names,
                          const int64_t *ref_lens, int32_t n_local, const int64_t *crb, const int32_t *ref_id,
                          int32_t level, int32_t flags, int64_t name_base) {
  const int64_t N = o->n_reads;
  const int T = nthreads();
  const int64_t kBlk = 65280;
  FILE *f = fopen(path, (flags & 4) ? "ab" : "wb");
  if (!f) return 1;
  std::string data;  // uncompressed bytes not yet in a full block
  auto put32 = [](std::string &s, uint32_t v) { s.append((const char *)&v, 4); };
  if (flags & 1) {
    std::string text = "@HD\tVN:1.6\tSO:coordinate\n";
    for (int32_t k = 0; k < n_ref; ++k)
      text += std::string("@SQ\tSN:") + ref_names[k] + "\tLN:" + std::to_string(ref_lens[k]) + "\n";
    data.append("BAM\1", 4);
    put32(data, (uint32_t)text.size());
    data += text;
    put32(data, (uint32_t)n_ref);
    for (int32_t k = 0; k < n_ref; ++k) {
      put32(data, (uint32_t)strlen(ref_names[k]) + 1);
      data.append(ref_names[k], strlen(ref_names[k]) + 1);
      put32(data, (uint32_t)ref_lens[k]);
    }
  }
  int rc = 0;
  auto flush = [&](bool all) {  // compress the whole blocks of `data` (all: the tail too)
    const int64_t nb = all ? ((int64_t)data.size() + kBlk - 1) / kBlk : (int64_t)data.size() / kBlk;
    if (nb <= 0) return;
    std::vector<std::string> comp((size_t)nb);
    parallel_for(nb, [&](int, int64_t a, int64_t e) {
      for (int64_t i = a; i < e; ++i)
        bgzf_block((const uint8_t *)data.data() + i * kBlk, std::min<int64_t>(kBlk, (int64_t)data.size() - i * kBlk),
                   level, comp[(size_t)i]);
    });
    for (auto &c : comp)
      if (!rc && fwrite(c.data(), 1, c.size(), f) != c.size()) rc = 2;
    data.erase(0, (size_t)std::min<int64_t>((int64_t)data.size(), nb * kBlk));
  };
  const int64_t chunk = std::max<int64_t>(1 << 16, (int64_t)T * 8192);
  std::vector<std::string> parts((size_t)T);
  for (int64_t c0 = 0; c0 < N && !rc; c0 += chunk) {
    const int64_t c1 = std::min(N, c0 + chunk);
    parallel_for(c1 - c0, [&](int t, int64_t a, int64_t e) {
      parts[(size_t)t].clear();
      bam_records(o, c0 + a, c0 + e, crb, n_local, ref_id, name_base, parts[(size_t)t]);
    });
    for (auto &x : parts) {
      data += x;
      x.clear();
    }
    flush(false);
  }
  flush(true);
  if (!rc && (flags & 2)) {
    std::string eof;
    bgzf_block(nullptr, 0, level, eof);
    if (fwrite(eof.data(), 1, eof.size(), f) != eof.size()) rc = 2;
  }
  if (fclose(f) != 0 && !rc) rc = 2;
  return rc;
}

// The one-contig form (contig id 0, the whole file): the input of the ingest measurements.
int gq_synth_write_bam(const gq_synth_out *o, const char *path, const char *contig, int64_t contig_len,
                       int32_t level) {
  const int64_t crb[2] = {0, o->n_reads};
  const int32_t id = 0;
  return gq_synth_write_bam_ex(o, path, 1, &contig, &contig_len, 1, crb, &id, level, 3, 0);
}

}  // extern "C"
