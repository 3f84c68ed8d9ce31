// gq_somatic.hip — somatic-standard on MI355X (gfx950).
//
// Restates, per locus, SomaticStandard.Caller.findPotentialVariantAtLocus and the driver's
// filter chain (paths relative to /root/reference/src/main/scala/org/hammerlab/guacamole/):
//   commands/SomaticStandardCaller.scala:162-245 (caller), :124-151 (driver filters)
//   filters/PileupFilter.scala:29-89, filters/PileupElementsFilter.scala:25-36
//   likelihood/Likelihood.scala:48-201, variants/AlleleEvidence.scala:41-102
//   filters/SomaticGenotypeFilter.scala:58-307, variants/CalledSomaticAllele.scala:37-51
//   DistributedUtil.pileupFlatMapTwoRDDs (DistributedUtil.scala:316-335, skipEmpty = true)
//
// Two kernels:
//   somatic_tile<T>   one workgroup per tile of T loci: LDS histogram of the tumor reads
//                     (the germline sink) -> per-locus "tumor has a non-Match element / the
//                     MD reference is ambiguous" bit kept in registers; LDS re-zeroed, the
//                     normal reads histogrammed -> normal depth.  Loci visited by either
//                     sample are counted; loci with a tumor non-Match and normal depth > 0
//                     are queued (a superset of the loci the caller can emit at: filters
//                     only remove elements).
//                     A queued locus whose tumor pileup provably has the hom-ref genotype as
//                     its maximum-likelihood genotype is dropped (hom_ref_margin below): the
//                     caller returns nothing there whatever the odds and filters.
//   somatic_call      one wave per queued locus: exact elements of both pileups
//                     (classify), per-sample distinct-allele table in registers with the
//                     FP64 per-allele sums of log(2pc), log(pc + (1 - pc)), log(2(1 - pc)),
//                     genotype likelihoods for every (a_i, a_j), normalisation, the odds
//                     test, allele evidence (mean / median via LDS), filters, record.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gq_alleles.h"
#include <hipcub/hipcub.hpp>

#include "gq_host.h"
#include "gq_strictmath.h"
#include "gq_scala_order.h"

// The caller's FP64 arithmetic must round like the reference's: no fused multiply-add
// anywhere in this file (e.g. (agg + 0) - ln2 * depth would otherwise contract).
#pragma clang fp contract(off)

using namespace gq;

namespace {

#include "gq_winorder.h"

constexpr int kSomT = 1024;
constexpr int kEvCap = 1024;  // allele-supporting elements per sample held in LDS for medians

struct SomRec {  // one emitted CalledSomaticAllele
  uint64_t key;  // output ordinal << 12
  int32_t contig, pos;
  uint16_t ref_len, alt_len;
  uint8_t flags, pad[3];
  uint64_t allele;  // inline bytes (ref then alt) if ref_len + alt_len <= 8, else pool offset
  double log_odds;
  int32_t gq, pad2;
  gq_evidence tumor, normal;
};

// ------------------------------------------------------------------------------------------
// Hom-ref bound (the tumor side of findPotentialVariantAtLocus, SomaticStandardCaller.scala:
// 196-206).  The caller computes, over the filtered tumor pileup, genotype likelihoods
//   L(a1, a2) = sum_e log(P(e, a1) + P(e, a2)) (- D ln 2, common),  P(e, a) = pc_e if the
//   element's allele is a else 1 - pc_e,  pc_e = phredSuccess(base quality) * phredSuccess(mapq)
// (Likelihood.scala:149-201, IncludingAlignment) and emits nothing unless the maximum-likelihood
// genotype holds a variant allele.  At a locus whose elements are all single-base Match /
// Mismatch elements against one reference base r:
//   L(r, r)  = sum_match log(2 pc) + sum_mismatch log(2 (1 - pc))
//   L(g)    <= ln2 * n_mismatch + sum_match max(0, log(2 (1 - pc)))  for every other genotype g
// (each term is at most log 2; a Match element adds log 1 = 0 to (r, v) and log(2 (1 - pc)) to
// (v, w)).  So margin = sum_match [log(2 pc) - max(0, log(2 (1 - pc)))] + sum_mismatch
// [log(2 (1 - pc)) - ln 2] > 0 proves (r, r) is the unique maximum: no call at any odds.  The
// sum runs in FP32 (error far below the eps the test applies) over the reads the mapq filter
// keeps (QualityAlignedReadsFilter, PileupElementsFilter.scala:25-36).
__device__ __forceinline__ void hom_ref_margin_lane(const DevReads &R, int64_t r, int32_t L0, int32_t L1,
                                                    int min_mapq, const float *eq, const float *lsq, float *marg) {
  const int32_t s = R.start[r], e = R.end[r];
  if (e <= L0 || s >= L1) return;
  const int mq = (int)R.mapq[r];
  if (min_mapq > 0 && mq < min_mapq) return;
  const int32_t nmd = R.n_md[r];
  if (nmd < 0) return;  // GQ_E_NO_MD is raised by the histogram pass
  const float em = exp2f(-0.33219281f * (float)mq);  // 10^(-mapq/10)
  // log phredSuccess(mapq) = log(1 - em), -inf at mapq 0: taken from log1p, not from 1 - f below
  // (1 - f cancels catastrophically when pc -> 0 and would turn log(2 pc) = -inf into a finite
  // value, proving hom-ref where a mapq-0 Match read makes L(ref, ref) = -inf)
  const float lsm = log1pf(-em);
  const int64_t so = R.seq_off[r];
  const uint32_t *ev = R.md_ev + R.md_off[r];
  int k = 0;  // MD event cursor (events sorted by offset; runs visited in reference order)
  int32_t ev_off = nmd > 0 ? (int32_t)(ev[0] >> 8) : 0x7FFFFFFF;
  uint32_t ev_b = nmd > 0 ? (ev[0] & 0xFFu) : 0u;
  constexpr float kLn2 = 0.69314718f;
  // bases and qualities share offsets: both come in aligned 16-byte chunks (the pools are
  // device allocations, so the aligned chunk around a read's first / last byte is readable)
  auto run = [&](int32_t ra, int32_t rp0, int32_t len) {
    const int32_t a = ra > L0 ? ra : L0, b = (ra + len) < L1 ? (ra + len) : L1;
    for (int32_t l = a; l < b;) {
      const int64_t gp = so + rp0 + (l - ra);
      const int sh = (int)(gp & 15);
      uint4 ws, wq;
      if (gp - sh + 16 <= R.seq_cap) {  // uploaded pools carry a zeroed tail (seq and qual)
        ws = *reinterpret_cast<const uint4 *>(R.seq + (gp - sh));
        wq = *reinterpret_cast<const uint4 *>(R.qual + (gp - sh));
      } else {  // the end of a wrapped (caller-allocated) pool: byte loads only inside it
        uint32_t s4[4] = {0, 0, 0, 0}, q4[4] = {0, 0, 0, 0};
        for (int k = 0; k < 16 && gp - sh + k < R.seq_bytes; ++k) {
          s4[k >> 2] |= (uint32_t)R.seq[gp - sh + k] << (8 * (k & 3));
          q4[k >> 2] |= (uint32_t)R.qual[gp - sh + k] << (8 * (k & 3));
        }
        ws = make_uint4(s4[0], s4[1], s4[2], s4[3]);
        wq = make_uint4(q4[0], q4[1], q4[2], q4[3]);
      }
      const int nb = min(16 - sh, b - l);
      for (int j = 0; j < nb; ++j) {
        const int bi = sh + j, wi = bi >> 2, bs = 8 * (bi & 3);
        const uint32_t w_s = wi == 0 ? ws.x : wi == 1 ? ws.y : wi == 2 ? ws.z : ws.w;
        const uint32_t w_q = wi == 0 ? wq.x : wi == 1 ? wq.y : wi == 2 ? wq.z : wq.w;
        const uint32_t base = (w_s >> bs) & 0xFFu;
        const int q = (int)(int8_t)(uint8_t)(w_q >> bs);
        const int32_t off = l + j - s;
        while (ev_off < off) {
          ++k;
          ev_off = k < nmd ? (int32_t)(ev[k] >> 8) : 0x7FFFFFFF;
          ev_b = k < nmd ? (ev[k] & 0xFFu) : 0u;
        }
        const uint32_t m = ev_off == off ? ev_b : base;
        float t;
        if (q < 0) {
          t = -1e30f;  // outside the table: the exact kernel decides
        } else {
          const float eb = eq[q];
          const float f = eb + em - eb * em;  // 1 - pc
          if (base == m) t = kLn2 + lsq[q] + lsm - fmaxf(0.0f, kLn2 + __logf(f));
          else t = __logf(f);  // log(2 (1 - pc)) - ln 2
        }
        atomicAdd(&marg[l + j - L0], t);
      }
      l += nb;
    }
  };
  const int32_t lead = R.lead[r];
  if (lead >= 0) {
    run(s, lead, e - s);
    return;
  }
  const uint32_t *cg = R.cigar + R.cigar_off[r];
  const int32_t nc = R.n_cigar[r];
  int32_t ref = s, rp = 0;
  for (int c = 0; c < nc && ref < L1; ++c) {
    const int op = (int)(cg[c] & 15u);
    const int32_t len = (int32_t)(cg[c] >> 4);
    if (op == OP_M || op == OP_EQ || op == OP_X) {
      run(ref, rp, len);
      ref += len;
      rp += len;
    } else if (op == OP_I || op == OP_S) {
      rp += len;
    } else if (op == OP_D || op == OP_N) {
      ref += len;
    }
  }
}

#include "gq_somatic_proj.h"
#include "gq_direct_common.h"
#include "gq_somatic_direct.h"

// ------------------------------------------------------------------------------------------
// somatic_tile: candidate loci (the tiles somatic_proj cannot take)
// ------------------------------------------------------------------------------------------
template <int T>
// four waves per SIMD (<= 128 VGPRs).  The tiles somatic_proj hands over (list), a block per
// tile at a time; candidates go to the block's output partition (kPartsCols + block).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void somatic_tile(const Tile *__restrict__ tiles_t,
                                                       const Tile *__restrict__ tiles_n, DevReads RT, DevReads RN,
                                                       ComplexItem *__restrict__ cand, OutGeom og,
                                                       const int32_t *__restrict__ list, int min_mapq, Counters *ctr,
                                                       RefView ref, int no_bound = 0) {
  constexpr int S = T + 2 * kGuard;
  constexpr int KPT = T / kBlock;  // loci per thread
  static_assert(KPT <= 8, "per-thread flag bits");
  __shared__ __attribute__((aligned(16))) uint32_t cnt[W_N * S];
  __shared__ float marg[T];  // hom-ref margin of the tumor pileup
  __shared__ float eq[128];   // 10^(-q/10)
  __shared__ float lsq[128];  // log(1 - 10^(-q/10)) = log phredSuccess(q), -inf at q = 0
  const int part = kPartsCols + (int)(blockIdx.x & (kPartsWalk - 1));
  const unsigned long long pbase = og.slot(1, part, 0), pcap = og.capB[1];
  if (threadIdx.x < 128) {
    eq[threadIdx.x] = exp2f(-0.33219281f * (float)threadIdx.x);
    lsq[threadIdx.x] = log1pf(-eq[threadIdx.x]);
  }
  const int64_t n_list = (int64_t)ctr->n_slow;
  unsigned visited = 0;
  for (int64_t li = blockIdx.x; li < n_list; li += gridDim.x) {
  const int32_t tile = list[li];
  const Tile tt = tiles_t[tile], tn = tiles_n[tile];
  const int32_t L0 = tt.L0, L1 = tt.L1;
  const int nloci = L1 - L0;
  const bool wide = (tt.re - tt.rb) >= 65535 || (tn.re - tn.rb) >= 65535;
  if (wide) {  // 16-bit counters could overflow: every locus goes to the exact kernel
    for (int k = 0; k < KPT; ++k) {
      const int i = threadIdx.x + k * kBlock;
      const unsigned long long b = wave_reserve(&ctr->part[1][part], i < nloci ? 1u : 0u);
      if (i < nloci && b < pcap) cand[pbase + b] = ComplexItem{tile, L0 + i, 1};
    }
    continue;
  }
  uint4 *c4 = reinterpret_cast<uint4 *>(cnt);
  __syncthreads();  // the previous tile's readers are done
  for (int i = threadIdx.x; i < W_N * S / 4; i += blockDim.x) c4[i] = make_uint4(0u, 0u, 0u, 0u);
  for (int i = threadIdx.x; i < T; i += blockDim.x) marg[i] = 0.0f;
  __syncthreads();
  {
    GermSink<T, 0> sink{cnt, L0, &ctr->err, &ctr->err_pos};
    for (int64_t r = tt.rb + threadIdx.x; r < tt.re; r += blockDim.x) {
      walk_read_lane(RT, r, L0, L1, sink);
      hom_ref_margin_lane(RT, r, L0, L1, min_mapq, eq, lsq, marg);
    }
  }
  __syncthreads();
  uint32_t tflag = 0;  // bit k: tumor depth > 0 at locus tid + k * kBlock; bit 8 + k: tumor candidate
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int i = threadIdx.x + k * kBlock;
    if (i >= nloci) continue;
    const uint32_t wac = cnt[W_AC * S + kGuard + i], wtg = cnt[W_TG * S + kGuard + i],
                   wox = cnt[W_OX * S + kGuard + i], wnn = cnt[W_NN * S + kGuard + i];
    const uint32_t cA = wac & 0xFFFFu, cC = wac >> 16, cT = wtg & 0xFFFFu, cG = wtg >> 16, cN = wnn >> 16;
    const uint32_t cx = (wox & 0xFFFFu) + (wox >> 16);
    const uint32_t depth = cA + cC + cT + cG + cN + cx;
    if (depth == 0) continue;
    tflag |= 1u << k;
    uint32_t mask = cnt[W_MASK * S + kGuard + i] & 0xFu;
    const uint32_t eac = cnt[W_EAC * S + kGuard + i], etg = cnt[W_ETG * S + kGuard + i];
    if (cA > (eac & 0xFFFFu)) mask |= 1u;
    if (cC > (eac >> 16)) mask |= 2u;
    if (cT > (etg & 0xFFFFu)) mask |= 4u;
    if (cG > (etg >> 16)) mask |= 8u;
    const int rc = mask ? (__ffs((int)mask) - 1) : 4;
    const uint32_t c_ref = rc == 0 ? cA : rc == 1 ? cC : rc == 2 ? cT : rc == 3 ? cG : cN;
    const bool agree = !ref.b || ref_agrees(mask, ref.b[ref.off[tt.contig] + L0 + i]);
    if (!agree || __popc(mask) > 1 || cx > 0 || depth > c_ref) {
      // single-base elements only, one standard reference base, no N: the hom-ref bound applies
      const bool bound = !no_bound && agree && __popc(mask) == 1 && cx == 0 && cN == 0 && marg[i] > 0.02f + 2e-4f * (float)depth;
      if (!bound) tflag |= 1u << (8 + k);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < W_N * S / 4; i += blockDim.x) c4[i] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
  {
    GermSink<T, 0> sink{cnt, L0, &ctr->err, &ctr->err_pos};
    for (int64_t r = tn.rb + threadIdx.x; r < tn.re; r += blockDim.x) walk_read_lane(RN, r, L0, L1, sink);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int i = threadIdx.x + k * kBlock;
    bool q = false;
    if (i < nloci) {
      uint32_t dn = 0;
#pragma unroll
      for (int w = W_AC; w < W_NN; ++w) {
        const uint32_t v = cnt[w * S + kGuard + i];
        dn += (v & 0xFFFFu) + (v >> 16);
      }
      dn += cnt[W_NN * S + kGuard + i] >> 16;  // low bits of W_NN hold the reference mask
      if (((tflag >> k) & 1u) || dn > 0) ++visited;
      q = ((tflag >> (8 + k)) & 1u) && dn > 0;
    }
    const unsigned long long b = wave_reserve(&ctr->part[1][part], q ? 1u : 0u);
    if (q && b < pcap) cand[pbase + b] = ComplexItem{tile, L0 + i, 0};
  }
  }
  __shared__ unsigned red;
  if (threadIdx.x == 0) red = 0;
  __syncthreads();
  if (visited) atomicAdd(&red, visited);
  __syncthreads();
  if (threadIdx.x == 0 && red) atomicAdd(&ctr->spread[0][blockIdx.x & (kSpread - 1)], (unsigned long long)red);
}

// ------------------------------------------------------------------------------------------
// somatic_call: exact caller per queued locus (one wave per locus)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}


// ADAM PhredUtils.phredToSuccessProbability, 1 - 10^(-q/10) for q in [0, 255] (restated in
// oracle/oracle.cpp:201-207): a table filled on the host with the host's pow, so the device
// starts from the very bits the reference's arithmetic starts from.
__constant__ double g_succ[256];
__device__ __forceinline__ double phred_success(int q) { return g_succ[q > 255 ? 255 : (q < 0 ? 0 : q)]; }

__device__ int success_to_phred(double p) {  // successProbabilityToPhred: round(-10 log10(1 - p)) (Math.round)
  const double x = -10.0 * sm::log10(1.0 - p);
  if (isnan(x)) return 0;
  const double r = floor(x + 0.5);
  long long l;
  if (r >= 9.2233720368547758e18) l = 0x7FFFFFFFFFFFFFFFll;
  else if (r <= -9.2233720368547758e18) l = (long long)0x8000000000000000ull;
  else l = (long long)r;
  return (int)(int32_t)(uint32_t)(uint64_t)l;
}

// |a - b| within FP rounding noise of the threshold: reported as GQ_FLAG_KNIFE_EDGE (the
// outcome there depends on the exact bits of every term, which this kernel reproduces)
__device__ __forceinline__ bool near_edge(double a, double b) { return fabs(a - b) <= 1e-9 * fmax(1.0, fabs(b)); }
// successProbabilityToPhred(p) rounds -10 log10(1 - p); flag values within 1e-6 of a .5 step
__device__ __forceinline__ bool phred_rounding_edge(double p) {
  const double x = -10.0 * sm::log10(1.0 - p);
  if (!isfinite(x)) return false;
  return fabs((x - floor(x)) - 0.5) <= 1e-6;
}

// Element quality (PileupElement.qualityScore, PileupElement.scala:166-171; quality bytes are
// signed JVM bytes): SNV / Deletion = the base quality at the element's read position,
// Insertion = min over its bases, MidDeletion / Clipped = the read's mapping quality.
// (so, mapq: the read's seq_off and mapq, loaded by the caller beside its classify)
__device__ __forceinline__ int elem_quality(const DevReads &R, const AlleleDesc &d, int64_t so, int mapq) {
  const uint8_t *q = R.qual + so;
  switch (d.kind) {
    case K_SNV:
    case K_DEL: return (int)(int8_t)q[d.rp];
    case K_INS: {
      int m = 1 << 30;
      for (int i = 0; i < d.aux; ++i) m = min(m, (int)(int8_t)q[d.rp + i]);
      return m;
    }
    default: return mapq;
  }
}

__device__ __forceinline__ bool allele_is_variant(const DevReads &R, const AlleleDesc &a, int32_t pos) {  // Allele.isVariant
  const int rl = allele_ref_len(a), al = allele_alt_len(a);
  if (rl != al) return true;
  for (int i = 0; i < rl; ++i)
    if (allele_byte(R, a, pos, 0, i) != allele_byte(R, a, pos, 1, i)) return true;
  return false;
}
__device__ __forceinline__ bool allele_std_alt(const DevReads &R, const AlleleDesc &a, int32_t pos) {  // Likelihood.scala:106
  const int al = allele_alt_len(a);
  for (int i = 0; i < al; ++i)
    if (!std_bit(allele_byte(R, a, pos, 1, i))) return false;
  return true;
}

__device__ void raise_at(Counters *ctr, int code, int64_t where) {
  raise_error(&ctr->err, (int64_t *)&ctr->err_pos, code, where);
}

// The reads of a tile window [rb, re) covering pos, compacted into a per-wave LDS list (tile-
// relative indices) in pileup element order, so the per-read passes below run over ~depth
// lanes rather than every read of the window; deeper than the list: the passes walk the
// window in read order instead (with an initial group there: a capacity error).
constexpr int kCover = 768;
struct Cover {
  const int32_t *lst;
  int64_t rb, n;  // slots
  bool compact;
  bool deep;  // the list cannot hold what the pileup order needs: the deep instantiation's locus
  int sel;  // sample filter (-1: every read)
  // read of slot k and whether it covers pos
  __device__ __forceinline__ int64_t read(const DevReads &R, int64_t k, int32_t pos, bool *act) const {
    if (k >= n) {
      *act = false;
      return rb;
    }
    if (compact) {
      *act = true;
      return rb + lst[k];
    }
    const int64_t r = rb + k;
    *act = R.start[r] <= pos && pos < R.end[r] && (sel < 0 || (int)R.sample[r] == sel);
    return r;
  }
};
// lst holds `cap` reads, tmp 2 th words (the initial group's reorder: at most th reads).
__device__ __forceinline__ Cover make_cover(const DevReads &R, int64_t rb, int64_t re, int32_t pos, int32_t *lst, uint32_t *tmp,
                            int cap, int th, const WinInit &w, const int64_t *__restrict__ init_reads,
                            const int32_t *__restrict__ init_rank, Counters *ctr, int sel = -1) {
  const int lane = threadIdx.x & 63;
  int64_t n = 0;
  // the covering reads lie in [first pmax_end > pos, first start > pos)
  //  (searched together: every read before the first is also before the second)
  int64_t ra, rz;
  wave_first_true2(rb, re, [&](int64_t r) { return R.pmax_end[r] > pos; }, [&](int64_t r) { return R.start[r] > pos; },
                   ra, rz);
  for (int64_t r0 = ra; r0 < rz; r0 += 64) {
    const int64_t r = r0 + lane;
    const bool c = r < rz && R.start[r] <= pos && pos < R.end[r] && (sel < 0 || (int)R.sample[r] == sel);
    const unsigned long long b = __ballot(c);
    const int64_t at = n + (int64_t)__popcll(b & ((1ull << lane) - 1ull));
    if (c && at < cap) lst[at] = (int32_t)(r - rb);
    n += (int64_t)__popcll(b);
  }
  __builtin_amdgcn_wave_barrier();
  Cover cv;
  cv.lst = lst;
  cv.rb = rb;
  cv.compact = n <= cap;
  cv.n = cv.compact ? n : (re - rb);
  cv.sel = sel;
  cv.deep = false;
  if (w.n > 0 && pos < w.E) {
    if (!cv.compact) {  // the initial group's heap order needs the list
      cv.deep = true;
      return cv;
    }
    // the initial group's reads covering pos are a prefix of the list (they start at or
    // before F, every other covering read after F): reorder that prefix by heap rank
    int p = 0;
    for (int k0 = 0; k0 < (int)n; k0 += 64) {
      const int k = k0 + lane;
      p += (int)__popcll(__ballot(k < (int)n && R.start[rb + lst[k]] <= w.F));
    }
    if (p > th) {
      cv.deep = true;
      return cv;
    }
    for (int k = lane; k < p; k += 64) {
      const int64_t r = rb + lst[k];
      int lo = 0, hi = w.n;  // r in the group's ascending read list
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (init_reads[w.off + m] < r) lo = m + 1;
        else hi = m;
      }
      tmp[k] = (uint32_t)init_rank[w.off + lo];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int k = lane; k < p; k += 64) {
      int before = 0;
      for (int j = 0; j < p; ++j) before += tmp[j] < tmp[k] ? 1 : 0;
      tmp[th + before] = (uint32_t)lst[k];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int k = lane; k < p; k += 64) lst[k] = (int32_t)tmp[th + k];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  return cv;
}

// Pileup.referenceBaseAtLocus over the covering reads: the standard MD-derived bases present
// (ambiguous = more than one); the base itself when they agree.  Where they disagree the
// reference takes the first in heap order: the first pass lists the locus and the second
// receives the base from heap_ref_bases (ref_override >= 0).
__device__ __forceinline__ void pileup_ref(const DevReads &R, const Cover &cv, int32_t pos, Counters *ctr, int ref_override,
                           uint8_t &refbase, bool &ambiguous) {
  const int lane = threadIdx.x & 63;
  uint32_t mask = 0;
  for (int64_t k0 = 0; k0 < cv.n; k0 += 64) {
    bool cov;
    const int64_t r = cv.read(R, k0 + lane, pos, &cov);
    if (cov) {
      const int v = md_ref_at(R, r, pos);
      if (v < 0) raise_at(ctr, v == -4 ? GQ_E_NO_MD : v == -3 ? GQ_E_MD : GQ_E_ASSERT, pos);
      else mask |= std_bit((uint8_t)v);
    }
  }
  for (int d = 1; d < 64; d <<= 1) mask |= __shfl_xor(mask, d, 64);
  ambiguous = __popc(mask) > 1;
  refbase = 'N';
  if (ref_override >= 0) refbase = (uint8_t)ref_override;
  else if (mask) refbase = bit_base(mask);
}

// Per-sample pileup summary held by one wave: a distinct-allele table (slot s * 64 + lane
// lives in lane `lane`, register slot s) with per-allele element counts; 64 NS entries.
template <int NS>
struct SamplePile {
  uint64_t klo[NS], khi[NS];
  AlleleDesc desc[NS];
  uint32_t n_all[NS], n_f[NS];
  int nt;             // used table entries (wave-uniform)
  uint32_t depth_all; // elements
  uint32_t depth_f;   // elements passing the mapping-quality filter
  uint32_t fwd_f;     // ... on the positive strand
  uint8_t refbase;
  bool ambiguous, overflow;
};

// Build the allele table of one sample's pileup at pos (counts only: order-free).
template <int NS>
__device__ __forceinline__ void gather_sample(const DevReads &R, const Cover &cv, int32_t pos, int min_mapq, int ref_override,
                              Counters *ctr, SamplePile<NS> &P) {
  const int lane = threadIdx.x & 63;
  pileup_ref(R, cv, pos, ctr, ref_override, P.refbase, P.ambiguous);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    P.klo[s] = P.khi[s] = 0;
    P.n_all[s] = P.n_f[s] = 0;
  }
  P.nt = 0;
  P.depth_all = P.depth_f = P.fwd_f = 0;
  P.overflow = false;
  for (int64_t k0 = 0; k0 < cv.n; k0 += 64) {
    bool act;
    const int64_t r = cv.read(R, k0 + lane, pos, &act);
    AlleleDesc d;
    Key128 key{0, 0};
    bool pass = false;
    const int mq = act ? (int)R.mapq[r] : 0;  // issued with classify's loads
    const bool fwd = act && !(R.flags[r] & 1);
    if (act) {
      int errc = 0;
      if (!classify(R, r, pos, P.refbase, d, &errc)) {
        raise_at(ctr, errc, pos);
        act = false;
      } else {
        key = allele_key(R, d, pos, 0);
        pass = min_mapq <= 0 || mq >= min_mapq;  // QualityAlignedReadsFilter (PileupElementsFilter.scala:25-36)
      }
    }
    const unsigned long long actb = __ballot(act), passb = __ballot(act && pass);
    P.depth_all += (uint32_t)__popcll(actb);
    P.depth_f += (uint32_t)__popcll(passb);
    P.fwd_f += (uint32_t)__popcll(__ballot(act && pass && fwd));
    unsigned long long pending = actb;
    while (pending) {
      const int leader = __ffsll((long long)pending) - 1;
      const uint64_t klo = __shfl(key.lo, leader, 64), khi = __shfl(key.hi, leader, 64);
      const bool match = act && key.lo == klo && key.hi == khi;
      const unsigned long long mb = __ballot(match);
      const uint32_t na = (uint32_t)__popcll(mb), nf = (uint32_t)__popcll(mb & passb);
      int found = -1;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bool hit = (s * 64 + lane) < P.nt && P.klo[s] == klo && P.khi[s] == khi;
        const unsigned long long hb = __ballot(hit);
        if (found < 0 && hb) found = s * 64 + (__ffsll((long long)hb) - 1);
      }
      if (found < 0) {
        if (P.nt >= 64 * NS) {
          P.overflow = true;
        } else {
          found = P.nt++;
          const int owner = found & 63, sl = found >> 6;
          AlleleDesc ld;
          ld.read = __shfl(d.read, leader, 64);
          ld.aux = __shfl(d.aux, leader, 64);
          ld.rp = __shfl(d.rp, leader, 64);
          ld.kind = (uint8_t)__shfl((int)d.kind, leader, 64);
          ld.rb = (uint8_t)__shfl((int)d.rb, leader, 64);
          ld.base = (uint8_t)__shfl((int)d.base, leader, 64);
          ld.pad = 0;
#pragma unroll
          for (int s = 0; s < NS; ++s)
            if (s == sl && lane == owner) {
              P.klo[s] = klo;
              P.khi[s] = khi;
              P.desc[s] = ld;
            }
        }
      }
      if (found >= 0) {
        const int owner = found & 63, sl = found >> 6;
#pragma unroll
        for (int s = 0; s < NS; ++s)
          if (s == sl && lane == owner) {
            P.n_all[s] += na;
            P.n_f[s] += nf;
          }
      }
      pending &= ~mb;
    }
  }
}

template <int NS>
__device__ __forceinline__ AlleleDesc pile_desc(const SamplePile<NS> &P, int j) {
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

// Genotype likelihoods of one sample (Likelihood.likelihoodsOfAllPossibleGenotypesFromPileup,
// normalised, not log space).  Eligible alleles (filtered count > 0, standard alt bases) are
// ranked by Allele order into `order[0..n)` (LDS, per wave); genotype g <-> (i <= j) in the
// reference's enumeration order.
struct GenoResult {
  int n;          // eligible alleles
  int G;          // genotypes
  bool deep;      // more genotypes than ll holds: the deep instantiation's locus
  int best_g;     // maxBy (first maximum)
  double best_l;  // its normalised likelihood
  double var_sum; // sum of normalised likelihoods of genotypes with a variant allele
  int bi, bj;     // table entries of the best genotype's alleles
};

__device__ __forceinline__ void genotype_index(int g, int n, int &i, int &j) {  // g -> (i, j), i <= j, row-major
  int row = 0, rem = g;
  while (rem >= n - row) {
    rem -= n - row;
    ++row;
  }
  i = row;
  j = row + rem;
}

constexpr int kMaxG = 128;  // genotypes held per sample for the normalisation (15 eligible alleles)

// sum_e log(P(e, a1) + P(e, a2)) over the mapq-filtered elements of the pileup for the
// genotype (k1, k2) of each lane, P(e, a) = pc_e if e's allele is a else 1 - pc_e
// (Likelihood.scala:166-188).  The reference fills a Colt matrix and folds each genotype's row
// with DoubleMatrix1D.aggregate(plus, chain(log, plus)), which starts from the LAST element and
// adds the earlier ones in turn; the fold below runs in exactly that order over the elements
// in pileup order, with java.lang.StrictMath's log, so every genotype gets the reference's
// bits.  Lanes = elements compute the three possible terms log(pc + pc), log(pc + (1 - pc)),
// log((1 - pc) + (1 - pc)); then the wave walks the elements backwards, each lane (genotype)
// adding the term its alleles select.
__device__ __forceinline__ double fold_genotypes(const DevReads &R, const Cover &cv, int32_t pos, uint8_t refbase, int min_mapq,
                                 bool include_alignment, Key128 k1, Key128 k2, Counters *ctr) {
  const int lane = threadIdx.x & 63;
  double agg = 0.0;
  bool started = false;
  if (cv.n == 0) return agg;
  for (int64_t c0 = ((cv.n - 1) / 64) * 64; c0 >= 0; c0 -= 64) {
    bool act;
    const int64_t r = cv.read(R, c0 + lane, pos, &act);
    Key128 key{0, 0};
    double t2 = 0.0, th = 0.0, t0 = 0.0;
    bool pass = false;
    if (act) {
      AlleleDesc d;
      int errc = 0;
      const int mq = (int)R.mapq[r];  // issued with classify's loads
      const int64_t so = R.seq_off[r];
      if (classify(R, r, pos, refbase, d, &errc)) {
        pass = min_mapq <= 0 || mq >= min_mapq;
        if (pass) {
          key = allele_key(R, d, pos, 0);
          const int q = elem_quality(R, d, so, mq);
          if (q < 0) raise_at(ctr, GQ_E_ASSERT, pos);  // PhredUtils: negative phred
          double pc = phred_success(q);
          if (include_alignment) pc = pc * phred_success(mq);  // probabilityCorrectIncludingAlignment
          const double pw = 1.0 - pc;
          t2 = sm::log(pc + pc);
          th = sm::log(pc + pw);
          t0 = sm::log(pw + pw);
        }
      }
    }
    unsigned long long pb = __ballot(act && pass);
    while (pb) {
      const int j = 63 - __clzll((long long)pb);  // the chunk's last element first
      pb &= ~(1ull << j);
      const uint64_t klo = lane_u64(key.lo, j), khi = lane_u64(key.hi, j);
      const double a2 = lane_f64(t2, j), ah = lane_f64(th, j), a0 = lane_f64(t0, j);
      const bool m1 = k1.lo == klo && k1.hi == khi, m2 = k2.lo == klo && k2.hi == khi;
      const double term = (m1 && m2) ? a2 : (m1 || m2) ? ah : a0;
      agg = started ? agg + term : term;
      started = true;
    }
  }
  return agg;
}

template <int NS>
__device__ __forceinline__ GenoResult genotypes(const DevReads &R, const SamplePile<NS> &P, const Cover &cv, int32_t pos,
                                int min_mapq, bool include_alignment, int16_t *order, uint8_t *is_var,
                                double *ll_lds, int maxG, Counters *ctr, bool by_log = false) {
  const int lane = threadIdx.x & 63;
  GenoResult res{};
  // eligibility + variant flag per entry (entry j on lane j & 63, slot j >> 6)
  bool elig[NS], var[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int j = s * 64 + lane;
    elig[s] = j < P.nt && P.n_f[s] > 0 && allele_std_alt(R, P.desc[s], pos);
    var[s] = j < P.nt && allele_is_variant(R, P.desc[s], pos);
  }
  // rank of each eligible entry among eligible entries by Allele order
  int n = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) n += __popcll(__ballot(elig[s]));
  res.n = n;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int rank = 0;
    for (int k = 0; k < P.nt; ++k) {
      const AlleleDesc dk = pile_desc(P, k);
      bool ek = false;
      _Pragma("unroll") for (int t = 0; t < NS; ++t) if (t == (k >> 6)) ek = __shfl((int)elig[t], k & 63, 64);
      if (elig[s] && ek && k != s * 64 + lane && allele_cmp(R, dk, P.desc[s], pos) < 0) ++rank;
    }
    if (elig[s]) order[rank] = (int16_t)(s * 64 + lane);
    if (s * 64 + lane < 64 * NS) is_var[s * 64 + lane] = var[s] ? 1 : 0;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const int G = n * (n + 1) / 2;
  res.G = G;
  if (G == 0) return res;
  if (G > maxG) {
    res.deep = true;
    res.G = 0;
    return res;
  }
  // log-likelihood per genotype: the Colt fold, + log(prior = 1) - ln 2 * depth (Likelihood.scala:189)
  const double ln2d = sm::log(2.0) * (double)P.depth_f;
  for (int g0 = 0; g0 < G; g0 += 64) {
    const int g = g0 + lane;
    int i = 0, j = 0;
    if (g < G) genotype_index(g, n, i, j);
    const int ei = g < G ? order[i] : 0, ej = g < G ? order[j] : 0;
    // the table keys live on their owner lanes (entry e: lane e & 63, slot e >> 6)
    Key128 k1{~0ull, ~0ull}, k2{~0ull, ~0ull};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint64_t lo1 = __shfl(P.klo[s], ei & 63, 64), hi1 = __shfl(P.khi[s], ei & 63, 64);
      const uint64_t lo2 = __shfl(P.klo[s], ej & 63, 64), hi2 = __shfl(P.khi[s], ej & 63, 64);
      if (g < G && s == (ei >> 6)) k1 = Key128{lo1, hi1};
      if (g < G && s == (ej >> 6)) k2 = Key128{lo2, hi2};
    }
    const double agg = fold_genotypes(R, cv, pos, P.refbase, min_mapq, include_alignment, k1, k2, ctr);
    if (g < G) ll_lds[g] = agg + sm::log(1.0) - ln2d;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // normalisation in the reference's order (Likelihood.scala:190-199): total = the exp(ll)
  // added genotype by genotype, then exp(ll - log(total)); maxBy keeps the first maximum, the
  // normal's variant mass adds the variant genotypes in turn (SomaticStandardCaller.scala:206-217)
  double tot = 0.0;
  for (int g0 = 0; g0 < G; g0 += 64) {
    const double e = (g0 + lane < G) ? sm::exp(ll_lds[g0 + lane]) : 0.0;
    for (int j = 0; j < 64 && g0 + j < G; ++j) tot = tot + lane_f64(e, j);
  }
  const double lt = sm::log(tot);
  // by_log: the first maximum of the normalized log-likelihoods (logSpace = true,
  // GermlineStandardCaller.scala:105-111), its exp as the likelihood
  double best = 0.0, bestx = 0.0, vsum = 0.0;
  int bestg = -1;
  for (int g0 = 0; g0 < G; g0 += 64) {
    const int g = g0 + lane;
    double L = 0.0, X = 0.0;
    bool v = false;
    if (g < G) {
      X = ll_lds[g] - lt;
      L = sm::exp(X);
      int i, j;
      genotype_index(g, n, i, j);
      v = is_var[order[i]] || is_var[order[j]];
    }
    const unsigned long long vb = __ballot(v);
    for (int j = 0; j < 64 && g0 + j < G; ++j) {
      const double Lj = lane_f64(L, j);
      const double Xj = by_log ? lane_f64(X, j) : 0.0;
      if (bestg < 0 || (by_log ? Xj > bestx : Lj > best)) {
        best = Lj;
        bestx = Xj;
        bestg = g0 + j;
      }
      if ((vb >> j) & 1ull) vsum = vsum + Lj;
    }
  }
  res.best_g = bestg;
  res.best_l = best;
  res.var_sum = vsum;
  int i, j;
  genotype_index(bestg, n, i, j);
  res.bi = order[i];
  res.bj = order[j];
  return res;
}

// AlleleEvidence.apply (AlleleEvidence.scala:58-101) for the elements of one sample whose
// allele key is `target`.  Supporting elements' (mapq, quality, mismatches) go to `ev_lds`
// in element order for the running mean (Breeze, in element order) and the medians.
// Returns false when more elements support the allele than ev_lds holds (evcap): the deep
// instantiation's locus.
template <int NS>
__device__ __forceinline__ bool allele_evidence(const DevReads &R, const Cover &cv, int32_t pos, int min_mapq, const SamplePile<NS> &P,
                                Key128 target, double likelihood, uint32_t *ev_lds, uint32_t evcap, Counters *ctr,
                                gq_evidence &ev) {
  const int lane = threadIdx.x & 63;
  uint32_t n = 0, fwd = 0;
  for (int64_t k0 = 0; k0 < cv.n; k0 += 64) {
    bool cov;
    const int64_t r = cv.read(R, k0 + lane, pos, &cov);
    bool hit = false;
    uint32_t packed = 0;
    if (cov) {
      const int mq = (int)R.mapq[r];
      const int64_t so = R.seq_off[r];  // the read's scalars issued with classify's loads
      const int32_t nmd = R.n_md[r];
      const uint32_t nmm = (uint32_t)R.n_mismatch[r];
      if (min_mapq <= 0 || mq >= min_mapq) {
        AlleleDesc d;
        int errc = 0;
        if (classify(R, r, pos, P.refbase, d, &errc)) {
          const Key128 k = allele_key(R, d, pos, 0);
          if (k.lo == target.lo && k.hi == target.hi) {
            hit = true;
            if (nmd < 0) raise_at(ctr, GQ_E_NO_MD, pos);
            packed = (uint32_t)mq | ((uint32_t)(uint8_t)(int8_t)elem_quality(R, d, so, mq) << 8) | (nmm << 16);
          }
        }
      }
    }
    const unsigned long long hb = __ballot(hit);
    const uint32_t before = (uint32_t)__popcll(hb & ((1ull << lane) - 1ull));
    if (hit && n + before < evcap) ev_lds[n + before] = packed;
    fwd += (uint32_t)__popcll(__ballot(hit && !(R.flags[r] & 1)));
    n += (uint32_t)__popcll(hb);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  ev.likelihood = likelihood;
  ev.read_depth = (int32_t)P.depth_f;
  ev.forward_depth = (int32_t)P.fwd_f;
  ev.allele_read_depth = (int32_t)n;
  ev.allele_forward_depth = (int32_t)fwd;
  if (n == 0) {
    ev.mean_mq = ev.median_mq = ev.mean_bq = ev.median_bq = ev.median_mismatches = __builtin_nan("");
    return true;
  }
  if (n > evcap) return false;
  // breeze.stats.mean: running mean in element order
  double mq = 0.0, bq = 0.0;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t v = ev_lds[k];
    mq += ((double)(v & 0xFFu) - mq) / (double)(k + 1);
    bq += ((double)(int8_t)((v >> 8) & 0xFFu) - bq) / (double)(k + 1);
  }
  ev.mean_mq = mq;
  ev.mean_bq = bq;
  // k-th smallest by rank counting (lane-parallel over the elements)
  auto kth = [&](int field, uint32_t k) -> int {
    auto val = [&](uint32_t v) -> int {
      return field == 0 ? (int)(v & 0xFFu) : field == 1 ? (int)(int8_t)((v >> 8) & 0xFFu) : (int)(v >> 16);
    };
    int found = 0x7FFFFFFF;
    for (uint32_t e = lane; e < n; e += 64) {
      const int x = val(ev_lds[e]);
      uint32_t lt = 0, le = 0;
      for (uint32_t f = 0; f < n; ++f) {
        const int y = val(ev_lds[f]);
        lt += y < x;
        le += y <= x;
      }
      if (lt <= k && k < le) found = x;
    }
    for (int d = 1; d < 64; d <<= 1) found = min(found, __shfl_xor(found, d, 64));
    return found;
  };
  if (n & 1) {
    ev.median_mq = (double)kth(0, (n - 1) / 2);
    ev.median_bq = (double)kth(1, (n - 1) / 2);
    ev.median_mismatches = (double)kth(2, (n - 1) / 2);
  } else {
    ev.median_mq = ((double)kth(0, n / 2 - 1) + (double)kth(0, n / 2)) / 2.0;
    ev.median_bq = ((double)kth(1, n / 2 - 1) + (double)kth(1, n / 2)) / 2.0;
    ev.median_mismatches = (double)((kth(2, n / 2 - 1) + kth(2, n / 2)) / 2);  // Int median (parity unpinned)
  }
  return true;
}

constexpr int kSomWaves = kBlock / 64;

#ifndef GQ_CALL_WPE
#define GQ_CALL_WPE 3  // waves per SIMD the register budget must allow
#endif

#include "gq_somatic_call.h"

// ---- germline-standard: GermlineStandard.Caller.callVariantsAtLocus
// (commands/GermlineStandardCaller.scala:90-124) + GenotypeFilter (filters/GenotypeFilter.scala:
// 140-154) at the candidate loci somatic_proj / somatic_tile leave (the reads as both "tumor"
// and "normal"; the hom-ref bound with probabilityCorrectIgnoringAlignment).  One wave per
// locus: the pileup's reference base over every read, then per sample (bySample, in sample
// order) the QualityAlignedReadsFilter pileup's genotype likelihoods in log space, normalized,
// the first maximum, and each non-reference allele of that genotype (twice for a hom-alt) with
// its evidence over the sample's unfiltered pileup.  Records keep the sample in key bits 4-11.
// Capacities of the LDS working set (fast instantiation): covering reads kCover, supporting
// elements kEvCap, genotypes kMaxG, 128 distinct alleles per sample.  A locus past any of them is
// handed whole (from the sample it reached on) to the deep instantiation: per-wave global scratch
// sized from the deepest handed-over pileup and its largest allele table, 1024 alleles per
// sample — the reference (Pileup.scala:37-146, Likelihood.scala:99-113, VariantSupport.scala:
// 110-118) has no depth limit.
struct DeepSel {
  int64_t *out;              // fast: (list position << 3 | sample) of handed-over loci
  unsigned long long cap;    // out's / sel's capacity
  const int64_t *sel;        // deep: the handed-over entries
  int64_t n_sel;
  uint8_t *scratch;          // deep: one slice per wave (gs_wave_bytes)
  int scap, maxG;            // deep: reads per slice list, genotypes
};
constexpr int kDeepNS = 16;  // deep allele tables: 64 x 16 = 1024 distinct alleles per sample
__host__ __device__ __forceinline__ size_t gs_wave_bytes(int scap, int maxG) {
  return (size_t)maxG * 8 + (size_t)scap * 4 * 4 + 64 * kDeepNS * 3 + 64;
}
struct GsMem {
  int32_t *cov_a, *cov_s;
  uint32_t *ev;  // 2 scap words: the heap-order reorder, then the evidence values
  int16_t *order;
  uint8_t *is_var;
  double *ll;
  int cap, th, maxG;
};
__device__ __forceinline__ GsMem gs_deep_mem(uint8_t *base, int scap, int maxG) {
  GsMem m;
  uint8_t *p = base;
  m.ll = (double *)p;
  p += (size_t)maxG * 8;
  m.cov_a = (int32_t *)p;
  p += (size_t)scap * 4;
  m.cov_s = (int32_t *)p;
  p += (size_t)scap * 4;
  m.ev = (uint32_t *)p;
  p += (size_t)scap * 8;
  m.order = (int16_t *)p;
  p += 64 * kDeepNS * 2;
  m.is_var = p;
  m.cap = scap;
  m.th = scap;
  m.maxG = maxG;
  return m;
}

template <bool DEEP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DEEP ? 1 : GQ_CALL_WPE))) void germline_standard_call(
    const Tile *__restrict__ tiles, const ComplexItem *__restrict__ items, DevReads R, gq_germline_std_params prm,
    SomRec *__restrict__ recs, unsigned long long rec_cap, uint8_t *__restrict__ pool, unsigned long long pool_cap,
    OutGeom og, Counters *ctr, SomWin sw, AmbItem *__restrict__ amb_out, unsigned long long amb_cap,
    const AmbItem *__restrict__ amb_in, const uint8_t *__restrict__ amb_ref, int64_t n_amb_in, DeepSel dd) {
  constexpr int NS = DEEP ? kDeepNS : kSlots;
  constexpr int FW = DEEP ? 1 : kSomWaves;
  __shared__ int16_t order_lds[FW][64 * kSlots];
  __shared__ uint8_t var_lds[FW][64 * kSlots];
  __shared__ uint32_t ev_lds[FW][kEvCap];
  __shared__ int32_t cover_a[FW][kCover], cover_s[FW][kCover];
  __shared__ double ll_lds[FW][kMaxG];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t gwave = wave_id();
  const int64_t nwaves_total = ((int64_t)gridDim.x * blockDim.x) >> 6;
  GsMem m;
  if constexpr (DEEP) {
    m = gs_deep_mem(dd.scratch + (size_t)gwave * gs_wave_bytes(dd.scap, dd.maxG), dd.scap, dd.maxG);
  } else {
    m = GsMem{cover_a[wv], cover_s[wv], ev_lds[wv], order_lds[wv], var_lds[wv], ll_lds[wv], kCover, 512, kMaxG};
  }
  const unsigned long long n_items =
      DEEP ? (unsigned long long)dd.n_sel : amb_in ? (unsigned long long)n_amb_in : ctr->part_off[1][kParts];
  for (int64_t si = gwave; si < (int64_t)n_items; si += nwaves_total) {
    const int64_t li = DEEP ? (dd.sel[si] >> 3) : si;
    const int smp0 = DEEP ? (int)(dd.sel[si] & 7) : 0;  // the first sample the fast pass did not finish
    const int64_t it = amb_in ? amb_in[li].item : li;
    const ComplexItem item = items[part_slot_wave(ctr->part_off[1], (unsigned long long)it, og, 1)];
    const Tile tt = tiles[item.tile];
    const int32_t pos = item.pos;
    const int32_t win = sw.range_win[tt.range];
    // a locus (from sample smp on) the working set cannot hold: the deep instantiation's
    auto hand_over = [&](int smp, uint32_t depth, int nt) {
      if constexpr (!DEEP) {
        if (lane == 0) {
          const unsigned long long k = atomicAdd(&ctr->n_deep, 1ull);
          if (k < dd.cap) dd.out[k] = (li << 3) | smp;
          atomicMax(&ctr->deep_max, (unsigned long long)depth);
          atomicMax(&ctr->deep_nt, (unsigned long long)nt);
        }
      } else {
        raise_at(ctr, GQ_E_CAPACITY, pos);
      }
    };
    // the pileup's reference base (Pileup.referenceBaseAtLocus over every read)
    const Cover ca = make_cover(R, tt.rb, tt.re, pos, m.cov_a, m.ev, m.cap, m.th, sw.wi[2 * win], sw.init_reads,
                                sw.init_rank, ctr);
    if (ca.deep) {
      hand_over(0, (uint32_t)(tt.re - tt.rb), 64 * NS);
      continue;
    }
    uint8_t refbase;
    bool ambiguous;
    pileup_ref(R, ca, pos, ctr, amb_in ? (int)amb_ref[li] : -1, refbase, ambiguous);
    if (!amb_in && ambiguous) {  // heap order decides the reference base: list it
      if (lane == 0) {
        const unsigned long long k = atomicAdd(&ctr->n_amb, 1ull);
        if (k < amb_cap) amb_out[k] = AmbItem{item.tile, pos, it};
      }
      continue;
    }
    for (int smp = smp0; smp < R.n_samples; ++smp) {
      const Cover cs = R.n_samples == 1 ? ca
                                        : make_cover(R, tt.rb, tt.re, pos, m.cov_s, m.ev, m.cap, m.th, sw.wi[2 * win],
                                                     sw.init_reads, sw.init_rank, ctr, smp);
      if (cs.deep) {
        hand_over(smp, (uint32_t)(tt.re - tt.rb), 64 * NS);
        break;
      }
      SamplePile<NS> PF;
      gather_sample(R, cs, pos, prm.min_mapq, refbase, ctr, PF);
      if (PF.overflow) {
        hand_over(smp, (uint32_t)cs.n, 64 * kDeepNS);
        break;
      }
      if (PF.depth_f == 0) continue;  // no sample pileup, or nothing left after the mapq filter
      const GenoResult g =
          genotypes(R, PF, cs, pos, prm.min_mapq, false, m.order, m.is_var, m.ll, m.maxG, ctr, true);
      if (g.deep) {
        hand_over(smp, (uint32_t)cs.n, PF.nt);
        break;
      }
      if (g.G == 0) {
        raise_at(ctr, GQ_E_ASSERT, pos);  // empty.maxBy: no allele with standard bases
        continue;
      }
      const AlleleDesc a1 = pile_desc(PF, g.bi), a2 = pile_desc(PF, g.bj);
      const bool v1 = allele_is_variant(R, a1, pos), v2 = allele_is_variant(R, a2, pos);
      if (!v1 && !v2) continue;
      SamplePile<NS> PA;  // the sample's unfiltered pileup: AlleleEvidence's
      gather_sample(R, cs, pos, 0, refbase, ctr, PA);
      // both alleles' evidence first: a sample is handed over whole or not at all
      gq_evidence evs[2];
      bool fits = true;
      for (int sub = 0; sub < 2 && fits; ++sub)
        if (sub == 0 ? v1 : v2)
          fits = allele_evidence(R, cs, pos, 0, PA, allele_key(R, sub == 0 ? a1 : a2, pos, 0), g.best_l, m.ev,
                                 (uint32_t)(DEEP ? 2 * m.cap : kEvCap), ctr, evs[sub]);
      if (!fits || PA.overflow) {
        hand_over(smp, (uint32_t)cs.n, PF.nt);
        break;
      }
      for (int sub = 0; sub < 2; ++sub) {
        if (!(sub == 0 ? v1 : v2)) continue;
        const AlleleDesc al = sub == 0 ? a1 : a2;
        const gq_evidence ev = evs[sub];
        const int gqv = success_to_phred(ev.likelihood - 1e-10);
        if (prm.apply_filters) {
          if (!(ev.read_depth >= prm.min_read_depth && ev.read_depth < prm.max_read_depth)) continue;
          if (prm.min_alternate_read_depth > 0 && !(ev.allele_read_depth >= prm.min_alternate_read_depth)) continue;
          if (prm.min_likelihood > 0 && !(gqv >= prm.min_likelihood)) continue;
        }
        const int rl = allele_ref_len(al), alt_l = allele_alt_len(al);
        SomRec rr;
        rr.key = ((uint64_t)(tt.ordinal0 + (pos - tt.L0)) << 12) | ((uint64_t)smp << 4) | (uint64_t)sub;
        rr.contig = tt.contig;
        rr.pos = pos;
        rr.ref_len = (uint16_t)rl;
        rr.alt_len = (uint16_t)alt_l;
        rr.flags = amb_in ? 1 : 0;
        rr.pad[0] = rr.pad[1] = rr.pad[2] = 0;
        rr.log_odds = 0.0;
        rr.gq = gqv;
        rr.pad2 = 0;
        rr.tumor = ev;
        rr.normal = gq_evidence{};
        if (rl + alt_l <= 8) {
          uint64_t v = 0;
          int j = 0;
          for (int i = 0; i < rl; ++i) v |= (uint64_t)allele_byte(R, al, pos, 0, i) << (8 * j++);
          for (int i = 0; i < alt_l; ++i) v |= (uint64_t)allele_byte(R, al, pos, 1, i) << (8 * j++);
          rr.allele = v;
        } else {
          unsigned long long off = 0;
          if (lane == 0) off = atomicAdd(&ctr->pool_used, (unsigned long long)(rl + alt_l));
          off = __shfl(off, 0, 64);
          if (off + rl + alt_l <= pool_cap)
            for (int i = lane; i < rl + alt_l; i += 64)
              pool[off + i] = i < rl ? allele_byte(R, al, pos, 0, i) : allele_byte(R, al, pos, 1, i - rl);
          rr.allele = off;
        }
        if (lane == 0) {
          const unsigned long long k = atomicAdd(&ctr->n_rec, 1ull);
          if (k < rec_cap) recs[k] = rr;
        }
      }
    }
  }
}

// Exclusive offsets of the candidate partitions (clamped to their capacities), the total in
// n_complex and the largest overflow in part_max[1] (part_scan of gq_pileup.hip, which = 1).
__global__ __launch_bounds__(1024) void part_scan_som(Counters *ctr, OutGeom og) {
  constexpr int PER = kParts / 1024;
  __shared__ unsigned long long s[1024];
  __shared__ unsigned long long mx;
  const int t = threadIdx.x;
  unsigned long long v[PER], sum = 0, m = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const unsigned long long x = ctr->part[1][t * PER + j];
    const unsigned long long cap = og.cap(1, t * PER + j);
    m = x > cap && x - cap > m ? x - cap : m;
    v[j] = x < cap ? x : cap;
    sum += v[j];
  }
  if (t == 0) mx = 0;
  s[t] = sum;
  __syncthreads();
  if (m) atomicMax(&mx, m);
  for (int d = 1; d < 1024; d <<= 1) {
    const unsigned long long y = t >= d ? s[t - d] : 0ull;
    __syncthreads();
    s[t] += y;
    __syncthreads();
  }
  unsigned long long o = s[t] - sum;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    ctr->part_off[1][t * PER + j] = o;
    o += v[j];
  }
  if (t == 1023) {
    ctr->part_off[1][kParts] = s[t];
    ctr->n_complex = s[t];
    ctr->part_max[1] = mx;
  }
}

// ---- variant-support: VariantSupport.pileupToAlleleCounts (commands/VariantSupport.scala:110-118)
struct VsRec {
  uint64_t key;  // locus ordinal (position in the concatenated loci ranges)
  int32_t contig, pos;
  int32_t count;
  uint16_t ref_len, alt_len;
  uint8_t flags, sample, pad[6];
  uint64_t allele;  // ref then alt bytes: inline when they fit 8 bytes, else a pool offset
};
static_assert(sizeof(VsRec) == 40, "VsRec layout");

// One wave per locus of the loci set: the covering reads' pileup (every element, no filter),
// its distinct alleles and their element counts (gather_sample's table).  Loci whose reference
// base depends on heap order are listed first (amb_out) and redone with the replayed base.
// A locus with more distinct alleles than the fast table (128) goes whole to the deep
// instantiation (1024 alleles; the cover list is only a shortcut: past it the reads are walked).
template <bool DEEP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DEEP ? 1 : 2))) void variant_support_call(
    const Tile *__restrict__ tiles, int64_t n_tiles, int64_t n_items, DevReads R, VsRec *__restrict__ recs,
    unsigned long long rec_cap, uint8_t *__restrict__ pool, unsigned long long pool_cap, Counters *ctr,
    AmbItem *__restrict__ amb_out, unsigned long long amb_cap, const AmbItem *__restrict__ amb_in,
    const uint8_t *__restrict__ amb_ref, int64_t n_amb_in, DeepSel dd) {
  constexpr int NS = DEEP ? kDeepNS : kSlots;
  __shared__ int32_t cover[kSomWaves][kCover];
  __shared__ uint32_t tmp[kSomWaves][kEvCap];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t gwave = wave_id();
  const int64_t nwaves_total = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t n = DEEP ? dd.n_sel : amb_in ? n_amb_in : n_items;
  for (int64_t si = gwave; si < n; si += nwaves_total) {
    const int64_t li = DEEP ? dd.sel[si] : si;
    const int64_t k = amb_in ? amb_in[li].item : li;
    int64_t t;
    if (amb_in) {
      t = amb_in[li].tile;
    } else {  // last tile whose first ordinal <= k
      int64_t lo = 0, hi = n_tiles - 1;
      while (lo < hi) {
        const int64_t m = (lo + hi + 1) >> 1;
        if (tiles[m].ordinal0 <= k) lo = m;
        else hi = m - 1;
      }
      t = lo;
    }
    const Tile tt = tiles[t];
    const int64_t pos64 = (int64_t)tt.L0 + (k - tt.ordinal0);
    if (k < tt.ordinal0 || pos64 >= tt.L1) continue;
    const int32_t pos = (int32_t)pos64;
    WinInit w0{};
    const Cover cv = make_cover(R, tt.rb, tt.re, pos, cover[wv], tmp[wv], kCover, 512, w0, nullptr, nullptr, ctr);
    SamplePile<NS> P;
    gather_sample(R, cv, pos, 0, amb_in ? (int)amb_ref[li] : -1, ctr, P);
    if (P.depth_all == 0) continue;  // skipEmpty
    if (P.overflow) {
      if constexpr (!DEEP) {
        if (lane == 0) {
          const unsigned long long q = atomicAdd(&ctr->n_deep, 1ull);
          if (q < dd.cap) dd.out[q] = li;
        }
      } else {
        raise_at(ctr, GQ_E_CAPACITY, pos);
      }
      continue;
    }
    if (!amb_in && P.ambiguous) {
      if (lane == 0) {
        const unsigned long long a = atomicAdd(&ctr->n_amb, 1ull);
        if (a < amb_cap) amb_out[a] = AmbItem{(int32_t)t, pos, k};
      }
      continue;
    }
    // Pileup.sampleName = the head element's sample (Pileup.scala:51): the reads' one sample,
    // or (flag bit 1) the first covering read's where the pileup mixes samples
    int first = -1;
    bool mixed = false;
    for (int64_t k0 = 0; k0 < cv.n; k0 += 64) {
      bool act;
      const int64_t r = cv.read(R, k0 + lane, pos, &act);
      const int smp = act ? (int)R.sample[r] : -1;
      const unsigned long long b = __ballot(act);
      if (!b) continue;
      if (first < 0) first = __shfl(smp, __ffsll((long long)b) - 1, 64);
      mixed |= __ballot(act && smp != first) != 0;
    }
    const uint8_t flags = (uint8_t)((amb_in ? 1 : 0) | (mixed ? 2 : 0));
    for (int j = 0; j < P.nt; ++j) {
      const AlleleDesc d = pile_desc(P, j);
      uint32_t cnt = 0;
#pragma unroll
      for (int s2 = 0; s2 < NS; ++s2)
        if (s2 == (j >> 6)) cnt = (uint32_t)__shfl((int)P.n_all[s2], j & 63, 64);
      const int rl = allele_ref_len(d), al = allele_alt_len(d);
      VsRec rr;
      rr.key = (uint64_t)k;
      rr.contig = tt.contig;
      rr.pos = pos;
      rr.count = (int32_t)cnt;
      rr.ref_len = (uint16_t)rl;
      rr.alt_len = (uint16_t)al;
      rr.flags = flags;
      rr.sample = (uint8_t)first;
      for (int q = 0; q < 6; ++q) rr.pad[q] = 0;
      if (rl + al <= 8) {
        uint64_t v = 0;
        for (int i = 0; i < rl; ++i) v |= (uint64_t)allele_byte(R, d, pos, 0, i) << (8 * i);
        for (int i = 0; i < al; ++i) v |= (uint64_t)allele_byte(R, d, pos, 1, i) << (8 * (rl + i));
        rr.allele = v;
      } else {
        unsigned long long off = 0;
        if (lane == 0) off = atomicAdd(&ctr->pool_used, (unsigned long long)(rl + al));
        off = __shfl(off, 0, 64);
        if (off + rl + al <= pool_cap)
          for (int i = lane; i < rl + al; i += 64)
            pool[off + i] = i < rl ? allele_byte(R, d, pos, 0, i) : allele_byte(R, d, pos, 1, i - rl);
        rr.allele = off;
      }
      if (lane == 0) {
        const unsigned long long q = atomicAdd(&ctr->n_rec, 1ull);
        if (q < rec_cap) recs[q] = rr;
      }
    }
  }
}

}  // namespace (reopened below)

// The projection's pool and the margin projection filled together (ensure_projection with a
// MarginReq): the margin pool and its slice flags allocated and preset, the term table built, then
// one pm_fill_rw pass.
gq_status gq::fused_projection_fill(gq_ctx *c, const gq_dev_reads *t, uint8_t *proj_pool, const MarginReq &mr) {
  const int key = 2 * mr.min_mapq + (mr.incl_align ? 1 : 0);
  if (!t->mproj) {
    void *p = nullptr;
    HIP_TRY(t->dp.get(&p, (size_t)(128 * t->n_rows + 32)));
    t->mproj = p;
    void *q = nullptr;
    HIP_TRY(t->dp.get(&q, (size_t)t->n_slices + 16));
    t->mnb = q;
  }
  HIP_TRY(hipMemsetAsync(t->mproj, kMargin8Zero, (size_t)(128 * t->n_rows + 32), c->stream));
  HIP_TRY(hipMemsetAsync(t->mnb, 0, (size_t)t->n_slices + 16, c->stream));
  void *tab = nullptr;
  HIP_TRY(t->dp.get(&tab, 256 * 256));
  hipLaunchKernelGGL(margin_table, dim3(256), dim3(256), 0, c->stream, mr.incl_align ? 1 : 0, (uint8_t *)tab);
  HIP_TRY(hipGetLastError());
  if (t->d.n_reads > 0) {
    hipLaunchKernelGGL(pm_fill_rw, dim3((unsigned)((std::min<int64_t>((t->d.n_reads + 255) / 256, 1 << 20) + 7) & ~(int64_t)7)),
                       dim3(256), 0, c->stream, t->d, proj_pool, mr.min_mapq, (const uint8_t *)tab,
                       (uint8_t *)t->mproj, (uint8_t *)t->mnb, fill_dbg());
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  t->dp.put(tab);
  t->mproj_mapq = key;
  return GQ_OK;
}

namespace {

gq_status ensure_margin_projection(gq_ctx *c, const gq_dev_reads *t, int min_mapq, bool incl_align = true) {
  const int key = 2 * min_mapq + (incl_align ? 1 : 0);  // the projection's filter and probability model
  if (t->mproj && t->mproj_mapq == key) return GQ_OK;
  if (!t->mproj) {
    void *p = nullptr;
    HIP_TRY(t->dp.get(&p, (size_t)(128 * t->n_rows + 32)));  // a byte per locus: 8 per 4-byte word of codes
    t->mproj = p;
    void *q = nullptr;
    HIP_TRY(t->dp.get(&q, (size_t)t->n_slices + 16));
    t->mnb = q;
    HIP_TRY(hipMemsetAsync(q, 0, (size_t)t->n_slices + 16, c->stream));
  }
  // the words no piece covers: biased zero terms (a rebuild for another filter rewrites only
  // pieces); the cell fill writes every word itself
  const int mode = margin_fill_mode();
  const bool cells = mode == 1 || mode == 2;  // these write every word: no preset
  if (cells) HIP_TRY(hipMemsetAsync((uint8_t *)t->mproj + 128 * t->n_rows, kMargin8Zero, 32, c->stream));
  else HIP_TRY(hipMemsetAsync(t->mproj, kMargin8Zero, (size_t)(128 * t->n_rows + 32), c->stream));
  void *tab = nullptr;  // margin_term8 by (mapq, quality, match)
  HIP_TRY(t->dp.get(&tab, 256 * 256));
  hipLaunchKernelGGL(margin_table, dim3(256), dim3(256), 0, c->stream, incl_align ? 1 : 0, (uint8_t *)tab);
  HIP_TRY(hipGetLastError());
  if (t->n_slices > 0) {
    static const int fill_u = getenv("GQ_FILL_U") ? atoi(getenv("GQ_FILL_U")) : 0;  // A/B: words per lane and round
    if (mode == 2) {  // A/B: GQ_MFILL=pieces
      const int64_t blocks = std::min<int64_t>((t->n_slices + 3) / 4, 1 << 20);
      hipLaunchKernelGGL(mproj_fill_pieces, dim3((unsigned)blocks), dim3(256), 0, c->stream, t->d, t->n_slices, min_mapq,
                         (const uint8_t *)tab, (uint8_t *)t->mproj, (uint8_t *)t->mnb);
    } else if (mode == 1) {  // A/B: GQ_MFILL=cells
      unsigned long long *nd = nullptr;
      int64_t *dl = nullptr;
      HIP_TRY(t->dp.get((void **)&nd, sizeof(unsigned long long)));
      HIP_TRY(t->dp.get((void **)&dl, sizeof(int64_t) * (size_t)t->n_slices));
      HIP_TRY(hipMemsetAsync(nd, 0, sizeof(unsigned long long), c->stream));
      const int64_t blocks = std::min<int64_t>((t->n_slices + 3) / 4, 1 << 20);
      hipLaunchKernelGGL(mproj_fill_cells, dim3((unsigned)blocks), dim3(256), 0, c->stream, t->d, t->n_slices, min_mapq,
                         (const uint8_t *)tab, (uint8_t *)t->mproj, (uint8_t *)t->mnb, dl, nd);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(mproj_fill_deep, dim3((unsigned)std::min<int64_t>(blocks, 2048)), dim3(256), 0, c->stream, t->d,
                         (const int64_t *)dl, (const unsigned long long *)nd, min_mapq, (const uint8_t *)tab,
                         (uint8_t *)t->mproj, (uint8_t *)t->mnb);
      t->dp.put(nd);
      t->dp.put(dl);
    } else if (mode == 3 || fill_slice_major()) {  // A/B: the slice-major fill of round 4 (GQ_MFILL / GQ_FILL=slice)
      auto kf = fill_u == 4 ? mproj_fill<4> : fill_u == 2 ? mproj_fill<2> : mproj_fill<1>;
      hipLaunchKernelGGL(kf, dim3((unsigned)std::min<int64_t>((t->n_slices + 3) / 4, 1 << 20)), dim3(256), 0,
                         c->stream, t->d, t->n_slices, min_mapq, (const uint8_t *)tab, (uint8_t *)t->mproj,
                         (uint8_t *)t->mnb);
    } else if (t->d.n_reads > 0) {
      // mnb: set per slice by the words (a rebuild for another filter starts from zero)
      HIP_TRY(hipMemsetAsync(t->mnb, 0, (size_t)t->n_slices + 16, c->stream));
      static const int fill_w = getenv("GQ_FILL_W") ? atoi(getenv("GQ_FILL_W")) : 1;  // words per lane unit
      auto kf = fill_u == 2 ? mproj_fill_rw<2, 1>
                : fill_u == 4 ? mproj_fill_rw<4, 1>
                : fill_w == 2 ? mproj_fill_rw<1, 2>
                : fill_w == 4 ? mproj_fill_rw<1, 4>
                              : mproj_fill_rw<1, 1>;
      hipLaunchKernelGGL(kf, dim3((unsigned)((std::min<int64_t>((t->d.n_reads + 255) / 256, 1 << 20) + 7) & ~(int64_t)7)),
                         dim3(256), 0, c->stream, t->d, min_mapq, (const uint8_t *)tab, (uint8_t *)t->mproj,
                         (uint8_t *)t->mnb, fill_dbg());
    }
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  t->dp.put(tab);
  t->mproj_mapq = key;
  return GQ_OK;
}

// The records of a somatic / germline-standard pass (device SomRec array + allele pool) ->
// the caller's result arrays in output (key) order, built on the device: the (key, slot) pairs
// radix-sorted (hipcub, only the bits a key can use), the allele lengths scanned into pool
// offsets, then one kernel writes the result image [pool_len | SoA columns | allele pool] and
// one D2H copy brings it into the result block.  ev[4] marks the end of the D2H;
// timings.marshal_ms is the host time after it.
struct SomLayout {  // byte offsets inside the image; header = int64 pool_len
  size_t contig, pos, sample, ref_off, ref_len, alt_off, alt_len, log_odds, gq, tumor, normal, flags, pool, bytes;
};
SomLayout som_layout(int64_t n, int64_t dev_pool_used) {
  auto al = [](size_t x) { return (x + 63) & ~(size_t)63; };
  const size_t N = (size_t)n;
  SomLayout L;
  L.contig = 64;
  L.pos = al(L.contig + 4 * N);
  L.sample = al(L.pos + 8 * N);
  L.ref_off = al(L.sample + N);
  L.ref_len = al(L.ref_off + 8 * N);
  L.alt_off = al(L.ref_len + 4 * N);
  L.alt_len = al(L.alt_off + 8 * N);
  L.log_odds = al(L.alt_len + 4 * N);
  L.gq = al(L.log_odds + 8 * N);
  L.tumor = al(L.gq + 4 * N);
  L.normal = al(L.tumor + sizeof(gq_evidence) * N);
  L.flags = al(L.normal + sizeof(gq_evidence) * N);
  L.pool = al(L.flags + N);
  // inline alleles hold <= 8 bytes; longer ones live in the device pool (each used once)
  L.bytes = al(L.pool + 8 * N + (size_t)dev_pool_used + 1);
  return L;
}

__global__ void som_keys(const SomRec *__restrict__ recs, int64_t n, uint64_t *__restrict__ keys,
                         uint32_t *__restrict__ slot) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  keys[k] = recs[k].key;
  slot[k] = (uint32_t)k;
}

__global__ void som_lengths(const SomRec *__restrict__ recs, const uint32_t *__restrict__ order, int64_t n,
                            int64_t *__restrict__ len) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const SomRec &r = recs[order[k]];
  len[k] = (int64_t)r.ref_len + r.alt_len;
}

// Record k of the output (slot order[k]) into the image; its allele bytes at pool offset off[k].
__global__ void som_image(const SomRec *__restrict__ recs, const uint32_t *__restrict__ order,
                          const int64_t *__restrict__ off, const uint8_t *__restrict__ dpool, int64_t n, SomLayout L,
                          uint8_t *__restrict__ img) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const SomRec &r = recs[order[k]];
  const int64_t at = off[k];
  const int tot = r.ref_len + r.alt_len;
  ((int32_t *)(img + L.contig))[k] = r.contig;
  ((int64_t *)(img + L.pos))[k] = r.pos;
  img[L.sample + k] = (uint8_t)((r.key >> 4) & 0xFFu);  // germline-standard: the sample slot (somatic: 0)
  ((int64_t *)(img + L.ref_off))[k] = at;
  ((int32_t *)(img + L.ref_len))[k] = r.ref_len;
  ((int64_t *)(img + L.alt_off))[k] = at + r.ref_len;
  ((int32_t *)(img + L.alt_len))[k] = r.alt_len;
  ((double *)(img + L.log_odds))[k] = r.log_odds;
  ((int32_t *)(img + L.gq))[k] = r.gq;
  ((gq_evidence *)(img + L.tumor))[k] = r.tumor;
  ((gq_evidence *)(img + L.normal))[k] = r.normal;
  img[L.flags + k] = r.flags;
  uint8_t *o = img + L.pool + at;
  if (tot <= 8)
    for (int i = 0; i < tot; ++i) o[i] = (uint8_t)(r.allele >> (8 * i));
  else
    for (int i = 0; i < tot; ++i) o[i] = dpool[r.allele + (uint64_t)i];
  if (k == n - 1) *(int64_t *)img = at + tot;
}

gq_status fetch_somatic_records(gq_ctx *c, const Counters &hc, unsigned long long pool_cap, uint64_t key_bound,
                                gq_somatic_calls *res) {
  const int64_t n = (int64_t)hc.n_rec;
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  const SomLayout lay = som_layout(n, (int64_t)std::min<unsigned long long>(hc.pool_used, pool_cap));
  HIP_TRY(c->image.ensure(lay.bytes));
  if (n > 0) {
    HIP_TRY(c->keys.ensure(nn * 8));
    HIP_TRY(c->keys_sorted.ensure(nn * 8));
    HIP_TRY(c->idx.ensure(nn * 8));
    HIP_TRY(c->idx_sorted.ensure(nn * 8));
    const unsigned nb = (unsigned)((n + kBlock - 1) / kBlock);
    uint64_t *keys = (uint64_t *)c->keys.p, *keys2 = (uint64_t *)c->keys_sorted.p;
    uint32_t *slot = (uint32_t *)c->idx.p, *order = (uint32_t *)c->idx_sorted.p;
    int64_t *len = (int64_t *)c->keys.p, *off = (int64_t *)c->idx.p;  // reused once the sort is done
    hipLaunchKernelGGL(som_keys, dim3(nb), dim3(kBlock), 0, c->stream, (const SomRec *)c->srecs.p, n, keys, slot);
    HIP_TRY(hipGetLastError());
    const int end_bit = key_bound ? 64 - __builtin_clzll(key_bound) : 64;
    size_t tmp = 0, tmp2 = 0;
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, keys, keys2, slot, order, (int)n, 0, end_bit, c->stream));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp2, len, off, (int)n, c->stream));
    HIP_TRY(c->sort_tmp.ensure(std::max(tmp, tmp2)));
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(c->sort_tmp.p, tmp, keys, keys2, slot, order, (int)n, 0, end_bit,
                                               c->stream));
    hipLaunchKernelGGL(som_lengths, dim3(nb), dim3(kBlock), 0, c->stream, (const SomRec *)c->srecs.p,
                       (const uint32_t *)order, n, len);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(c->sort_tmp.p, tmp2, len, off, (int)n, c->stream));
    hipLaunchKernelGGL(som_image, dim3(nb), dim3(kBlock), 0, c->stream, (const SomRec *)c->srecs.p,
                       (const uint32_t *)order, (const int64_t *)off, (const uint8_t *)c->pool.p, n, lay,
                       (uint8_t *)c->image.p);
    HIP_TRY(hipGetLastError());
  } else {
    HIP_TRY(hipMemsetAsync(c->image.p, 0, 64, c->stream));
  }
  uint8_t *blk = (uint8_t *)malloc(lay.bytes);
  if (!blk) return set_err(GQ_E_NOMEM, "somatic result block of %zu bytes", lay.bytes);
  const hipError_t e = hipMemcpyAsync(blk, c->image.p, lay.bytes, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) (void)hipEventRecord(c->ev[4], c->stream);
  if (e != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
    free(blk);
    return set_err(GQ_E_HIP, "somatic result image D2H");
  }
  const auto m0 = std::chrono::steady_clock::now();
  res->n = n;
  res->block_ = blk;
  res->contig = (int32_t *)(blk + lay.contig);
  res->pos = (int64_t *)(blk + lay.pos);
  res->sample = blk + lay.sample;
  res->ref_off = (int64_t *)(blk + lay.ref_off);
  res->ref_len = (int32_t *)(blk + lay.ref_len);
  res->alt_off = (int64_t *)(blk + lay.alt_off);
  res->alt_len = (int32_t *)(blk + lay.alt_len);
  res->log_odds = (double *)(blk + lay.log_odds);
  res->gq = (int32_t *)(blk + lay.gq);
  res->tumor = (gq_evidence *)(blk + lay.tumor);
  res->normal = (gq_evidence *)(blk + lay.normal);
  res->flags = blk + lay.flags;
  res->allele_pool = blk + lay.pool;
  res->pool_len = n > 0 ? *(const int64_t *)blk : 0;
  c->timings.marshal_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - m0).count();
  return GQ_OK;
}

}  // namespace

// A reference genome resident in HBM (ReferenceBroadcast.scala:39-55): the contigs of a read
// set's contig list, each at a 512-aligned offset and padded with 'N' to a whole 512-locus block
// past its end (somatic_proj reads 8 bases per lane of an aligned block).
struct gq_reference {
  int device = 0;
  int32_t n_contigs = 0;
  void *bytes = nullptr;
  int64_t *d_off = nullptr;
  std::vector<int64_t> off, len;  // host copies; off = -1 for a contig the reference lacks
};

extern "C" {

gq_status gq_reference_upload(gq_ctx *c, int32_t n_contigs, const uint8_t *const *bases, const int64_t *lengths,
                              gq_reference **out) {
  if (!c || n_contigs < 0 || (n_contigs > 0 && (!bases || !lengths)) || !out)
    return set_err(GQ_E_ARG, "gq_reference_upload: bad argument");
  HIP_TRY(hipSetDevice(c->device));
  gq_reference *r = new gq_reference();
  r->device = c->device;
  r->n_contigs = n_contigs;
  r->off.assign((size_t)n_contigs, -1);
  r->len.assign((size_t)n_contigs, -1);
  int64_t tot = 0;
  for (int32_t k = 0; k < n_contigs; ++k) {
    if (!bases[k] || lengths[k] < 0) continue;
    r->off[(size_t)k] = tot;
    r->len[(size_t)k] = lengths[k];
    tot += (lengths[k] + 1023) / 512 * 512;
  }
  auto fail = [&](gq_status st) {
    gq_reference_free(r);
    return st;
  };
  if (hipMalloc(&r->bytes, (size_t)std::max<int64_t>(tot, 512)) != hipSuccess ||
      hipMalloc((void **)&r->d_off, sizeof(int64_t) * (size_t)std::max(n_contigs, 1)) != hipSuccess)
    return fail(set_err(GQ_E_HIP, "gq_reference_upload: hipMalloc of %lld bytes failed", (long long)tot));
  if (hipMemsetAsync(r->bytes, 'N', (size_t)std::max<int64_t>(tot, 512), c->stream) != hipSuccess)
    return fail(set_err(GQ_E_HIP, "gq_reference_upload: memset failed"));
  for (int32_t k = 0; k < n_contigs; ++k)
    if (r->off[(size_t)k] >= 0 && lengths[k] > 0 &&
        hipMemcpyAsync((uint8_t *)r->bytes + r->off[(size_t)k], bases[k], (size_t)lengths[k], hipMemcpyHostToDevice,
                       c->stream) != hipSuccess)
      return fail(set_err(GQ_E_HIP, "gq_reference_upload: copy of contig %d failed", k));
  if (n_contigs > 0 && hipMemcpyAsync(r->d_off, r->off.data(), sizeof(int64_t) * (size_t)n_contigs,
                                      hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return fail(set_err(GQ_E_HIP, "gq_reference_upload: offsets copy failed"));
  if (hipStreamSynchronize(c->stream) != hipSuccess) return fail(set_err(GQ_E_HIP, "gq_reference_upload: sync failed"));
  *out = r;
  return GQ_OK;
}

void gq_reference_free(gq_reference *r) {
  if (!r) return;
  (void)hipSetDevice(r->device);
  if (r->bytes) (void)hipFree(r->bytes);
  if (r->d_off) (void)hipFree(r->d_off);
  delete r;
}

gq_status gq_somatic_standard(gq_ctx *c, const gq_dev_reads *t, const gq_dev_reads *n, const gq_loci *loci,
                              const gq_somatic_params *p, gq_somatic_calls **out) {
  return gq_somatic_standard_ref(c, t, n, loci, nullptr, p, out);
}

gq_status gq_somatic_standard_ref(gq_ctx *c, const gq_dev_reads *t, const gq_dev_reads *n, const gq_loci *loci,
                                  const gq_reference *ref, const gq_somatic_params *p, gq_somatic_calls **out) {
  if (!c || !t || !n || !loci || !p || !out) return set_err(GQ_E_ARG, "gq_somatic_standard: null argument");
  if (t->d.n_contigs != n->d.n_contigs)
    return set_err(GQ_E_ARG, "tumor and normal read sets must share the contig list (%d vs %d contigs)",
                   t->d.n_contigs, n->d.n_contigs);
  const int dbg = getenv("GQ_DBG") ? atoi(getenv("GQ_DBG")) : 0;  // diagnostics only (read per call)
  RefView rv{nullptr, nullptr};
  std::vector<int32_t> lc;
  std::vector<int64_t> ls, le, lt;
  gq_loci trimmed{};
  if (ref) {
    // The reference looks a base up for every pileup (getReferenceBase, ReferenceBroadcast.scala:
    // 26-30): a contig it lacks, or a locus past its end, fails the job where a read covers it.
    // Loci no read reaches are trimmed away (no pileup forms there).
    if (ref->n_contigs != t->d.n_contigs)
      return set_err(GQ_E_ARG, "reference covers %d contigs, the read sets %d", ref->n_contigs, t->d.n_contigs);
    if (ref->device != c->device) return set_err(GQ_E_ARG, "reference uploaded to another device");
    HIP_TRY(hipSetDevice(c->device));
    // does a read of either sample overlap [a, b) of contig ci (a pileup forms there)?
    auto covered = [&](int32_t ci, int64_t a, int64_t b, bool *hit) -> gq_status {
      *hit = false;
      for (const gq_dev_reads *sr : {t, n}) {
        std::vector<char> o;
        const gq_status s2 = reads_overlap(c, sr, ci, {{a, b}}, o);
        if (s2) return s2;
        if (o[0]) *hit = true;
      }
      return GQ_OK;
    };
    for (int64_t k = 0; k < loci->n_ranges; ++k) {
      const int32_t ci = loci->contig[k];
      const int64_t s0 = loci->start[k];
      int64_t e0 = loci->end[k];
      if (e0 <= s0) continue;
      if (ci < 0 || ci >= ref->n_contigs) return set_err(GQ_E_ARG, "loci range on contig %d: no such contig", ci);
      bool hit = false;
      if (ref->off[(size_t)ci] < 0) {
        const gq_status s2 = covered(ci, s0, e0, &hit);
        if (s2) return s2;
        if (hit) return set_err(GQ_E_ARG, "contig %d does not exist in the current reference", ci);
        continue;
      }
      const int64_t len = ref->len[(size_t)ci];
      if (e0 > len) {
        // only a pileup at a locus of THIS range past the contig's end fails (getReferenceBase)
        const gq_status s2 = covered(ci, std::max(len, s0), e0, &hit);
        if (s2) return s2;
        if (hit)
          return set_err(GQ_E_ARG, "locus %lld of contig %d is past the end of the reference contig (length %lld)",
                         (long long)std::max(len, s0), ci, (long long)len);
        e0 = len;
        if (e0 <= s0) continue;
      }
      lc.push_back(ci);
      ls.push_back(s0);
      le.push_back(e0);
      lt.push_back(loci->task ? loci->task[k] : 0);
    }
    trimmed = gq_loci{(int64_t)lc.size(), lc.data(), ls.data(), le.data(), loci->task ? lt.data() : nullptr};
    loci = &trimmed;
    rv = RefView{(const uint8_t *)ref->bytes, ref->d_off};
  }
  HIP_TRY(hipSetDevice(c->device));
  const auto h0 = std::chrono::steady_clock::now();
  c->timings = gq_timings{};
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  // one loci plan per sample, 512-locus tiles aligned to 512-locus blocks (somatic_proj)
  Plan pt, pn;
  // somatic_direct (straight from the reads) unless GQ_SOM=proj asks for somatic_proj over the
  // projection and margin projection (A/B; the same candidates)
  static const bool som_proj = getenv("GQ_SOM") && strcmp(getenv("GQ_SOM"), "proj") == 0;
  const bool direct = !som_proj && t->d.seq_cap >= 8;
  const MarginReq mreq{(int)p->min_mapq, true};  // (with the projection, the margin projection in the same pass)
  gq_status st = direct ? GQ_OK : ensure_projection(c, t, &mreq);  // (derived on first use)
  if (st) return st;
  st = plan(c, t, loci, SomProjCfg::kT, pt, c->tiles, 0, 0, 0, true);
  if (st) return st;
  st = plan(c, n, loci, SomProjCfg::kT, pn, c->tiles2, 0, 0, 0, true);
  if (st) return st;
  gq_somatic_calls *res = (gq_somatic_calls *)calloc(1, sizeof(gq_somatic_calls));
  if (!res) return set_err(GQ_E_NOMEM, "calloc");
  if (pt.n_tiles == 0) {
    *out = res;
    return GQ_OK;
  }
  // PhredUtils.phredToSuccessProbability table: the host's pow, the bits the reference starts from
  {
    static_assert(sizeof(double) == 8, "FP64");
    double succ[256];
    for (int q = 0; q < 256; ++q) succ[q] = 1.0 - std::pow(10.0, -q / 10.0);
    HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_succ), succ, sizeof succ, 0, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  // pileup element order: each window's first visited locus and initial (heap-ordered) group
  SomWin sw{};
  st = build_somwin(c, pt, t, n, sw);
  if (st) {
    free(res);
    return st;
  }
  // the tumor's margin projection for this mapq filter (derived once per read set and filter);
  // somatic_direct: only the term table
  if (direct) {
    if (c->mtab_key != 1) {
      HIP_TRY(c->mtab.ensure(256 * 256));
      hipLaunchKernelGGL(margin_table, dim3(256), dim3(256), 0, c->stream, 1, (uint8_t *)c->mtab.p);
      HIP_TRY(hipGetLastError());
      c->mtab_key = 1;
    }
  } else {
    st = ensure_margin_projection(c, t, (int)p->min_mapq);
  }
  if (st) {
    free(res);
    return st;
  }
  // candidates: one output partition per somatic_proj workgroup (capA) and per somatic_tile
  // block (capB), grown on overflow (part_scan's part_max)
  OutGeom og{};
  {
    if (c->n_cu <= 0 &&
        hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess)
      c->n_cu = 256;
    int &wg_cu = direct ? c->somd_wg_per_cu : c->som_wg_per_cu;
    if (wg_cu <= 0) {
      int nb = 0;
      const hipError_t e =
          direct ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, somatic_direct<false>, SomDirCfg::kThreads, 0)
                 : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, somatic_proj<false>, SomProjCfg::kThreads, 0);
      if (e != hipSuccess || nb <= 0) nb = direct ? 2 : 4;
      wg_cu = nb;
    }
    og.ncols = (int)std::max<int64_t>(1, std::min<int64_t>({(pt.n_tiles + SomProjCfg::kWaves - 1) / SomProjCfg::kWaves,
                                                           (int64_t)wg_cu * c->n_cu, (int64_t)kPartsCols}));
    const unsigned long long wg_loci = (unsigned long long)((pt.n_tiles + og.ncols - 1) / og.ncols) * SomProjCfg::kT;
    og.capA[1] = wg_loci / 16 + 256;
    og.capB[1] = (unsigned long long)pt.n_loci / 65536 + 1024;
  }
  unsigned long long rec_cap = 1 << 16, pool_cap = 1 << 20, amb_cap = 4096, deep_cap = 4096;
  Counters hc{};
  float call_ms = 0, deep_ms = 0, front_ms = 0;
  // GQ_CALL_SPLIT=1: the split caller (somatic_front + the back end over stored records).  Measured
  // slower at chr1 60x/30x (front 3.9 ms + back 5.5 ms against 8.6 ms for the one kernel,
  // profiles/r04_a5_kernel_stats.csv), so the one kernel is the default.
  static const bool split = getenv("GQ_CALL_SPLIT") && atoi(getenv("GQ_CALL_SPLIT")) != 0;
  // GQ_CALL_WPE=2: the one-kernel caller built for 2 waves per SIMD (no spills) instead of 3
  static const bool wpe2 = getenv("GQ_CALL_WPE") && atoi(getenv("GQ_CALL_WPE")) == 2;
  for (int attempt = 0; attempt < 3; ++attempt) {
    HIP_TRY(c->amb.ensure(amb_cap * sizeof(AmbItem)));
    HIP_TRY(c->cplx.ensure(og.total(1) * sizeof(ComplexItem)));
    HIP_TRY(c->srecs.ensure(rec_cap * sizeof(SomRec)));
    HIP_TRY(c->pool.ensure(pool_cap));
    HIP_TRY(c->slow.ensure((size_t)pt.n_tiles * sizeof(int32_t)));
    HIP_TRY(c->counters.ensure(sizeof(Counters)));
    Counters *ctr = (Counters *)c->counters.p;
    HIP_TRY(hipMemsetAsync(ctr, 0, sizeof(Counters), c->stream));
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    if (direct) {
      if (rv.b)
        hipLaunchKernelGGL(somatic_direct<true>, dim3((unsigned)og.ncols), dim3(SomDirCfg::kThreads), 0, c->stream,
                           (const Tile *)c->tiles.p, (const Tile *)c->tiles2.p, pt.n_tiles, t->d, n->d.start, n->d.end,
                           (const uint8_t *)c->mtab.p, (int)p->min_mapq, (ComplexItem *)c->cplx.p, og, ctr,
                           (int32_t *)c->slow.p, rv, 0, (dbg >> 16) & 0xFF);
      else
        hipLaunchKernelGGL(somatic_direct<false>, dim3((unsigned)og.ncols), dim3(SomDirCfg::kThreads), 0, c->stream,
                           (const Tile *)c->tiles.p, (const Tile *)c->tiles2.p, pt.n_tiles, t->d, n->d.start, n->d.end,
                           (const uint8_t *)c->mtab.p, (int)p->min_mapq, (ComplexItem *)c->cplx.p, og, ctr,
                           (int32_t *)c->slow.p, rv, 0, (dbg >> 16) & 0xFF);
    } else if (rv.b)
      hipLaunchKernelGGL(somatic_proj<true>, dim3((unsigned)og.ncols), dim3(SomProjCfg::kThreads), 0, c->stream,
                         (const Tile *)c->tiles.p, (const Tile *)c->tiles2.p, pt.n_tiles, t->d,
                         (const uint8_t *)t->mproj, (const uint8_t *)t->mnb, n->d.start, n->d.end, (ComplexItem *)c->cplx.p, og, ctr,
                         (int32_t *)c->slow.p, rv);
    else
      hipLaunchKernelGGL(somatic_proj<false>, dim3((unsigned)og.ncols), dim3(SomProjCfg::kThreads), 0, c->stream,
                         (const Tile *)c->tiles.p, (const Tile *)c->tiles2.p, pt.n_tiles, t->d,
                         (const uint8_t *)t->mproj, (const uint8_t *)t->mnb, n->d.start, n->d.end, (ComplexItem *)c->cplx.p, og, ctr,
                         (int32_t *)c->slow.p, rv);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL((somatic_tile<SomProjCfg::kT>), dim3((unsigned)std::min<int64_t>(pt.n_tiles, 2048)), dim3(kBlock), 0,
                       c->stream, (const Tile *)c->tiles.p, (const Tile *)c->tiles2.p, t->d, n->d,
                       (ComplexItem *)c->cplx.p, og, (const int32_t *)c->slow.p, (int)p->min_mapq, ctr, rv);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(part_scan_som, dim3(1), dim3(1024), 0, c->stream, ctr, og);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    unsigned long long n_cand = 0;
    {  // candidate overflow: grow and re-run the tile kernels before the (costly) caller runs
      unsigned long long pm = 0;
      HIP_TRY(hipMemcpyAsync(&pm, &ctr->part_max[1], sizeof(pm), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipMemcpyAsync(&n_cand, &ctr->part_off[1][kParts], sizeof(n_cand), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      if (pm) {
        og.capA[1] += pm + 64;
        og.capB[1] += pm + 64;
        if (attempt == 2) {
          free(res);
          return set_err(GQ_E_CAPACITY, "candidate capacity retries exhausted");
        }
        continue;
      }
    }
    // the exact caller: the fast kernel (pileups up to kFastCap reads per sample, element
    // records in LDS), then the deep kernel over the deeper candidates it listed, then the
    // deep kernel again over the loci whose reference base heap order decides
    HIP_TRY(c->deep_list.ensure(2 * deep_cap * sizeof(int64_t)));  // the deep list, then the wide list
    // persistent: the resident workgroups, each wave over every (grid)-th candidate (a grid of
    // many generations leaves a tail of idle SIMDs behind the last ones)
    if (c->call_wg_per_cu <= 0) {
      int nb = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, split ? (const void *)somatic_call_k<false, true>
                                                             : wpe2 ? (const void *)somatic_call_k<false, false, 2>
                                                                    : (const void *)somatic_call_k<false, false, 3>,
                                                       kBlock, 0) != hipSuccess ||
          nb <= 0)
        nb = 3;
      c->call_wg_per_cu = nb;
    }
    static const int grid_env = getenv("GQ_CALL_GRID") ? atoi(getenv("GQ_CALL_GRID")) : 0;  // A/B: 0 = resident
    const int64_t grid_cap = grid_env > 0 ? (int64_t)grid_env : (int64_t)c->call_wg_per_cu * c->n_cu;
    const int cblocks = (int)std::min<int64_t>(std::max<int64_t>(pt.n_tiles, 1), grid_cap);
    const DeepIO dio{(int64_t *)c->deep_list.p, deep_cap, 0, nullptr, 0, 0};
    // the candidates' records in list order (every caller kernel below reads them)
    HIP_TRY(c->cands.ensure(sizeof(CandRec) * (size_t)std::max<unsigned long long>(n_cand, 1)));
    hipLaunchKernelGGL(cand_prep, dim3((unsigned)((kParts + kSomWaves - 1) / kSomWaves)), dim3(kBlock), 0, c->stream,
                       (const Tile *)c->tiles.p, (const Tile *)c->tiles2.p, (const ComplexItem *)c->cplx.p, og,
                       (const Counters *)ctr, sw, t->d, n->d, (CandRec *)c->cands.p);
    HIP_TRY(hipGetLastError());
    front_ms = 0;
    if (!split) {
      auto k1 = wpe2 ? somatic_call_k<false, false, 2> : somatic_call_k<false, false, 3>;
      hipLaunchKernelGGL(k1, dim3(cblocks), dim3(kBlock), 0, c->stream, (const CandRec *)c->cands.p, t->d, n->d, *p,
                         (SomRec *)c->srecs.p, rec_cap, (uint8_t *)c->pool.p, pool_cap, og, ctr, sw, (AmbItem *)c->amb.p,
                         amb_cap, (const AmbItem *)nullptr, (const uint8_t *)nullptr, (int64_t)0, rv, dbg, dio,
                         ElemStore{});
      HIP_TRY(hipGetLastError());
    } else {
      // the split caller, in batches of at most kStoreBatch candidates (the store: 5 KiB each):
      // somatic_front (covers + element records, latency-bound, many waves) then the back end
      // (tables, FP64 genotypes, evidence) over the stored records
      constexpr int64_t kStoreBatch = 1 << 20;
      const int64_t nb = std::min<int64_t>((int64_t)n_cand, kStoreBatch);
      const size_t hdr_b = ((size_t)std::max<int64_t>(nb, 1) * sizeof(uint4) + 255) & ~(size_t)255;
      const size_t el_b = (size_t)std::max<int64_t>(nb, 1) * 2 * kFastCap * sizeof(uint4);
      const size_t cov_b = (size_t)std::max<int64_t>(nb, 1) * 2 * kFastCap * sizeof(int32_t);
      HIP_TRY(c->el_store.ensure(hdr_b + el_b + cov_b));
      if (c->front_wg_per_cu <= 0) {
        int fb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&fb, somatic_front, kBlock, 0) != hipSuccess || fb <= 0) fb = 6;
        c->front_wg_per_cu = fb;
      }
      uint8_t *sb = (uint8_t *)c->el_store.p;
      for (int64_t b0 = 0; b0 < (int64_t)n_cand; b0 += kStoreBatch) {
        const int64_t b1 = std::min<int64_t>((int64_t)n_cand, b0 + kStoreBatch);
        const ElemStore es{(uint4 *)sb, (uint4 *)(sb + hdr_b), (int32_t *)(sb + hdr_b + el_b), b0, b1};
        const int64_t waves = b1 - b0;
        const unsigned fblocks = (unsigned)std::min<int64_t>((waves + kSomWaves - 1) / kSomWaves,
                                                            (int64_t)c->front_wg_per_cu * c->n_cu);
        const unsigned bblocks = (unsigned)std::min<int64_t>((waves + kSomWaves - 1) / kSomWaves, grid_cap);
        if (b0 > 0) {  // the previous batch's front time (its back end keeps the GPU busy meanwhile)
          HIP_TRY(hipEventSynchronize(c->ev[7]));
          float ms = 0;
          (void)hipEventElapsedTime(&ms, c->ev[6], c->ev[7]);
          front_ms += ms;
        }
        HIP_TRY(hipEventRecord(c->ev[6], c->stream));
        hipLaunchKernelGGL(somatic_front, dim3(fblocks), dim3(kBlock), 0, c->stream, (const CandRec *)c->cands.p, t->d,
                           n->d, *p, ctr, sw, dbg, dio, es);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ev[7], c->stream));
        hipLaunchKernelGGL((somatic_call_k<false, true>), dim3(bblocks), dim3(kBlock), 0, c->stream,
                           (const CandRec *)c->cands.p, t->d, n->d, *p, (SomRec *)c->srecs.p, rec_cap, (uint8_t *)c->pool.p, pool_cap, og, ctr, sw,
                           (AmbItem *)c->amb.p, amb_cap, (const AmbItem *)nullptr, (const uint8_t *)nullptr, (int64_t)0,
                           rv, dbg, dio, es);
        HIP_TRY(hipGetLastError());
      }
    }
    HIP_TRY(hipEventRecord(c->ev[3], c->stream));
    HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    (void)hipEventElapsedTime(&call_ms, c->ev[2], c->ev[3]);
    if (split && n_cand > 0) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, c->ev[6], c->ev[7]);
      front_ms += ms;
    }
    deep_ms = 0;
    bool retry = false;
    if (hc.n_deep > deep_cap) {
      deep_cap = hc.n_deep + 1024;
      retry = true;
    }
    // the deep kernel's per-wave scratch: the deepest listed pileup (at least kFastCap: the
    // genotype keys share its evidence words)
    auto run_deep = [&](int64_t n_items, const AmbItem *ain, const uint8_t *aref) -> gq_status {
      const int scap = (int)std::max<unsigned long long>(hc.deep_max, (unsigned long long)kFastCap);
      const int64_t nw = std::min<int64_t>(n_items, 4096);
      const size_t wb = deep_wave_bytes(scap, kMaxG);
      HIP_TRY(c->deep_scratch.ensure((size_t)nw * wb + 256));
      HIP_TRY(hipEventRecord(c->ev[5], c->stream));
      const unsigned blocks = (unsigned)((nw + kSomWaves - 1) / kSomWaves);
      hipLaunchKernelGGL((somatic_call_k<true, false>), dim3(blocks), dim3(kBlock), 0, c->stream,
                         (const CandRec *)c->cands.p, t->d, n->d, *p,
                         (SomRec *)c->srecs.p, rec_cap, (uint8_t *)c->pool.p, pool_cap, og, ctr, sw,
                         (AmbItem *)(ain ? nullptr : c->amb.p), ain ? (unsigned long long)0 : amb_cap, ain, aref,
                         ain ? n_items : (int64_t)0, ain ? RefView{nullptr, nullptr} : rv, dbg,
                         DeepIO{(int64_t *)c->deep_list.p, 0, ain ? 0 : n_items, (uint8_t *)c->deep_scratch.p, scap,
                                kMaxG, (int64_t *)c->deep_list.p + deep_cap, deep_cap},
                         ElemStore{});
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipEventRecord(c->ev[3], c->stream));
      HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      float ms = 0;
      (void)hipEventElapsedTime(&ms, c->ev[5], c->ev[3]);
      deep_ms += ms;
      return GQ_OK;
    };
    if (!retry && hc.n_deep > 0 && !hc.err) {
      st = run_deep((int64_t)hc.n_deep, nullptr, nullptr);
      if (st) {
        free(res);
        return st;
      }
    }
    if (hc.n_wide > deep_cap) {
      deep_cap = hc.n_wide + 1024;
      retry = true;
    }
    // the wide kernel: the candidates past the deep kernel's allele table or genotype scratch
    // (64 kWideNS distinct alleles per sample, every genotype of them in its scratch); a few
    // waves, each with a large scratch slice.  ain: a heap-order replay's hand-over (the list
    // holds positions in ain, whose resolved reference bases the kernel reads from aref).
    auto run_wide = [&](int64_t n_items, const AmbItem *ain, const uint8_t *aref, int64_t n_ain) -> gq_status {
      const int scap = (int)std::max<unsigned long long>(hc.deep_max, (unsigned long long)kFastCap);
      const int maxg = 64 * kWideNS * (64 * kWideNS + 1) / 2;
      const int64_t nw = std::min<int64_t>(n_items, 16);  // (12.6 MB of genotype scratch per wave)
      const size_t wb = deep_wave_bytes(scap, maxg, kWideNS);
      HIP_TRY(c->deep_scratch.ensure((size_t)nw * wb + 256));
      HIP_TRY(hipEventRecord(c->ev[5], c->stream));
      hipLaunchKernelGGL((somatic_call_k<true, false, 3, kWideNS>), dim3((unsigned)((nw + kSomWaves - 1) / kSomWaves)),
                         dim3(kBlock), 0, c->stream, (const CandRec *)c->cands.p, t->d, n->d, *p, (SomRec *)c->srecs.p,
                         rec_cap, (uint8_t *)c->pool.p, pool_cap, og, ctr, sw, (AmbItem *)(ain ? nullptr : c->amb.p),
                         ain ? (unsigned long long)0 : amb_cap, ain, aref, ain ? n_ain : (int64_t)0,
                         ain ? RefView{nullptr, nullptr} : rv, dbg,
                         DeepIO{(int64_t *)c->deep_list.p + deep_cap, 0, n_items, (uint8_t *)c->deep_scratch.p,
                                scap, maxg, nullptr, 0},
                         ElemStore{});
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipEventRecord(c->ev[3], c->stream));
      HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      float ms = 0;
      (void)hipEventElapsedTime(&ms, c->ev[5], c->ev[3]);
      deep_ms += ms;
      return GQ_OK;
    };
    if (!retry && hc.n_wide > 0 && !hc.err) {
      st = run_wide((int64_t)hc.n_wide, nullptr, nullptr, 0);
      if (st) {
        free(res);
        return st;
      }
    }
    if (hc.n_amb > amb_cap) {
      amb_cap = hc.n_amb + 1024;
      retry = true;
    }
    if (!retry && hc.n_amb > 0 && !hc.err) {
      // loci where a sample's reference base depends on heap order: replay both windows'
      // queues, then the deep caller over just those loci with the resolved bases
      std::vector<AmbItem> amb((size_t)hc.n_amb);
      HIP_TRY(hipMemcpyAsync(amb.data(), c->amb.p, amb.size() * sizeof(AmbItem), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(c->amb_ref.ensure(2 * amb.size()));
      st = heap_ref_bases(c, pt, c->tiles, {t, n}, amb, (uint8_t *)c->amb_ref.p);
      if (st) {
        free(res);
        return st;
      }
      // (the hand-over list of the replay starts empty: loci past the deep table go to the wide kernel)
      HIP_TRY(hipMemsetAsync(&ctr->n_wide, 0, sizeof(ctr->n_wide), c->stream));
      st = run_deep((int64_t)amb.size(), (const AmbItem *)c->amb.p, (const uint8_t *)c->amb_ref.p);
      if (st) {
        free(res);
        return st;
      }
      if (hc.n_wide > deep_cap) {
        deep_cap = hc.n_wide + 1024;
        retry = true;
      }
      if (!retry && hc.n_wide > 0 && !hc.err) {
        st = run_wide((int64_t)hc.n_wide, (const AmbItem *)c->amb.p, (const uint8_t *)c->amb_ref.p, (int64_t)amb.size());
        if (st) {
          free(res);
          return st;
        }
      }
    }
    if (hc.n_rec > rec_cap) {
      rec_cap = hc.n_rec + 1024;
      retry = true;
    }
    if (hc.pool_used > pool_cap) {
      pool_cap = hc.pool_used + 4096;
      retry = true;
    }
    if (!retry) break;
    if (attempt == 2) {
      free(res);
      return set_err(GQ_E_CAPACITY, "output capacity retries exhausted");
    }
  }
  for (int k = 0; k < kSpread; ++k) hc.visited += hc.spread[0][k];
  if ((dbg & 16) && hc.prof[5])
    fprintf(stderr, "gq somatic_call prof (cycles/candidate/wave): front|records %.0f (tumor fold %.0f) tables %.0f "
            "tumor-genotypes %.0f normal-genotypes+evidence %.0f (%llu candidates reached)\n", (double)hc.prof[0] / hc.prof[5],
            (double)hc.prof[1] / hc.prof[5], (double)hc.prof[2] / hc.prof[5], (double)hc.prof[3] / hc.prof[5],
            (double)hc.prof[4] / hc.prof[5], hc.prof[5]);
  st = check_device_error(c, hc);
  if (st) {
    free(res);
    return st;
  }
  st = fetch_somatic_records(c, hc, pool_cap, (uint64_t)std::max<int64_t>(pt.n_loci, 1) << 12, res);
  if (st) {
    free(res);
    return st;
  }
  res->visited_loci = (int64_t)hc.visited;
  res->candidate_loci = (int64_t)hc.n_complex;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[2]);
  c->timings.pileup_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
  c->timings.complex_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[3], c->ev[4]);
  c->timings.finalize_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[4]);
  c->timings.total_ms = ms;
  c->timings.pileup_launches = 1;
  c->timings.tiles = pt.n_tiles;
  c->timings.walk_tiles = (int64_t)hc.n_slow;
  c->timings.deep_loci = (int64_t)hc.n_deep;
  c->timings.deep_max = (int64_t)hc.deep_max;
  c->timings.call_ms = call_ms;
  c->timings.deep_ms = deep_ms;
  c->timings.front_ms = front_ms;
  c->timings.host_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - h0).count();
  *out = res;
  return GQ_OK;
}

gq_status gq_variant_support(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, gq_allele_counts **out) {
  if (!c || !rd || !loci || !out) return set_err(GQ_E_ARG, "gq_variant_support: null argument");
  HIP_TRY(hipSetDevice(c->device));
  const auto h0 = std::chrono::steady_clock::now();
  c->timings = gq_timings{};
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  Plan pl;
  gq_status st = ensure_columns(c, rd);
  if (st) return st;
  st = plan(c, rd, loci, 512, pl, c->tiles);
  if (st) return st;
  gq_allele_counts *res = (gq_allele_counts *)calloc(1, sizeof(gq_allele_counts));
  if (!res) return set_err(GQ_E_NOMEM, "calloc");
  auto fail = [&](gq_status e) {
    gq_free_allele_counts(res);
    return e;
  };
  unsigned long long rec_cap = (unsigned long long)std::max<int64_t>(pl.n_loci * 2, 1024), pool_cap = 1 << 16,
                     amb_cap = 4096, deep_cap = 1024;
  Counters hc{};
  const int blocks = (int)std::min<int64_t>(std::max<int64_t>((pl.n_loci + kSomWaves - 1) / kSomWaves, 1), 8192);
  for (int attempt = 0; pl.n_tiles > 0; ++attempt) {
    HIP_TRY(c->amb.ensure(amb_cap * sizeof(AmbItem)));
    HIP_TRY(c->srecs.ensure(rec_cap * sizeof(VsRec)));
    HIP_TRY(c->pool.ensure(pool_cap));
    HIP_TRY(c->counters.ensure(sizeof(Counters)));
    HIP_TRY(c->deep_list.ensure(deep_cap * sizeof(int64_t)));
    Counters *ctr = (Counters *)c->counters.p;
    HIP_TRY(hipMemsetAsync(ctr, 0, sizeof(Counters), c->stream));
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    int64_t *dl = (int64_t *)c->deep_list.p;
    const DeepSel fast{dl, deep_cap, nullptr, 0, nullptr, 0, 0};
    // the loci the fast table handed over [from, hc.n_deep): the deep instantiation, same mode
    auto run_deep = [&](int64_t from, const AmbItem *ain, const uint8_t *aref, int64_t n_ain) -> gq_status {
      HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      const int64_t nd = (int64_t)std::min<unsigned long long>(hc.n_deep, deep_cap) - from;
      if (nd <= 0 || hc.err) return GQ_OK;
      const DeepSel deep{nullptr, deep_cap, dl + from, nd, nullptr, 0, 0};
      const int db = (int)std::min<int64_t>((nd + kSomWaves - 1) / kSomWaves, 64);
      hipLaunchKernelGGL(variant_support_call<true>, dim3((unsigned)db), dim3(kBlock), 0, c->stream,
                         (const Tile *)c->tiles.p, pl.n_tiles, pl.n_loci, rd->d, (VsRec *)c->srecs.p, rec_cap,
                         (uint8_t *)c->pool.p, pool_cap, ctr, ain ? (AmbItem *)nullptr : (AmbItem *)c->amb.p,
                         ain ? (unsigned long long)0 : amb_cap, ain, aref, n_ain, deep);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      return GQ_OK;
    };
    hipLaunchKernelGGL(variant_support_call<false>, dim3((unsigned)blocks), dim3(kBlock), 0, c->stream,
                       (const Tile *)c->tiles.p, pl.n_tiles, pl.n_loci, rd->d, (VsRec *)c->srecs.p, rec_cap,
                       (uint8_t *)c->pool.p, pool_cap, ctr, (AmbItem *)c->amb.p, amb_cap, (const AmbItem *)nullptr,
                       (const uint8_t *)nullptr, (int64_t)0, fast);
    HIP_TRY(hipGetLastError());
    st = run_deep(0, nullptr, nullptr, 0);
    if (st) return fail(st);
    bool retry = false;
    if (hc.n_amb > amb_cap) {
      amb_cap = hc.n_amb + 1024;
      retry = true;
    }
    if (hc.n_deep > deep_cap) {
      deep_cap = hc.n_deep + 1024;
      retry = true;
    }
    if (!retry && hc.n_amb > 0 && !hc.err) {  // heap-order reference bases: replay, then redo those loci
      std::vector<AmbItem> amb((size_t)hc.n_amb);
      HIP_TRY(hipMemcpyAsync(amb.data(), c->amb.p, amb.size() * sizeof(AmbItem), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(c->amb_ref.ensure(amb.size()));
      st = heap_ref_bases(c, pl, c->tiles, {rd}, amb, (uint8_t *)c->amb_ref.p);
      if (st) return fail(st);
      const int ab = (int)std::min<int64_t>(((int64_t)amb.size() + kSomWaves - 1) / kSomWaves, 8192);
      const int64_t from = (int64_t)hc.n_deep;
      hipLaunchKernelGGL(variant_support_call<false>, dim3((unsigned)ab), dim3(kBlock), 0, c->stream,
                         (const Tile *)c->tiles.p, pl.n_tiles, pl.n_loci, rd->d, (VsRec *)c->srecs.p, rec_cap,
                         (uint8_t *)c->pool.p, pool_cap, ctr, (AmbItem *)nullptr, (unsigned long long)0,
                         (const AmbItem *)c->amb.p, (const uint8_t *)c->amb_ref.p, (int64_t)amb.size(), fast);
      HIP_TRY(hipGetLastError());
      st = run_deep(from, (const AmbItem *)c->amb.p, (const uint8_t *)c->amb_ref.p, (int64_t)amb.size());
      if (st) return fail(st);
      if (hc.n_deep > deep_cap) {
        deep_cap = hc.n_deep + 1024;
        retry = true;
      }
    }
    if (hc.n_rec > rec_cap) {
      rec_cap = hc.n_rec + 1024;
      retry = true;
    }
    if (hc.pool_used > pool_cap) {
      pool_cap = hc.pool_used + 4096;
      retry = true;
    }
    if (!retry || hc.err) break;
    if (attempt == 2) return fail(set_err(GQ_E_CAPACITY, "variant-support output capacity retries exhausted"));
  }
  HIP_TRY(hipEventRecord(c->ev[2], c->stream));
  st = check_device_error(c, hc);
  if (st) return fail(st);
  const int64_t nr = pl.n_tiles > 0 ? (int64_t)hc.n_rec : 0;
  std::vector<VsRec> recs((size_t)nr);
  std::vector<uint8_t> hpool((size_t)std::min<unsigned long long>(hc.pool_used, pool_cap));
  if (nr) HIP_TRY(hipMemcpyAsync(recs.data(), c->srecs.p, (size_t)nr * sizeof(VsRec), hipMemcpyDeviceToHost, c->stream));
  if (!hpool.empty()) HIP_TRY(hipMemcpyAsync(hpool.data(), c->pool.p, hpool.size(), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  // loci in call order; a locus's alleles by (ref, alt) bytes (the reference iterates a HashMap)
  auto bytes = [&](const VsRec &r) {
    std::string b((size_t)(r.ref_len + r.alt_len), '\0');
    for (int i = 0; i < r.ref_len + r.alt_len; ++i)
      b[(size_t)i] = (char)(r.ref_len + r.alt_len <= 8 ? (uint8_t)(r.allele >> (8 * i)) : hpool[(size_t)r.allele + (size_t)i]);
    return b;
  };
  std::vector<std::string> ab((size_t)nr);
  for (int64_t k = 0; k < nr; ++k) ab[(size_t)k] = bytes(recs[(size_t)k]);
  std::vector<int64_t> ord((size_t)nr);
  for (int64_t k = 0; k < nr; ++k) ord[(size_t)k] = k;
  std::sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) {
    const VsRec &a = recs[(size_t)x], &b = recs[(size_t)y];
    if (a.key != b.key) return a.key < b.key;
    const std::string ra = ab[(size_t)x].substr(0, a.ref_len), rb2 = ab[(size_t)y].substr(0, b.ref_len);
    if (ra != rb2) return ra < rb2;
    return ab[(size_t)x].substr(a.ref_len) < ab[(size_t)y].substr(b.ref_len);
  });
  const size_t N = (size_t)std::max<int64_t>(nr, 1);
  res->n = nr;
  res->contig = (int32_t *)malloc(N * 4);
  res->pos = (int64_t *)malloc(N * 8);
  res->sample = (int32_t *)malloc(N * 4);
  res->count = (int32_t *)malloc(N * 4);
  res->ref_off = (int64_t *)malloc(N * 8);
  res->alt_off = (int64_t *)malloc(N * 8);
  res->ref_len = (int32_t *)malloc(N * 4);
  res->alt_len = (int32_t *)malloc(N * 4);
  res->flags = (uint8_t *)malloc(N);
  std::string apool;
  for (int64_t q = 0; q < nr; ++q) {
    const int64_t k = ord[(size_t)q];
    const VsRec &r = recs[(size_t)k];
    res->contig[q] = r.contig;
    res->pos[q] = r.pos;
    res->sample[q] = r.sample;
    res->count[q] = r.count;
    res->ref_len[q] = r.ref_len;
    res->alt_len[q] = r.alt_len;
    res->ref_off[q] = (int64_t)apool.size();
    res->alt_off[q] = (int64_t)apool.size() + r.ref_len;
    res->flags[q] = r.flags;
    apool += ab[(size_t)k];
  }
  res->pool_len = (int64_t)apool.size();
  res->allele_pool = (uint8_t *)malloc(std::max<size_t>(apool.size(), 1));
  if (!apool.empty()) memcpy(res->allele_pool, apool.data(), apool.size());
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[2]);
  c->timings.pileup_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[2]);
  c->timings.total_ms = ms;
  c->timings.tiles = pl.n_tiles;
  c->timings.host_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - h0).count();
  *out = res;
  return GQ_OK;
}

void gq_free_allele_counts(gq_allele_counts *r) {
  if (!r) return;
  free(r->contig);
  free(r->pos);
  free(r->sample);
  free(r->count);
  free(r->ref_off);
  free(r->alt_off);
  free(r->ref_len);
  free(r->alt_len);
  free(r->allele_pool);
  free(r->flags);
  free(r);
}

gq_status gq_germline_standard(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, const gq_germline_std_params *p,
                               gq_somatic_calls **out) {
  if (!c || !rd || !loci || !p || !out) return set_err(GQ_E_ARG, "gq_germline_standard: null argument");
  HIP_TRY(hipSetDevice(c->device));
  const auto h0 = std::chrono::steady_clock::now();
  c->timings = gq_timings{};
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  Plan pt;
  const MarginReq mreq{(int)p->min_mapq, false};  // (with the projection, the margin projection in the same pass)
  gq_status st = ensure_projection(c, rd, &mreq);  // (derived on first use)
  if (st) return st;
  st = plan(c, rd, loci, SomProjCfg::kT, pt, c->tiles, 0, 0, 0, true);
  if (st) return st;
  gq_somatic_calls *res = (gq_somatic_calls *)calloc(1, sizeof(gq_somatic_calls));
  if (!res) return set_err(GQ_E_NOMEM, "calloc");
  auto fail = [&](gq_status e) {
    free(res);
    return e;
  };
  if (pt.n_tiles == 0) {
    *out = res;
    return GQ_OK;
  }
  {
    double succ[256];
    for (int q = 0; q < 256; ++q) succ[q] = 1.0 - std::pow(10.0, -q / 10.0);
    HIP_TRY(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_succ), succ, sizeof succ, 0, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  SomWin sw{};
  st = build_somwin(c, pt, rd, rd, sw);
  if (st) return fail(st);
  // the hom-ref bound with probabilityCorrectIgnoringAlignment; with several samples the bound
  // over the pooled elements proves nothing per sample, so every non-Match locus is a candidate
  st = ensure_margin_projection(c, rd, (int)p->min_mapq, false);
  if (st) return fail(st);
  const int no_bound = rd->d.n_samples > 1 ? 1 : 0;
  const bool direct = false;  // (germline-standard keeps somatic_proj over its margin projection)
  OutGeom og{};
  {
    if (c->n_cu <= 0 &&
        hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess)
      c->n_cu = 256;
    int &wg_cu = direct ? c->somd_wg_per_cu : c->som_wg_per_cu;
    if (wg_cu <= 0) {
      int nb = 0;
      const hipError_t e =
          direct ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, somatic_direct<false>, SomDirCfg::kThreads, 0)
                 : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, somatic_proj<false>, SomProjCfg::kThreads, 0);
      if (e != hipSuccess || nb <= 0) nb = direct ? 2 : 4;
      wg_cu = nb;
    }
    og.ncols = (int)std::max<int64_t>(1, std::min<int64_t>({(pt.n_tiles + SomProjCfg::kWaves - 1) / SomProjCfg::kWaves,
                                                           (int64_t)wg_cu * c->n_cu, (int64_t)kPartsCols}));
    const unsigned long long wg_loci = (unsigned long long)((pt.n_tiles + og.ncols - 1) / og.ncols) * SomProjCfg::kT;
    og.capA[1] = wg_loci / 16 + 256;
    og.capB[1] = (unsigned long long)pt.n_loci / 65536 + 1024;
  }
  unsigned long long rec_cap = 1 << 16, pool_cap = 1 << 20, amb_cap = 4096, deep_cap = 4096;
  Counters hc{};
  for (int attempt = 0; attempt < 3; ++attempt) {
    HIP_TRY(c->amb.ensure(amb_cap * sizeof(AmbItem)));
    HIP_TRY(c->cplx.ensure(og.total(1) * sizeof(ComplexItem)));
    HIP_TRY(c->srecs.ensure(rec_cap * sizeof(SomRec)));
    HIP_TRY(c->pool.ensure(pool_cap));
    HIP_TRY(c->slow.ensure((size_t)pt.n_tiles * sizeof(int32_t)));
    HIP_TRY(c->counters.ensure(sizeof(Counters)));
    Counters *ctr = (Counters *)c->counters.p;
    HIP_TRY(hipMemsetAsync(ctr, 0, sizeof(Counters), c->stream));
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    hipLaunchKernelGGL(somatic_proj<false>, dim3((unsigned)og.ncols), dim3(SomProjCfg::kThreads), 0, c->stream,
                       (const Tile *)c->tiles.p, (const Tile *)c->tiles.p, pt.n_tiles, rd->d, (const uint8_t *)rd->mproj, (const uint8_t *)rd->mnb,
                       rd->d.start, rd->d.end, (ComplexItem *)c->cplx.p, og, ctr, (int32_t *)c->slow.p,
                       RefView{nullptr, nullptr}, no_bound);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL((somatic_tile<SomProjCfg::kT>), dim3((unsigned)std::min<int64_t>(pt.n_tiles, 2048)), dim3(kBlock), 0,
                       c->stream, (const Tile *)c->tiles.p, (const Tile *)c->tiles.p, rd->d, rd->d, (ComplexItem *)c->cplx.p,
                       og, (const int32_t *)c->slow.p, (int)p->min_mapq, ctr, RefView{nullptr, nullptr}, 1);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(part_scan_som, dim3(1), dim3(1024), 0, c->stream, ctr, og);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    {
      unsigned long long pm = 0;
      HIP_TRY(hipMemcpyAsync(&pm, &ctr->part_max[1], sizeof(pm), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      if (pm) {
        og.capA[1] += pm + 64;
        og.capB[1] += pm + 64;
        if (attempt == 2) return fail(set_err(GQ_E_CAPACITY, "candidate capacity retries exhausted"));
        continue;
      }
    }
    const int cblocks = (int)std::min<int64_t>(std::max<int64_t>(pt.n_tiles, 1), 8192);
    HIP_TRY(c->deep_list.ensure(deep_cap * sizeof(int64_t)));
    int64_t *dl = (int64_t *)c->deep_list.p;
    const DeepSel fast{dl, deep_cap, nullptr, 0, nullptr, 0, 0};
    // the loci the fast working set handed over [from, hc.n_deep): the deep instantiation, same
    // mode, its per-wave scratch sized from the deepest of them and their largest allele table
    auto run_deep = [&](int64_t from, AmbItem *aout, unsigned long long acap, const AmbItem *ain, const uint8_t *aref,
                        int64_t n_ain) -> gq_status {
      HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      const int64_t nd = (int64_t)std::min<unsigned long long>(hc.n_deep, deep_cap) - from;
      if (nd <= 0 || hc.err) return GQ_OK;
      const int scap = (int)std::max<unsigned long long>(hc.deep_max, 64);
      const int64_t nt = (int64_t)std::min<unsigned long long>(std::max<unsigned long long>(hc.deep_nt, 2), 64 * kDeepNS);
      const int maxG = (int)std::max<int64_t>(nt * (nt + 1) / 2, 16);
      const int64_t waves = std::min<int64_t>(nd, 256);
      HIP_TRY(c->deep_scratch.ensure((size_t)waves * gs_wave_bytes(scap, maxG) + 256));
      const DeepSel deep{nullptr, deep_cap, dl + from, nd, (uint8_t *)c->deep_scratch.p, scap, maxG};
      hipLaunchKernelGGL(germline_standard_call<true>, dim3((unsigned)((waves + kSomWaves - 1) / kSomWaves)),
                         dim3(kBlock), 0, c->stream, (const Tile *)c->tiles.p, (const ComplexItem *)c->cplx.p, rd->d, *p,
                         (SomRec *)c->srecs.p, rec_cap, (uint8_t *)c->pool.p, pool_cap, og, ctr, sw, aout, acap, ain,
                         aref, n_ain, deep);
      HIP_TRY(hipGetLastError());
      HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      return GQ_OK;
    };
    hipLaunchKernelGGL(germline_standard_call<false>, dim3(cblocks), dim3(kBlock), 0, c->stream, (const Tile *)c->tiles.p,
                       (const ComplexItem *)c->cplx.p, rd->d, *p, (SomRec *)c->srecs.p, rec_cap, (uint8_t *)c->pool.p,
                       pool_cap, og, ctr, sw, (AmbItem *)c->amb.p, amb_cap, (const AmbItem *)nullptr,
                       (const uint8_t *)nullptr, (int64_t)0, fast);
    HIP_TRY(hipGetLastError());
    st = run_deep(0, (AmbItem *)c->amb.p, amb_cap, nullptr, nullptr, 0);
    if (st) return fail(st);
    HIP_TRY(hipEventRecord(c->ev[3], c->stream));
    bool retry = false;
    if (hc.n_amb > amb_cap) {
      amb_cap = hc.n_amb + 1024;
      retry = true;
    }
    if (hc.n_deep > deep_cap) {
      deep_cap = hc.n_deep + 1024;
      retry = true;
    }
    if (!retry && hc.n_amb > 0 && !hc.err) {  // heap-order reference bases: replay, then those loci again
      std::vector<AmbItem> amb((size_t)hc.n_amb);
      HIP_TRY(hipMemcpyAsync(amb.data(), c->amb.p, amb.size() * sizeof(AmbItem), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(c->amb_ref.ensure(amb.size()));
      st = heap_ref_bases(c, pt, c->tiles, {rd}, amb, (uint8_t *)c->amb_ref.p);
      if (st) return fail(st);
      const int ablocks = (int)std::min<int64_t>(((int64_t)amb.size() + 3) / 4, 8192);
      const int64_t from = (int64_t)hc.n_deep;
      hipLaunchKernelGGL(germline_standard_call<false>, dim3(ablocks), dim3(kBlock), 0, c->stream,
                         (const Tile *)c->tiles.p, (const ComplexItem *)c->cplx.p, rd->d, *p, (SomRec *)c->srecs.p,
                         rec_cap, (uint8_t *)c->pool.p, pool_cap, og, ctr, sw, (AmbItem *)nullptr,
                         (unsigned long long)0, (const AmbItem *)c->amb.p, (const uint8_t *)c->amb_ref.p,
                         (int64_t)amb.size(), fast);
      HIP_TRY(hipGetLastError());
      st = run_deep(from, (AmbItem *)nullptr, (unsigned long long)0, (const AmbItem *)c->amb.p,
                    (const uint8_t *)c->amb_ref.p, (int64_t)amb.size());
      if (st) return fail(st);
      HIP_TRY(hipEventRecord(c->ev[3], c->stream));
      if (hc.n_deep > deep_cap) {
        deep_cap = hc.n_deep + 1024;
        retry = true;
      }
    }
    if (hc.n_rec > rec_cap) {
      rec_cap = hc.n_rec + 1024;
      retry = true;
    }
    if (hc.pool_used > pool_cap) {
      pool_cap = hc.pool_used + 4096;
      retry = true;
    }
    if (!retry) break;
    if (attempt == 2) return fail(set_err(GQ_E_CAPACITY, "output capacity retries exhausted"));
  }
  for (int k = 0; k < kSpread; ++k) hc.visited += hc.spread[0][k];
  st = check_device_error(c, hc);
  if (st) return fail(st);
  st = fetch_somatic_records(c, hc, pool_cap, (uint64_t)std::max<int64_t>(pt.n_loci, 1) << 12, res);
  if (st) return fail(st);
  res->visited_loci = (int64_t)hc.visited;
  res->candidate_loci = (int64_t)hc.n_complex;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[2]);
  c->timings.pileup_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
  c->timings.complex_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[3], c->ev[4]);
  c->timings.finalize_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[4]);
  c->timings.total_ms = ms;
  c->timings.tiles = pt.n_tiles;
  c->timings.host_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - h0).count();
  *out = res;
  return GQ_OK;
}

void gq_free_somatic(gq_somatic_calls *r) {
  if (!r) return;
  if (r->block_) {  // one block holds every array (fetch_somatic_records)
    free(r->block_);
    free(r);
    return;
  }
  free(r->contig);
  free(r->pos);
  free(r->sample);
  free(r->ref_off);
  free(r->alt_off);
  free(r->ref_len);
  free(r->alt_len);
  free(r->allele_pool);
  free(r->log_odds);
  free(r->gq);
  free(r->tumor);
  free(r->normal);
  free(r->flags);
  free(r);
}

}  // extern "C"

namespace {
__global__ void warm_k() {}
}  // namespace
hipError_t gq::warm_somatic(hipStream_t s) {
  hipLaunchKernelGGL(warm_k, dim3(1), dim3(64), 0, s);
  return hipGetLastError();
}
