// gq_germline_common.h — the pieces of the germline-threshold path shared by its kernels:
// germline_decide (the GermlineThreshold decision over a tile's LDS histogram, for the walker),
// germline_expand (variant candidates -> Genotype records), the run counters, and
// germline_walk (the lane-per-read walker for the tiles germline_proj hands over).
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
struct LdsOut {  // one partition per workgroup, counters in LDS
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
  // reg (one locus per thread): this thread's locus's A C T G N counts held in
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
    // (ref C with G and N alleles present: their Scala map order depends on first occurrences,
    // gq_scala_order.h; germline_complex decides those)
    const bool cgn = low == 2u && c[3] > 0 && c[4] > 0;
    const bool to_complex = (wide && in) || (live && (ambiguous || cx > 0 || multi_sample || cgn));
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
// Allele (ref, b) keys: count << 16 | (255 - Scala map rank) << 8 | category: sorting the keys
// descending = sortBy(-count), a stable sort of the counts map's iteration order
// (GermlineThresholdCaller.scala:103-104, gq_scala_order.h).  Unused slots get a key past
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
    // categories: (ref, A) (ref, C) (ref, T) (ref, G) (ref, N), and 5 the MidDeletion allele
    // (ref, "") (Alignment.scala:87-92; its count in alt_len)
    constexpr int NC = 6;
    const uint32_t c[NC] = {(uint32_t)(cand.allele & 0xFFFFu), (uint32_t)((cand.allele >> 16) & 0xFFFFu),
                            (uint32_t)((cand.allele >> 32) & 0xFFFFu), (uint32_t)(cand.allele >> 48), cand.ref_len,
                            cand.alt_len};
    const uint32_t depth = c[0] + c[1] + c[2] + c[3] + c[4] + c[5];
    const uint8_t ref = cand.gt0;
    // the counts map's Scala order over the alleles present: up to four, the mutable map's
    // (bucket descending; no two share a bucket here: the pairs that could went to
    // germline_complex), five or more: the HashTrieMap's (gq_scala_order.h)
    int npres = 0;
#pragma unroll
    for (int cat = 0; cat < NC; ++cat) npres += c[cat] > 0 ? 1 : 0;
    uint64_t sk[NC];
#pragma unroll
    for (int cat = 0; cat < NC; ++cat) {
      scala::SeqHasher hr, ha;
      hr.add_byte(ref);
      if (cat < 5) ha.add_byte(cat_base(cat));
      const uint32_t h = scala::allele_hash(hr.result(), ha.result());
      sk[cat] = npres <= 4 ? (uint64_t)(15u - scala::mutable_bucket(h, 4)) : scala::trie_key(h);
    }
    uint32_t k0 = 0, k1 = 0, k2 = 0;  // top three passing keys: count << 16 | (255 - map rank) << 8 | category
    int npass = 0;
#pragma unroll
    for (int cat = 0; cat < NC; ++cat) {
      const uint32_t cc = c[cat];
      if (cc == 0 || !passes(cc, depth)) continue;
      ++npass;
      int rank = 0;
#pragma unroll
      for (int o = 0; o < NC; ++o)
        if (o != cat && c[o] > 0 && (sk[o] < sk[cat] || (sk[o] == sk[cat] && o < cat))) ++rank;
      uint32_t key = (cc << 16) | ((uint32_t)(255 - rank) << 8) | (uint32_t)cat;
      if (key > k0) { const uint32_t t = k0; k0 = key; key = t; }
      if (key > k1) { const uint32_t t = k1; k1 = key; key = t; }
      if (key > k2) { k2 = key; }
    }
    const bool tie = npass >= 2 && ((k0 >> 16) == (k1 >> 16) || (npass >= 3 && (k1 >> 16) == (k2 >> 16)));
    if (tie) ++ties;
    const uint8_t fl = tie ? GQ_FLAG_TIE : 0;
    // the case split (GermlineThresholdCaller.scala:118-176) -> up to two records (g0, g1, the
    // allele's category or the symbolic <ALT>).  Allele.isVariant: ref != alt; the MidDeletion
    // allele (ref, "") is a variant with an empty alt.
    const int t0 = (int)(k0 & 0xFFu), t1 = (int)(k1 & 0xFFu);
    auto is_var = [&](int cat) { return cat == 5 || cat_base(cat) != ref; };
    int nout = 0, aa = 0, ab = 0;
    uint8_t ga0 = 0, ga1 = 0, gb0 = 0, gb1 = 0;
    bool syma = false;
    if (npass == 0) {
      if (emit_no_call) nout = 1, ga0 = ga1 = GQ_GT_NOCALL, syma = true;
    } else if (npass == 1 && !is_var(t0)) {
      if (emit_ref) nout = 1, ga0 = ga1 = GQ_GT_REF, syma = true;
    } else if (npass == 1) {
      nout = 1, ga0 = ga1 = GQ_GT_ALT, aa = t0;
    } else {
      const bool v1 = is_var(t0), v2 = is_var(t1);
      if ((!v1 || !v2) && ((t0 == 5) != (t1 == 5))) {
        // heterozygous deletion (an empty alt beside a non-variant allele): no record
      } else if (v1 != v2) {
        nout = 1, ga0 = GQ_GT_REF, ga1 = GQ_GT_ALT, aa = v1 ? t0 : t1;
      } else if (v1 && v2) {
        nout = 2, ga0 = gb0 = GQ_GT_ALT, ga1 = gb1 = GQ_GT_OTHERALT, aa = t0, ab = t1;
      }
      // two non-variant alleles cannot occur (every Match allele is (ref, ref))
    }
    // the pair's two slots are consecutive in the partition (reserved together); an unused
    // slot gets the dead key.  Records are written as two 16-byte halves (CallRec layout).
    auto put = [&](unsigned long long at, bool live, int sub, uint8_t g0, uint8_t g1, int cat, bool sym) {
      const uint64_t key = live ? (cand.key | (uint64_t)sub) : dead_key;
      const uint32_t alt_len = sym ? 5u : cat == 5 ? 0u : 1u;
      const uint64_t allele = sym ? ((uint64_t)ref | kAltSym)
                                  : ((uint64_t)ref | (cat == 5 ? 0ull : (uint64_t)cat_base(cat) << 8));
      const uint32_t w3 = (uint32_t)cand.sample | ((uint32_t)g0 << 8) | ((uint32_t)g1 << 16) |
                          ((uint32_t)(live ? fl : 0) << 24);
      const uint32_t w4 = 1u | (alt_len << 16);  // ref_len 1, alt_len
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

// The tiles germline_proj handed over: every read walked lane-per-read (walk_read_lane,
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
