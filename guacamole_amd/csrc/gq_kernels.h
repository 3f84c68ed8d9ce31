// gq_kernels.h — device-side building blocks shared by the pileup kernels.
//
// Element semantics restate PileupElement.alignment / advanceToLocus
// (/root/reference/src/main/scala/org/hammerlab/guacamole/pileup/PileupElement.scala:68-248)
// and Pileup.referenceBaseAtLocus (pileup/Pileup.scala:157-165).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gq {

enum : int { OP_M = 0, OP_I = 1, OP_D = 2, OP_N = 3, OP_S = 4, OP_H = 5, OP_P = 6, OP_EQ = 7, OP_X = 8 };

__device__ __forceinline__ bool consumes_ref(int op) {
  return op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X;
}
__device__ __forceinline__ bool consumes_read(int op) {
  return op == OP_M || op == OP_I || op == OP_S || op == OP_EQ || op == OP_X;
}

// element kinds (pileup/Alignment.scala:32-94)
enum : int { K_SNV = 0, K_INS = 1, K_DEL = 2, K_MID = 3, K_CLIP = 4 };
// SNV = Match or Mismatch (decided against the pileup reference base later)

// Device view of a resident read set (device pointers).
struct DevReads {
  int64_t n_reads;
  int32_t n_contigs, n_samples;
  const int64_t *contig_read_begin;
  const int32_t *start, *end, *pmax_end;
  const uint8_t *mapq, *flags, *sample;
  const int64_t *seq_off;
  const int32_t *seq_len;
  const int64_t *cigar_off;
  const int32_t *n_cigar;
  const int64_t *md_off;
  const int32_t *n_md;
  const uint16_t *n_mismatch;
  const uint8_t *seq, *qual;
  const uint32_t *cigar, *md_ev;
};

// One locus tile: contiguous loci [L0, L1) of one contig, plus the index range
// [rb, re) of reads that can overlap it (pmax_end > L0, start < L1).
struct Tile {
  int64_t ordinal0;  // output ordinal of L0 (position in the concatenated loci ranges)
  int64_t rb, re;
  int32_t contig, L0, L1, range;
};

// Per-call record written by the germline kernels, sorted by `key` afterwards.
struct CallRec {
  uint64_t key;  // ordinal << 12 | sample << 4 | sub
  int32_t contig;
  int32_t pos;
  uint8_t sample, gt0, gt1, flags;
  uint16_t ref_len, alt_len;
  uint64_t allele;  // inline bytes (ref then alt) if ref_len + alt_len <= 8, else pool offset
};
static_assert(sizeof(CallRec) == 32, "CallRec layout");

struct ComplexItem {
  int32_t tile;
  int32_t pos;
};

enum : int { ERR_NONE = 0 };

__device__ __forceinline__ void raise_error(int *err, int64_t *err_pos, int code, int64_t where) {
  if (atomicCAS(err, 0, code) == 0) *err_pos = where;
}

__device__ __forceinline__ int base_cat(uint8_t b) {
  switch (b) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    case 'N': return 4;
    default: return 5;
  }
}
__device__ __forceinline__ uint32_t std_bit(uint8_t b) {
  switch (b) {
    case 'A': return 1u;
    case 'C': return 2u;
    case 'G': return 4u;
    case 'T': return 8u;
    default: return 0u;
  }
}
__device__ __forceinline__ uint8_t bit_base(uint32_t m) {  // lowest set bit of a std mask -> base
  return (m & 1u) ? 'A' : (m & 2u) ? 'C' : (m & 4u) ? 'G' : 'T';
}

// MD event lookup for reference offset `off` (events sorted by offset).
__device__ __forceinline__ int md_find(const uint32_t *ev, int32_t n, int32_t off) {
  int lo = 0, hi = n;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    int32_t o = (int32_t)(ev[mid] >> 8);
    if (o < off) lo = mid + 1;
    else hi = mid;
  }
  if (lo < n && (int32_t)(ev[lo] >> 8) == off) return (int)(ev[lo] & 0xFFu);
  return -1;
}

// Wave-cooperative walk of one read's CIGAR over the loci [L0, L1): lanes take 64
// consecutive loci of each reference-consuming op.  `sink.elem(l, kind, base, mdb, ev)`
// receives every pileup element (l, kind), the sequenced base for SNV/anchor
// elements, the read's MD-derived reference base at l (MDTagUtils.getReference),
// and whether an MD event (mismatch / deleted base) sits at l.
template <class Sink>
__device__ __forceinline__ void walk_read(const DevReads &R, int64_t r, int32_t L0, int32_t L1, Sink &sink) {
  const int lane = threadIdx.x & 63;
  const int32_t s = R.start[r];
  const int32_t e = R.end[r];
  if (e <= L0 || s >= L1) return;
  const int64_t seq_off = R.seq_off[r];
  const int32_t slen = R.seq_len[r];
  const int64_t cig_off = R.cigar_off[r];
  const int32_t ncig = R.n_cigar[r];
  const int64_t md_off = R.md_off[r];
  const int32_t nmd = R.n_md[r];
  const uint8_t fl = R.flags[r];
  if (nmd < 0) {  // MappedRead.mdTagReferenceBases on a read without MD (MappedRead.scala:57-60)
    sink.error(4 /*GQ_E_NO_MD*/, ((int64_t)s));
    return;
  }
  const uint32_t *ev = R.md_ev + md_off;
  // events preloaded into lanes (first 64); longer lists fall back to a binary search
  const uint32_t ev_lane = lane < nmd ? ev[lane] : 0xFFFFFFFFu;
  const int nev_reg = nmd < 64 ? nmd : 64;

  int32_t ref = s;
  int32_t rpos = 0;
  bool lead_ins = false;  // I before any reference-consuming op on a read at locus 0 (PileupElement.scala:102-103, 240-245)
  bool seen_ref = false;
  for (int k = 0; k < ncig; ++k) {
    const uint32_t c = R.cigar[cig_off + k];
    const int op = (int)(c & 15u);
    const int32_t len = (int32_t)(c >> 4);
    const int nextop = (k + 1 < ncig) ? (int)(R.cigar[cig_off + k + 1] & 15u) : -1;
    if (op == OP_I && !seen_ref && s == 0) lead_ins = true;
    if (op == OP_P) sink.error(1 /*GQ_E_ASSERT*/, (int64_t)ref);
    if (consumes_ref(op)) {
      seen_ref = true;
      const int32_t a = ref > L0 ? ref : L0;
      const int32_t b = (ref + len) < L1 ? (ref + len) : L1;
      for (int32_t l0 = a; l0 < b; l0 += 64) {
        const int32_t l = l0 + lane;
        const int32_t off = l - s;
        // MD event at this reference offset (all lanes participate: readlane is uniform)
        int mdv = -1;
        for (int j = 0; j < nev_reg; ++j) {
          const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)ev_lane, j);
          if ((int32_t)(v >> 8) == off) mdv = (int)(v & 0xFFu);
        }
        if (nmd > 64 && mdv < 0 && l < b) mdv = md_find(ev, nmd, off);
        if (l < b) {
          if (op == OP_M || op == OP_EQ || op == OP_X) {
            const int32_t rp = rpos + (l - ref);
            uint8_t base = 0;
            if (rp < slen) base = R.seq[seq_off + rp];
            else sink.error(1, (int64_t)l);
            const bool fin = (l == ref + len - 1);
            int kind = K_SNV;
            if (lead_ins && l == 0) kind = K_INS;
            else if (fin && (op == OP_M || op == OP_EQ) && nextop == OP_I) kind = K_INS;
            else if (fin && nextop == OP_D) kind = K_DEL;
            const uint8_t mdb = mdv >= 0 ? (uint8_t)mdv : base;
            sink.elem(l, kind, base, mdb, mdv >= 0, fl);
          } else if (op == OP_D) {
            if (mdv < 0) sink.error(3 /*GQ_E_MD*/, (int64_t)l);
            sink.elem(l, K_MID, (uint8_t)0, mdv >= 0 ? (uint8_t)mdv : (uint8_t)'N', true, fl);
          } else {  // N: Clipped, MD-derived reference 'N'
            sink.elem(l, K_CLIP, (uint8_t)0, (uint8_t)'N', false, fl);
          }
        }
      }
      ref += len;
    }
    if (consumes_read(op)) rpos += len;
    if (ref >= L1) break;
  }
}

}  // namespace gq
