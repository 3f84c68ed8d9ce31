// gq_alleles.h — exact per-element classification and allele identity on device
// (PileupElement.alignment, PileupElement.scala:68-135; Allele, variants/Allele.scala:26-43;
// MappedRead.getReferenceBaseAtLocus, reads/MappedRead.scala:57-76).  Used by the
// general-allele germline kernel and the somatic candidate kernel.
#pragma once
#include "gq_kernels.h"
#include "gq_scala_order.h"

namespace gq {
namespace {

struct AlleleDesc {  // enough to regenerate an allele's bytes
  int64_t read;      // read index (for INS / DEL / MID byte access)
  int32_t aux;       // INS: number of alt bytes; DEL: deleted length
  int32_t rp;        // INS: first alt byte position in the read
  uint8_t kind;
  uint8_t rb;        // pileup ref base (SNV / DEL)
  uint8_t base;      // SNV sequenced base / MID deleted base
  uint8_t pad;
};

__device__ __forceinline__ int allele_ref_len(const AlleleDesc &d) {
  switch (d.kind) {
    case K_SNV: return 1;
    case K_INS: return d.aux > 0 ? 1 : 0;
    case K_DEL: return 1 + d.aux;
    case K_MID: return 1;
    default: return 0;
  }
}
__device__ __forceinline__ int allele_alt_len(const AlleleDesc &d) {
  switch (d.kind) {
    case K_SNV: return 1;
    case K_INS: return d.aux;
    case K_DEL: return 1;
    default: return 0;
  }
}
// Byte i of the ref (which=0) / alt (which=1) allele.  DEL bytes 1.. come from the
// read's MD deletion events at pos+1.. (PileupElement.scala:108-114).
__device__ __forceinline__ uint8_t allele_byte(const DevReads &R, const AlleleDesc &d, int32_t pos, int which, int i) {
  switch (d.kind) {
    case K_SNV: return which == 0 ? d.rb : d.base;
    case K_INS: {
      const uint8_t *s = R.seq + R.seq_off[d.read];
      return which == 0 ? s[d.rp] : s[d.rp + i];
    }
    case K_DEL: {
      if (which == 1 || i == 0) return d.rb;
      const int32_t s = R.start[d.read];
      const int v = md_find(R.md_ev + R.md_off[d.read], R.n_md[d.read], pos + i - s);
      return v < 0 ? (uint8_t)'?' : (uint8_t)v;
    }
    case K_MID: return d.base;
    default: return 0;
  }
}

// An allele's bytes (ref then alt, little-endian in w) gathered with every load of the
// allele issued together, instead of one dependent load chain per byte (allele_byte; a
// deletion's bytes after the first each took an MD search).  ok = false when ref + alt is
// longer than 13 bytes: callers then take allele_byte.
struct AlleleBytes {
  uint32_t w[4];
  int rl, al;
  bool ok;
  // byte k of ref ++ alt (k a compile-time constant after unrolling: no indexed array)
  __device__ __forceinline__ uint8_t byte(int k) const { return (uint8_t)(w[k >> 2] >> (8 * (k & 3))); }
};
__device__ __forceinline__ AlleleBytes allele_bytes(const DevReads &R, const AlleleDesc &d, int32_t pos) {
  AlleleBytes a;
  a.rl = allele_ref_len(d);
  a.al = allele_alt_len(d);
  a.w[0] = a.w[1] = a.w[2] = a.w[3] = 0;
  const int n = a.rl + a.al;
  a.ok = n <= 13;  // key_from's exact packing (longer alleles: allele_byte)
  if (!a.ok) return a;
  uint32_t b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) b[i] = 0;
  if (d.kind == K_SNV) {
    b[0] = d.rb;
    b[1] = d.base;
  } else if (d.kind == K_MID) {
    b[0] = d.base;
  } else if (d.kind == K_INS) {
    // ref: the anchor s[0] (when aux > 0), alt: s[0 .. aux); reads past the read's end stay
    // inside the pool (its zeroed tail) and are masked off
    const uint8_t *sq = R.seq + R.seq_off[d.read] + d.rp;
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = sq[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) b[i] = i < n ? ((a.rl == 1 && i > 0) ? v[i - 1] : v[i]) : 0u;
  } else if (d.kind == K_DEL) {
    // ref: the pileup base, then the MD deleted bases at pos + 1 .. (consecutive events: one
    // search, then one batch of loads); alt: the pileup base
    const int64_t r = d.read;
    const uint32_t *ev = R.md_ev + R.md_off[r];
    const int32_t nmd = R.n_md[r], off = pos + 1 - R.start[r];
    int lo = 0, hi = nmd;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((int32_t)(ev[mid] >> 8) < off) lo = mid + 1;
      else hi = mid;
    }
    uint32_t e[15];
#pragma unroll
    for (int i = 0; i < 15; ++i) e[i] = nmd > 0 ? ev[min(lo + i, nmd - 1)] : 0u;
    b[0] = d.rb;
#pragma unroll
    for (int i = 0; i < 15; ++i) {
      const bool hit = lo + i < nmd && (int32_t)(e[i] >> 8) == off + i;
      if (1 + i < a.rl) b[1 + i] = hit ? (e[i] & 0xFFu) : (uint32_t)'?';
    }
#pragma unroll
    for (int i = 1; i < 16; ++i)
      if (i == a.rl) b[i] = d.rb;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) a.w[i >> 2] |= (b[i] & 0xFFu) << (8 * (i & 3));
  return a;
}

struct Key128 {
  uint64_t lo, hi;
};
// 128-bit allele identity: exact packing (lengths, sample, bytes) when ref + alt <= 13
// bytes, else two independent 64-bit hashes with marker 0xFFFF in the length bytes.
// byte(which, i) returns byte i of the ref (which = 0) or alt (which = 1) allele.
template <class F>
__device__ __forceinline__ Key128 key_from(int rl, int al, int sample, F byte) {
  Key128 k{0, 0};
  if (rl + al <= 13) {
    k.lo = (uint64_t)(uint8_t)rl | ((uint64_t)(uint8_t)al << 8) | ((uint64_t)(uint8_t)sample << 16);
    int j = 3;
    auto put = [&](uint8_t x) {
      if (j < 8) k.lo |= (uint64_t)x << (8 * j);
      else k.hi |= (uint64_t)x << (8 * (j - 8));
      ++j;
    };
    for (int i = 0; i < rl; ++i) put(byte(0, i));
    for (int i = 0; i < al; ++i) put(byte(1, i));
  } else {
    uint64_t h1 = 0xcbf29ce484222325ull ^ (uint64_t)rl, h2 = 0x9e3779b97f4a7c15ull ^ ((uint64_t)al << 32);
    auto mix = [&](uint8_t x) {
      h1 = (h1 ^ x) * 0x100000001b3ull;
      h2 = (h2 + x + 0x632be59bd9b4e019ull) * 0xff51afd7ed558ccdull;
      h2 ^= h2 >> 29;
    };
    for (int i = 0; i < rl; ++i) mix(byte(0, i));
    mix(0xFE);
    for (int i = 0; i < al; ++i) mix(byte(1, i));
    k.lo = (h1 & ~0xFFFFFFull) | 0xFFFFull | ((uint64_t)sample << 16);
    k.hi = h2;
  }
  return k;
}
// kGather: the bytes through allele_bytes (one batch of loads; more registers)
// key_from over gathered bytes, with every byte at a constant position (registers only)
__device__ __forceinline__ Key128 key_from_bytes(const AlleleBytes &ab, int sample) {
  Key128 k{0, 0};
  const uint64_t lo = (uint64_t)ab.w[0] | ((uint64_t)ab.w[1] << 32), hi = (uint64_t)ab.w[2] | ((uint64_t)ab.w[3] << 32);
  // key_from's exact packing (allele_bytes gathers n <= 13 only): lengths, sample, then the
  // bytes from byte 3
  k.lo = (uint64_t)(uint8_t)ab.rl | ((uint64_t)(uint8_t)ab.al << 8) | ((uint64_t)(uint8_t)sample << 16) | (lo << 24);
  k.hi = (lo >> 40) | (hi << 24);
  return k;
}
template <bool kGather = false>
__device__ __forceinline__ Key128 allele_key(const DevReads &R, const AlleleDesc &d, int32_t pos, int sample) {
  if constexpr (kGather) {
    const AlleleBytes ab = allele_bytes(R, d, pos);
    if (ab.ok) return key_from_bytes(ab, sample);
  }
  return key_from(allele_ref_len(d), allele_alt_len(d), sample,
                  [&](int which, int i) { return allele_byte(R, d, pos, which, i); });
}

// Allele ordering (variants/Allele.scala:31-36): ref string, then alt string.
__device__ __forceinline__ int allele_cmp(const DevReads &R, const AlleleDesc &a, const AlleleDesc &b, int32_t pos) {
  for (int which = 0; which < 2; ++which) {
    const int la = which ? allele_alt_len(a) : allele_ref_len(a);
    const int lb = which ? allele_alt_len(b) : allele_ref_len(b);
    const int n = la < lb ? la : lb;
    for (int i = 0; i < n; ++i) {
      const int x = allele_byte(R, a, pos, which, i), y = allele_byte(R, b, pos, which, i);
      if (x != y) return x < y ? -1 : 1;
    }
    if (la != lb) return la < lb ? -1 : 1;
  }
  return 0;
}

__device__ __forceinline__ int md_ref_at(const DevReads &R, int64_t r, int32_t pos);

// Locate the PileupElement of read r at `pos` (PileupElement.apply + advanceToLocus) and
// classify it (PileupElement.alignment).  Returns false and sets *errc on a reference error.
// With mdv != nullptr the same CIGAR walk also yields md_ref_at(R, r, pos) in *mdv (always
// set, also when classify fails).
__device__ __forceinline__ bool classify(const DevReads &R, int64_t r, int32_t pos, uint8_t refbase, AlleleDesc &d, int *errc,
                                         int *mdv = nullptr) {
  const int32_t s = R.start[r];
  const int64_t cig_off = R.cigar_off[r];
  const int32_t ncig = R.n_cigar[r];
  const int32_t slen = R.seq_len[r];  // loaded with the other scalars: the base load below
  const int64_t so = R.seq_off[r];    // then waits for the CIGAR walk only
  const int32_t nmd = mdv ? R.n_md[r] : 0;
  const int64_t mdo = mdv ? R.md_off[r] : 0;
  int ci = 0;
  int32_t ci_locus = s, within = 0, rp = 0;
  for (;;) {
    if (ci >= ncig) {
      if (mdv) *mdv = -1;
      *errc = 1;
      return false;
    }
    const uint32_t c = R.cigar[cig_off + ci];
    const int op = (int)(c & 15u);
    const int32_t len = (int32_t)(c >> 4);
    const int32_t rlen = consumes_ref(op) ? len : 0;
    if (ci_locus <= pos && pos < ci_locus + rlen) {
      if (consumes_read(op)) rp += pos - ci_locus - within;
      within = pos - ci_locus;
      break;
    } else if (pos == 0 && op == OP_I) {
      break;
    } else {
      if (consumes_read(op)) rp += len - within;
      ci_locus += rlen;
      ++ci;
      within = 0;
    }
  }
  const uint32_t c = R.cigar[cig_off + ci];
  const int op = (int)(c & 15u);
  const int32_t len = (int32_t)(c >> 4);
  if (mdv) {  // md_ref_at's answer from this walk (rp is the read offset at pos in a read op)
    if (op == OP_I) {
      *mdv = md_ref_at(R, r, pos);  // (pos 0 behind a leading insertion)
    } else if (nmd < 0) {
      *mdv = -4;
    } else {
      const bool seq_elem = op != OP_D && op != OP_N && rp < slen;
      const int b = seq_elem ? (int)R.seq[so + rp] : -1;
      const int v = md_find(R.md_ev + mdo, nmd, pos - s);
      *mdv = op == OP_D ? (v < 0 ? -3 : v) : op == OP_N ? (int)'N' : v >= 0 ? v : b;
    }
  }
  const bool fin = within == len - 1;
  const bool has_next = ci + 1 < ncig;
  const uint32_t cn = has_next ? R.cigar[cig_off + ci + 1] : 0u;
  const int nextop = fin ? (has_next ? (int)(cn & 15u) : -1) : op;
  d.read = r;
  d.rb = refbase;
  d.pad = 0;
  if ((op == OP_M || op == OP_EQ) && nextop == OP_I) {
    const int32_t ilen = (int32_t)(cn >> 4);  // I consumes read bases
    int32_t from = rp, until = rp + ilen + 1;
    from = from < 0 ? 0 : (from > slen ? slen : from);
    until = until > slen ? slen : until;
    if (until < from) until = from;
    d.kind = K_INS;
    d.rp = from;
    d.aux = until - from;
    d.base = 0;
    if (d.aux == 0) {
      *errc = 1;
      return false;
    }
  } else if (op == OP_I && nextop != -1 && ci_locus == 0) {
    int32_t from = rp, until = rp + len + 1;
    from = from < 0 ? 0 : (from > slen ? slen : from);
    until = until > slen ? slen : until;
    if (until < from) until = from;
    d.kind = K_INS;
    d.rp = from;
    d.aux = until - from;
    d.base = 0;
    if (d.aux == 0) {
      *errc = 1;
      return false;
    }
  } else if (op == OP_I) {
    *errc = 2;  // InvalidCigarElementException
    return false;
  } else if ((op == OP_M || op == OP_EQ || op == OP_X) && nextop == OP_D) {
    d.kind = K_DEL;
    d.aux = (int32_t)(cn >> 4);
    d.rp = rp;
    d.base = 0;
    const uint32_t *ev = R.md_ev + R.md_off[r];
    const int nmd = R.n_md[r];
    for (int i = 1; i <= d.aux; ++i)
      if (md_find(ev, nmd, pos + i - s) < 0) {
        *errc = 3;
        return false;
      }
  } else if (op == OP_D) {
    const int v = md_find(R.md_ev + R.md_off[r], R.n_md[r], pos - s);
    if (v < 0) {
      *errc = 3;
      return false;
    }
    d.kind = K_MID;
    d.base = (uint8_t)v;
    d.aux = 0;
    d.rp = 0;
  } else if (nextop == OP_D) {
    *errc = 1;
    return false;
  } else if (op == OP_M || op == OP_EQ || op == OP_X) {
    if (rp >= slen) {
      *errc = 1;
      return false;
    }
    d.kind = K_SNV;
    d.base = R.seq[so + rp];
    d.aux = 0;
    d.rp = rp;
  } else if (op == OP_S || op == OP_N || op == OP_H) {
    d.kind = K_CLIP;
    d.base = 0;
    d.aux = 0;
    d.rp = 0;
  } else {
    *errc = 1;
    return false;
  }
  return true;
}

// MD-derived reference base of read r at pos (MappedRead.getReferenceBaseAtLocus) or -1 on error.
__device__ __forceinline__ int md_ref_at(const DevReads &R, int64_t r, int32_t pos) {
  // the read's scalars are loaded together up front, and the read base at pos is loaded beside
  // the MD search: one latency round each instead of a chain
  const int32_t s = R.start[r];
  const int64_t cig_off = R.cigar_off[r];
  const int32_t ncig = R.n_cigar[r];
  const int32_t nmd = R.n_md[r];
  const int64_t mdo = R.md_off[r];
  const int64_t so = R.seq_off[r];
  const int32_t sl = R.seq_len[r];
  int32_t ref = s, rp = 0;
  for (int k = 0; k < ncig; ++k) {
    const uint32_t c = R.cigar[cig_off + k];
    const int op = (int)(c & 15u);
    const int32_t len = (int32_t)(c >> 4);
    if (consumes_ref(op)) {
      if (pos < ref + len) {
        if (nmd < 0) return -4;
        const int32_t q = rp + (pos - ref);
        const bool seq_elem = op != OP_D && op != OP_N && q < sl;
        const int b = seq_elem ? (int)R.seq[so + q] : -1;
        const int v = md_find(R.md_ev + mdo, nmd, pos - s);
        if (op == OP_D) return v < 0 ? -3 : v;
        if (op == OP_N) return 'N';
        if (v >= 0) return v;
        return b;  // -1 past the read's bases
      }
      ref += len;
    }
    if (consumes_read(op)) rp += len;
  }
  return -1;
}

constexpr int kSlots = 2;  // table capacity = 64 * kSlots distinct (sample, allele) keys per locus

// Scala hash (Allele(refBases, altBases).hashCode, gq_scala_order.h) of an allele from its bytes
__device__ __forceinline__ uint32_t allele_scala_hash(const DevReads &R, const AlleleDesc &a, int32_t pos) {
  scala::SeqHasher hr, ha;
  const int rl = allele_ref_len(a), al = allele_alt_len(a);
  for (int i = 0; i < rl; ++i) hr.add_byte(allele_byte(R, a, pos, 0, i));
  for (int i = 0; i < al; ++i) ha.add_byte(allele_byte(R, a, pos, 1, i));
  return scala::allele_hash(hr.result(), ha.result());
}

// Value of lane j (wave-uniform j) broadcast to every lane, for 64-bit types.
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int j) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), j);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ double lane_f64(double v, int j) {
  return __builtin_bit_cast(double, lane_u64(__builtin_bit_cast(uint64_t, v), j));
}
// Minimum / maximum over the wave (every lane active).
__device__ __forceinline__ int wave_min_i32(int v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v = min(v, __shfl_xor(v, d, 64));
  return v;
}
__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v = max(v, __shfl_xor(v, d, 64));
  return v;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t o = (int64_t)(((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)v, d, 64)) |
                                ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)((uint64_t)v >> 32), d, 64) << 32));
    v = o < v ? o : v;
  }
  return v;
}

}  // namespace
}  // namespace gq
