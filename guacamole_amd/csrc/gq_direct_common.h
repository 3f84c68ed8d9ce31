// gq_direct_common.h — device helpers shared by the kernels that count pileups straight from
// the resident reads (germline_direct in gq_pileup.hip, somatic_direct in gq_somatic.hip):
// general_segments (a general CIGAR as count / complex / MidDeletion segments) and wave
// scans.  Included inside each translation unit's anonymous namespace.
#pragma once

// (gq_kernels.h, gq_host.h: included by the translation unit before this header)

// the rotated slot schedule (every group on a slot at the same iteration): somatic_direct's
// bases and qualities are fetched once instead of ~2.6 times (chr20 60x: FETCH 22.9 -> 8.7 GB,
// 7.06 -> 6.58 ms); germline_direct, not bound by its fetches, measured 3 % slower with it
#ifndef GQ_DIR_ROT
#define GQ_DIR_ROT 1   // somatic_direct
#endif
#ifndef GQ_GDIR_ROT
#define GQ_GDIR_ROT 0  // germline_direct
#endif
#ifndef GQ_DIR_GROUP
#define GQ_DIR_GROUP 4  // lanes (columns) walking their slots together: 1, 2, 4, 8, 16, 32 or 64
#endif

// Column-kernel records (derived once at upload, after the read shapes).  A general-CIGAR read
// (not a single (M|=|X) block) becomes segments for the in-kernel path, PileupElement's rules
// (PileupElement.scala:68-248, as walk_read_lane) over the whole read:
//   count   loci [ref_off, ref_off + len) are Match/Mismatch elements whose bases start at
//           sequence offset seq_off;
//   complex loci [ref_off, ref_off + len) hold an insertion / deletion anchor, mid-deletions
//           or clipped (N) elements: the exact kernel decides them;
//   middel  loci [ref_off, ref_off + len) of a D op whose MD deleted bases are all A/C/G/T:
//           MidDeletion elements (counted by germline_proj, complex for the other kernels).
// Returns false if the in-kernel path cannot take the read (P op, M bases past the sequence,
// a deleted locus without its MD base, sizes beyond the packed fields): such reads keep the
// exact walker, which raises the reference's error where it applies.
// (segment kinds kSegCount / kSegComplex / kSegMidDel: gq_host.h)
template <class Emit>
__device__ bool general_segments(const DevReads &R, int64_t r, Emit emit) {
  const int32_t s = R.start[r], nmd = R.n_md[r], slen = R.seq_len[r], ncig = R.n_cigar[r];
  if (ncig < 1 || ncig > 32 || slen >= 16384) return false;
  const uint32_t *cg = R.cigar + R.cigar_off[r];
  const uint32_t *ev = R.md_ev + R.md_off[r];
  // the first five operations in one round of loads (past the last: the last again)
  uint32_t c5[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) c5[j] = cg[j < ncig ? j : ncig - 1];
  auto cig = [&](int32_t q) {
    return q < 5 ? (q == 0 ? c5[0] : q == 1 ? c5[1] : q == 2 ? c5[2] : q == 3 ? c5[3] : c5[4]) : cg[q];
  };
  int32_t ref = 0, rpos = 0, k = 0, nseg = 0;
  bool lead_ins = false, seen_ref = false;
  for (int32_t q = 0; q < ncig; ++q) {
    const uint32_t cq = cig(q);
    const int op = (int)(cq & 15u);
    const int32_t len = (int32_t)(cq >> 4);
    const int nextop = q + 1 < ncig ? (int)(cig(q + 1) & 15u) : -1;
    if (op == OP_P || op > OP_X) return false;
    if (op == OP_I && !seen_ref && s == 0) lead_ins = true;
    if (consumes_ref(op)) {
      seen_ref = true;
      const int32_t ra = ref, rb = ref + len;
      if (op == OP_M || op == OP_EQ || op == OP_X) {
        if (rpos + len > slen) return false;
        const bool first_ins = lead_ins && s + ra == 0;
        const bool anchor = ((op == OP_M || op == OP_EQ) && nextop == OP_I) || nextop == OP_D;
        const int32_t lo = first_ins ? ra + 1 : ra, hi = anchor ? rb - 1 : rb;
        if (hi > lo) emit(kSegCount, lo, hi - lo, rpos + (lo - ra), nseg++);
        if (first_ins) emit(kSegComplex, ra, 1, 0, nseg++);
        if (anchor && !(first_ins && rb - 1 == ra)) emit(kSegComplex, rb - 1, 1, 0, nseg++);
      } else {
        bool std_bases = op == OP_D;
        if (op == OP_D)
          for (int32_t l = ra; l < rb; ++l) {
            while (k < nmd && (int32_t)(ev[k] >> 8) < l) ++k;
            if (k >= nmd || (int32_t)(ev[k] >> 8) != l) return false;
            std_bases = std_bases && std_bit((uint8_t)(ev[k] & 0xFFu)) != 0u;
          }
        emit(std_bases ? kSegMidDel : kSegComplex, ra, len, 0, nseg++);
      }
      ref += len;
    }
    if (consumes_read(op)) rpos += len;
  }
  return nseg <= 255;
}

// bytes [a, b) of a 64-bit word (0 <= a, b <= 8)
__device__ __forceinline__ uint64_t byte_range_mask(int32_t a, int32_t b) {
  const uint64_t lt = b > 0 ? (~0ull >> (64 - 8 * b)) : 0ull;
  const uint64_t ge = a < 8 ? (~0ull << (8 * a)) : 0ull;
  return lt & ge;
}

// Inclusive prefix maximum / suffix minimum over the 64 lanes (every lane active).
__device__ __forceinline__ int32_t wave_incl_max_i(int32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t y = __shfl_up(v, d, 64);
    if (lane >= d) v = max(v, y);
  }
  return v;
}
__device__ __forceinline__ int32_t wave_suffix_min_i(int32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t y = __shfl_down(v, d, 64);
    if (lane + d < 64) v = min(v, y);
  }
  return v;
}

