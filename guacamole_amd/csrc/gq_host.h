// gq_host.h — internals shared by the library's translation units (gq_pileup.hip,
// gq_somatic.hip): error reporting, run counters, device buffers, the context and
// resident read-set handles, tile planning.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

#include "../../include/gqpileup.h"
#include "gq_kernels.h"

namespace gq {

gq_status set_err(gq_status s, const char *fmt, ...);  // thread-local message for gq_last_error

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return set_err(GQ_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
  } while (0)

constexpr int kBlock = 256;
constexpr int kGermT = 512;  // loci per germline tile
constexpr int kCountT = 512;  // loci per counts tile
constexpr size_t kSeqPad = 2048;  // zeroed tail of the uploaded sequence pool  // LDS staging of a read batch's sequence bytes

constexpr int kSpread = 64;
constexpr int kPartsCols = 2048;  // [0, 2048): one output partition per germline workgroup
constexpr int kPartsWalk = 1024;  // then one per walker / complex-kernel wave (modulo)
constexpr int kParts = kPartsCols + kPartsWalk;  // output partitions (see Counters::part)

struct Counters {  // device-side run counters (one allocation, zeroed per call)
  unsigned long long n_rec;
  unsigned long long n_complex;
  unsigned long long visited;
  unsigned long long ambiguous;
  unsigned long long ties;
  unsigned long long pool_used;
  int err;
  int pad;
  long long err_pos;
  unsigned long long n_slow;       // tiles germline_proj handed to germline_walk
  unsigned long long n_dead;       // record slots germline_expand left unused
  unsigned long long part_max[2];  // largest partition count of records / complex items (part_scan)
  unsigned long long n_amb;        // loci listed for the heap-order reference base (AmbItem list)
  unsigned long long n_ord;        // germline loci whose Scala map order depends on element order
  unsigned long long n_deep;       // somatic candidates handed to the deep caller
  unsigned long long n_wide;       // somatic candidates the deep caller handed to the wide one (> 128 alleles)
  unsigned long long n_gdeep[3];   // germline_complex loci handed to the wide table (first pass, order, heap-order runs)
  unsigned long long deep_max;     // deepest per-sample pileup among them and the listed loci
  unsigned long long deep_nt;      // germline-standard: largest allele table among the loci handed to the deep caller
  unsigned long long n_out;        // germline records in the result image (calls_image)
  unsigned long long out_pool;     // their allele bytes (the image's pool length)
  // per-tile run counters, spread over kSpread addresses (summed on the host)
  unsigned long long spread[4][64];  // visited, ambiguous, ties, dead record slots
  unsigned long long prof[8];  // diagnostic phase clocks (GQ_DBG=16 only)
  // ---- device-only tail (the host copies the head, up to `part`)
  // germline outputs: records (0) and complex items (1) are reserved per partition — a
  // writer appends to partition p at slot p * capacity + k — so no single counter serialises
  // every writer on the chip.  part_off = exclusive offsets of the kept counts (part_scan).
  unsigned long long part[2][kParts];
  unsigned long long part_off[2][kParts + 1];
};
constexpr size_t kCountersHead = offsetof(Counters, part);

// Wave-aggregated reservation of `n` slots on a global counter.
__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long *ctr, unsigned n) {
  if (__ballot(n != 0) == 0) return 0;  // nothing to reserve in this wave (the common case)
  const int lane = threadIdx.x & 63;
  // inclusive scan of n across the wave
  unsigned x = n;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    unsigned y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  const unsigned total = __shfl(x, 63, 64);
  unsigned long long base = 0;
  if (lane == 63 && total) base = atomicAdd(ctr, (unsigned long long)total);
  base = __shfl(base, 63, 64);
  return base + (x - n);
}

// Geometry of the partitioned germline outputs (records: which = 0, complex items: 1).
// Partitions [0, ncols) belong to germline_proj workgroups (capacity capA each), partitions
// [kPartsCols, kParts) to walker / complex-kernel waves (capacity capB each); the others are
// unused.  slot(which, p, k) is the buffer index of element k of partition p.
struct OutGeom {
  int ncols;
  int pad_;
  unsigned long long capA[2], capB[2];
  __host__ __device__ __forceinline__ unsigned long long cap(int which, int p) const {
    return p < kPartsCols ? capA[which] : capB[which];
  }
  __host__ __device__ __forceinline__ unsigned long long slot(int which, int p, unsigned long long k) const {
    return p < kPartsCols ? (unsigned long long)p * capA[which] + k
                          : (unsigned long long)ncols * capA[which] + (unsigned long long)(p - kPartsCols) * capB[which] + k;
  }
  __host__ __device__ __forceinline__ unsigned long long total(int which) const {
    return (unsigned long long)ncols * capA[which] + (unsigned long long)(kParts - kPartsCols) * capB[which];
  }
};

// Buffer index of the k-th kept element of a partitioned output: the partition q with
// off[q] <= k < off[q + 1] (off = part_off[which], kParts + 1 entries), then its slot.
__device__ __forceinline__ unsigned long long part_slot(const unsigned long long *off, unsigned long long k,
                                                        const OutGeom &g, int which) {
  int lo = 0, hi = kParts - 1;  // last q with off[q] <= k
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (off[m] <= k) lo = m;
    else hi = m - 1;
  }
  return g.slot(which, lo, k - off[lo]);
}

// First index in [lo, hi) whose monotone predicate (false ... true) holds, hi if none: 64
// probes per round (wave-uniform bounds; every lane active).  A window of n reads takes
// ceil(log64 n) dependent loads.
template <class P>
__device__ __forceinline__ int64_t wave_first_true(int64_t lo, int64_t hi, P &&pred) {
  const int lane = threadIdx.x & 63;
  while (hi - lo > 64) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t p = lo + (int64_t)lane * step;
    const unsigned long long b = __ballot(p >= hi || pred(p));
    if (!b) {
      lo = lo + 63 * step + 1;
      continue;
    }
    const int f = __ffsll((long long)b) - 1;
    if (f == 0) return lo;
    const int64_t nhi = lo + (int64_t)f * step;  // true there (or hi)
    lo = lo + (int64_t)(f - 1) * step + 1;
    hi = nhi < hi ? nhi : hi;
  }
  const int64_t p = lo + lane;
  const unsigned long long b = __ballot(p >= hi || pred(p));
  return b ? lo + (__ffsll((long long)b) - 1) : hi;
}

// Two wave_first_true searches over the same [lo, hi) in lockstep: each round issues both
// searches' probes before either ballot is read, so the two dependent-load chains overlap.
template <class P1, class P2>
__device__ __forceinline__ void wave_first_true2(int64_t lo, int64_t hi, P1 &&pred1, P2 &&pred2, int64_t &out1,
                                                 int64_t &out2) {
  const int lane = threadIdx.x & 63;
  int64_t lo1 = lo, hi1 = hi, lo2 = lo, hi2 = hi;
  bool done1 = false, done2 = false;
  // one round of one search: narrows [l, h) or finishes it (wave-uniform)
  auto round = [&](int64_t &l, int64_t &h, bool &done, int64_t &out, bool hit) {
    if (done) return;
    if (h - l > 64) {
      const int64_t step = (h - l + 63) / 64;
      const unsigned long long b = __ballot(hit);
      if (!b) {
        l = l + 63 * step + 1;
        return;
      }
      const int f = __ffsll((long long)b) - 1;
      if (f == 0) {
        out = l;
        done = true;
        return;
      }
      const int64_t nh = l + (int64_t)f * step;
      l = l + (int64_t)(f - 1) * step + 1;
      h = nh < h ? nh : h;
    } else {
      const unsigned long long b = __ballot(hit);
      out = b ? l + (__ffsll((long long)b) - 1) : h;
      done = true;
    }
  };
  while (!(done1 && done2)) {
    // this round's probe of each unfinished search (both loads in flight together)
    const int64_t s1 = hi1 - lo1 > 64 ? (hi1 - lo1 + 63) / 64 : 1, s2 = hi2 - lo2 > 64 ? (hi2 - lo2 + 63) / 64 : 1;
    const int64_t p1 = lo1 + (int64_t)lane * s1, p2 = lo2 + (int64_t)lane * s2;
    const bool h1 = !done1 && (p1 >= hi1 || pred1(p1));
    const bool h2 = !done2 && (p2 >= hi2 || pred2(p2));
    round(lo1, hi1, done1, out1, h1);
    round(lo2, hi2, done2, out2, h2);
  }
}

// part_slot for a wave-uniform k, the search spread over the lanes: two rounds of 64 probes
// (two dependent loads instead of a twelve-step binary search).  Every lane must be active.
__device__ __forceinline__ unsigned long long part_slot_wave(const unsigned long long *off, unsigned long long k,
                                                             const OutGeom &g, int which) {
  constexpr int kStep = (kParts + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int q1 = lane * kStep;
  const bool le1 = q1 < kParts && off[q1 < kParts ? q1 : 0] <= k;
  const int base = (63 - __clzll((long long)__ballot(le1))) * kStep;  // off[0] = 0 <= k: lane 0 always
  const int q2 = base + lane;
  const bool le2 = lane < kStep && q2 < kParts && off[q2 < kParts ? q2 : 0] <= k;
  const int q = base + (63 - __clzll((long long)__ballot(le2)));
  return g.slot(which, q, k - off[q]);
}

// This wave's index in the grid (blockDim a multiple of 64), known wave-uniform to the compiler:
// loads indexed by it go to scalar registers.
__device__ __forceinline__ int64_t wave_id() {
  return (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP row shifts and row broadcasts
// (no LDS round trips).  Every lane must be active.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Projection slice `slot` (the block-row pool, ProjRec in gq_kernels.h): its contig c, its
// 16-column span [qc0, qc0 + 16) and its read window [ra, rz) — the reads of the contig with
// pmax_end > the slice's first locus and start < its end, in read order (every read with a piece
// in the slice, and the reads between them).
struct SliceWin {
  int32_t c, qc0;
  int64_t ra, rz;
};
__device__ __forceinline__ SliceWin slice_window(const DevReads &R, int64_t slot) {
  int lo = 0, hi = R.n_contigs - 1;  // contig: last c with qoff[c] <= slot
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (R.qoff[m] <= slot) lo = m;
    else hi = m - 1;
  }
  const int c = lo;
  const int32_t q = (int32_t)(slot - R.qoff[c]);
  const int32_t L = 128 * q;
  const int64_t cb = R.contig_read_begin[c], ce = R.contig_read_begin[c + 1];
  // the block index (block_index: per 512-locus block g, the first read with pmax_end past its
  // start and the first read starting in or after it) bounds both searches to the block's reads:
  // ra >= blk_rb[g] (L is past the block's start) and every window read starts before the next
  // block's first read, blk_rs[g + 1] (the contig's end for its last block)
  int64_t a0 = cb, a1 = ce;
  if (R.blk_rb) {
    const int64_t g = slot >> 2;  // (qoff[c] is a multiple of 4: slot / 4 is the global block)
    a0 = R.blk_rb[g];
    if (((slot >> 2) + 1) < (R.qoff[c + 1] >> 2)) a1 = R.blk_rs[g + 1];
  }
  const int64_t hi0 = a1;
  while (a0 < a1) {  // first read with pmax_end > L
    const int64_t m = (a0 + a1) >> 1;
    if (R.pmax_end[m] > L) a1 = m;
    else a0 = m + 1;
  }
  const int64_t ra = a0;
  a1 = hi0;
  while (a0 < a1) {  // first read with start >= L + 128
    const int64_t m = (a0 + a1) >> 1;
    if (R.start[m] >= L + 128) a1 = m;
    else a0 = m + 1;
  }
  return SliceWin{c, 16 * q, ra, a0};
}

// Slice `slot` with its stored window (slice_windows + the scan of its sizes).
__device__ __forceinline__ SliceWin slice_stored(const DevReads &R, int64_t slot) {
  int lo = 0, hi = R.n_contigs - 1;  // contig: last c with qoff[c] <= slot
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (R.qoff[m] <= slot) lo = m;
    else hi = m - 1;
  }
  const int64_t ra = R.sra[slot];
  return SliceWin{lo, 16 * (int32_t)(slot - R.qoff[lo]), ra, ra + (R.soff[slot + 1] - R.soff[slot])};
}

// Read r's piece in a slice: first column (slice-relative s0 - qc0 = its offset) and length in
// columns; sl = 0: no piece (the read ends before the slice, or the projection cannot take it).
__device__ __forceinline__ void piece_of(const ProjRec &p, int32_t qc0, int32_t &s0, int32_t &sl) {
  s0 = qc0;
  sl = 0;
  if (p.col1 != kProjNone) {
    s0 = p.col0 > qc0 ? p.col0 : qc0;
    const int32_t e = p.col1 < qc0 + 16 ? p.col1 : qc0 + 16;
    sl = e > s0 ? e - s0 : 0;
  }
}
__device__ __forceinline__ void slice_piece(const DevReads &R, int64_t r, int32_t qc0, int32_t &s0, int32_t &sl) {
  s0 = qc0;
  sl = 0;
  const ProjRec p = R.prec[r];
  if (p.col1 != kProjNone) {
    s0 = p.col0 > qc0 ? p.col0 : qc0;
    const int32_t e = p.col1 < qc0 + 16 ? p.col1 : qc0 + 16;
    sl = e > s0 ? e - s0 : 0;
  }
}

// One wave over slice `slot` with window [ra, rz): each piece (a read's columns inside the slice)
// takes the first row that is free from its first column — greedy interval partitioning over
// pieces sorted by first column, which is read order (reads are sorted by start; pieces of reads
// that began before the slice all start at its column 0): as many rows as the slice's deepest
// column has reads.  Each read's row goes to rows[r - ra] (0xFFFF: no piece), so the fill kernels
// place words without redoing this pass.  Returns the slice's rows, or -1 past kSliceRowsMax.
//
// The pieces that start at one column are placed together: the rows free at that column (row
// k's end column rend[k] <= c) are listed in ascending order by one wave-wide compaction, and
// the group's t-th piece takes the t-th of them (new rows past the list) — what placing the
// group's pieces one by one, each on the first free row, gives, since a placed piece's row is
// busy at c.  rend (kSliceRowsMax bytes) and fl (kSliceRowsMax u16) are this wave's LDS.
__device__ __forceinline__ int32_t slice_assign_rows(const DevReads &R, const SliceWin &W, uint16_t *__restrict__ rows,
                                                     uint8_t *__restrict__ rend, uint16_t *__restrict__ fl) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  int32_t nrows = 0;
  bool over = false;
  for (int64_t r0 = W.ra; r0 < W.rz; r0 += 64) {
    const int64_t r = r0 + lane;
    int32_t s0 = W.qc0, sl = 0;
    if (r < W.rz) slice_piece(R, r, W.qc0, s0, sl);
    const int32_t c = s0 - W.qc0, e = c + sl;
    int32_t myrow = -1;
    unsigned long long pend = __ballot(sl > 0);
    while (pend) {  // the batch's groups of equal first column, in read order (uniform)
      const int pl = __ffsll((long long)pend) - 1;
      const int32_t cg = __builtin_amdgcn_readlane(c, pl);
      const unsigned long long mem = __ballot(sl > 0 && c == cg);
      pend &= ~mem;
      const uint32_t S = (uint32_t)__popcll(mem);
      // the first S rows free at column cg, ascending (rows k0..k0+3 on lane (k0 / 4) % 64)
      uint32_t nf = 0;
      const uint32_t lim = (uint32_t)(cg + 1) * 0x01010101u;
      for (int32_t j0 = 0; j0 < nrows && nf < S; j0 += 256) {  // uniform
        const int32_t k0 = j0 + 4 * lane;
        uint32_t x = 0x7F7F7F7Fu;  // 0x7F: no such row (never free)
        if (k0 < nrows) {
          x = *reinterpret_cast<const uint32_t *>(rend + k0);
          const int32_t nb = nrows - k0;
          if (nb < 4) {
            const uint32_t keep = (1u << (8 * nb)) - 1u;
            x = (x & keep) | (0x7F7F7F7Fu & ~keep);
          }
        }
        uint32_t fr = ~((x | 0x80808080u) - lim) & 0x80808080u;  // bytes <= cg (no borrows: each >= 0x80)
        const uint32_t n = (uint32_t)__popc(fr);
        const uint32_t incl = wave_incl_scan(n);
        uint32_t at = nf + incl - n;
        while (fr) {
          fl[at++] = (uint16_t)(k0 + (__builtin_ctz(fr) >> 3));
          fr &= fr - 1u;
        }
        nf += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if ((mem >> lane) & 1ull) {
        const uint32_t t = (uint32_t)__popcll(mem & below);
        const int32_t k = t < nf ? (int32_t)fl[t] : nrows + (int32_t)(t - nf);
        if (k >= kSliceRowsMax) {
          over = true;
        } else {
          rend[k] = (uint8_t)e;
          myrow = k;
        }
      }
      nrows += S > nf ? (int32_t)(S - nf) : 0;
      if (nrows > kSliceRowsMax) nrows = kSliceRowsMax;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (rows && r < W.rz) rows[r - W.ra] = myrow >= 0 ? (uint16_t)myrow : (uint16_t)0xFFFFu;
  }
  return __ballot(over) ? -1 : nrows;
}

// Inclusive prefix minimum over the 64 lanes of a wave (signed), DPP as wave_incl_scan; lanes
// shifted in from outside the row / wave contribute INT32_MAX.
__device__ __forceinline__ int32_t wave_incl_min(int32_t v) {
  constexpr int kMax = 0x7FFFFFFF;
  v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x111, 0xF, 0xF, false));  // row_shr:1
  v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x112, 0xF, 0xF, false));  // row_shr:2
  v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x114, 0xF, 0xF, false));  // row_shr:4
  v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x118, 0xF, 0xF, false));  // row_shr:8
  v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = min(v, __builtin_amdgcn_update_dpp(kMax, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return v;
}

// Rows of slice W's pieces without a sequential pass (one wave): greedy interval partitioning
// in read order (= first column order) that reuses the row freed EARLIEST — as optimal as
// first-fit (any greedy in start order that opens a row only when none is free uses as many rows
// as the deepest column holds pieces), and computable in parallel.  With pieces k = 0, 1, ... in
// read order, A_k = pieces ending at or before piece k's first column (a column histogram of the
// ends), and U_k = reuses among pieces 0..k-1: U_{k+1} = min(U_k + 1, A_k), so
// U_k = k + min(0, min_{j<k}(A_j - j) - 1) (a prefix minimum).  Piece k reuses a row iff
// A_k > U_k: the row of E[U_k], the U_k-th piece in end order (which ended before k began, so it
// precedes k); otherwise it opens row k - U_k.  Rows resolve by following E (chains inside a
// 64-piece batch, a few steps).  Each window read's row goes to rows[r - ra] (0xFFFF: no piece).
// lds: 2 * kRowsLdsPieces u16 (E and the pieces' rows) + 32 u32.  Returns the slice's rows, -1
// past kSliceRowsMax, or -2 when the slice has more than kRowsLdsPieces pieces (the caller
// takes slice_assign_rows there).
constexpr int kRowsLdsPieces = 1024;
__device__ __forceinline__ int32_t slice_rows_fifo(const DevReads &R, const SliceWin &W, uint16_t *__restrict__ rows,
                                                   uint16_t *__restrict__ eord, uint16_t *__restrict__ prow_k,
                                                   uint32_t *__restrict__ hist) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  constexpr int32_t kInf = 0x7FFFFFFF;
  if (lane < 32) hist[lane] = 0;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // pass 1: a histogram of the pieces' end columns (1..16) and the piece count (the first
  // batch's pieces kept for pass 2: most windows are one batch)
  int32_t n = 0;
  int32_t s0_first = W.qc0, sl_first = 0;
  for (int64_t r0 = W.ra; r0 < W.rz; r0 += 64) {
    const int64_t r = r0 + lane;
    int32_t s0 = W.qc0, sl = 0;
    if (r < W.rz) slice_piece(R, r, W.qc0, s0, sl);
    if (r0 == W.ra) {
      s0_first = s0;
      sl_first = sl;
    }
    if (sl > 0) atomicAdd(&hist[s0 - W.qc0 + sl], 1u);
    n += (int32_t)__popcll(__ballot(sl > 0));
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (n > kRowsLdsPieces) return -2;
  // lane v (0..16): cum = pieces ending at or before column v
  const uint32_t cum = wave_incl_scan(lane <= 16 ? hist[lane] : 0u);
  uint32_t seen = 0;  // lane v: pieces ending at column v already ranked
  int32_t runmin = kInf, base = 0;
  for (int64_t r0 = W.ra; r0 < W.rz; r0 += 64) {
    const int64_t r = r0 + lane;
    int32_t s0 = s0_first, sl = sl_first;
    if (r0 != W.ra) {  // (uniform: later batches load their pieces again)
      s0 = W.qc0;
      sl = 0;
      if (r < W.rz) slice_piece(R, r, W.qc0, s0, sl);
    }
    const bool has = sl > 0;
    const int32_t c0 = has ? s0 - W.qc0 : 0, c1 = c0 + sl;
    const unsigned long long hm = __ballot(has);
    const int32_t k = base + (int32_t)__popcll(hm & below);
    // E[rank] = k, rank = pieces ending before piece k's end + those with its end ranked before it
    int32_t rank = 0;
    unsigned long long pend = hm;
    while (pend) {  // the batch's distinct end columns (uniform)
      const int pl = __ffsll((long long)pend) - 1;
      const int32_t v = __builtin_amdgcn_readlane(c1, pl);
      const unsigned long long m = __ballot(has && c1 == v);
      pend &= ~m;
      const uint32_t before = (uint32_t)__builtin_amdgcn_readlane((int)cum, v - 1);
      const uint32_t sv = (uint32_t)__builtin_amdgcn_readlane((int)seen, v);
      if (has && c1 == v) rank = (int32_t)(before + sv + (uint32_t)__popcll(m & below));
      seen += lane == v ? (uint32_t)__popcll(m) : 0u;
    }
    if (has) eord[rank] = (uint16_t)k;
    // U_k = k + min(0, min_{j<k}(A_j - j) - 1), A_k = cum[c0]
    const int32_t A = __builtin_amdgcn_ds_bpermute(4 * c0, (int)cum);
    const int32_t incl = wave_incl_min(has ? A - k : kInf);
    const int32_t excl = min(runmin, __builtin_amdgcn_update_dpp(kInf, incl, 0x138, 0xF, 0xF, false));  // wave_shr:1
    const int32_t U = k + min(0, excl == kInf ? 0 : excl - 1);
    const bool reuse = has && A > U;
    if (has) prow_k[k] = reuse ? (uint16_t)0xFFFFu : (uint16_t)(k - U);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int32_t parent = reuse ? (int32_t)eord[U] : 0;
    int32_t row = has && !reuse ? k - U : -1;
    // a reused row is its parent's (the parent precedes it; chains inside the batch take a few rounds)
    while (__ballot(reuse && row < 0)) {
      if (reuse && row < 0) {
        const uint32_t pr = prow_k[parent];
        if (pr != 0xFFFFu) {
          row = (int32_t)pr;
          prow_k[k] = (uint16_t)pr;
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (rows && r < W.rz) rows[r - W.ra] = has && row < kSliceRowsMax ? (uint16_t)row : (uint16_t)0xFFFFu;
    runmin = min(runmin, __builtin_amdgcn_readlane(incl, 63));
    base += (int32_t)__popcll(hm);
  }
  const int32_t nrows = n - (n + min(0, runmin == kInf ? 0 : runmin - 1));
  return nrows > kSliceRowsMax ? -1 : nrows;
}

// A piece of a 64-read batch, for the word-per-lane fills (slice_fill): set up once by the
// piece's lane, read from LDS by the lanes of its words.
// Bytes [lo, hi) of an 8-byte word (clamped to [0, 8)) as a mask: an edge word's loci inside its read.
__device__ __forceinline__ uint64_t edge_mask(int32_t lo, int32_t hi) {
  lo = lo < 0 ? 0 : lo;
  hi = hi > 8 ? 8 : hi;
  if (hi <= lo) return 0;
  const uint64_t top = hi == 8 ? ~0ull : (1ull << (8 * hi)) - 1ull;
  return top & ~((1ull << (8 * lo)) - 1ull);
}

struct __attribute__((aligned(16))) PieceMeta {
  int64_t p0;         // pool offset of locus 0: a column-eligible read's base / quality at locus l is p0 + l
  int32_t s, e;       // the read's [start, end)
  int32_t s0, row;    // the piece's first column and its row
  uint32_t info, mq;  // ColDesc info, mapping quality
  uint32_t ev[4];     // MD events at the piece's loci: bit i = locus 8 s0 + i (margin fill)
};
static_assert(sizeof(PieceMeta) == 48, "PieceMeta: three 16-byte LDS reads");

// Inclusive prefix maximum over the 64 lanes of a wave (values >= 0), DPP as wave_incl_scan.
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true));  // row_shr:1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true));  // row_shr:2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true));  // row_shr:4
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true));  // row_shr:8
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return v;
}

// Once per word of the slice's pieces, a lane per word (a batch's words in piece order:
// consecutive words of a piece on consecutive lanes, so the loads of a piece's bases and the
// stores of its row coalesce): raw = fetch(read, meta, column, events) (the word's loads), then
// emit(act, raw, read, meta, column, events).  events: the word's eight MD-event bits (EV only).
// Each lane takes kU words per round and issues all their loads before the first emit.  A word
// finds its piece without a search: the pieces starting inside the round's words mark their first
// word in LDS (owner), a prefix maximum carries each mark over the piece's words, and one ballot
// gives the piece already running at each 64-word window's start.  setup(read, meta, md_off)
// runs once per piece on the piece's lane (meta's read fields filled) and returns false to drop it.  meta: this wave's 64 LDS entries;
// owner: its kU * 64 LDS words.
template <bool EV, int kU, class S, class F, class E>
__device__ __forceinline__ void slice_fill(const DevReads &R, const SliceWin &W, const uint16_t *__restrict__ rows,
                                           PieceMeta *__restrict__ meta, uint32_t *__restrict__ owner, S &&setup,
                                           F &&fetch, E &&emit) {
  const int lane = threadIdx.x & 63;
  for (int64_t r0 = W.ra; r0 < W.rz; r0 += 64) {
    const int64_t r = r0 + lane;
    int32_t s0 = W.qc0, sl = 0;
    // the read's records in one round, loaded whether or not it has a piece here (a valid read
    // index either way): no load waits on another
    const bool in = r < W.rz;
    const int64_t rr = in ? r : W.ra;
    const uint16_t k = rows[rr - W.ra];
    const ProjRec pr = R.prec[rr];
    const ColDesc d = R.cdesc[rr];
    const int64_t so = R.seq_off[rr];
    const int32_t ld = R.lead[rr];
    uint32_t mq = 0;
    int64_t mdo = 0;
    if constexpr (EV) {
      mq = R.mapq[rr];
      mdo = R.md_off[rr];
    }
    if (in && k != 0xFFFFu) {
      piece_of(pr, W.qc0, s0, sl);
      if (sl > 0) {
        PieceMeta m;
        m.s0 = s0;
        m.row = k;
        m.s = d.start;
        m.e = d.end;
        m.info = d.info;
        m.mq = mq;
        m.p0 = so + (ld > 0 ? ld : 0) - d.start;
        if (setup(r, m, mdo)) meta[lane] = m;
        else sl = 0;
      }
    }
    const uint32_t len = (uint32_t)sl;
    const uint32_t incl = wave_incl_scan(len), ex = incl - len;
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    for (uint32_t w0 = 0; w0 < tot; w0 += 64 * kU) {
#pragma unroll
      for (int u = 0; u < kU; ++u) owner[64 * u + lane] = 0;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (len > 0 && ex > w0 && ex < w0 + 64 * kU) owner[ex - w0] = (uint32_t)lane + 1;  // the piece's first word
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      int kk[kU];
      int32_t col[kU];
      bool act[kU];
      PieceMeta pm[kU];
      uint32_t evb[kU];
      decltype(fetch((int64_t)0, pm[0], (int32_t)0, 0u)) raw[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const uint32_t wb = w0 + 64 * u, w = wb + (uint32_t)lane;
        const unsigned long long run = __ballot(len > 0 && ex <= wb);  // the last of them runs at wb
        const uint32_t k_at = run ? 64u - (uint32_t)__clzll((long long)run) : 0u;  // its lane + 1
        const uint32_t k1 = max(wave_incl_max(owner[64 * u + lane]), k_at);
        act[u] = w < tot;
        const int k = act[u] ? (int)k1 - 1 : 0;
        kk[u] = k;
        const uint4 *src = reinterpret_cast<const uint4 *>(meta + k);
        const uint4 a = src[0], b = src[1];
        PieceMeta &m = pm[u];
        m.p0 = (int64_t)((uint64_t)a.x | ((uint64_t)a.y << 32));
        m.s = (int32_t)a.z;
        m.e = (int32_t)a.w;
        m.s0 = (int32_t)b.x;
        m.row = (int32_t)b.y;
        m.info = b.z;
        m.mq = b.w;
        const uint32_t kex = (uint32_t)__shfl((int)ex, k, 64);
        col[u] = m.s0 + (int32_t)(w - kex);
        evb[u] = 0;
        if constexpr (EV) {
          const uint4 c = src[2];
          const int32_t i0 = 8 * (col[u] - m.s0);  // bit of the word's first locus
          const int iw = i0 >> 5;
          const uint32_t ew = (iw & 2) ? ((iw & 1) ? c.w : c.z) : ((iw & 1) ? c.y : c.x);
          evb[u] = (ew >> (i0 & 31)) & 0xFFu;
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (act[u]) raw[u] = fetch(r0 + kk[u], pm[u], col[u], evb[u]);
#pragma unroll
      for (int u = 0; u < kU; ++u) emit(act[u], raw[u], r0 + kk[u], pm[u], col[u], evb[u]);
    }
    __builtin_amdgcn_wave_barrier();  // (the next batch rewrites meta)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

// ---- Projection words (proj_fill / proj_fill_rw and the somatic fused fill) ----
// A general CIGAR's count segments (col_derive): Match/Mismatch runs, complex runs, MidDeletion runs.
constexpr uint32_t kSegCount = 0, kSegComplex = 1, kSegMidDel = 2;
__device__ __forceinline__ uint32_t proj_code(uint8_t b) {  // A 1, C 3, T 4, G 7; N and the rest 0
  return (b == 'A' || b == 'C' || b == 'G' || b == 'T') ? (uint32_t)(b & 7u) : 0u;
}

// Byte codes of four ASCII bases (proj_code, SWAR): A 1, C 3, G 7, T 4, anything else 0.
__device__ __forceinline__ uint32_t proj_codes4(uint32_t x) {
  auto eq = [x](uint32_t pat) {  // 0x80 in the bytes equal to pat's (exact: no carries between bytes)
    const uint32_t z = x ^ pat;
    return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z | 0x7F7F7F7Fu);
  };
  const uint32_t m = eq(0x41414141u) | eq(0x43434343u) | eq(0x47474747u) | eq(0x54545454u);
  return x & ((m >> 7) * 7u);
}

typedef uint64_t gq_u64u __attribute__((aligned(1)));  // unaligned 8-byte loads (gfx950 global memory)

// The projection word of read r at column col (loci [8 col, 8 col + 8)): byte j = code of locus
// 8 col + j | code of locus 8 col + j + 4 << 4 (4-bit codes, proj_code).  m: the read's piece
// (slice_fill).  proj_fetch loads the word's eight bases (one 8-byte load inside a column-eligible
// read; a general CIGAR's word is complete here); proj_code8 turns them into the word.
struct ProjRaw {
  uint64_t b;     // the bases, byte q = locus 8 col + q (0 outside the read)
  uint32_t word;  // general CIGAR: the word itself
  uint32_t gen;
};
__device__ __forceinline__ ProjRaw proj_fetch(const DevReads &R, int64_t r, const PieceMeta &m, int32_t col) {
  const int32_t s = m.s, e = m.e;
  const int32_t lb = 8 * col;  // locus of byte 0
  ProjRaw x{0, 0, 0};
  if (m.info & kColEligible) {  // [S|H]* (M|=|X) [S|H]*: locus l holds base p0 + l
    const int64_t a = m.p0 + lb;
    if (a >= 0 && a + 8 <= R.seq_cap) {  // one load; an edge word's loci outside the read masked
      x.b = *reinterpret_cast<const gq_u64u *>(R.seq + a) & edge_mask(s - lb, e - lb);
    } else {
      for (int q = 0; q < 8; ++q) {
        const int32_t l = lb + q;
        if (l >= s && l < e) x.b |= (uint64_t)R.seq[m.p0 + l] << (8 * q);
      }
    }
    return x;
  }
  // general CIGAR: the count segments (ref_off | len << 16, seq_off | kind << 16)
  const int32_t nmd = (int32_t)(m.info & 0xFFFFu), nseg = (int32_t)((m.info >> 18) & 0xFFu);
  const uint32_t *sg = R.cev + R.caux_off[r] + nmd;
  const int64_t so = R.seq_off[r];
  uint32_t v[2] = {0, 0};
  for (int32_t q2 = 0; q2 < nseg; ++q2) {
    const uint32_t a = sg[2 * q2], b = sg[2 * q2 + 1];
    if ((b >> 16) != kSegCount) continue;
    const int32_t ra = s + (int32_t)(a & 0xFFFFu), rl = (int32_t)(a >> 16), sp = (int32_t)(b & 0xFFFFu);
    if (ra >= lb + 8 || ra + rl <= lb) continue;
    for (int q = 0; q < 8; ++q) {
      const int32_t l = lb + q;
      if (l >= ra && l < ra + rl) v[q >> 2] |= proj_code(R.seq[so + sp + (l - ra)]) << (8 * (q & 3));
    }
  }
  x.word = v[0] | (v[1] << 4);
  x.gen = 1;
  return x;
}

// The cell fills' record offset of a read whose bytes are not in the window's byte run (a
// wrapped pool in another order, or past 2 GiB of it): its cells take the slow path.
constexpr uint32_t kCell3Far = 0x80000000u;

// ---- Piece fills: a wave per slice, a lane per piece, rows built in LDS (A/B: GQ_FILL=pieces) ----
// A wave takes a slice: each lane takes one of its window reads and, if the read has a piece in
// the slice, issues the loads of all the piece's words at once (up to 16 columns), turns them into
// words and writes them into the slice's rows in LDS (kPieceRows rows at a time, padded to 17
// words per row against bank conflicts); the rows then leave LDS as whole rows, 64 consecutive
// words per store (every word written, so the pool needs no preset).  A window over 64 reads
// takes several batches, a slice over kPieceRows rows several row chunks.
constexpr int kPieceRows = 64;
constexpr int kPieceStride = 17;  // LDS words per row
struct PieceRec {                 // a window read as one lane holds it
  int64_t p0;                     // pool offset of locus 0 (column-eligible reads)
  int32_t s, e;                   // [start, end)
  uint32_t info, mq;              // ColDesc info, mapping quality
  int64_t md_off;                 // its MD events
  uint32_t ev[4];                 // (EV fills) its first four MD events (0xFFFFFFFF: none)
};
// proj_codes4 for the bytes of a column-eligible read (A C G T N only, zero outside the read):
// A 1, C 3, G 7, T 4 are the low three bits, N (6) and zero bytes give 0.
__device__ __forceinline__ uint32_t proj_codes4_clean(uint32_t x) {
  const uint32_t y = x & 0x07070707u;
  const uint32_t n = y ^ 0x06060606u;                                   // zero bytes: N
  const uint32_t keep = (((n & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | n) & 0x80808080u;  // 0x80: not N
  return y & ((keep >> 7) * 0xFFu);
}
__device__ __forceinline__ PieceMeta piece_rec_meta(const PieceRec &m) {
  PieceMeta p;
  p.p0 = m.p0;
  p.s = m.s;
  p.e = m.e;
  p.s0 = 0;
  p.row = 0;
  p.info = m.info;
  p.mq = m.mq;
  return p;
}

// For every slice (grid-stride over waves): for each row chunk, rows zeroed in `lds` (words of
// type T, `zero`), then each window read r with a piece whose row lies in the chunk:
//   keep(rec)                      false: the piece writes nothing (its cells keep `zero`);
//   fast(rec, col, raw) for each of its columns, all issued before any is used (false: that
//                                  word takes slow(rec, r, col) instead, out of the unrolled path);
//   word(rec, col, raw) -> T       the word;
// then the chunk's rows go to pool (T words, 16 per row) at the slice's rows.  done(slot, flag)
// closes the slice with the OR over its lanes of flag(word) (e.g. a kMargin8None term).  pbad
// slices get `zero` rows.
template <class T, class Raw, bool EV, class K, class F, class Wd, class S, class G, class D>
__device__ __forceinline__ void piece_fill(const DevReads &R, int64_t n_slices, T *__restrict__ lds, T *__restrict__ pool,
                                           T zero, K &&keep, F &&fast, Wd &&word, S &&slow, G &&flag, D &&done) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t slot = wave_id(); slot < n_slices; slot += nw) {
    const int64_t g0 = R.srow[slot];
    const int32_t nr = (int32_t)(R.srow[slot + 1] - g0);
    if (nr <= 0) continue;
    T *out = pool + 16 * g0;
    if (R.pbad[slot]) {
      for (int32_t c = lane; c < 16 * nr; c += 64) out[c] = zero;
      continue;
    }
    const SliceWin W = slice_stored(R, slot);
    const uint16_t *prw = R.prow + R.soff[slot];
    bool any = false;
    for (int32_t k0 = 0; k0 < nr; k0 += kPieceRows) {
      const int32_t nk = nr - k0 < kPieceRows ? nr - k0 : kPieceRows;
      for (int32_t c = lane; c < kPieceStride * nk; c += 64) lds[c] = zero;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      for (int64_t r0 = W.ra; r0 < W.rz; r0 += 64) {
        const int64_t r = r0 + lane;
        const bool in = r < W.rz;
        const int64_t rr = in ? r : W.ra;
        const int32_t row = in ? (int32_t)prw[rr - W.ra] : 0xFFFF;
        const ProjRec pr = R.prec[rr];
        const ColDesc d = R.cdesc[rr];
        const int32_t ld = R.lead[rr];
        const int64_t so = R.seq_off[rr];
        PieceRec m;
        m.mq = R.mapq[rr];
        m.md_off = R.md_off[rr];
        m.p0 = so + (ld > 0 ? ld : 0) - d.start;
        m.s = d.start;
        m.e = d.end;
        m.info = d.info;
        int32_t s0 = W.qc0, sl = 0;
        piece_of(pr, W.qc0, s0, sl);
        const bool mine = in && row != 0xFFFF && row >= k0 && row < k0 + nk && sl > 0 && keep(m);
        if (!__ballot(mine)) continue;
        if constexpr (EV) {
          const int32_t nmd = (int32_t)(m.info & 0xFFFFu);
          const uint32_t *ev = R.md_ev + m.md_off;
#pragma unroll
          for (int q = 0; q < 4; ++q) m.ev[q] = mine && q < nmd ? ev[q] : 0xFFFFFFFFu;
        }
        const int32_t c0 = s0 - W.qc0;
        T *lrow = lds + kPieceStride * (mine ? row - k0 : 0);
        uint32_t sm = 0;
        const int32_t nj = mine ? sl : 0;
        for (int32_t j0 = 0; __ballot(j0 < nj); j0 += 4) {  // four words at a time, their loads together
          Raw raw[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            raw[j] = Raw{};
            if (j0 + j < nj && !fast(m, s0 + j0 + j, raw[j])) sm |= 1u << (j0 + j);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j0 + j < nj && !((sm >> (j0 + j)) & 1u)) lrow[c0 + j0 + j] = word(m, s0 + j0 + j, raw[j]);
        }
#pragma unroll 1
        for (int j = 0; j < 16; ++j)  // the rare words off the fast path, one copy of their code
          if (mine && ((sm >> j) & 1u)) lrow[c0 + j] = slow(m, r, s0 + j);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      T *o = out + 16 * k0;
      for (int32_t c = lane; c < 16 * nk; c += 64) {
        const T w = lds[kPieceStride * (c >> 4) + (c & 15)];
        o[c] = w;
        any = any || flag(w);
      }
      __builtin_amdgcn_wave_barrier();  // (the next chunk rezeroes the rows)
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    done(slot, __ballot(any) != 0);
  }
}

// ---- Read-major fills (the default; slice_fill above is the A/B alternative, GQ_FILL=slice) ----
inline int fill_dbg() {  // GQ_FILL_DBG (read_fill): diagnostics and the XCD-contiguous order
  static const int v = getenv("GQ_FILL_DBG") ? atoi(getenv("GQ_FILL_DBG")) : 0;
  return v;
}
inline bool fill_slice_major() {
  static const bool v = getenv("GQ_FILL") && strcmp(getenv("GQ_FILL"), "slice") == 0;
  return v;
}
// The cell / piece fills (a wave per slice, a lane per cell / piece) are the default; GQ_FILL=rw / slice: the
// read-major / slice-major fills of round 4 (A/B alternatives).
inline bool fill_pieces() {  // the cell or piece fills (no preset of the pool)
  static const bool v = !getenv("GQ_FILL") || strcmp(getenv("GQ_FILL"), "pieces") == 0 ||
                        strcmp(getenv("GQ_FILL"), "cells") == 0 || strcmp(getenv("GQ_FILL"), "cellsb") == 0;
  return v;
}
inline int fill_mode() {  // 0: cells (the projection's default), 1: pieces (GQ_FILL=pieces), 2: a workgroup per slice (cellsb)
  static const int v = getenv("GQ_FILL") && strcmp(getenv("GQ_FILL"), "pieces") == 0   ? 1
                       : getenv("GQ_FILL") && strcmp(getenv("GQ_FILL"), "cellsb") == 0 ? 2
                                                                                        : 0;
  return v;
}
// The margin projection's fill: read-major by default (chr20 60x: 5.5 ms against 8.6 ms by cells
// and 15.7 ms by pieces); GQ_MFILL=cells / pieces / slice pick the others.
inline int margin_fill_mode() {  // 0 read-major, 1 cells, 2 pieces, 3 slice-major
  static const int v = !getenv("GQ_MFILL") ? 0
                       : strcmp(getenv("GQ_MFILL"), "cells") == 0 ? 1
                       : strcmp(getenv("GQ_MFILL"), "pieces") == 0 ? 2
                       : strcmp(getenv("GQ_MFILL"), "slice") == 0 ? 3 : 0;
  return v;
}
// One wave per batch of 64 consecutive reads, a lane per word of the batch's projections: a
// read's words (its columns [col0, col1)) sit on consecutive lanes in column order, so its bases /
// qualities load as one contiguous run and each of its pieces' words lands in one row segment.
// No slice window is walked: each read looks up its pieces' rows once (the rows row_count stored
// per (slice, window read)) and keeps their global row numbers in its LDS record, so a round of
// words has no dependent record loads.  kU rounds' loads are issued before the first store.
struct __attribute__((aligned(16))) ReadMeta {
  int64_t p0;         // pool offset of locus 0 (column-eligible reads: base / quality of locus l at p0 + l)
  int32_t s, e;       // the read's [start, end)
  uint32_t info, mq;  // ColDesc info, mapping quality
  int32_t col0;       // first column
  uint32_t evin;      // 1: its MD events are all in ev01 / ev23 (read_fill<true>), else at md_off
  int64_t md_off;     // its MD events
  int64_t qoff;       // its contig's first slice
  int64_t grow[3];    // global row of its first three pieces (-1: no row / pbad slice)
  uint32_t ev01, ev23;  // up to four MD-event offsets from the read's start, 16 bits each (0xFFFF: none)
};
static_assert(sizeof(ReadMeta) == 80, "ReadMeta: five 16-byte LDS reads");
constexpr int kReadPieces = 3;  // pieces per read held in ReadMeta (a 150 bp read spans <= 3 slices)

__device__ __forceinline__ PieceMeta piece_meta(const ReadMeta &m) {  // the fields the word fetches read
  PieceMeta p;
  p.p0 = m.p0;
  p.s = m.s;
  p.e = m.e;
  p.s0 = 0;
  p.row = 0;
  p.info = m.info;
  p.mq = m.mq;
  return p;
}

// Global row of read r's piece in slice `slot` (-1: the slice is pbad or the read has no row there).
__device__ __forceinline__ int64_t piece_grow(const DevReads &R, int64_t r, int64_t slot) {
  if (R.pbad[slot]) return -1;
  const uint16_t k = R.prow[R.soff[slot] + (r - R.sra[slot])];
  return k == 0xFFFFu ? -1 : R.srow[slot] + (int64_t)k;
}

// Global rows of read r's pieces in slices q0 .. q0 + npc - 1 (npc <= kReadPieces; -1: none).
// Every load is issued together — the slices past the read's last piece load that piece's slice
// again — so the pieces cost two dependent rounds of loads, not four each (a load under a
// per-piece branch waits for the one before).  r lies in each of its pieces' slice windows.
__device__ __forceinline__ void piece_grows(const DevReads &R, int64_t r, int64_t q0, int32_t npc,
                                            int64_t (&g)[kReadPieces]) {
  if (npc <= 0) {
#pragma unroll
    for (int j = 0; j < kReadPieces; ++j) g[j] = -1;
    return;
  }
  int64_t so[kReadPieces], sa[kReadPieces], sr[kReadPieces];
  uint32_t pb[kReadPieces], k[kReadPieces];
#pragma unroll
  for (int j = 0; j < kReadPieces; ++j) {
    const int64_t sl = q0 + (j < npc ? j : npc - 1);
    pb[j] = R.pbad[sl];
    so[j] = R.soff[sl];
    sa[j] = R.sra[sl];
    sr[j] = R.srow[sl];
  }
#pragma unroll
  for (int j = 0; j < kReadPieces; ++j) k[j] = R.prow[so[j] + (r - sa[j])];
#pragma unroll
  for (int j = 0; j < kReadPieces; ++j) g[j] = j < npc && !pb[j] && k[j] != 0xFFFFu ? sr[j] + (int64_t)k[j] : -1;
}

// Batches of 64 reads from batch b0 on, stride nb (grid-stride over waves).  For each word of
// each kept read: raw = fetch(read, meta, column) (its loads), then emit(act, raw, read, meta,
// column, grow, slot).  keep(meta) decides per read (false: no words); batch(first read) runs
// at each batch's start (every lane).  meta: this wave's 64 LDS records; owner: its kU * 64 LDS
// words.
// dbg (diagnostics, GQ_FILL_DBG; the pool is wrong when set): 1 no word loads, 2 no word stores;
// 4: XCD-contiguous batches (workgroup i runs on XCD i % 8: each XCD takes one contiguous
// eighth of the batches, so rows that pieces of neighbouring batches share meet in one L2).
// EV: each read's MD events (up to four) are loaded with its records into ev01 / ev23.
// kW: consecutive words of a read per lane (the lane-to-word mapping is done once per kW words).
// src (R.seq or R.qual; nullptr: none): fetch(read, meta, column, pre, fast) gets the word's
// eight bytes at src + p0 + 8 column already loaded when fast (a column-eligible read's word
// inside the pool).
template <int kU, bool EV, int kW, class B, class K, class F, class E>
__device__ __forceinline__ void read_fill(const DevReads &R, ReadMeta *__restrict__ meta, uint32_t *__restrict__ owner,
                                          int dbg, const uint8_t *src, B &&batch, K &&keep, F &&fetch, E &&emit) {
  const int lane = threadIdx.x & 63;
  const int64_t nbat = (R.n_reads + 63) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  int64_t wid = wave_id();
  if (dbg & 4) {
    const int64_t per = (int64_t)gridDim.x >> 3;  // (the grid is a multiple of 8)
    wid = ((int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3)) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    wid = __builtin_amdgcn_readfirstlane((int)wid);
  }
  for (int64_t b = wid; b < nbat; b += nw) {
    batch(64 * b);
    const int64_t r = 64 * b + lane;
    const bool in = r < R.n_reads;
    const int64_t rr = in ? r : 64 * b;
    // the read's records in one round of loads
    const ProjRec pr = R.prec[rr];
    const ColDesc d = R.cdesc[rr];
    const int64_t so = R.seq_off[rr];
    const int32_t ld = R.lead[rr];
    const uint32_t mq = R.mapq[rr];
    const int64_t mdo = R.md_off[rr];
    int lo = 0, hi = R.n_contigs - 1;  // contig: last c with contig_read_begin[c] <= r
    while (lo < hi) {
      const int m = (lo + hi + 1) >> 1;
      if (R.contig_read_begin[m] <= rr) lo = m;
      else hi = m - 1;
    }
    ReadMeta m;
    m.p0 = so + (ld > 0 ? ld : 0) - d.start;
    m.s = d.start;
    m.e = d.end;
    m.info = d.info;
    m.mq = mq;
    m.col0 = pr.col0;
    m.evin = 0;
    m.ev01 = m.ev23 = 0xFFFFFFFFu;
    m.md_off = mdo;
    if constexpr (EV) {
      const int32_t nmd = (int32_t)(d.info & 0xFFFFu);
      if (in && nmd <= 4 && d.end - d.start < 0xFFF0) {  // (no word of the read reaches the 0xFFFF marker)
        // (the four loads issued together: past the read's last event its last one again)
        uint32_t v[4];
        if (nmd > 0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = R.md_ev[mdo + (k < nmd ? k : nmd - 1)];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = k < nmd ? v[k] : 0xFFFFFFFFu;
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = v[k] >> 8;  // offsets (none: 0xFFFFFF)
        bool ok = true;
#pragma unroll
        for (int k = 0; k < 4; ++k) ok = ok && (k >= nmd || o[k] < 0xFFFFu);
        if (ok) {
          m.evin = 1;
          m.ev01 = (o[0] & 0xFFFFu) | ((o[1] & 0xFFFFu) << 16);
          m.ev23 = (o[2] & 0xFFFFu) | ((o[3] & 0xFFFFu) << 16);
        }
      }
    }
    m.qoff = R.qoff[lo];
    uint32_t len = in && pr.col1 != kProjNone && pr.col1 > pr.col0 ? (uint32_t)(pr.col1 - pr.col0) : 0u;
    if (len && !keep(m)) len = 0;
    const uint32_t nun = (len + (uint32_t)kW - 1u) / (uint32_t)kW;  // the read's lane units
    {
      const int64_t q0 = m.qoff + (pr.col0 >> 4);
      const int32_t npc = len ? ((pr.col1 - 1) >> 4) - (pr.col0 >> 4) + 1 : 0;
      int64_t g[kReadPieces];
      piece_grows(R, rr, q0, npc < kReadPieces ? npc : kReadPieces, g);
#pragma unroll
      for (int j = 0; j < kReadPieces; ++j) m.grow[j] = g[j];
    }
    if (len) meta[lane] = m;
    const uint32_t incl = wave_incl_scan(nun), ex = incl - nun;
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    for (uint32_t w0 = 0; w0 < tot; w0 += 64 * kU) {
#pragma unroll
      for (int u = 0; u < kU; ++u) owner[64 * u + lane] = 0;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (nun > 0 && ex > w0 && ex < w0 + 64 * kU) owner[ex - w0] = (uint32_t)lane + 1;  // the read's first unit
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      constexpr int N = kU * kW;
      int kk[N];
      int32_t col[N];
      bool act[N];
      int64_t grow[N], slot[N];
      ReadMeta pm[kU];
      decltype(fetch((int64_t)0, pm[0], (int32_t)0, 0ull, false)) raw[N];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const uint32_t wb = w0 + 64 * u, w = wb + (uint32_t)lane;
        const unsigned long long run = __ballot(nun > 0 && ex <= wb);  // the last of them runs at wb
        const uint32_t k_at = run ? 64u - (uint32_t)__clzll((long long)run) : 0u;  // its lane + 1
        const uint32_t k1 = max(wave_incl_max(owner[64 * u + lane]), k_at);
        const bool au = w < tot;
        const int k = au ? (int)k1 - 1 : 0;
        const uint4 *src = reinterpret_cast<const uint4 *>(meta + k);
        const uint4 a = src[0], bq = src[1], c = src[2], dq = src[3], eq = src[4];
        ReadMeta &mm = pm[u];
        mm.p0 = (int64_t)((uint64_t)a.x | ((uint64_t)a.y << 32));
        mm.s = (int32_t)a.z;
        mm.e = (int32_t)a.w;
        mm.info = bq.x;
        mm.mq = bq.y;
        mm.col0 = (int32_t)bq.z;
        mm.evin = bq.w;
        mm.ev01 = eq.z;
        mm.ev23 = eq.w;
        mm.md_off = (int64_t)((uint64_t)c.x | ((uint64_t)c.y << 32));
        mm.qoff = (int64_t)((uint64_t)c.z | ((uint64_t)c.w << 32));
        const int64_t g0 = (int64_t)((uint64_t)dq.x | ((uint64_t)dq.y << 32));
        const int64_t g1 = (int64_t)((uint64_t)dq.z | ((uint64_t)dq.w << 32));
        const int64_t g2 = (int64_t)((uint64_t)eq.x | ((uint64_t)eq.y << 32));
        const uint32_t kex = (uint32_t)__shfl((int)ex, k, 64);
        const int32_t cbase = mm.col0 + kW * (int32_t)(w - kex);
        const int32_t col1 = (mm.e + 7) >> 3;  // the read's column end (prec_fill)
#pragma unroll
        for (int q = 0; q < kW; ++q) {
          const int i = kW * u + q;
          kk[i] = k;
          col[i] = cbase + q;
          act[i] = au && col[i] < col1;
          const int32_t pj = (col[i] >> 4) - (mm.col0 >> 4);
          slot[i] = mm.qoff + (col[i] >> 4);
          grow[i] = pj == 0 ? g0 : pj == 1 ? g1 : pj == 2 ? g2 : -2;
        }
      }
#pragma unroll
      for (int i = 0; i < N; ++i) {
        if (act[i] && grow[i] == -2) grow[i] = piece_grow(R, 64 * b + kk[i], slot[i]);  // a long read's later piece
        act[i] = act[i] && grow[i] >= 0;
      }
      // The N words' 8-byte loads first, every lane's (a word off the fast path loads src[0],
      // unused): a load under a per-word branch, or its mask applied right after it, would make
      // the wave wait for each before issuing the next.
      uint64_t pre[N];
      bool fast[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const ReadMeta &mi = pm[i / kW];
        const int64_t a = mi.p0 + 8 * (int64_t)col[i];
        fast[i] = src != nullptr && act[i] && (mi.info & kColEligible) && a >= 0 && a + 8 <= R.seq_cap;
        pre[i] = src != nullptr && R.seq_cap >= 8 && !(dbg & 1)
                     ? *reinterpret_cast<const gq_u64u *>(src + (fast[i] ? a : 0))
                     : 0ull;
      }
#pragma unroll
      for (int i = 0; i < N; ++i) {
        if (act[i] && !(dbg & 1)) raw[i] = fetch(64 * b + kk[i], pm[i / kW], col[i], pre[i], fast[i]);
        else raw[i] = {};
      }
#pragma unroll
      for (int i = 0; i < N; ++i)
        emit(act[i] && !(dbg & 2), raw[i], 64 * b + kk[i], pm[i / kW], col[i], grow[i], slot[i]);
    }
    __builtin_amdgcn_wave_barrier();  // (the next batch rewrites meta)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

// Wave-aggregated reservation of n <= 3 slots per lane on an LDS counter: lane prefixes
// from two ballots, one returning LDS atomic by the first active lane (a few hundred
// cycles, not the microseconds of a returning device-scope atomic).
__device__ __forceinline__ unsigned wave_reserve_lds(unsigned *ctr, unsigned n) {
  const uint64_t b1 = __ballot(n & 1u), b2 = __ballot(n & 2u);
  if ((b1 | b2) == 0) return 0;
  const uint64_t lt = __builtin_amdgcn_read_exec() & ((1ull << (threadIdx.x & 63)) - 1ull);
  const unsigned pre = (unsigned)__popcll(b1 & lt) + 2u * (unsigned)__popcll(b2 & lt);
  const unsigned total = (unsigned)__popcll(b1) + 2u * (unsigned)__popcll(b2);
  unsigned base = 0;
  if (lt == 0) base = atomicAdd(ctr, total);  // the first active lane
  base = (unsigned)__builtin_amdgcn_readfirstlane((int)base);
  return base + pre;
}

struct Plan {
  int64_t n_tiles = 0;
  int64_t n_loci = 0;
  int T = 0;
  bool aligned = false;  // tiles are pieces of T-aligned locus blocks (germline_proj)
  // the non-empty loci ranges in call order (host copies): contig, [start, end), first tile,
  // task, and the window each belongs to.  A window = a maximal run of ranges of one (task,
  // contig): one SlidingWindow per task and contig (DistributedUtil.scala:473-486).
  std::vector<int32_t> rc, rwin;
  std::vector<int64_t> rs, re, rt, rtask;
  struct Win {
    int32_t contig;
    int64_t r0, r1;  // ranges [r0, r1)
  };
  std::vector<Win> wins;
  // device copies (plan(), in the context's ranges buffer: valid until its next plan()): the
  // ranges' starts / ends, each range's window, each window's contig and first range (+ end)
  const int64_t *d_rs = nullptr, *d_re = nullptr, *d_wroff = nullptr;
  const int32_t *d_rwin = nullptr, *d_wcontig = nullptr;
  int64_t range_of_tile(int64_t t) const {  // last range whose first tile <= t
    return (int64_t)(std::upper_bound(rt.begin(), rt.end(), t) - rt.begin()) - 1;
  }
  int64_t tiles_of(int64_t r) const {
    const int64_t s = rs[(size_t)r], e = re[(size_t)r];
    return aligned ? (e - 1) / T - s / T + 1 : (e - s + T - 1) / T;
  }
};

// A locus whose pileup reference base depends on the queue's heap order (the reads' MD tags
// disagree there): listed by the kernels, resolved by heap_ref_bases.
struct AmbItem {
  int32_t tile, pos;
  int64_t item;  // the kernel's own item index (complex item / candidate)
};

}  // namespace gq

// ==========================================================================================
// Host side: context, resident read sets
// ==========================================================================================
namespace gq {
struct DevBuf {
  void *p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    size_t want = std::max(bytes, (size_t)256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) n = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};
}  // namespace gq

struct gq_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[8] = {};
  hipEvent_t dev_ev[4] = {};  // the derivation's device spans (gq_reads_info: derive / projection / fill)
  // a second stream for derivation kernels independent of the main stream's (the pool scan beside
  // the read checks, the sparse entries beside the projection fill), joined by side_ev
  hipStream_t side = nullptr;
  hipEvent_t side_ev[4] = {};
  gq_timings timings{};
  int germ_tile = gq::kGermT;
  int n_cu = 0;
  int proj_wg_per_cu = 0;  // resident germline_proj workgroups per CU (occupancy query, once)
  int dir_wg_per_cu = 0;   // resident germline_direct workgroups per CU (occupancy query, once)
  int som_wg_per_cu = 0;   // resident somatic_proj workgroups per CU
  int somd_wg_per_cu = 0;  // resident somatic_direct workgroups per CU
  gq::DevBuf mtab;         // somatic_direct: the margin-term table (margin_table, 64 KiB)
  int mtab_key = -1;       // its probability model (1: including alignment), -1: not built
  int call_wg_per_cu = 0;  // resident somatic_call_k<false> workgroups per CU
  gq::DevBuf ranges, tiles, recs, recs_sorted, keys, keys_sorted, idx, idx_sorted, cplx, pool, counters, sort_tmp, image, tiles2, srecs;
  gq::DevBuf c_depth, c_pos, c_base, c_indel, c_ref, c_rb, c_amb, slow, deep_tiles;
  gq::DevBuf amb, amb_ref, heap_off, heap_reads;  // heap-order reference bases (heap_ref_bases)
  gq::DevBuf win_meta, win_grp;                    // somatic pileup element order (window_first / _group)
  gq::DevBuf deep_list, deep_scratch;              // somatic: the deep caller's list and per-wave scratch
  int front_wg_per_cu = 0;                         // somatic_front: resident workgroups per CU
  gq::DevBuf cands;                                // somatic: the candidates' records (CandRec)
  gq::DevBuf el_store;                             // somatic: the split caller's element store (ElemStore)
  gq::DevBuf win_bound;                            // germline: window bounds (window_bounds)
  gq::DevBuf bkt;                                  // germline output order: bucket counts / offsets / fill
  // The bulk host -> device staging (H2DStager): two pinned chunks kept for the context's life
  // and allocated by `prep`, a helper thread gq_open starts (pinning 128 MB takes ~20 ms, and
  // freeing it as long: neither belongs on a load's path).  prep also loads the library's code
  // objects onto the device (a no-op launch per translation unit), which HIP otherwise does at a
  // module's first launch (~30 ms).
  void *stage[2] = {nullptr, nullptr};
  hipEvent_t stage_done[2] = {};
  bool stage_used[2] = {false, false};
  std::mutex stage_m;
  std::condition_variable stage_cv;
  bool stage_ready = false;
  hipError_t stage_err = hipSuccess;
  std::thread prep;
  hipError_t wait_stage() {
    std::unique_lock<std::mutex> lk(stage_m);
    stage_cv.wait(lk, [this] { return stage_ready; });
    return stage_err;
  }
  void *pin = nullptr;                             // pinned host staging for the small per-call copies
  size_t pin_n = 0;
  hipError_t pinned(size_t bytes) {                // pin has >= bytes (contents not kept)
    if (bytes <= pin_n) return hipSuccess;
    if (pin) (void)hipHostFree(pin);
    pin = nullptr;
    pin_n = 0;
    const size_t want = std::max(bytes, (size_t)65536);
    hipError_t e = hipHostMalloc(&pin, want, hipHostMallocDefault);
    if (e == hipSuccess) pin_n = want;
    return e;
  }
};

// Device buffers of the structures derived from a resident read set's SoA (the upload-time
// derivation, the projection, the margin projection) and of their temporaries.  A temporary goes
// back to `spare` when done; gq_reads_rederive hands every live buffer back, and a derivation of
// the same read set then takes its sizes from the spares: no hipMalloc / hipFree (each an
// implicit device synchronisation) on a re-derivation.
struct DerivedPool {
  std::vector<std::pair<void *, size_t>> live, spare;
  hipError_t get(void **p, size_t bytes) {
    bytes = std::max(bytes, (size_t)16);
    size_t best = spare.size();
    for (size_t i = 0; i < spare.size(); ++i)  // the smallest spare that fits without much waste
      if (spare[i].second >= bytes && spare[i].second <= bytes + bytes / 4 + 65536 &&
          (best == spare.size() || spare[i].second < spare[best].second))
        best = i;
    if (best < spare.size()) {
      *p = spare[best].first;
      live.push_back(spare[best]);
      spare.erase(spare.begin() + (long)best);
      return hipSuccess;
    }
    *p = nullptr;
    const hipError_t e = hipMalloc(p, bytes);
    if (e == hipSuccess) live.emplace_back(*p, bytes);
    return e;
  }
  void put(void *p) {  // (stream-ordered: later work on the same stream may reuse it)
    for (size_t i = 0; i < live.size(); ++i)
      if (live[i].first == p) {
        spare.push_back(live[i]);
        live.erase(live.begin() + (long)i);
        return;
      }
  }
  void release_all() {
    spare.insert(spare.end(), live.begin(), live.end());
    live.clear();
  }
  void free_all() {
    for (auto &x : live) (void)hipFree(x.first);
    for (auto &x : spare) (void)hipFree(x.first);
    live.clear();
    spare.clear();
  }
};

struct gq_dev_reads {
  gq_ctx *ctx = nullptr;
  gq::DevReads d{};
  std::vector<int64_t> contig_read_begin;  // host copy
  std::vector<void *> owned;               // device allocations of the SoA owned by this handle
  mutable DerivedPool dp;                  // the derived structures' buffers
  int64_t seq_bytes = 0;
  int64_t proj_bytes = 0, pev_count = 0, proj_reads = 0;  // projection sizes (derive_shape)
  int64_t n_slices = 0;                                    // projection slices (128 loci) over all contigs
  int64_t n_rows = 0;                                      // projection rows (kProjRowBytes each, ProjRec)
  float h2d_ms = 0, derive_ms = 0;                         // upload wall times (gq_reads_info)
  bool columns = false;            // the column records and base classes are derived (ensure_columns)
  bool ev_bases = false;           // ev_rb is derived (ensure_ev_bases)
  bool projected = false;          // the projection is derived (ensure_projection)
  void *nnb = nullptr;             // N bases per read (pool_clean), for the projection's sparse entries
  float proj_ms = 0;               // ensure_projection's wall time
  float fill_ms = 0;               // its pool fill kernel(s), HIP events on the context's stream
  float proj_dev_ms = 0;           // its device span (first kernel to last), HIP events
  float derive_dev_ms = 0;         // the upload-time derivation's device span, HIP events
  // A re-derivation does not wait for its spans: their events (derive start / end, projection
  // start, fill start / end, projection end) and the taken-read counters are read when the
  // figures are asked for (gq_reads_get_info) or before the next re-derivation (settle_stats).
  hipEvent_t tev[6] = {};
  unsigned pending = 0;            // 1: derivation span, 2: projection span, fill and proj_reads
  unsigned long long *nok = nullptr;  // proj_prep's spread counters (kOkSpread words) while pending & 2
  mutable void *mproj = nullptr;  // somatic margin projection (a biased byte per locus-read), for mproj_mapq
  mutable int mproj_mapq = -1;
  mutable void *mnb = nullptr;    // per slice: 1 if a margin term there is kMargin8None (no bound)
};

namespace gq {
// H2D of large pageable host arrays at PCIe rate: a copy from pageable memory goes through the
// runtime's own small bounce buffer (≈ 3 GB/s measured for the 4 GB bench shard); here the host
// bytes are copied by several threads into one of two pinned 64 MiB chunks while the DMA engine
// drains the other.
struct H2DStager {
  static constexpr size_t kChunk = size_t(64) << 20;
  gq_ctx *c;
  hipStream_t stream;
  void **buf = nullptr;
  hipEvent_t *done = nullptr;
  bool *used = nullptr;
  int slot = 0;
  unsigned threads = 1;
  explicit H2DStager(gq_ctx *ctx) : c(ctx), stream(ctx->stream) {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    threads = std::min(16u, hw);  // the GPU box's CPU share is 16 threads
  }
  ~H2DStager() {  // the chunks stay with the context; its copies must have drained
    for (int i = 0; done && i < 2; ++i)
      if (used[i]) (void)hipEventSynchronize(done[i]);
  }
  hipError_t init() {
    const hipError_t e = c->wait_stage();
    if (e != hipSuccess) return e;
    buf = c->stage;
    done = c->stage_done;
    used = c->stage_used;
    return hipSuccess;
  }
  // out[0, k) <- bytes [o, o + k) of the logical source, split over the threads
  template <class F>
  void fill(uint8_t *out, size_t o, size_t k, const F &src_range) const {
    const unsigned t = (unsigned)std::min<size_t>(threads, std::max<size_t>(1, k >> 22));  // >= 4 MiB / thread
    if (t <= 1) {
      src_range(out, o, k);
      return;
    }
    std::vector<std::thread> th;
    const size_t per = (k + t - 1) / t;
    for (unsigned i = 0; i < t; ++i) {
      const size_t a = (size_t)i * per;
      if (a >= k) break;
      th.emplace_back([&, a] { src_range(out + a, o + a, std::min(per, k - a)); });
    }
    for (auto &x : th) x.join();
  }
  // landed(end): called after each chunk's copy is enqueued on the stream (bytes [0, end) are
  // then in order on it), e.g. to start work on another stream behind an event
  template <class F, class G>
  hipError_t copy_from(void *dst, size_t bytes, const F &src_range, const G &landed) {
    for (size_t o = 0; o < bytes; o += kChunk) {
      const size_t k = std::min(kChunk, bytes - o);
      if (used[slot]) {
        hipError_t e = hipEventSynchronize(done[slot]);
        if (e != hipSuccess) return e;
      }
      fill((uint8_t *)buf[slot], o, k, src_range);
      hipError_t e = hipMemcpyAsync((char *)dst + o, buf[slot], k, hipMemcpyHostToDevice, stream);
      if (e == hipSuccess) e = hipEventRecord(done[slot], stream);
      if (e != hipSuccess) return e;
      used[slot] = true;
      slot ^= 1;
      e = landed(o + k);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  template <class F>
  hipError_t copy_from(void *dst, size_t bytes, const F &src_range) {
    return copy_from(dst, bytes, src_range, [](size_t) { return hipSuccess; });
  }
  hipError_t copy(void *dst, const void *src, size_t bytes) {
    return copy_from(dst, bytes, [src](uint8_t *out, size_t o, size_t k) { memcpy(out, (const uint8_t *)src + o, k); });
  }
};

// Upload-time derivation of a resident read set whose SoA arrays (and host copy of
// contig_read_begin) are in place: validation, read shape, projection pool, block index.
gq_status derive_shape(gq_ctx *c, gq_dev_reads *d, int64_t md_len);
// The column records (ColDesc, the auxiliary list, clean / N-base counts), derived on first use.
gq_status ensure_columns(gq_ctx *c, const gq_dev_reads *d);
// ev_rb (the read base under each MD event) of a resident read set, derived on first use
gq_status ensure_ev_bases(gq_ctx *c, const gq_dev_reads *d);
// The projection (ProjRec) of a resident read set, derived on first use.
// A margin projection wanted with the projection (the somatic tumor, germline-standard): with
// GQ_FILL_ONE both are filled in one read-major pass (fused_projection_fill) when the projection
// is derived — an A/B alternative: at chr20 60x it took 9.0 ms against 2.8 + 5.6 ms for the two
// passes, so the default keeps them separate.
struct MarginReq {
  int min_mapq;
  bool incl_align;
};
gq_status ensure_projection(gq_ctx *c, const gq_dev_reads *d, const MarginReq *mr = nullptr);
gq_status fused_projection_fill(gq_ctx *c, const gq_dev_reads *d, uint8_t *proj_pool, const MarginReq &mr);
// No-op launches that load each translation unit's code object onto the device (gq_open's prep).
hipError_t warm_pileup(hipStream_t s);
hipError_t warm_somatic(hipStream_t s);
hipError_t warm_heapref(hipStream_t s);
hipError_t warm_bamdev(hipStream_t s);

// Loci ranges -> locus tiles of T loci with each tile's read window in `rd`, written to `tiles`.
gq_status plan(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, int T, Plan &pl, DevBuf &tiles,
               int stage_cap = 0, int meta_cap = 0, int ev_cap = 0, bool aligned = false);
gq_status check_device_error(gq_ctx *c, const Counters &h);
// Pileup.referenceBaseAtLocus in the reference's heap order at each listed locus, for each of
// the read sets (advanced together, as the somatic caller's two windows are): the queues are
// replayed on the host (gq_replay.h) and the bases read on the device.  out_ref (device,
// n * sets.size() bytes) receives item i's base for set k at i * sets.size() + k.  `tiles`
// are the plan's device tiles (the same loci plan for every set).
gq_status heap_ref_bases(gq_ctx *c, const Plan &pl, const DevBuf &tiles_buf,
                         const std::vector<const gq_dev_reads *> &sets, const std::vector<AmbItem> &items,
                         uint8_t *out_ref);

// For each locus range [a, b) of `ranges` on contig `contig`: does a read of `set` overlap it
// (out[i] = 1)?  A device search: the first read with pmax_end > a is the first read ending
// past a, and a read overlaps [a, b) iff that one starts before b.
gq_status reads_overlap(gq_ctx *c, const gq_dev_reads *set, int32_t contig,
                        const std::vector<std::pair<int64_t, int64_t>> &ranges, std::vector<char> &out);
}  // namespace gq

