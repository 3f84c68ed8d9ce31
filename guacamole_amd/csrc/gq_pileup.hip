// gq_pileup.hip — MI355X (gfx950) pileup + per-locus germline-threshold engine.
//
// Kernels (see DESIGN.md for the roofline of each):
//   plan_tiles          one thread per locus tile: range lookup + binary search of the
//                       tile's read window [rb, re) (prefix-max end / start).
//   germline_tile<T>    one workgroup per tile of T loci: waves walk overlapping reads
//                       (lanes = 64 consecutive loci of a CIGAR op) and histogram
//                       elements into LDS with ds_add; then one thread per locus
//                       makes the GermlineThreshold decision on-device for "simple"
//                       loci (only Match/Mismatch elements with A/C/G/T/N bases and
//                       an unambiguous MD-derived reference base) and queues the
//                       rest for germline_complex.
//   germline_complex    one wave per queued locus: exact PileupElement semantics,
//                       variable-length alleles grouped by a 128-bit allele key in
//                       registers, GermlineThreshold case split.
//   counts_tile<T>      raw per-locus histogram (gq_pileup_counts).
//   + hipcub radix sort of the call records by output ordinal.
//
// Semantics restated from /root/reference/src/main/scala/org/hammerlab/guacamole/:
//   commands/GermlineThresholdCaller.scala:90-179, pileup/PileupElement.scala:68-248,
//   pileup/Pileup.scala:49-186, DistributedUtil.scala:260-306, windowing/SlidingWindow.scala.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gqpileup.h"
#include "gq_host.h"
#include "gq_alleles.h"

using namespace gq;

// ---- Exclusive scan of 32-bit per-read counts into 64-bit offsets (reduce, then scan) ------
// Tiles of 4096 counts (256 threads x 16 consecutive counts): tile sums, one workgroup scanning
// the tile sums, then each tile scanned again from its offset.  Reads the counts twice and
// writes the offsets once.
namespace {
constexpr int kScanT = 256, kScanV = 16, kScanTile = kScanT * kScanV;

__device__ __forceinline__ void scan_load16(const uint32_t *__restrict__ in, int64_t n, int64_t i0, uint32_t (&v)[kScanV]) {
  if (i0 + kScanV <= n) {
    const uint4 *p = reinterpret_cast<const uint4 *>(in + i0);
#pragma unroll
    for (int k = 0; k < kScanV / 4; ++k) {
      const uint4 w = p[k];
      v[4 * k] = w.x, v[4 * k + 1] = w.y, v[4 * k + 2] = w.z, v[4 * k + 3] = w.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kScanV; ++k) v[k] = i0 + k < n ? in[i0 + k] : 0u;
  }
}
// Exclusive prefix of x over the workgroup's kScanT threads (LDS, Hillis-Steele); *total: the sum.
__device__ __forceinline__ int64_t block_excl_i64(int64_t x, int64_t *lds, int64_t *total) {
  const int t = threadIdx.x;
  lds[t] = x;
  __syncthreads();
  for (int d = 1; d < kScanT; d <<= 1) {
    const int64_t y = t >= d ? lds[t - d] : 0;
    __syncthreads();
    lds[t] += y;
    __syncthreads();
  }
  const int64_t incl = lds[t];
  if (total) *total = lds[kScanT - 1];
  __syncthreads();
  return incl - x;
}
__global__ __launch_bounds__(kScanT) void scan_tile_sums(const uint32_t *__restrict__ in, int64_t n,
                                                         int64_t *__restrict__ sums) {
  __shared__ int64_t lds[kScanT];
  uint32_t v[kScanV];
  scan_load16(in, n, (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanV, v);
  int64_t x = 0;
#pragma unroll
  for (int k = 0; k < kScanV; ++k) x += v[k];
  int64_t tot = 0;
  (void)block_excl_i64(x, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}
// One workgroup: sums[0 .. nt) -> their exclusive prefix, in place.
__global__ __launch_bounds__(kScanT) void scan_sums_excl(int64_t *__restrict__ sums, int64_t nt) {
  __shared__ int64_t lds[kScanT];
  const int64_t per = (nt + kScanT - 1) / kScanT;
  const int64_t a = (int64_t)threadIdx.x * per, b = a + per < nt ? a + per : nt;
  int64_t x = 0;
  for (int64_t i = a; i < b; ++i) x += sums[i];
  int64_t run = block_excl_i64(x, lds, nullptr);
  for (int64_t i = a; i < b; ++i) {
    const int64_t y = sums[i];
    sums[i] = run;
    run += y;
  }
}
__global__ __launch_bounds__(kScanT) void scan_tiles(const uint32_t *__restrict__ in, int64_t n,
                                                     const int64_t *__restrict__ base, int64_t *__restrict__ out) {
  __shared__ int64_t lds[kScanT];
  const int64_t i0 = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanV;
  uint32_t v[kScanV];
  scan_load16(in, n, i0, v);
  int64_t x = 0;
#pragma unroll
  for (int k = 0; k < kScanV; ++k) x += v[k];
  int64_t run = base[blockIdx.x] + block_excl_i64(x, lds, nullptr);
  int64_t o[kScanV];
#pragma unroll
  for (int k = 0; k < kScanV; ++k) {
    o[k] = run;
    run += v[k];
  }
  if (i0 + kScanV <= n) {
    int4 *q = reinterpret_cast<int4 *>(out + i0);
#pragma unroll
    for (int k = 0; k < kScanV / 2; ++k)
      q[k] = make_int4((int)(uint32_t)o[2 * k], (int)(uint32_t)((uint64_t)o[2 * k] >> 32), (int)(uint32_t)o[2 * k + 1],
                       (int)(uint32_t)((uint64_t)o[2 * k + 1] >> 32));
  } else {
#pragma unroll
    for (int k = 0; k < kScanV; ++k)
      if (i0 + k < n) out[i0 + k] = o[k];
  }
}
}  // namespace

// out[i] = in[0] + ... + in[i - 1] for i < n (in and out 16-byte aligned).
static hipError_t scan_u32_to_i64(DerivedPool &dp, const uint32_t *in, int64_t *out, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t nt = (n + kScanTile - 1) / kScanTile;
  void *sums = nullptr;
  hipError_t e = dp.get(&sums, sizeof(int64_t) * (size_t)nt);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(scan_tile_sums, dim3((unsigned)nt), dim3(kScanT), 0, st, in, n, (int64_t *)sums);
  hipLaunchKernelGGL(scan_sums_excl, dim3(1), dim3(kScanT), 0, st, (int64_t *)sums, nt);
  hipLaunchKernelGGL(scan_tiles, dim3((unsigned)nt), dim3(kScanT), 0, st, in, n, (const int64_t *)sums, out);
  e = hipGetLastError();
  dp.put(sums);
  return e;
}

namespace gq {
thread_local std::string g_err;

gq_status set_err(gq_status s, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return s;
}

}  // namespace gq

namespace {
// ------------------------------------------------------------------------------------------
// Tile planning
// ------------------------------------------------------------------------------------------
// The block index of the reads (DevReads::blk_rb / blk_rs): one thread per 512-locus block.
__global__ void block_index(DevReads R, int64_t n_blocks, int64_t *__restrict__ blk_rb, int64_t *__restrict__ blk_rs) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_blocks) return;
  int lo = 0, hi = R.n_contigs - 1;  // the contig: last c with qoff[c] / 4 <= g
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if ((R.qoff[m] >> 2) <= g) lo = m;
    else hi = m - 1;
  }
  const int c = lo;
  const int64_t blk = (g - (R.qoff[c] >> 2)) * 512;
  const int64_t b = R.contig_read_begin[c], e = R.contig_read_begin[c + 1];
  int64_t a0 = b, a1 = e;
  while (a0 < a1) {
    const int64_t m = (a0 + a1) >> 1;
    if ((int64_t)R.pmax_end[m] > blk) a1 = m;
    else a0 = m + 1;
  }
  blk_rb[g] = a0;
  a1 = e;
  while (a0 < a1) {
    const int64_t m = (a0 + a1) >> 1;
    if ((int64_t)R.start[m] >= blk) a1 = m;
    else a0 = m + 1;
  }
  blk_rs[g] = a0;
}

__global__ void plan_tiles(const int32_t *__restrict__ r_contig, const int64_t *__restrict__ r_start,
                           const int64_t *__restrict__ r_end, const int64_t *__restrict__ r_ord,
                           const int64_t *__restrict__ r_tile0, int64_t n_ranges, int64_t n_tiles, int T,
                           DevReads R, Tile *__restrict__ tiles, int stage_cap, int meta_cap, int ev_cap,
                           int aligned, TileX *__restrict__ tilex) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  int64_t lo = 0, hi = n_ranges - 1;  // largest r with r_tile0[r] <= t
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if (r_tile0[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  const int64_t r = lo;
  // aligned: tiles are the range's pieces of the T-aligned blocks it meets (T a power of two)
  const int64_t blk = (r_start[r] / T + (t - r_tile0[r])) * (int64_t)T;
  const int64_t L0 = aligned ? max(r_start[r], blk) : r_start[r] + (t - r_tile0[r]) * (int64_t)T;
  const int64_t L1 = aligned ? min(blk + (int64_t)T, r_end[r]) : min(L0 + (int64_t)T, r_end[r]);
  const int32_t c = r_contig[r];
  int64_t b = R.contig_read_begin[c], e = R.contig_read_begin[c + 1];
  // rb: first read with pmax_end > L0 (pmax_end non-decreasing within the contig); aligned
  // tiles start their window at the block (every read with words in the block's projection
  // slices, so that a read's place in a slice is the sum of the window's earlier pieces)
  const int64_t W0 = aligned ? blk : L0;
  int64_t a0 = b, a1 = e;
  // aligned tiles: the window from the upload-time block index (blocks past the contig's
  // last read end hold no reads: [e, e))
  const int64_t g0 = aligned && T == 512 && R.blk_rb ? (R.qoff[c] >> 2) + blk / 512 : -1, g1 = aligned ? (R.qoff[c + 1] >> 2) : -1;
  if (g0 >= 0) {
    if (g0 >= g1) {
      a0 = a1 = e;
    } else {
      a0 = R.blk_rb[g0];
      // re in [first start >= blk, first start >= blk + 512]
      a1 = g0 + 1 < g1 ? R.blk_rs[g0 + 1] : e;
      if (L1 < blk + (int64_t)T) {
        int64_t s0 = max(a0, R.blk_rs[g0]);
        while (s0 < a1) {
          int64_t m = (s0 + a1) >> 1;
          if ((int64_t)R.start[m] >= L1) a1 = m;
          else s0 = m + 1;
        }
      }
    }
  } else {
    while (a0 < a1) {
      int64_t m = (a0 + a1) >> 1;
      if ((int64_t)R.pmax_end[m] > W0) a1 = m;
      else a0 = m + 1;
    }
  }
  const int64_t rb = a0;
  if (g0 >= 0) {
    a0 = a1;  // re
  } else {
    a0 = rb;
    a1 = e;  // re: first read with start >= L1
    while (a0 < a1) {
      int64_t m = (a0 + a1) >> 1;
      if ((int64_t)R.start[m] >= L1) a1 = m;
      else a0 = m + 1;
    }
  }
  Tile tl;
  tl.ordinal0 = r_ord[r] + (L0 - r_start[r]);
  tl.rb = rb;
  tl.re = a0;
  tl.contig = c;
  tl.L0 = (int32_t)L0;
  tl.L1 = (int32_t)L1;
  tl.range = (int32_t)r;
  // the germline column kernel stages the whole read window of a tile in LDS: at most
  // meta_cap reads, sequence bytes within stage_cap (1 KiB pieces), at most ev_cap MD events
  // (4-event aligned).  Otherwise sbytes = 0 and the tile goes to the walker kernel.
  tl.sb0 = 0;
  tl.sbytes = 0;
  tl.mb0 = 0;
  tl.mcnt = 0;
  if (stage_cap > 0 && a0 > rb && a0 - rb <= meta_cap) {
    const int64_t B0 = R.seq_off[rb] & ~(int64_t)15;
    const int64_t nb = R.seq_off[a0 - 1] + R.seq_len[a0 - 1] - B0;
    const int64_t M0 = R.caux_off[rb] & ~(int64_t)3;
    const int64_t nm = R.caux_off[a0] - M0;
    if (nb > 0 && ((nb + 1023) >> 10) * 1024 <= stage_cap && B0 + ((nb + 1023) >> 10) * 1024 <= R.seq_cap &&
        nm >= 0 && nm <= ev_cap) {
      tl.sb0 = B0;
      tl.sbytes = (int32_t)nb;
      tl.mb0 = M0;
      tl.mcnt = (int32_t)nm;
    }
  }
  // (the projection kernels' aligned tiles are planned without staging: mb0 is free for qs, so
  //  their setup skips a dependent qoff load)
  if (aligned && stage_cap == 0 && R.qoff) tl.qs = R.qoff[c] + blk / 128;
  tiles[t] = tl;
  if (tilex) {  // aligned projection tiles: germline_proj's per-tile setup, resolved here
    TileX x{};
    if (R.srow && R.qoff && a0 > rb) {
      const int64_t qs = tl.qs;
      x.row0 = R.srow[qs];
#pragma unroll
      for (int g = 0; g < 4; ++g) x.nr[g] = (int32_t)(R.srow[qs + g + 1] - R.srow[qs + g]);
      x.e0 = R.pev_off[rb];
      x.e1 = R.pev_off[a0];
      uint32_t bad = 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) bad |= (R.pbad[qs + g] ? 1u : 0u) << (8 * g);
      x.pbad4 = bad;
    }
    tilex[t] = x;
  }
}

#include "gq_direct_common.h"  // general_segments (a general-CIGAR read as segments), wave scans

__device__ __forceinline__ bool col_base_ok(const DevReads &R, int64_t r) {
  const int32_t s = R.start[r], e = R.end[r], nmd = R.n_md[r];
  return R.clean[r] && nmd >= 0 && nmd < 65536 && e - s < 32768 && e > s;
}

// Words of each read's auxiliary list (MD events, then two per segment of a general read).
__global__ void col_count(DevReads R, uint32_t *__restrict__ n_aux) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > R.n_reads) return;
  if (r == R.n_reads) {
    n_aux[r] = 0;
    return;
  }
  int32_t nseg = 0;
  if (R.lead[r] < 0 && col_base_ok(R, r) &&
      !general_segments(R, r, [&](uint32_t, int32_t, int32_t, int32_t, int32_t) { ++nseg; }))
    nseg = 0;
  n_aux[r] = (uint32_t)(R.n_md[r] > 0 ? R.n_md[r] : 0) + 2u * (uint32_t)nseg;
}

// The packed ColDesc of each read and its auxiliary list at aux_off[r]: one u32 per MD event
// (offset << 16 | MD base << 8 | read base), then per segment (ref_off | len << 16,
// seq_off | kind << 16).
// aux_bound: the list's allocated words.  The list is sized from the pools (MD events + 6 words
// per CIGAR op), which bounds it only when no two reads share MD or CIGAR pool words; a read whose
// list would end past the allocation gets none (not column-eligible: the walkers take it).
__global__ void col_derive(DevReads R, const int64_t *__restrict__ aux_off, ColDesc *__restrict__ cd,
                           uint32_t *__restrict__ aux, int64_t aux_bound) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R.n_reads) return;
  const int32_t s = R.start[r], e = R.end[r], lead = R.lead[r];
  const bool fits = aux_off[r + 1] <= aux_bound;
  const int32_t nmd = R.n_md[r];
  const bool base_ok = fits && col_base_ok(R, r);
  const bool ok = lead >= 0 && base_ok;
  uint32_t *o = aux + aux_off[r];
  const int32_t nev = nmd > 0 ? nmd : 0;
  int32_t nseg = 0;
  bool gen = false;
  if (lead < 0 && base_ok && aux_off[r + 1] - aux_off[r] > nev) {  // col_count found segments
    gen = general_segments(R, r, [&](uint32_t kind, int32_t ref_off, int32_t len, int32_t seq_off, int32_t q) {
      o[nev + 2 * q] = (uint32_t)ref_off | ((uint32_t)len << 16);
      o[nev + 2 * q + 1] = (uint32_t)seq_off | (kind << 16);
      nseg = q + 1;
    });
  }
  ColDesc d;
  d.start = s;
  d.end = e;
  d.pmax_end = R.pmax_end[r];
  d.info = (uint32_t)(nmd > 0 ? (nmd < 65536 ? nmd : 65535) : 0) | (ok ? kColEligible : 0u) |
           (gen ? kColGeneral | ((uint32_t)nseg << 18) : 0u);
  d.seq_lo = (uint32_t)(uint64_t)(R.seq_off[r] + (lead > 0 ? lead : 0));
  d.md_lo = (uint32_t)(uint64_t)aux_off[r];
  cd[r] = d;
  if (fits && nmd > 0) {  // four events per round of loads (past the last: the last again)
    const uint32_t *ev = R.md_ev + R.md_off[r];
    const uint8_t *rb = R.ev_rb + R.md_off[r];
    for (int32_t k0 = 0; k0 < nmd; k0 += 4) {
      uint32_t e4[4], b4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t k = k0 + j < nmd ? k0 + j : nmd - 1;
        e4[j] = ev[k];
        b4[j] = rb[k];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t off = e4[j] >> 8;
        if (k0 + j < nmd) o[k0 + j] = off < 32768u ? (off << 16) | ((e4[j] & 0xFFu) << 8) | b4[j] : 0xFFFFFFFFu;
      }
    }
  }
}

// ---- Projections (germline_proj, ProjRec in gq_kernels.h), derived after col_derive -------
__device__ __forceinline__ bool proj_ok(uint32_t info) { return (info & (kColEligible | kColGeneral)) != 0; }
// Codes of four bases of a column-eligible read (A C G T N, 0 outside the read): the low three
// bits index a v_perm table (A 1, C 3, T 4, N 0, G 7, 0 -> 0) — proj_codes4 for such bytes.
__device__ __forceinline__ uint32_t perm_codes4(uint32_t x) {
  return __builtin_amdgcn_perm(0x07000004u, 0x03000100u, x & 0x07070707u);
}

// Each slice's read window (slice_window), thread per slice: its first read and its number of
// reads (scanned into the offsets of their rows); entry n_slices: 0.
__global__ void slice_windows(DevReads R, int64_t n_slices, int64_t *__restrict__ sra, int64_t *__restrict__ scnt) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q > n_slices) return;
  if (q == n_slices) {
    sra[q] = 0;
    scnt[q] = 0;
    return;
  }
  const SliceWin W = slice_window(R, q);
  sra[q] = W.ra;
  scnt[q] = W.rz - W.ra;
}

// The projection's per-read records in one pass (thread per read, record n: zeros): ProjRec
// (prec_fill), the pbad slices of the reads the projection cannot take (slice_bad), the sparse
// entries per read (proj_count) and the reads it takes, counted into kSpread words (proj_count_ok).
constexpr int kOkSpread = 1024;  // proj_prep's count words (summed on the host)
__global__ void proj_prep(DevReads R, const uint32_t *__restrict__ n_nbase, ProjRec *__restrict__ prec,
                          uint8_t *__restrict__ pbad, uint32_t *__restrict__ nents, unsigned long long *__restrict__ n_ok) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  ProjRec p{0, 0};
  int64_t e = 0;
  bool ok = false;
  if (r < R.n_reads) {
    const ColDesc d = R.cdesc[r];
    ok = proj_ok(d.info);
    p.col0 = d.start >> 3;
    p.col1 = ok ? (d.end + 7) >> 3 : kProjNone;
    if (ok) {
      const int32_t nmd = (int32_t)(d.info & 0xFFFFu);
      e = nmd + (int64_t)n_nbase[r];
      if (d.info & kColGeneral) {
        const int32_t nseg = (int32_t)((d.info >> 18) & 0xFFu);
        const uint32_t *sg = R.cev + R.caux_off[r] + nmd;
        for (int32_t q = 0; q < nseg; ++q) e += (sg[2 * q + 1] >> 16) != kSegCount ? 1 : 0;
      }
    } else {  // its slices go to the walkers
      int lo = 0, hi = R.n_contigs - 1;
      while (lo < hi) {
        const int m = (lo + hi + 1) >> 1;
        if (R.contig_read_begin[m] <= r) lo = m;
        else hi = m - 1;
      }
      const int64_t q0 = R.qoff[lo];
      const int32_t s = R.start[r], en = R.end[r];
      if (en > s && s >= 0)
        for (int32_t q = s >> 7; q <= (en - 1) >> 7; ++q) pbad[q0 + q] = 1;
    }
  }
  if (r <= R.n_reads) {
    prec[r] = p;
    nents[r] = (uint32_t)e;
  }
  // the block's count: one LDS add per wave, one global add per block, spread over kOkSpread words
  __shared__ unsigned long long s_ok;
  if (threadIdx.x == 0) s_ok = 0;
  __syncthreads();
  const unsigned long long k = (unsigned long long)__popcll(__ballot(ok));
  if ((threadIdx.x & 63) == 0 && k) atomicAdd(&s_ok, k);
  __syncthreads();
  if (threadIdx.x == 0 && s_ok) atomicAdd(&n_ok[blockIdx.x & (kOkSpread - 1)], s_ok);
}

// Rows of each slice and each of its reads' row (slice_assign_rows, one wave per slice); past
// kSliceRowsMax the slice is pbad (and gets no rows).
__global__ __launch_bounds__(256) void row_count(DevReads R, int64_t n_slices, uint16_t *__restrict__ prow,
                                                 int32_t *__restrict__ srows, uint8_t *__restrict__ pbad,
                                                 int first_fit) {
  __shared__ __attribute__((aligned(16))) uint8_t s_rend[4][kSliceRowsMax];
  __shared__ uint16_t s_fl[4][kSliceRowsMax];
  const int wv = threadIdx.x >> 6;
  const int64_t w0 = wave_id();
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t slot = w0; slot < n_slices; slot += nw) {
    const SliceWin W = slice_stored(R, slot);
    // the parallel assignment (its E / row lists in the first-fit pass's LDS), first-fit past it
    int32_t n = first_fit ? -2
                                 : slice_rows_fifo(R, W, prow + R.soff[slot], reinterpret_cast<uint16_t *>(s_rend[wv]),
                                                   s_fl[wv], reinterpret_cast<uint32_t *>(s_fl[wv] + kRowsLdsPieces));
    if (n == -2) n = slice_assign_rows(R, W, prow + R.soff[slot], s_rend[wv], s_fl[wv]);
    if ((threadIdx.x & 63) == 0) {
      srows[slot] = n < 0 ? 0 : (n + kRowPad - 1) & ~(kRowPad - 1);  // zero rows up to a multiple of kRowPad
      if (n < 0) pbad[slot] = 1;
    }
  }
}
__global__ void rows64(int64_t n, const int32_t *__restrict__ srows, int64_t *__restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q <= n) out[q] = q < n ? srows[q] : 0;
}

// The projection pool in block rows, one wave per slice, a lane per word (the rows row_count
// assigned, stored; pbad slices stay zero: their blocks go to the walker).
// KU: words per lane per round (GQ_FILL_U picks 1 or 4: fewer registers and more waves, or more
// loads in flight per wave; measured at chr20 60x: 1 word 4.8 ms, 4 words 5.8 ms, so 1 is the default)
template <int KU>
__global__ __launch_bounds__(256) void proj_fill(DevReads R, int64_t n_slices, uint8_t *__restrict__ proj) {
  __shared__ PieceMeta s_meta[4][64];
  __shared__ uint32_t s_owner[4][KU * 64];
  PieceMeta *meta = s_meta[threadIdx.x >> 6];
  uint32_t *owner = s_owner[threadIdx.x >> 6];
  const int64_t w0 = wave_id();
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t slot = w0; slot < n_slices; slot += nw) {
    if (R.pbad[slot]) continue;  // uniform
    uint32_t *out = reinterpret_cast<uint32_t *>(proj) + 16 * R.srow[slot];  // the slice's block rows
    slice_fill<false, KU>(
        R, slice_stored(R, slot), R.prow + R.soff[slot], meta, owner,
        [&](int64_t, PieceMeta &, int64_t) { return true; },
        [&](int64_t r, const PieceMeta &m, int32_t col, uint32_t) { return proj_fetch(R, r, m, col); },
        [&](bool act, const ProjRaw &x, int64_t, const PieceMeta &m, int32_t col, uint32_t) {
          if (act)
            out[16 * (int64_t)m.row + (col & 15)] =
                x.gen ? x.word : proj_codes4((uint32_t)x.b) | (proj_codes4((uint32_t)(x.b >> 32)) << 4);
        });
  }
}

// The projection pool, read-major (read_fill): a wave per 64 consecutive reads, a lane per word.
template <int KU, int KW>
__global__ __launch_bounds__(256) void proj_fill_rw(DevReads R, uint8_t *__restrict__ proj, int dbg) {
  __shared__ ReadMeta s_meta[4][64];
  __shared__ uint32_t s_owner[4][KU * 64];
  uint32_t *out = reinterpret_cast<uint32_t *>(proj);
  read_fill<KU, false, KW>(
      R, s_meta[threadIdx.x >> 6], s_owner[threadIdx.x >> 6], dbg, R.seq, [](int64_t) {},
      [](const ReadMeta &) { return true; },
      [&](int64_t r, const ReadMeta &m, int32_t col, uint64_t pre, bool fast) {
        if (fast) return ProjRaw{pre & edge_mask(m.s - 8 * col, m.e - 8 * col), 0u, 0u};
        return proj_fetch(R, r, piece_meta(m), col);
      },
      [&](bool act, const ProjRaw &x, int64_t, const ReadMeta &, int32_t col, int64_t grow, int64_t) {
        if (act)  // (an eligible read's bytes are A C G T N: the v_perm lookup)
          out[16 * grow + (col & 15)] =
              x.gen ? x.word : perm_codes4((uint32_t)x.b) | (perm_codes4((uint32_t)(x.b >> 32)) << 4);
      });
}

// ---- The projection pool by cells (the default) ----
// A wave per slice, a lane per cell (row k, column c) of its rows, every word written (zeros where
// no piece lies: the pool needs no preset), 64 consecutive words per store.  The window's reads
// are staged in LDS as 16-byte records (pool offset of locus 0 relative to the window's first
// read, start, end, ColDesc info) and a map cell -> window read (u8) is marked from each piece's
// stored row; a cell then costs one map read, one record read, one 8-byte load of its bases from
// the pool (a 32-bit offset on the window's base), a v_perm code lookup and its store.  Slices
// with more than kCell3Win window reads are listed in deep (their rows zeroed) for the
// slice-major fill.
constexpr int kCell3Win = 255;    // window reads a u8 map can name
constexpr int kCell3Rows = 64;    // rows per map chunk
static_assert(kCell3Rows % kRowPad == 0, "chunks hold whole kRowPad row groups");
struct __attribute__((aligned(16))) Cell3Rec {
  uint32_t a;         // seq_off + leading clip - seq_off[window's first read]
  int32_t s, e;       // [start, end)
  uint32_t info;      // ColDesc info (bit kColEligible: the fast path)
};
template <int CU>  // cells per lane whose loads issue together (4; A/B GQ_FILL_U=8)
__global__ __launch_bounds__(256) void proj_fill_cells(DevReads R, int64_t n_slices, uint8_t *__restrict__ proj,
                                                       int64_t *__restrict__ deep, unsigned long long *__restrict__ n_deep,
                                                       int dbg) {
  __shared__ Cell3Rec s_rec[4][kCell3Win];
  __shared__ uint8_t s_map[4][kCell3Rows * 16];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Cell3Rec *rec = s_rec[wv];
  uint8_t *map = s_map[wv];
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t slot = wave_id(); slot < n_slices; slot += nw) {
    const int64_t g0 = R.srow[slot];
    const int32_t nr = (int32_t)(R.srow[slot + 1] - g0);
    if (nr <= 0) continue;
    uint32_t *out = reinterpret_cast<uint32_t *>(proj) + 16 * g0;
    const SliceWin W = slice_stored(R, slot);
    const int32_t nwin = (int32_t)(W.rz - W.ra);
    if (R.pbad[slot] || nwin > kCell3Win || nwin <= 0) {
      for (int32_t c = lane; c < 16 * nr; c += 64) out[c] = 0u;
      if (!R.pbad[slot] && nwin > kCell3Win && lane == 0) deep[atomicAdd(n_deep, 1ull)] = slot;
      continue;
    }
    const int64_t base = R.seq_off[W.ra];  // the window's bytes: [base, ...) in read order
    const uint8_t *pool = R.seq + base;
    const int64_t span = R.seq_cap - base;  // readable bytes from pool
    const uint16_t *prw = R.prow + R.soff[slot];
    int32_t prow_i = 0xFFFF, pc0 = 0, psl = 0;  // this lane's window read (first batch) and its piece
    for (int32_t i = lane; i < nwin; i += 64) {
      const int64_t r = W.ra + i;
      const ColDesc d = R.cdesc[r];
      const int32_t ld = R.lead[r];
      const int64_t so = R.seq_off[r];
      const ProjRec pr = R.prec[r];
      const int32_t row = prw[i];
      // a read whose bytes do not follow the window's first read's (a wrapped pool in another
      // order) takes the slow path: a = kCell3Far
      const int64_t av = so + (ld > 0 ? ld : 0) - base;
      Cell3Rec m;
      m.a = R.pool_ordered && av >= 0 && av < (int64_t)kCell3Far ? (uint32_t)av : kCell3Far;
      m.s = d.start;
      m.e = d.end;
      m.info = d.info;
      rec[i] = m;
      int32_t s0, sl;
      piece_of(pr, W.qc0, s0, sl);
      if (i < 64) {
        prow_i = row;
        pc0 = s0 - W.qc0;
        psl = row == 0xFFFF ? 0 : sl;
      }
    }
    if (dbg & 16) continue;  // ablation: the window's records only
    for (int32_t k0 = 0; k0 < nr; k0 += kCell3Rows) {
      const int32_t nk = nr - k0 < kCell3Rows ? nr - k0 : kCell3Rows;
      for (int32_t c = lane; c < 16 * nk; c += 64) map[c] = 0xFFu;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      for (int32_t i = lane; i < nwin; i += 64) {  // each piece marks its cells in the chunk
        int32_t row = prow_i, c0 = pc0, sl = psl;
        if (i >= 64) {  // (windows over 64 reads: the later batches' pieces reloaded)
          row = prw[i];
          int32_t s0;
          piece_of(R.prec[W.ra + i], W.qc0, s0, sl);
          c0 = s0 - W.qc0;
          sl = row == 0xFFFF ? 0 : sl;
        }
        if (sl <= 0 || row < k0 || row >= k0 + nk) continue;
        uint8_t *mp = map + 16 * (row - k0) + c0;
        for (int32_t j = 0; j < sl; ++j) mp[j] = (uint8_t)i;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      uint32_t *o = out + 16 * k0;
      for (int32_t c00 = (dbg & 8) ? 16 * nk : 0; c00 < 16 * nk; c00 += 64 * CU) {  // CU cells per lane, loads together
        uint64_t b[CU], mk[CU];
        uint32_t slow = 0;
        // Every lane loads (an empty or slow cell the window's first word, masked off): a load
        // under a divergent branch, or a mask applied right after it, makes the wave wait for it
        // before the next cell's — one load in flight instead of CU.
#pragma unroll
        for (int u = 0; u < CU; ++u) {
          const int32_t c = c00 + 64 * u + lane;
          const uint32_t pp = c < 16 * nk ? map[c] : 0xFFu;
          const Cell3Rec m = rec[pp != 0xFFu ? pp : 0];
          const int32_t lb = 8 * (W.qc0 + (c & 15));
          const int64_t v = (int64_t)m.a + lb - m.s;
          const bool ok = (m.info & kColEligible) && m.a != kCell3Far && v >= 0 && v + 8 <= span;
          if (pp != 0xFFu && !ok) slow |= 1u << u;
          mk[u] = pp != 0xFFu && ok ? edge_mask(m.s - lb, m.e - lb) : 0ull;
          const uint32_t off = pp != 0xFFu && ok ? (uint32_t)v : 0u;
          b[u] = (dbg & 1) || span < 8 ? (uint64_t)off  // (ablation bit 0: no loads)
                                       : *reinterpret_cast<const gq_u64u *>(pool + off);
        }
        uint32_t x[CU];
#pragma unroll
        for (int u = 0; u < CU; ++u) {
          const uint64_t y = b[u] & mk[u];
          x[u] = perm_codes4((uint32_t)y) | (perm_codes4((uint32_t)(y >> 32)) << 4);
        }
        // Stores under a wave-uniform bound only (16 nk is a multiple of 64: rows are padded to
        // kRowPad), slow cells included — their slow path below rewrites them: stores under
        // divergent branches are each made to wait for the last one.
#pragma unroll
        for (int u = 0; u < CU; ++u)
          if (c00 + 64 * u < 16 * nk) o[c00 + 64 * u + lane] = x[u];
        if (slow) {  // rare: a general CIGAR, a word at the pool's end
#pragma unroll 1
          for (int u = 0; u < CU; ++u) {
            if (!((slow >> u) & 1u)) continue;
            const int32_t c = c00 + 64 * u + lane;
            const uint32_t p = map[c];
            const Cell3Rec m = rec[p];
            const int64_t r = W.ra + p;
            const int32_t ld = R.lead[r];
            PieceMeta pm;
            pm.p0 = R.seq_off[r] + (ld > 0 ? ld : 0) - m.s;  // (from the read itself: any pool order)
            pm.s = m.s;
            pm.e = m.e;
            pm.s0 = 0;
            pm.row = 0;
            pm.info = m.info;
            pm.mq = 0;
            const ProjRaw x = proj_fetch(R, r, pm, W.qc0 + (c & 15));
            o[c] = x.gen ? x.word : proj_codes4((uint32_t)x.b) | (proj_codes4((uint32_t)(x.b >> 32)) << 4);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();  // (the next chunk rewrites the map)
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
  }
}

// The cell fill with a workgroup per slice (GQ_FILL=cellsb, A/B): the window's records in one
// round (a thread per window read), the map marked by all four waves, each thread four cells.
__global__ __launch_bounds__(256) void proj_fill_cellsb(DevReads R, int64_t n_slices, uint8_t *__restrict__ proj,
                                                        int64_t *__restrict__ deep, unsigned long long *__restrict__ n_deep,
                                                        int dbg) {
  __shared__ Cell3Rec rec[kCell3Win + 1];
  __shared__ uint8_t map[kCell3Rows * 16];
  const int tid = threadIdx.x;
  for (int64_t slot = blockIdx.x; slot < n_slices; slot += gridDim.x) {
    const int64_t g0 = R.srow[slot];
    const int32_t nr = (int32_t)(R.srow[slot + 1] - g0);
    if (nr <= 0) continue;
    uint32_t *out = reinterpret_cast<uint32_t *>(proj) + 16 * g0;
    const SliceWin W = slice_stored(R, slot);
    const int32_t nwin = (int32_t)(W.rz - W.ra);
    if (R.pbad[slot] || nwin > kCell3Win || nwin <= 0) {
      for (int32_t c = tid; c < 16 * nr; c += 256) out[c] = 0u;
      if (!R.pbad[slot] && nwin > kCell3Win && tid == 0) deep[atomicAdd(n_deep, 1ull)] = slot;
      continue;
    }
    const int64_t base = R.seq_off[W.ra];
    const uint8_t *pool = R.seq + base;
    const int64_t span = R.seq_cap - base;
    int32_t prow_i = 0xFFFF, pc0 = 0, psl = 0;
    if (tid < nwin) {
      const int64_t r = W.ra + tid;
      const ColDesc d = R.cdesc[r];
      const int32_t ld = R.lead[r];
      const int64_t so = R.seq_off[r];
      const ProjRec pr = R.prec[r];
      const int32_t row = R.prow[R.soff[slot] + tid];
      const int64_t av = so + (ld > 0 ? ld : 0) - base;
      Cell3Rec m;
      m.a = R.pool_ordered && av >= 0 && av < (int64_t)kCell3Far ? (uint32_t)av : kCell3Far;
      m.s = d.start;
      m.e = d.end;
      m.info = d.info;
      rec[tid] = m;
      int32_t s0, sl;
      piece_of(pr, W.qc0, s0, sl);
      prow_i = row;
      pc0 = s0 - W.qc0;
      psl = row == 0xFFFF ? 0 : sl;
    }
    for (int32_t k0 = 0; k0 < nr; k0 += kCell3Rows) {
      const int32_t nk = nr - k0 < kCell3Rows ? nr - k0 : kCell3Rows;
      for (int32_t c = tid; c < 16 * nk; c += 256) map[c] = 0xFFu;
      __syncthreads();
      if (psl > 0 && prow_i >= k0 && prow_i < k0 + nk) {
        uint8_t *mp = map + 16 * (prow_i - k0) + pc0;
        for (int32_t j = 0; j < psl; ++j) mp[j] = (uint8_t)tid;
      }
      __syncthreads();
      uint32_t *o = out + 16 * k0;
      uint64_t b[4], mk[4];
      uint32_t slow = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int32_t c = 256 * u + tid;
        const uint32_t pp = c < 16 * nk ? map[c] : 0xFFu;
        const Cell3Rec m = rec[pp != 0xFFu ? pp : 0];
        const int32_t lb = 8 * (W.qc0 + (c & 15));
        const int64_t v = (int64_t)m.a + lb - m.s;
        const bool ok = (m.info & kColEligible) && m.a != kCell3Far && v >= 0 && v + 8 <= span;
        if (pp != 0xFFu && !ok) slow |= 1u << u;
        mk[u] = pp != 0xFFu && ok ? edge_mask(m.s - lb, m.e - lb) : 0ull;
        const uint32_t off = pp != 0xFFu && ok ? (uint32_t)v : 0u;
        b[u] = span < 8 ? (uint64_t)off : *reinterpret_cast<const gq_u64u *>(pool + off);
      }
      uint32_t x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint64_t y = b[u] & mk[u];
        x[u] = perm_codes4((uint32_t)y) | (perm_codes4((uint32_t)(y >> 32)) << 4);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)  // (a wave's 64 cells lie all inside or all past 16 nk: rows padded to kRowPad)
        if (256 * u + (tid & ~63) < 16 * nk) o[256 * u + tid] = x[u];
      if (slow) {
#pragma unroll 1
        for (int u = 0; u < 4; ++u) {
          if (!((slow >> u) & 1u)) continue;
          const int32_t c = 256 * u + tid;
          const uint32_t p = map[c];
          const Cell3Rec m = rec[p];
          const int64_t r = W.ra + p;
          const int32_t ld = R.lead[r];
          PieceMeta pm;
          pm.p0 = R.seq_off[r] + (ld > 0 ? ld : 0) - m.s;
          pm.s = m.s;
          pm.e = m.e;
          pm.s0 = 0;
          pm.row = 0;
          pm.info = m.info;
          pm.mq = 0;
          const ProjRaw xx = proj_fetch(R, r, pm, W.qc0 + (c & 15));
          o[c] = xx.gen ? xx.word : proj_codes4((uint32_t)xx.b) | (proj_codes4((uint32_t)(xx.b >> 32)) << 4);
        }
      }
      __syncthreads();  // (the next chunk rewrites the map, the next slice the records)
    }
  }
}

// The listed (deep) slices, slice-major (their rows zeroed by proj_fill_cells).
__global__ __launch_bounds__(256) void proj_fill_deep(DevReads R, const int64_t *__restrict__ deep,
                                                      const unsigned long long *__restrict__ n_deep,
                                                      uint8_t *__restrict__ proj) {
  __shared__ PieceMeta s_meta[4][64];
  __shared__ uint32_t s_owner[4][64];
  PieceMeta *meta = s_meta[threadIdx.x >> 6];
  uint32_t *owner = s_owner[threadIdx.x >> 6];
  const int64_t nd = (int64_t)*n_deep;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave_id(); i < nd; i += nw) {
    const int64_t slot = deep[i];
    uint32_t *out = reinterpret_cast<uint32_t *>(proj) + 16 * R.srow[slot];
    slice_fill<false, 1>(
        R, slice_stored(R, slot), R.prow + R.soff[slot], meta, owner,
        [&](int64_t, PieceMeta &, int64_t) { return true; },
        [&](int64_t r, const PieceMeta &m, int32_t col, uint32_t) { return proj_fetch(R, r, m, col); },
        [&](bool act, const ProjRaw &x, int64_t, const PieceMeta &m, int32_t col, uint32_t) {
          if (act)
            out[16 * (int64_t)m.row + (col & 15)] =
                x.gen ? x.word : proj_codes4((uint32_t)x.b) | (proj_codes4((uint32_t)(x.b >> 32)) << 4);
        });
  }
}

// The projection pool slice by slice (piece_fill in gq_host.h): a wave per slice, a lane per
// piece, the rows built in LDS and written whole (zeros where no piece lies: no preset).
__global__ __launch_bounds__(256) void proj_fill_pieces(DevReads R, int64_t n_slices, uint8_t *__restrict__ proj,
                                                        int dbg) {
  __shared__ uint32_t s_rows[4][kPieceRows * kPieceStride];
  piece_fill<uint32_t, uint64_t, false>(
      R, n_slices, s_rows[threadIdx.x >> 6], reinterpret_cast<uint32_t *>(proj), 0u,
      [](const PieceRec &) { return true; },
      [&](const PieceRec &m, int32_t col, uint64_t &b) {  // a column-eligible read's eight bases, one load
        const int32_t lb = 8 * col;
        const int64_t a = m.p0 + lb;
        if (!(m.info & kColEligible) || a < 0 || a + 8 > R.seq_cap) return false;
        if (dbg & 1) {  // ablation: no loads
          b = (uint64_t)a;
          return true;
        }
        b = *reinterpret_cast<const gq_u64u *>(R.seq + a);
        if (m.s > lb || m.e < lb + 8) b &= edge_mask(m.s - lb, m.e - lb);  // (the read's first / last word)
        return true;
      },
      [](const PieceRec &, int32_t, uint64_t b) {
        return proj_codes4_clean((uint32_t)b) | (proj_codes4_clean((uint32_t)(b >> 32)) << 4);
      },
      [&](const PieceRec &m, int64_t r, int32_t col) {
        const ProjRaw x = proj_fetch(R, r, piece_rec_meta(m), col);
        return x.gen ? x.word : proj_codes4((uint32_t)x.b) | (proj_codes4((uint32_t)(x.b >> 32)) << 4);
      },
      [](uint32_t) { return false; }, [](int64_t, bool) {});
}

// The sparse entries of each read (thread per read): MD events, N bases (without an event),
// complex segments; unused slots of the N bound are padding.
__global__ void pev_fill(DevReads R, const int64_t *__restrict__ eoff, uint2 *__restrict__ pev) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R.n_reads) return;
  const ColDesc d = R.cdesc[r];
  if (!proj_ok(d.info)) return;
  int64_t o = eoff[r];
  const int64_t o1 = eoff[r + 1];
  const int32_t s = d.start, nmd = (int32_t)(d.info & 0xFFFFu);
  const uint32_t *ev = R.md_ev + R.md_off[r];
  const uint8_t *evb = R.ev_rb + R.md_off[r];
  for (int32_t k = 0; k < nmd; ++k) {
    const uint32_t x = ev[k];
    const uint8_t rb = evb[k];
    const int c = rb == 0 ? 7 : base_cat(rb);
    pev[o++] = make_uint2((uint32_t)(s + (int32_t)(x >> 8)), std_bit((uint8_t)(x & 0xFFu)) | ((uint32_t)(c <= 4 ? c : 7) << 4));
  }
  // N bases of the Match/Mismatch elements that carry no MD event (an event entry counts those)
  auto n_run = [&](int32_t ra, int32_t len, int64_t p) {  // loci [ra, ra + len) at pool offset p
    int32_t k = 0;
    for (int32_t i = 0; i < len && o < o1; ++i) {
      if (R.seq[p + i] != 'N') continue;
      const int32_t off = ra + i - s;
      while (k < nmd && (int32_t)(ev[k] >> 8) < off) ++k;
      if (k < nmd && (int32_t)(ev[k] >> 8) == off) continue;
      pev[o++] = make_uint2((uint32_t)(ra + i), 4u << 4);
    }
  };
  if (d.info & kColGeneral) {
    const int32_t nseg = (int32_t)((d.info >> 18) & 0xFFu);
    const uint32_t *sg = R.cev + R.caux_off[r] + nmd;
    for (int32_t q = 0; q < nseg; ++q) {
      const uint32_t a = sg[2 * q], b = sg[2 * q + 1];
      const int32_t ra = s + (int32_t)(a & 0xFFFFu), rl = (int32_t)(a >> 16);
      if ((b >> 16) != kSegCount)
        pev[o++] = make_uint2((uint32_t)ra, kPevComplex | ((b >> 16) == kSegMidDel ? kPevMidDel : 0u) | (uint32_t)rl);
      else if (o < o1) n_run(ra, rl, R.seq_off[r] + (int32_t)(b & 0xFFFFu));
    }
  } else if (o < o1) {
    n_run(s, d.end - s, R.seq_off[r] + (R.lead[r] > 0 ? R.lead[r] : 0));
  }
  for (; o < o1; ++o) pev[o] = make_uint2(0x80000000u, kPevNone);
}

// Upload-time checks, one thread per read (bits of *bad): 1 = reads not sorted by start within
// their contig, or pmax_end not the running maximum of end (SlidingWindow.scala:55-56 "Regions
// must be sorted"; plan_tiles binary-searches both); 2 = an offset / length outside its pool or
// a sample slot >= n_samples (would read out of bounds); 4 = the sequence pool is not in read
// order (flags only: such tiles take the walker).
__device__ __forceinline__ int validate_one(const DevReads &R, int64_t r) {
  int lo = 0, hi = R.n_contigs;  // contig of r: last c with contig_read_begin[c] <= r
  while (lo < hi) {
    const int m = (lo + hi + 1) >> 1;
    if (R.contig_read_begin[m] <= r) lo = m;
    else hi = m - 1;
  }
  // every field in one round of loads (read r - 1's as read 0's own for r = 0), then the tests
  // without short-circuits (a load behind a || would wait for the one before)
  const int64_t rp = r > 0 ? r - 1 : r;
  const bool first = R.contig_read_begin[lo] == r;
  const int32_t s = R.start[r], e = R.end[r], pm = R.pmax_end[r], s1 = R.start[rp], pm1 = R.pmax_end[rp];
  const int64_t so = R.seq_off[r], so1 = R.seq_off[rp], co = R.cigar_off[r], mo = R.md_off[r];
  const int32_t sl = R.seq_len[r], sl1 = R.seq_len[rp], nc = R.n_cigar[r], nm = R.n_md[r];
  const int smp = (int)R.sample[r];
  int b = 0;
  b |= ((e < s) | (s < 0)) ? 1 : 0;
  b |= (first ? pm != e : ((s < s1) | (pm != max(pm1, e)))) ? 1 : 0;
  b |= ((so < 0) | (sl < 0) | (so + sl > R.seq_bytes)) ? 2 : 0;
  b |= ((co < 0) | (nc < 0) | (co + nc > R.cigar_len)) ? 2 : 0;
  b |= ((nm > 0) & ((mo < 0) | (mo + nm > R.md_len))) ? 2 : 0;
  b |= smp >= R.n_samples ? 2 : 0;
  b |= ((r > 0) & (so < so1 + sl1)) ? 4 : 0;
  return b;
}

// clean[r] = every sequenced byte of read r is one of A C G T N (the germline column path's
// precondition).  Pool in read order: 16 bytes per thread, coalesced; the rare other bytes
// find their read by binary search of seq_off and clear its flag (clean preset to 1).
__global__ void pool_clean(DevReads R, uint8_t *__restrict__ clean, uint32_t *__restrict__ n_nbase) {
  // two 16-byte chunks per thread (both loads in flight before either is checked), kBlock apart
  const int64_t c0 = (int64_t)blockIdx.x * (2 * kBlock) + threadIdx.x;
  uint32_t ws[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t b0 = (c0 + (int64_t)h * kBlock) * 16;
    ws[h][0] = ws[h][1] = ws[h][2] = ws[h][3] = 0x41414141u;  // past the pool: nothing to check
    if (b0 >= R.seq_bytes) continue;
    if (b0 + 16 <= R.seq_cap) {  // uploaded pools have a zeroed tail; a wrapped one may end anywhere
      const uint4 w = *reinterpret_cast<const uint4 *>(R.seq + b0);
      ws[h][0] = w.x, ws[h][1] = w.y, ws[h][2] = w.z, ws[h][3] = w.w;
    } else {
      ws[h][0] = ws[h][1] = ws[h][2] = ws[h][3] = 0;
      for (int k = 0; k < 16 && b0 + k < R.seq_bytes; ++k) ws[h][k >> 2] |= (uint32_t)R.seq[b0 + k] << (8 * (k & 3));
    }
  }
  // bytes equal to A, C, G or T: 0x80 in their byte (exact SWAR compare, no carries between bytes)
  auto acgt = [](uint32_t x) {
    auto eq = [x](uint32_t pat) {
      const uint32_t z = x ^ pat;
      return ~(((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z | 0x7F7F7F7Fu);
    };
    return eq(0x41414141u) | eq(0x43434343u) | eq(0x47474747u) | eq(0x54545454u);
  };
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t b0 = (c0 + (int64_t)h * kBlock) * 16;
    if (b0 >= R.seq_bytes) continue;
    if ((acgt(ws[h][0]) & acgt(ws[h][1]) & acgt(ws[h][2]) & acgt(ws[h][3])) == 0x80808080u) continue;  // the common chunk
    for (int k = 0; k < 16; ++k) {
      const uint8_t x = (uint8_t)(ws[h][k >> 2] >> (8 * (k & 3)));
      if (b0 + k >= R.seq_bytes || x == 'A' || x == 'C' || x == 'G' || x == 'T') continue;
      int64_t lo = 0, hi = R.n_reads - 1;  // last read with seq_off <= b0 + k
      while (lo < hi) {
        const int64_t m = (lo + hi + 1) >> 1;
        if (R.seq_off[m] <= b0 + k) lo = m;
        else hi = m - 1;
      }
      // zero-length reads share an offset with their neighbour: every read holding the byte.
      // An N keeps the read clean and is counted (the projection's N-base entries).
      for (int64_t r = lo; r >= 0 && R.seq_off[r] + R.seq_len[r] > b0 + k; --r)
        if (R.seq_off[r] <= b0 + k) {
          if (x == 'N') atomicAdd(&n_nbase[r], 1u);
          else clean[r] = 0;
        }
    }
  }
}
// The same per read (a wrapped pool in another order), one thread per read.
__global__ void read_clean(DevReads R, uint8_t *__restrict__ clean, uint32_t *__restrict__ n_nbase) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R.n_reads) return;
  const uint8_t *q = R.seq + R.seq_off[r];
  bool ok = true;
  uint32_t nn = 0;
  for (int32_t k = 0; k < R.seq_len[r]; ++k) {
    const uint8_t b = q[k];
    ok = ok && (b == 'A' || b == 'C' || b == 'G' || b == 'T' || b == 'N');
    nn += b == 'N' ? 1u : 0u;
  }
  clean[r] = ok ? 1 : 0;
  n_nbase[r] = nn;
}

// CIGAR shape per read (derived once at upload): leading soft clip if the CIGAR is
// [S|H]* (M|=|X) [S|H]* and the sequence covers it, else -(1 + the (M|=|X) operations) (general
// walker; germline_direct reserves that many count segments).
__device__ __forceinline__ void shape_one(const DevReads &R, int64_t r, int16_t *__restrict__ lead, bool bad) {
  // a read whose offsets lie outside their pools (bad) reads nothing: n = 0
  const int64_t off = R.cigar_off[r];
  const int32_t n = bad ? 0 : R.n_cigar[r];
  // the first four CIGAR operations in one round of loads (past the last: the last again), ahead
  // of the shape test that decides what they mean (indexes clamped into the pool: the loads do
  // not wait for validate_one's verdict)
  uint32_t c4[4] = {0u, 0u, 0u, 0u};
  const int32_t n_raw = R.n_cigar[r];
  auto clampi = [](int64_t x, int64_t len) { return x < 0 ? (int64_t)0 : x >= len ? len - 1 : x; };
  if (R.cigar_len > 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) c4[j] = R.cigar[clampi(off + (j < n_raw ? j : n_raw - 1), R.cigar_len)];
  }
  int32_t ld = 0, mlen = 0, n_m = 0;  // (n_m: the (M|=|X) operations)
  int mi = -1;
  bool simple = n > 0;
  for (int k = 0; k < n; ++k) {
    const uint32_t c = k < 4 ? (k == 0 ? c4[0] : k == 1 ? c4[1] : k == 2 ? c4[2] : c4[3]) : R.cigar[off + k];
    const int op = (int)(c & 15u);
    if (op == OP_M || op == OP_EQ || op == OP_X) {
      if (mi >= 0) simple = false;
      mi = k;
      mlen = (int32_t)(c >> 4);
      n_m += n_m < 32766 ? 1 : 0;
    } else if (op == OP_S) {
      if (mi < 0) ld += (int32_t)(c >> 4);
    } else if (op != OP_H) {
      simple = false;
    }
  }
  if (mi < 0 || ld > 32767 || ld + mlen > R.seq_len[r]) simple = false;
  lead[r] = bad ? (int16_t)-1 : simple ? (int16_t)ld : (int16_t)(-1 - n_m);
}

// ev_rb: the sequenced base under each MD event (0 where the event sits on a deletion or
// outside the Match/Mismatch operations), one thread per read, derived on first use
// (ensure_ev_bases) by the kernels that read it: the column records and the projection.  The
// walkers and germline_direct take the base from the pool where they meet the event.
__global__ void ev_bases(DevReads R, uint8_t *__restrict__ ev_rb) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R.n_reads) return;
  const int32_t nmd = R.n_md[r];
  if (nmd <= 0) return;
  const int64_t mdo = R.md_off[r];
  const uint32_t *ev = R.md_ev + mdo;
  uint8_t *rb = ev_rb + mdo;
  const int32_t ld = R.lead[r];
  if (ld >= 0) {  // [S|H]* (M|=|X) [S|H]*: the event at reference offset o reads base lead + o
    const int64_t so = R.seq_off[r];
    const int32_t mlen = R.end[r] - R.start[r];  // (lead + mlen <= seq_len: read_prep's shape test)
    for (int k0 = 0; k0 < nmd; k0 += 4) {  // four events, then their bases, per round of loads
      uint32_t o4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o4[j] = ev[k0 + j < nmd ? k0 + j : nmd - 1] >> 8;
      uint8_t b4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool in = (int32_t)o4[j] < mlen;
        b4[j] = R.seq[in ? so + ld + (int32_t)o4[j] : so];
        b4[j] = in ? b4[j] : (uint8_t)0;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (k0 + j < nmd) rb[k0 + j] = b4[j];
    }
    return;
  }
  const int64_t off = R.cigar_off[r];
  const int32_t n = R.n_cigar[r];
  int32_t ref = 0, rp = 0;
  int k = 0;
  for (int c = 0; c < n && k < nmd; ++c) {
    const uint32_t cc = R.cigar[off + c];
    const int op = (int)(cc & 15u);
    const int32_t len = (int32_t)(cc >> 4);
    if (consumes_ref(op)) {
      while (k < nmd && (int32_t)(ev[k] >> 8) < ref + len) {
        const int32_t o = (int32_t)(ev[k] >> 8);
        uint8_t v = 0;
        if ((op == OP_M || op == OP_EQ || op == OP_X) && o >= ref) {
          const int32_t q = rp + (o - ref);
          if (q < R.seq_len[r]) v = R.seq[R.seq_off[r] + q];
        }
        rb[k++] = v;
      }
      ref += len;
    }
    if (consumes_read(op)) rp += len;
  }
  for (; k < nmd; ++k) rb[k] = 0;
}
// The upload-time checks (validate_one) and the read shapes (shape_one) in one pass over the
// reads: a read whose own offsets lie outside their pools (bit 2) gets no shape (the upload fails
// on the flag anyway).
__global__ void read_prep(DevReads R, int *__restrict__ bad, int16_t *__restrict__ lead) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R.n_reads) return;
  const int b = validate_one(R, r);
  if (b) atomicOr(bad, b);
  shape_one(R, r, lead, (b & 2) != 0);  // (its loads go out beside validate_one's)
}

__device__ __forceinline__ uint64_t pack_inline(uint8_t r0, const uint8_t *alt, int alt_len) {
  uint64_t v = r0;
  for (int i = 0; i < alt_len; ++i) v |= (uint64_t)alt[i] << (8 * (1 + i));
  return v;
}

// ------------------------------------------------------------------------------------------
// germline_tile: LDS histogram + on-device decision for simple loci
// ------------------------------------------------------------------------------------------

#include "gq_germline_common.h"
#include "gq_germline_proj.h"
#include "gq_germline_direct.h"
#include "gq_winorder.h"

// ------------------------------------------------------------------------------------------
// germline_complex: exact per-element classification for queued loci (one wave per locus)
// ------------------------------------------------------------------------------------------

// The hand-off of loci from the fast germline_complex (64 NS = 128 table keys) to the wide one:
// the fast launch appends the positions (in its item list) of loci whose table overflows to
// `out` (at most cap, counted in *n_out: more means a retry with a larger list); the wide
// launch over the same item list takes those positions from `sel`, *n_sel of them (read on the
// device, so the pair runs without a host round trip).
struct DeepList {
  int64_t *out;
  unsigned long long *n_out;
  const int64_t *sel;
  const unsigned long long *n_sel;
  unsigned long long cap;
};

// four waves per SIMD (128 VGPRs; a few spills) beat three without spills: the kernel is latency-bound
#ifndef GQ_CPLX_WPE
#define GQ_CPLX_WPE 3  // waves per SIMD the register budget must allow (4: 120 B/lane of spills)
#endif
template <int NS>  // allele-table slots: 64 NS distinct (sample, allele) keys per locus
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(NS > 2 ? 1 : GQ_CPLX_WPE))) void germline_complex(const Tile *__restrict__ tiles,
                                                           const ComplexItem *__restrict__ items, DevReads R,
                                                           int threshold, int emit_ref, int emit_no_call,
                                                           CallRec *__restrict__ recs, OutGeom og,
                                                           uint8_t *__restrict__ pool, unsigned long long pool_cap,
                                                           Counters *ctr, AmbItem *__restrict__ amb_out,
                                                           unsigned long long amb_cap,
                                                           const AmbItem *__restrict__ amb_in,
                                                           const uint8_t *__restrict__ amb_ref, int64_t n_amb_in,
                                                           int dbg, SomWin sw, DeepList dl) {
  // amb_in == nullptr: every queued item; a locus whose reads' MD-derived bases disagree
  // (Pileup.referenceBaseAtLocus then depends on the queue's heap order) is only listed in
  // amb_out.  amb_in != nullptr: the listed loci again, with their reference base resolved
  // in heap order (heap_ref_bases) in amb_ref, and the element order of each window (sw: the
  // initial group's heap ranks) for the Scala map orders below.
  //
  // Output order (GermlineThresholdCaller.scala:100-104): the per-sample records come in the
  // order of Pileup.bySample (a groupBy over sample names, Pileup.scala:57-61) and count ties
  // among passing alleles keep the order of the counts' groupBy map (sortBy is stable): the
  // Scala 2.10 Map iteration orders restated in gq_scala_order.h.  Both depend on the first
  // occurrence of a key in pileup element order only where two keys share a mutable.HashMap
  // bucket (up to four keys); such loci are listed with the heap-order ones (amb_out) and
  // redone with the windows' element order.
  const int lane = threadIdx.x & 63;
  const int64_t gwave = wave_id();
  const int64_t nwaves_total = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // items beyond a partition's capacity were never written (the host retries with larger ones)
  //
  // Table capacity: the fast instantiation (NS = 2) hands a locus with more than 128 distinct
  // (sample, allele) keys to the wide one (deep_out, whole: nothing of it is counted or written
  // here), which runs over that list (sel: positions in this launch's item list) with 1024
  // keys in registers; Pileup.scala:37-146 has no such limit, and 1024 distinct keys at one
  // locus is past any real pileup's depth-bounded allele count.
  const unsigned long long n_list = amb_in ? (unsigned long long)n_amb_in : ctr->part_off[1][kParts];
  const unsigned long long n_items = dl.sel ? min(*dl.n_sel, dl.cap) : n_list;
  const int rpart = kPartsCols + (int)(gwave & (kPartsWalk - 1));  // this wave's record partition
  // the reads covering the locus, compacted (tile-relative indices): the two per-read passes
  // then run over ~depth lanes instead of every read of the tile (one latency chain, not three)
  constexpr int kCover = 256;
  __shared__ int32_t cover_buf[kBlock / 64][kCover];
  int32_t *cover = cover_buf[threadIdx.x >> 6];
  // dbg & 32: phase clocks per item (cover, reference base, elements, decision + records, items)
  uint64_t clk[6] = {0, 0, 0, 0, 0, 0}, tk = 0;
  auto tick = [&](int k) {
    if (dbg & 32) {
      const uint64_t t = __builtin_readcyclecounter();
      if (k >= 0) clk[k] += t - tk;
      tk = t;
    }
  };
  for (int64_t si = gwave; si < (int64_t)n_items; si += nwaves_total) {
    tick(-1);
    if (dbg & 32) clk[4] += 1;
    const int64_t li = dl.sel ? dl.sel[si] : si;
    const int64_t it = amb_in ? amb_in[li].item : li;
    const ComplexItem item = items[part_slot_wave(ctr->part_off[1], (unsigned long long)it, og, 1)];
    const Tile tl = tiles[item.tile];
    const int32_t pos = item.pos;
    int ncov = 0;
    bool compact = true;
    // the covering reads lie in [first pmax_end > pos, first start > pos)
    //  (both searched over the window together: every read before the first is also before the
    //  second, as start < end <= pmax_end)
    int64_t ra, rz;
    wave_first_true2(tl.rb, tl.re, [&](int64_t r) { return R.pmax_end[r] > pos; },
                     [&](int64_t r) { return R.start[r] > pos; }, ra, rz);
    for (int64_t r0 = ra; r0 < rz; r0 += 64) {
      const int64_t r = r0 + lane;
      const bool c = r < rz && R.start[r] <= pos && pos < R.end[r];
      const unsigned long long b = __ballot(c);
      const int at = ncov + (int)__popcll(b & ((1ull << lane) - 1ull));
      if (c && at < kCover) cover[at] = (int32_t)(r - tl.rb);
      ncov += (int)__popcll(b);
    }
    if (ncov > kCover) compact = false;  // deeper than the buffer: walk the tile's reads
    __builtin_amdgcn_wave_barrier();
    // read slot k of a pass: the k-th covering read (compact) or read rb + k (every read)
    const int64_t n_slots = compact ? ncov : (tl.re - tl.rb);
    auto slot_read = [&](int64_t k, bool *act) -> int64_t {
      if (k >= n_slots) {
        *act = false;
        return tl.rb;
      }
      if (compact) {
        *act = true;
        return tl.rb + cover[k];
      }
      const int64_t r = tl.rb + k;
      *act = R.start[r] <= pos && pos < R.end[r];
      return r;
    };
    tick(0);
    // ---- pass 1: pileup reference base (Pileup.referenceBaseAtLocus).  When every covering
    //      read fits one batch, the same CIGAR walk classifies the element too (pass 2 then
    //      only sets its reference base): one latency chain instead of two
    const bool fused = n_slots <= 64;  // uniform
    AlleleDesc fd;
    fd.rb = 0;
    int ferr = 0, fsmp = 0;
    bool fact = false, fok = false;
    int64_t fr = tl.rb;
    uint32_t mask = 0;  // standard MD-derived bases present
    for (int64_t k0 = 0; k0 < n_slots; k0 += 64) {
      bool cv;
      const int64_t r = slot_read(k0 + lane, &cv);
      if (cv) {
        int v;
        if (fused) {
          fsmp = R.sample[r] & 7;
          fok = classify(R, r, pos, 0, fd, &ferr, &v);
          fact = true;
          fr = r;
        } else {
          v = md_ref_at(R, r, pos);
        }
        if (v < 0) {
          raise_error(&ctr->err, (int64_t *)&ctr->err_pos, v == -4 ? GQ_E_NO_MD : v == -3 ? GQ_E_MD : GQ_E_ASSERT,
                      pos);
        } else {
          mask |= std_bit((uint8_t)v);
        }
      }
    }
    for (int d = 1; d < 64; d <<= 1) mask |= __shfl_xor(mask, d, 64);
    const bool ambiguous = __popc(mask) > 1;
    uint8_t refbase = 'N';
    if (amb_in && amb_ref) {
      refbase = amb_ref[li];
    } else if (ambiguous && !amb_in) {
      // listed for the heap-order replay; a wide tile's visit is counted here, once
      if (lane == 0) {
        if (item.flags & 1) {
          atomicAdd(&ctr->visited, 1ull);
          atomicAdd(&ctr->ambiguous, 1ull);
        }
        const unsigned long long k = atomicAdd(&ctr->n_amb, 1ull);
        if (k < amb_cap) amb_out[k] = AmbItem{item.tile, pos, it};
      }
      continue;
    } else if (mask) {
      refbase = bit_base(mask);
    }
    tick(1);
    // ---- pass 2: classify elements, group alleles per (sample, allele) in registers
    uint64_t tlo[NS], thi[NS];
    uint32_t tcnt[NS];
    int64_t tfirst[NS];  // first occurrence (element-order key) of each entry
    AlleleDesc tdesc[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      tlo[s] = thi[s] = 0;
      tcnt[s] = 0;
      tfirst[s] = INT64_MAX;
    }
    int nt = 0;  // used slots (uniform)
    bool overflow = false;
    uint32_t st_lane = 0;  // lane s < 8: elements of sample s (read back with readlane: no scratch array)
    int64_t st_first = INT64_MAX;  // lane s < 8: the first element of sample s (element-order key)
    // the window's initial group (element order): only the re-runs carry it
    const WinInit wio = sw.init_reads ? sw.wi[2 * sw.range_win[tl.range]] : WinInit{INT32_MAX, INT32_MIN, 0, 0, 0};
    // one batch of elements (up to 64, in read order) into the table and the per-sample totals
    auto add_batch = [&](bool act, int64_t r, const AlleleDesc &d, int smp, const Key128 &key) {
      const int64_t okey = act ? element_order_key(R, r, pos, wio, sw.init_reads, sw.init_rank) : INT64_MAX;
      // slots run in read order, so with no initial-group read in the batch the first element
      // of a group is its lowest lane (no wave reduction)
      const bool by_lane = __ballot(act && okey < (1ll << 40)) == 0;
      // per-sample totals and first elements
      for (int sm = 0; sm < R.n_samples && sm < 8; ++sm) {
        const unsigned long long b = __ballot(act && smp == sm);
        if (!b) continue;  // uniform
        const int64_t f = by_lane ? lane_u64(okey, __ffsll((long long)b) - 1)
                                  : wave_min_i64(act && smp == sm ? okey : INT64_MAX);
        if (lane == sm) {
          st_lane += (uint32_t)__popcll(b);
          st_first = f < st_first ? f : st_first;
        }
      }
      unsigned long long pending = __ballot(act);
      while (pending) {
        const int leader = __ffsll((long long)pending) - 1;
        const uint64_t klo = __shfl(key.lo, leader, 64), khi = __shfl(key.hi, leader, 64);
        const bool match = act && key.lo == klo && key.hi == khi;
        const unsigned long long mb = __ballot(match);
        const uint32_t n = (uint32_t)__popcll(mb);
        // find the key in the table
        int found = -1;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bool hit = (s * 64 + lane) < nt && tlo[s] == klo && thi[s] == khi;
          const unsigned long long hb = __ballot(hit);
          if (found < 0 && hb) found = s * 64 + (__ffsll((long long)hb) - 1);
        }
        if (found < 0) {
          if (nt >= 64 * NS) {
            overflow = true;
          } else {
            found = nt++;
            // leader's descriptor -> owning lane of the slot
            const int owner = found & 63, sl = found >> 6;
            AlleleDesc ld;
            ld.read = __shfl(d.read, leader, 64);
            ld.aux = __shfl(d.aux, leader, 64);
            ld.rp = __shfl(d.rp, leader, 64);
            ld.kind = (uint8_t)__shfl((int)d.kind, leader, 64);
            ld.rb = (uint8_t)__shfl((int)d.rb, leader, 64);
            ld.base = (uint8_t)__shfl((int)d.base, leader, 64);
            ld.pad = (uint8_t)smp;  // sample in pad
            ld.pad = (uint8_t)__shfl((int)smp, leader, 64);
#pragma unroll
            for (int s = 0; s < NS; ++s)
              if (s == sl && lane == owner) {
                tlo[s] = klo;
                thi[s] = khi;
                tcnt[s] = 0;
                tdesc[s] = ld;
              }
          }
        }
        if (found >= 0) {
          const int owner = found & 63, sl = found >> 6;
          const int64_t f = by_lane ? lane_u64(okey, leader) : wave_min_i64(match ? okey : INT64_MAX);
#pragma unroll
          for (int s = 0; s < NS; ++s)
            if (s == sl && lane == owner) {
              tcnt[s] += n;
              tfirst[s] = f < tfirst[s] ? f : tfirst[s];
            }
        }
        pending &= ~mb;
      }
    };
    if (fused) {
      bool act = fact;
      AlleleDesc d = fd;
      d.rb = refbase;
      int smp = act ? fsmp : 0;
      Key128 key{0, 0};
      if (act && !fok) {
        raise_error(&ctr->err, (int64_t *)&ctr->err_pos, ferr, pos);
        act = false;
        smp = 0;
      }
      if (act) key = allele_key<true>(R, d, pos, smp);
      add_batch(act, fr, d, smp, key);
    } else {
      for (int64_t k0 = 0; k0 < n_slots; k0 += 64) {
        bool act;
        const int64_t r = slot_read(k0 + lane, &act);
        AlleleDesc d;
        Key128 key{0, 0};
        int smp = act ? (R.sample[r] & 7) : 0;  // issued with classify's loads
        if (act) {
          int errc = 0;
          if (!classify(R, r, pos, refbase, d, &errc)) {
            raise_error(&ctr->err, (int64_t *)&ctr->err_pos, errc, pos);
            act = false;
            smp = 0;
          } else {
            key = allele_key<true>(R, d, pos, smp);
          }
        }
        add_batch(act, r, d, smp, key);
      }
    }
    if (overflow) {
      if (NS <= 2 && dl.out) {  // the wide instantiation's, whole
        if (lane == 0) {
          const unsigned long long k = atomicAdd(dl.n_out, 1ull);
          if (k < dl.cap) dl.out[k] = li;
        }
      } else {
        raise_error(&ctr->err, (int64_t *)&ctr->err_pos, GQ_E_CAPACITY, pos);
      }
      continue;
    }
    if ((item.flags & 1) && !amb_in) {  // queued from a wide tile: count the visit here
      const uint32_t tot = (uint32_t)__ballot(lane < 8 && st_lane > 0);
      if (tot == 0) continue;
      if (lane == 0) {
        atomicAdd(&ctr->visited, 1ull);
        if (ambiguous) atomicAdd(&ctr->ambiguous, 1ull);
      }
    }
    tick(2);
    // ---- Scala map orders (gq_scala_order.h): each entry's order key within its sample's
    //      counts map, each present sample's within bySample, and whether either depends on
    //      first occurrences (two keys in one mutable.HashMap bucket, up to four keys)
    const int ns_all = R.n_samples < 8 ? R.n_samples : 8;
    uint64_t tkey[NS];
    bool dep = false;
    int tsm[NS];
    bool tpass[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bool live = s * 64 + lane < nt;
      tsm[s] = live ? (int)tdesc[s].pad : -1;
      const uint32_t tot = (uint32_t)__shfl((int)st_lane, tsm[s] < 0 ? 0 : tsm[s], 64);
      tpass[s] = live && tot > 0 && (long long)tcnt[s] * 100 / (long long)tot > threshold;
      tkey[s] = 0;
    }
    // the map order only decides between passing entries of one sample with equal counts
    bool tie_any = false;
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) {
      unsigned long long pb = __ballot(tpass[s2]);
      while (pb && !tie_any) {
        const int ow = __ffsll((long long)pb) - 1;
        pb &= pb - 1;
        const int smj = __builtin_amdgcn_readlane(tsm[s2], ow);
        const int cj = __builtin_amdgcn_readlane((int)tcnt[s2], ow);
        bool hit = false;
#pragma unroll
        for (int s = 0; s < NS; ++s)
          hit |= tpass[s] && tsm[s] == smj && (int)tcnt[s] == cj && !(s == s2 && lane == ow);
        tie_any = __ballot(hit) != 0;
      }
    }
    if (tie_any) {
      uint32_t tb[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const uint32_t h = tsm[s] >= 0 ? allele_scala_hash(R, tdesc[s], pos) : 0u;
        tb[s] = scala::mutable_bucket(h, 4);
        tkey[s] = scala::trie_key(h);  // five or more alleles in the sample: HashTrieMap order
      }
      // entries of the same sample, and same-bucket ties among passing ones
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        int n_same = 0;
        bool pair = false;
        for (int k = 0; k < nt; ++k) {
          const int ow = k & 63, sl = k >> 6;
          int ksm = -1;
          uint32_t kb = 0, kc = 0;
          bool kp = false;
#pragma unroll
          for (int t = 0; t < NS; ++t)
            if (t == sl) {
              ksm = __shfl(tsm[t], ow, 64);
              kb = (uint32_t)__shfl((int)tb[t], ow, 64);
              kc = (uint32_t)__shfl((int)tcnt[t], ow, 64);
              kp = __shfl((int)tpass[t], ow, 64) != 0;
            }
          if (ksm == tsm[s] && tsm[s] >= 0) {
            ++n_same;
            if (k != s * 64 + lane && kb == tb[s] && kp && tpass[s] && kc == tcnt[s]) pair = true;
          }
        }
        // up to four keys: Map1..Map4 in the mutable map's order (bucket descending, a chain
        // newest first = the later first occurrence first)
        if (tsm[s] >= 0 && n_same <= 4)
          tkey[s] = ((uint64_t)(15u - tb[s]) << 42) | (((1ull << 42) - 1ull) - (uint64_t)tfirst[s]);
        if (tsm[s] >= 0 && n_same <= 4 && pair) dep = true;
      }
    }
    // samples: lane sm < 8 holds its rank among the present samples
    int srank = 0;
    const bool present = lane < ns_all && st_lane > 0;
    const int np = __popcll(__ballot(present));
    if (np > 1) {
      uint64_t sk = ~0ull;
      uint32_t sb = 16u + (uint32_t)lane;
      if (R.sample_hash && present) {
        const uint32_t h = R.sample_hash[lane];
        sb = scala::mutable_bucket(h, 4);
        sk = np <= 4 ? (((uint64_t)(15u - sb) << 42) | (((1ull << 42) - 1ull) - (uint64_t)st_first)) : scala::trie_key(h);
      } else if (present) {
        sk = (uint64_t)lane;  // no sample names given: slot order
      }
      int rk = 0;
      bool same_bucket = false;
      for (int t = 0; t < 8; ++t) {
        const uint64_t tk2 = lane_u64(sk, t);
        const uint32_t tb2 = (uint32_t)__builtin_amdgcn_readlane((int)sb, t);
        if (t != lane && tk2 != ~0ull && present) {
          if (tk2 < sk || (tk2 == sk && t < lane)) ++rk;
          if (R.sample_hash && np <= 4 && tb2 == sb) same_bucket = true;
        }
      }
      srank = rk;
      if (__ballot(same_bucket) != 0) dep = true;
    }
    // (sw without init_reads: window bounds only; past a window's initial group the elements
    //  are in read order, which the keys above already used)
    // (a first pass has the window bounds only: past E the read order above is the element order)
    if (__ballot(dep) != 0 && !amb_in && (sw.init_reads || !sw.wi || pos < sw.wi[2 * sw.range_win[tl.range]].E)) {
      // the order depends on first occurrences: listed (after the amb list's capacity) and
      // redone with the windows' element order (amb_ref == nullptr: the base is not ambiguous)
      if (lane == 0) {
        const unsigned long long k = atomicAdd(&ctr->n_ord, 1ull);
        if (k < amb_cap) amb_out[amb_cap + k] = AmbItem{item.tile, pos, it};
      }
      continue;
    }
    tick(5);
    // ---- pass 3: GermlineThreshold decision per sample (uniform serial code)
    const uint64_t ord = (uint64_t)(tl.ordinal0 + (pos - tl.L0));
    for (int sm = 0; sm < R.n_samples && sm < 8; ++sm) {
      const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)st_lane, sm);
      if (total == 0) continue;
      const int rank_sm = __builtin_amdgcn_readlane(srank, sm);
      // select top-3 passing entries by (count desc, map order); three named slots, not an
      // indexed array (a dynamically indexed array would live in scratch)
      uint32_t topc[3] = {0, 0, 0};
      uint64_t topk[3] = {0, 0, 0};
      AlleleDesc topd[3];
      int npass = 0;
      for (int j = 0; j < nt; ++j) {
        const int owner = j & 63, sl = j >> 6;
        uint32_t cj = 0;
        uint64_t kj = 0;
        AlleleDesc dj;
#pragma unroll
        for (int s = 0; s < NS; ++s)
          if (s == sl) {
            kj = lane_u64(tkey[s], owner);
            cj = (uint32_t)__shfl((int)tcnt[s], owner, 64);
            dj.read = __shfl(tdesc[s].read, owner, 64);
            dj.aux = __shfl(tdesc[s].aux, owner, 64);
            dj.rp = __shfl(tdesc[s].rp, owner, 64);
            dj.kind = (uint8_t)__shfl((int)tdesc[s].kind, owner, 64);
            dj.rb = (uint8_t)__shfl((int)tdesc[s].rb, owner, 64);
            dj.base = (uint8_t)__shfl((int)tdesc[s].base, owner, 64);
            dj.pad = (uint8_t)__shfl((int)tdesc[s].pad, owner, 64);
          }
        if (dj.pad != sm) continue;
        if ((long long)cj * 100 / (long long)total <= threshold) continue;
        const int f = npass < 3 ? npass : 3;  // entries held before this one (sorted)
        ++npass;
        auto better = [&](uint32_t ce, uint64_t ke) { return ce < cj || (ce == cj && kj < ke); };
        // insertion position: past every held entry this one does not beat
        const bool b2 = f > 2 && better(topc[2], topk[2]);
        const bool b1 = f > 1 && (b2 || f == 2) && better(topc[1], topk[1]);
        const bool b0 = f > 0 && (b1 || f == 1) && better(topc[0], topk[0]);
        const int p = b0 ? 0 : b1 ? 1 : (b2 || f == 2) ? 2 : f;
        if (p == 0) {
          topc[2] = topc[1];
          topk[2] = topk[1];
          topd[2] = topd[1];
          topc[1] = topc[0];
          topk[1] = topk[0];
          topd[1] = topd[0];
          topc[0] = cj;
          topk[0] = kj;
          topd[0] = dj;
        } else if (p == 1) {
          topc[2] = topc[1];
          topk[2] = topk[1];
          topd[2] = topd[1];
          topc[1] = cj;
          topk[1] = kj;
          topd[1] = dj;
        } else if (p == 2) {
          topc[2] = cj;
          topk[2] = kj;
          topd[2] = dj;
        }
      }
      const bool tie = npass >= 2 && (topc[0] == topc[1] || (npass >= 3 && topc[1] == topc[2]));
      const uint8_t fl = (tie ? GQ_FLAG_TIE : 0) | (ambiguous ? GQ_FLAG_AMBIGUOUS_REF : 0);
      if (lane == 0 && tie) atomicAdd(&ctr->ties, 1ull);
      // emit helper: alleles from descriptors, or symbolic "<ALT>" with an explicit ref
      // (descriptors by value: a pointer into topd would put the array in scratch memory, one
      //  global-latency load per field read)
      auto emit = [&](const AlleleDesc a, uint8_t sym_ref_kind, const AlleleDesc ref_src, uint8_t g0, uint8_t g1,
                      int sub) {
        // sym_ref_kind: 0 => allele `a`; 1 => (refbase, <ALT>); 2 => (ref of ref_src, <ALT>)
        int rl, al;
        if (sym_ref_kind == 0) {
          rl = allele_ref_len(a);
          al = allele_alt_len(a);
        } else if (sym_ref_kind == 1) {
          rl = 1;
          al = 5;
        } else {
          rl = allele_ref_len(ref_src);
          al = 5;
        }
        auto byte_at = [&](int which, int i) -> uint8_t {
          if (sym_ref_kind == 0) return allele_byte(R, a, pos, which, i);
          if (which == 1) return (uint8_t)"<ALT>"[i];
          if (sym_ref_kind == 1) return refbase;
          return allele_byte(R, ref_src, pos, 0, i);
        };
        CallRec rr;
        rr.key = (ord << 12) | ((uint64_t)rank_sm << 4) | (uint64_t)sub;  // bySample order
        rr.contig = tl.contig;
        rr.pos = pos;
        rr.sample = (uint8_t)sm;
        rr.gt0 = g0;
        rr.gt1 = g1;
        rr.flags = fl;
        rr.ref_len = (uint16_t)rl;
        rr.alt_len = (uint16_t)al;
        if (rl + al <= 8) {
          // lane i fetches byte i (one load chain for all of them, not one per byte: a
          // deletion's bytes each take an MD search), then the bytes are packed by readlane
          uint32_t bv = 0;
          if (lane < rl + al) bv = byte_at(lane < rl ? 0 : 1, lane < rl ? lane : lane - rl);
          uint64_t v = 0;
          for (int i = 0; i < rl + al; ++i) v |= (uint64_t)(uint8_t)__builtin_amdgcn_readlane((int)bv, i) << (8 * i);
          rr.allele = v;
        } else {
          unsigned long long off = 0;
          if (lane == 0) off = atomicAdd(&ctr->pool_used, (unsigned long long)(rl + al));
          off = __shfl(off, 0, 64);
          if (off + rl + al <= pool_cap) {
            for (int i = lane; i < rl + al; i += 64)
              pool[off + i] = i < rl ? byte_at(0, i) : byte_at(1, i - rl);
          }
          rr.allele = off;
        }
        if (lane == 0) {
          const unsigned long long k = atomicAdd(&ctr->part[0][rpart], 1ull);
          if (k < og.capB[0]) recs[og.slot(0, rpart, k)] = rr;
        }
      };
      if (npass == 0) {
        if (emit_no_call) emit(AlleleDesc{}, 1, AlleleDesc{}, GQ_GT_NOCALL, GQ_GT_NOCALL, 0);
      } else {
        auto isvar = [&](const AlleleDesc &a) {  // Allele.isVariant: refBases != altBases
          const int rl = allele_ref_len(a), al = allele_alt_len(a);
          if (rl != al) return true;
          for (int i = 0; i < rl; ++i)
            if (allele_byte(R, a, pos, 0, i) != allele_byte(R, a, pos, 1, i)) return true;
          return false;
        };
        const bool v1 = isvar(topd[0]);
        if (npass == 1 && !v1) {
          if (emit_ref) emit(AlleleDesc{}, 1, AlleleDesc{}, GQ_GT_REF, GQ_GT_REF, 0);
        } else if (npass == 1) {
          emit(topd[0], 0, AlleleDesc{}, GQ_GT_ALT, GQ_GT_ALT, 0);
        } else {
          const bool v2 = isvar(topd[1]);
          const bool e1 = allele_alt_len(topd[0]) == 0, e2 = allele_alt_len(topd[1]) == 0;
          if ((!v1 || !v2) && (e1 != e2)) {
            // heterozygous deletion: no call (GermlineThresholdCaller.scala:146-149)
          } else if (v1 != v2) {
            emit(v1 ? topd[0] : topd[1], 0, AlleleDesc{}, GQ_GT_REF, GQ_GT_ALT, 0);
          } else if (v1 && v2) {
            emit(topd[0], 0, AlleleDesc{}, GQ_GT_ALT, GQ_GT_OTHERALT, 0);
            emit(topd[1], 0, AlleleDesc{}, GQ_GT_ALT, GQ_GT_OTHERALT, 1);
          } else {
            const bool n1 = allele_ref_len(topd[0]) == 1 && allele_byte(R, topd[0], pos, 0, 0) == 'N';
            const bool n2 = allele_ref_len(topd[1]) == 1 && allele_byte(R, topd[1], pos, 0, 0) == 'N';
            if (n1 || n2) emit(AlleleDesc{}, 2, n1 ? topd[1] : topd[0], GQ_GT_REF, GQ_GT_REF, 0);
            else raise_error(&ctr->err, (int64_t *)&ctr->err_pos, GQ_E_MULTI_REF, pos);
          }
        }
      }
    }
    tick(3);
  }
  if ((dbg & 32) && (threadIdx.x & 63) == 0 && clk[4])
    for (int k = 0; k < 6; ++k) atomicAdd(&ctr->prof[k], (unsigned long long)clk[k]);
}

// ------------------------------------------------------------------------------------------
// counts_tile: dense raw histogram (gq_pileup_counts)
// ------------------------------------------------------------------------------------------
enum : int { K2_A = 0, K2_C, K2_T, K2_G, K2_N, K2_O, K2_INS, K2_DEL, K2_MID, K2_CLIP, K2_POS, K2_MASK, K2_EVA, K2_EVC,
             K2_EVT, K2_EVG, K2_NCAT };  // base_cat order

template <int T>
struct CountSink {
  uint32_t *cnt;
  int32_t L0;
  int *err;
  long long *err_pos;
  __device__ __forceinline__ void elem(int32_t l, int kind, uint8_t base, uint8_t mdb, bool ev, uint8_t fl) {
    elem_i(l - L0, kind, base, mdb, ev, fl);
  }
  __device__ __forceinline__ void bases4_clean(int i, uint32_t w, uint32_t valid4, uint8_t fl) {
    bases4(i, w, valid4, fl);
  }
  __device__ __forceinline__ void bases4(int i, uint32_t w, uint32_t valid4, uint8_t fl) {
    for (int j = 0; j < 4; ++j)
      if (((valid4 >> j) & 1u) && i + j >= 0 && i + j < T) elem_i(i + j, K_SNV, (uint8_t)(w >> (8 * j)), 0, false, fl);
  }
  __device__ __forceinline__ void event_i(int i, uint8_t b, uint8_t m, uint8_t) {
    const int bc = base_cat(b);
    if (bc < 4) atomicAdd(&cnt[(K2_EVA + bc) * T + i], 1u);
    const uint32_t bit = std_bit(m);
    if (bit) atomicOr(&cnt[K2_MASK * T + i], bit);
  }
  __device__ __forceinline__ void elem_i(int i, int kind, uint8_t base, uint8_t mdb, bool ev, uint8_t fl) {
    int c;
    switch (kind) {
      case K_SNV: c = base_cat(base); break;
      case K_INS: c = K2_INS; break;
      case K_DEL: c = K2_DEL; break;
      case K_MID: c = K2_MID; break;
      default: c = K2_CLIP; break;
    }
    atomicAdd(&cnt[c * T + i], 1u);
    if (!(fl & 1)) atomicAdd(&cnt[K2_POS * T + i], 1u);
    const uint32_t b = std_bit(mdb);
    if (kind == K_SNV && !ev) return;  // mask derived from base counts below
    if (kind == K_SNV && ev) {
      const int bc = base_cat(base);
      if (bc < 4) atomicAdd(&cnt[(K2_EVA + bc) * T + i], 1u);
    }
    if (b) atomicOr(&cnt[K2_MASK * T + i], b);
  }
  __device__ __forceinline__ void clip_run(int i0, int i1, uint8_t fl) {
    for (int i = i0; i < i1; ++i) elem_i(i, K_CLIP, 0, (uint8_t)'N', false, fl);
  }
  __device__ __forceinline__ void error(int code, int64_t where) { raise_error(err, (int64_t *)err_pos, code, where); }
};

template <int T>
__global__ __launch_bounds__(kBlock) void counts_tile(const Tile *__restrict__ tiles, DevReads R,
                                                      int32_t *__restrict__ depth, int32_t *__restrict__ pos_depth,
                                                      int32_t *__restrict__ base_counts,
                                                      int32_t *__restrict__ indel_counts,
                                                      int32_t *__restrict__ ref_depth, uint8_t *__restrict__ ref_base,
                                                      uint8_t *__restrict__ ambiguous, Counters *ctr) {
  __shared__ uint32_t cnt[K2_NCAT * T];
  const Tile tl = tiles[blockIdx.x];
  const int32_t L0 = tl.L0, L1 = tl.L1;
  for (int i = threadIdx.x; i < K2_NCAT * T; i += blockDim.x) cnt[i] = 0u;
  __syncthreads();
  CountSink<T> sink{cnt, L0, &ctr->err, &ctr->err_pos};
  for (int64_t r = tl.rb + threadIdx.x; r < tl.re; r += blockDim.x) walk_read_lane(R, r, L0, L1, sink);
  __syncthreads();
  for (int i = threadIdx.x; i < L1 - L0; i += blockDim.x) {
    const int64_t o = tl.ordinal0 + i;
    uint32_t dsum = 0;
    for (int k = 0; k <= K2_CLIP; ++k) dsum += cnt[k * T + i];
    uint32_t mask = cnt[K2_MASK * T + i];
    for (int k = 0; k < 4; ++k)
      if (cnt[k * T + i] > cnt[(K2_EVA + k) * T + i]) mask |= 1u << k;
    const uint8_t rb = mask ? bit_base(mask) : (uint8_t)'N';
    depth[o] = (int32_t)dsum;
    pos_depth[o] = (int32_t)cnt[K2_POS * T + i];
    const int out_order[6] = {K2_A, K2_C, K2_G, K2_T, K2_N, K2_O};  // output: A C G T N other
    for (int k = 0; k < 6; ++k) base_counts[o * 6 + k] = (int32_t)cnt[out_order[k] * T + i];
    for (int k = 0; k < 4; ++k) indel_counts[o * 4 + k] = (int32_t)cnt[(K2_INS + k) * T + i];
    ref_depth[o] = (int32_t)cnt[base_cat(rb) * T + i];
    ref_base[o] = rb;
    ambiguous[o] = __popc(mask) > 1 ? 1 : 0;
  }
}

// vaf_tile: VAFHistogram's per-locus variant allele frequency (VariantLocus.apply,
// commands/VAFHistogram.scala:31-37) binned on the device (generateVAFHistogram, :188-196).
// Loci whose reference base depends on heap order are listed with their counts (the host
// bins them after the replay).  hist: 64 spread copies of the 101 bins.
struct VafAmb {
  int32_t depth, base[6];  // depth, Match/Mismatch elements by base (A C G T N other)
};
template <int T>
__global__ __launch_bounds__(kBlock) void vaf_tile(const Tile *__restrict__ tiles, DevReads R, int bins,
                                                   int min_depth, int min_vaf, unsigned long long *__restrict__ hist,
                                                   AmbItem *__restrict__ amb, VafAmb *__restrict__ amb_cnt,
                                                   unsigned long long amb_cap, Counters *ctr) {
  __shared__ uint32_t cnt[K2_NCAT * T];
  __shared__ uint32_t h[101];
  const Tile tl = tiles[blockIdx.x];
  const int32_t L0 = tl.L0, L1 = tl.L1;
  for (int i = threadIdx.x; i < K2_NCAT * T; i += blockDim.x) cnt[i] = 0u;
  for (int i = threadIdx.x; i < 101; i += blockDim.x) h[i] = 0u;
  __syncthreads();
  CountSink<T> sink{cnt, L0, &ctr->err, &ctr->err_pos};
  for (int64_t r = tl.rb + threadIdx.x; r < tl.re; r += blockDim.x) walk_read_lane(R, r, L0, L1, sink);
  __syncthreads();
  const int bin_size = 100 / bins;
  unsigned visited = 0, variant = 0;
  for (int i = threadIdx.x; i < L1 - L0; i += blockDim.x) {
    uint32_t dsum = 0;
    for (int k = 0; k <= K2_CLIP; ++k) dsum += cnt[k * T + i];
    if (dsum == 0) continue;  // skipEmpty
    ++visited;
    uint32_t mask = cnt[K2_MASK * T + i];
    for (int k = 0; k < 4; ++k)
      if (cnt[k * T + i] > cnt[(K2_EVA + k) * T + i]) mask |= 1u << k;
    if (__popc(mask) > 1) {  // the reference base comes from heap order: the host bins it
      const unsigned long long k = atomicAdd(&ctr->n_amb, 1ull);
      if (k < amb_cap) {
        amb[k] = AmbItem{(int32_t)blockIdx.x, L0 + i, (int64_t)k};
        VafAmb v;
        v.depth = (int32_t)dsum;
        const int out_order[6] = {K2_A, K2_C, K2_G, K2_T, K2_N, K2_O};
        for (int q = 0; q < 6; ++q) v.base[q] = (int32_t)cnt[out_order[q] * T + i];
        amb_cnt[k] = v;
      }
      continue;
    }
    const uint8_t rb = mask ? bit_base(mask) : (uint8_t)'N';
    const uint32_t ref = cnt[base_cat(rb) * T + i];
    if (ref == dsum) continue;  // no VariantLocus
    // (depth - referenceDepth).toFloat / depth; depth >= minReadDepth; vaf >= minVAF / 100.0
    const float vaf = (float)(int32_t)(dsum - ref) / (float)(int32_t)dsum;
    if (!((int32_t)dsum >= min_depth) || !((double)vaf >= (double)min_vaf / 100.0)) continue;
    ++variant;
    const int pct = (int)(vaf * 100.0f);
    atomicAdd(&h[pct - pct % bin_size], 1u);
  }
  __syncthreads();
  unsigned long long *hh = hist + (size_t)(blockIdx.x & 63) * 101;
  for (int i = threadIdx.x; i < 101; i += blockDim.x)
    if (h[i]) atomicAdd(&hh[i], (unsigned long long)h[i]);
  for (int d = 32; d >= 1; d >>= 1) {
    visited += __shfl_xor(visited, d, 64);
    variant += __shfl_xor(variant, d, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (visited) atomicAdd(&ctr->spread[0][blockIdx.x & (kSpread - 1)], (unsigned long long)visited);
    if (variant) atomicAdd(&ctr->spread[1][blockIdx.x & (kSpread - 1)], (unsigned long long)variant);
  }
}

// ------------------------------------------------------------------------------------------
// Result image: the gq_calls arrays built on device in output order (one D2H copy)
// ------------------------------------------------------------------------------------------
struct CallsLayout {  // byte offsets inside the image; header = int64 pool_len, int64 n
  size_t contig, pos, ref_off, alt_off, ref_len, alt_len, sample, gt0, gt1, flags, pool, bytes;
};
__host__ __device__ inline CallsLayout calls_layout(int64_t n, int64_t dev_pool_used) {
  auto al = [](size_t x) { return (x + 63) & ~(size_t)63; };
  const size_t N = (size_t)n;
  CallsLayout L;
  L.contig = 64;
  L.pos = al(L.contig + 4 * N);
  L.ref_off = al(L.pos + 8 * N);
  L.alt_off = al(L.ref_off + 8 * N);
  L.ref_len = al(L.alt_off + 8 * N);
  L.alt_len = al(L.ref_len + 4 * N);
  L.sample = al(L.alt_len + 4 * N);
  L.gt0 = al(L.sample + N);
  L.gt1 = al(L.gt0 + N);
  L.flags = al(L.gt1 + N);
  L.pool = al(L.flags + N);
  // inline alleles hold <= 8 bytes; longer ones live in the device pool (each used once)
  L.bytes = al(L.pool + 8 * N + (size_t)dev_pool_used + 1);
  return L;
}

// Exclusive offsets of the per-partition counts (clamped to the capacity) of one output kind,
// their total (n_rec / n_complex) and the largest count (part_max); one block of 1024
// threads, kParts / 1024 partitions each.
__global__ __launch_bounds__(1024) void part_scan(Counters *ctr, int which, OutGeom og) {
  constexpr int PER = kParts / 1024;
  __shared__ unsigned long long s[1024];
  __shared__ unsigned long long mx;
  const int t = threadIdx.x;
  unsigned long long v[PER], sum = 0, m = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const unsigned long long x = ctr->part[which][t * PER + j];
    const unsigned long long cap = og.cap(which, t * PER + j);
    m = x > cap && x - cap > m ? x - cap : m;  // largest overflow
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
  unsigned long long o = s[t] - sum;  // exclusive
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    ctr->part_off[which][t * PER + j] = o;
    o += v[j];
  }
  if (t == 1023) {
    ctr->part_off[which][kParts] = s[t];
    if (which == 0) ctr->n_rec = s[t];
    else ctr->n_complex = s[t];
    ctr->part_max[which] = mx;  // 0: every partition within its capacity
  }
}

// Dense (key, slot) pairs of the partitioned records, for the radix sort.
__global__ void gather_keys(const CallRec *__restrict__ recs, const Counters *__restrict__ ctr, OutGeom og,
                            int64_t n, uint64_t *__restrict__ keys,
                            int32_t *__restrict__ slot) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const unsigned long long src = part_slot(ctr->part_off[0], (unsigned long long)k, og, 0);
  keys[k] = recs[src].key;
  slot[k] = (int32_t)src;
}

// Output order without a comparison sort.  Records fall into buckets of 2^bshift output
// ordinals (key >> (12 + bshift)); the buckets are scanned, and a record's place inside its
// bucket is the number of the bucket's records with a smaller key (keys of live records are
// unique).  Buckets hold few records: 512 loci of a sparse call set (bshift 9), one locus when
// every locus emits (bshift 0).  Unused candidate slots (dead_key) are dropped.
//
// The chain reads every size from the device (record slots: part_scan's n_rec; records: the
// bucket scan's total), so it is launched right behind the pileup kernels with grid-stride
// loops and no host round trip; the host reads the counters once, at the end.
constexpr int kFinBlocks = 1024;  // grid of the record-slot kernels
constexpr int kImgBlocks = 512;   // calls_image chunks (one workgroup each)
// (a record whose key lies past every bucket — a slot a kernel reserved and never wrote — is
// dropped and raises GQ_E_ASSERT at the slot: an internal fault, reported instead of a wild write)
__global__ __launch_bounds__(kBlock) void bucket_count(const CallRec *__restrict__ recs, Counters *__restrict__ ctr,
                                                        OutGeom og, uint64_t dead_key, int bshift, int64_t nbk,
                                                        uint64_t *__restrict__ keys, int32_t *__restrict__ slot,
                                                        int64_t *__restrict__ bkt, uint32_t *__restrict__ cnt) {
  const int64_t n_all = (int64_t)ctr->n_rec;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_all; k += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long src = part_slot(ctr->part_off[0], (unsigned long long)k, og, 0);
    const uint64_t key = recs[src].key;
    keys[k] = key;
    slot[k] = (int32_t)src;
    int64_t b = key == dead_key ? -1 : (int64_t)(key >> (12 + bshift));
    if (b >= nbk) {
      if (atomicCAS(&ctr->err, 0, 1 /*GQ_E_ASSERT*/) == 0) {  // (the record, for the host's message)
        const CallRec r = recs[src];
        ctr->err_pos = (long long)src;
        ctr->prof[0] = key;
        ctr->prof[1] = ((unsigned long long)(uint32_t)r.contig << 32) | (uint32_t)r.pos;
        ctr->prof[2] = ((unsigned long long)r.flags << 24) | ((unsigned long long)r.gt1 << 16) | ((unsigned long long)r.gt0 << 8) | r.sample;
        ctr->prof[3] = (unsigned long long)k;
        ctr->prof[4] = ctr->n_rec;
      }
      b = -1;
    }
    bkt[k] = b;
    if (b >= 0) atomicAdd(&cnt[b], 1u);
  }
}

__global__ void bucket_scatter(const Counters *__restrict__ ctr, const int64_t *__restrict__ bkt,
                               const uint32_t *__restrict__ off, uint32_t *__restrict__ fill,
                               int32_t *__restrict__ members) {
  const int64_t n_all = (int64_t)ctr->n_rec;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_all; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = bkt[k];
    if (b >= 0) members[off[b] + atomicAdd(&fill[b], 1u)] = (int32_t)k;
  }
}

__global__ void bucket_rank(int64_t nbk, const uint32_t *__restrict__ off, const int32_t *__restrict__ members,
                            const uint64_t *__restrict__ keys, const int32_t *__restrict__ slot,
                            const int64_t *__restrict__ bkt, int32_t *__restrict__ order) {
  const int64_t n = off[nbk];  // live records
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = members[p];
    const int64_t b = bkt[k];
    const uint32_t lo = off[b], hi = off[b + 1];
    const uint64_t key = keys[k];
    uint32_t rank = 0;
    for (uint32_t q = lo; q < hi; ++q) rank += keys[members[q]] < key ? 1u : 0u;
    order[lo + rank] = slot[k];
  }
}

__global__ void zero_u32(uint32_t *__restrict__ v, int64_t n) {  // one launch for the bucket words (memsets split in four)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) v[i] = 0u;
}

__global__ void iota_i32(int32_t *__restrict__ v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (int32_t)i;
}

// calls_image works in kImgBlocks contiguous chunks of the n records (output order); the pool
// offsets are a scan of the records' allele lengths: chunk sums (img_sums), their exclusive
// scan (img_scan, one workgroup), then each chunk's own scan inside calls_image.
__device__ __forceinline__ void img_chunk(int64_t n, int64_t &a, int64_t &b) {
  const int64_t per = (n + kImgBlocks - 1) / kImgBlocks;
  a = min(n, (int64_t)blockIdx.x * per);
  b = min(n, a + per);
}
__device__ __forceinline__ uint32_t rec_len(const CallRec &r) { return (uint32_t)r.ref_len + (uint32_t)r.alt_len; }

__global__ __launch_bounds__(kBlock) void img_sums(const CallRec *__restrict__ recs, const int32_t *__restrict__ order,
                                                    const uint32_t *__restrict__ off, int64_t nbk,
                                                    int64_t *__restrict__ bsum) {
  __shared__ unsigned long long red;
  if (threadIdx.x == 0) red = 0;
  __syncthreads();
  int64_t a, b;
  img_chunk((int64_t)off[nbk], a, b);
  unsigned long long s = 0;
  for (int64_t k = a + threadIdx.x; k < b; k += blockDim.x) s += rec_len(recs[order[k]]);
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(&red, s);
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = (int64_t)red;
}

__global__ __launch_bounds__(kImgBlocks) void img_scan(int64_t *__restrict__ bsum) {  // in place, exclusive; total at [kImgBlocks]
  __shared__ int64_t s[kImgBlocks];
  const int t = threadIdx.x;
  const int64_t v = bsum[t];
  s[t] = v;
  __syncthreads();
  for (int d = 1; d < kImgBlocks; d <<= 1) {
    const int64_t y = t >= d ? s[t - d] : 0;
    __syncthreads();
    s[t] += y;
    __syncthreads();
  }
  bsum[t] = s[t] - v;
  if (t == kImgBlocks - 1) bsum[kImgBlocks] = s[t];
}

__global__ __launch_bounds__(kBlock) void calls_image(const CallRec *__restrict__ recs, const int32_t *__restrict__ order,
                                                       const uint32_t *__restrict__ off, int64_t nbk,
                                                       const int64_t *__restrict__ bsum, const uint8_t *__restrict__ dpool,
                                                       Counters *__restrict__ ctr, uint8_t *__restrict__ img) {
  __shared__ uint32_t wsum[kBlock / 64];
  const int64_t n = (int64_t)off[nbk];
  const CallsLayout L = calls_layout(n, 0);
  int64_t a, b;
  img_chunk(n, a, b);
  int64_t prefix = bsum[blockIdx.x];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t base = a; base < b; base += blockDim.x) {  // uniform trip count per workgroup
    const int64_t k = base + threadIdx.x;
    CallRec r{};
    if (k < b) r = recs[order[k]];
    const uint32_t tot = k < b ? rec_len(r) : 0u;
    const uint32_t inc = wave_incl_scan(tot);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      before += w < wv ? wsum[w] : 0u;
      all += wsum[w];
    }
    __syncthreads();
    if (k < b) {
      const int64_t o = prefix + before + inc - tot;
      reinterpret_cast<int32_t *>(img + L.contig)[k] = r.contig;
      reinterpret_cast<int64_t *>(img + L.pos)[k] = r.pos;
      reinterpret_cast<int64_t *>(img + L.ref_off)[k] = o;
      reinterpret_cast<int64_t *>(img + L.alt_off)[k] = o + r.ref_len;
      reinterpret_cast<int32_t *>(img + L.ref_len)[k] = r.ref_len;
      reinterpret_cast<int32_t *>(img + L.alt_len)[k] = r.alt_len;
      img[L.sample + k] = r.sample;
      img[L.gt0 + k] = r.gt0;
      img[L.gt1 + k] = r.gt1;
      img[L.flags + k] = r.flags;
      uint8_t *dst = img + L.pool + o;
      if (tot <= 8) {
        for (uint32_t i = 0; i < tot; ++i) dst[i] = (uint8_t)(r.allele >> (8 * i));
      } else {
        for (uint32_t i = 0; i < tot; ++i) dst[i] = dpool[r.allele + i];
      }
    }
    prefix += all;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // header and the counters the host reads back
    const int64_t pool_len = bsum[kImgBlocks];
    reinterpret_cast<int64_t *>(img)[0] = pool_len;
    reinterpret_cast<int64_t *>(img)[1] = n;
    ctr->n_out = (unsigned long long)n;
    ctr->out_pool = (unsigned long long)pool_len;
  }
}

}  // namespace

// ==========================================================================================
// Host side: context, resident read sets, entry points
// ==========================================================================================
namespace {
__global__ void warm_k() {}
}  // namespace
hipError_t gq::warm_pileup(hipStream_t s) {
  hipLaunchKernelGGL(warm_k, dim3(1), dim3(64), 0, s);
  return hipGetLastError();
}

extern "C" {

const char *gq_version(void) { return "guacamole-amd gqpileup 0.1 (gfx950)"; }
const char *gq_last_error(void) { return g_err.c_str(); }

gq_status gq_open(int device, gq_ctx **out) {
  if (!out) return set_err(GQ_E_ARG, "gq_open: null out");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return set_err(GQ_E_ARG, "gq_open: device %d out of range (%d devices)", device, n);
  HIP_TRY(hipSetDevice(device));
  gq_ctx *c = new gq_ctx();
  c->device = device;
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIP_TRY(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
  for (auto &e : c->ev) HIP_TRY(hipEventCreate(&e));
  for (auto &e : c->dev_ev) HIP_TRY(hipEventCreate(&e));
  for (auto &e : c->side_ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // the staging chunks first (a load may wait on them), then the code objects
  c->prep = std::thread([c] {
    hipError_t e = hipSetDevice(c->device);
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
      e = hipHostMalloc(&c->stage[i], H2DStager::kChunk, hipHostMallocDefault);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&c->stage_done[i], hipEventDisableTiming);
    }
    {
      std::lock_guard<std::mutex> lk(c->stage_m);
      c->stage_err = e;
      c->stage_ready = true;
    }
    c->stage_cv.notify_all();
    if (e == hipSuccess) e = gq::warm_pileup(c->stream);
    if (e == hipSuccess) e = gq::warm_somatic(c->stream);
    if (e == hipSuccess) e = gq::warm_heapref(c->stream);
    if (e == hipSuccess) e = gq::warm_bamdev(c->stream);
    (void)e;  // (a failed warm-up only leaves the loading to the first launch)
  });
  *out = c;
  return GQ_OK;
}


void gq_close(gq_ctx *c) {
  if (!c) return;
  if (c->prep.joinable()) c->prep.join();
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (int i = 0; i < 2; ++i) {
    if (c->stage_done[i]) (void)hipEventDestroy(c->stage_done[i]);
    if (c->stage[i]) (void)hipHostFree(c->stage[i]);
  }
  for (DevBuf *b : {&c->ranges, &c->tiles, &c->recs, &c->recs_sorted, &c->keys, &c->keys_sorted, &c->idx,
                    &c->idx_sorted, &c->cplx, &c->pool, &c->counters, &c->sort_tmp, &c->image, &c->tiles2, &c->srecs, &c->c_depth, &c->c_pos,
                    &c->c_base, &c->c_indel, &c->c_ref, &c->c_rb, &c->c_amb, &c->slow, &c->amb, &c->amb_ref,
                    &c->heap_off, &c->heap_reads, &c->win_meta, &c->win_grp, &c->bkt})
    b->release();
  for (auto &e : c->ev) (void)hipEventDestroy(e);
  for (auto &e : c->dev_ev) (void)hipEventDestroy(e);
  for (auto &e : c->side_ev) (void)hipEventDestroy(e);
  if (c->side) {
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamDestroy(c->side);
  }
  if (c->pin) (void)hipHostFree(c->pin);
  (void)hipStreamDestroy(c->stream);
  delete c;
}

gq_status gq_get_timings(const gq_ctx *c, gq_timings *out) {
  if (!c || !out) return set_err(GQ_E_ARG, "gq_get_timings: null argument");
  *out = c->timings;
  return GQ_OK;
}

gq_status gq_set_tile(gq_ctx *c, int32_t t) {
  if (!c) return set_err(GQ_E_ARG, "null ctx");
  if (t == 0) t = kGermT;
  if (t != 512) return set_err(GQ_E_ARG, "tile must be 512 (the germline column kernel's geometry)");
  c->germ_tile = t;
  return GQ_OK;
}

static gq_status validate_reads(const gq_reads *h) {
  if (!h) return set_err(GQ_E_ARG, "null read set");
  if (h->n_reads < 0 || h->n_contigs <= 0) return set_err(GQ_E_ARG, "bad read-set sizes");
  if (h->n_samples < 1 || h->n_samples > 8) return set_err(GQ_E_ARG, "n_samples must be in [1, 8]");
  return GQ_OK;
}

// The spans a re-derivation recorded without waiting (gq_dev_reads::pending): wait for them now.
static gq_status settle_stats(gq_dev_reads *d) {
  if (d->pending & 1) {
    HIP_TRY(hipEventSynchronize(d->tev[1]));
    (void)hipEventElapsedTime(&d->derive_dev_ms, d->tev[0], d->tev[1]);
  }
  if (d->pending & 2) {
    HIP_TRY(hipEventSynchronize(d->tev[5]));
    (void)hipEventElapsedTime(&d->fill_ms, d->tev[3], d->tev[4]);
    (void)hipEventElapsedTime(&d->proj_dev_ms, d->tev[2], d->tev[5]);
    std::vector<unsigned long long> hk(kOkSpread);
    HIP_TRY(hipMemcpy(hk.data(), d->nok, sizeof(unsigned long long) * kOkSpread, hipMemcpyDeviceToHost));
    d->proj_reads = 0;
    for (unsigned long long x : hk) d->proj_reads += (int64_t)x;
    d->dp.put(d->nok);
    d->nok = nullptr;
  }
  d->pending = 0;
  return GQ_OK;
}

static gq_status derive_shape_impl(gq_ctx *c, gq_dev_reads *d, int64_t md_len, bool lazy = false) {
  for (hipEvent_t &e : d->tev)
    if (!e) HIP_TRY(hipEventCreate(&e));
  HIP_TRY(hipEventRecord(d->tev[0], c->stream));
  {  // contig_read_begin: 0, non-decreasing, n_reads (host copy)
    const auto &b = d->contig_read_begin;
    bool ok = !b.empty() && b.front() == 0 && b.back() == d->d.n_reads;
    for (size_t i = 1; i < b.size() && ok; ++i) ok = b[i] >= b[i - 1];
    if (!ok) return set_err(GQ_E_UNSORTED, "contig_read_begin must run from 0 to n_reads, non-decreasing");
  }
  void *p = nullptr;
  HIP_TRY(d->dp.get(&p, sizeof(int16_t) * (size_t)std::max<int64_t>(d->d.n_reads, 1)));
  d->d.lead = (const int16_t *)p;
  d->d.ev_rb = nullptr;  // (derived on first use: ensure_ev_bases)
  d->ev_bases = false;
  int unordered = 0;
  const int nc = d->d.n_contigs;
  std::vector<int32_t> last((size_t)nc, 0);  // each contig's largest read end (pmax_end of its last read)
  if (d->d.n_reads > 0) {
    void *flag = nullptr;
    HIP_TRY(d->dp.get(&flag, sizeof(int)));
    HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), c->stream));
    const unsigned nb = (unsigned)((d->d.n_reads + kBlock - 1) / kBlock);
    // validation and the read shapes in one pass (a read out of its pools gets no shape)
    hipLaunchKernelGGL(read_prep, dim3(nb), dim3(kBlock), 0, c->stream, d->d, (int *)flag, (int16_t *)p);
    HIP_TRY(hipGetLastError());
    int bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    const auto &crb = d->contig_read_begin;
    for (int k = 0; k < nc; ++k)
      if (crb[(size_t)k + 1] > crb[(size_t)k])
        HIP_TRY(hipMemcpyAsync(&last[(size_t)k], d->d.pmax_end + (crb[(size_t)k + 1] - 1), sizeof(int32_t),
                               hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (bad & 1)
      return set_err(GQ_E_UNSORTED, "Regions must be sorted by start locus: reads are not sorted by (contig, start), "
                                    "or pmax_end is not the running maximum of end within each contig");
    if (bad & 2)
      return set_err(GQ_E_ARG, "read set: an offset or length lies outside its pool, or a sample slot >= n_samples");
    unordered = (bad & 4) ? 1 : 0;
  }
  {  // the projections' slices (whole 512-locus blocks up to each contig's largest read end) and
     // the block index of the reads (plan_tiles' windows of aligned tiles); the projection
     // itself is derived on first use (ensure_projection)
    std::vector<int64_t> qoff((size_t)nc + 1, 0);
    for (int k = 0; k < nc; ++k) {
      const int64_t col1 = ((int64_t)std::max(last[(size_t)k], 0) + 7) >> 3;
      qoff[(size_t)k + 1] = qoff[(size_t)k] + 4 * ((col1 + 63) >> 6);
    }
    void *qo = nullptr;
    HIP_TRY(d->dp.get(&qo, sizeof(int64_t) * ((size_t)nc + 1)));
    HIP_TRY(hipMemcpyAsync(qo, qoff.data(), sizeof(int64_t) * ((size_t)nc + 1), hipMemcpyHostToDevice, c->stream));
    d->d.qoff = (const int64_t *)qo;
    d->n_slices = qoff[(size_t)nc];
    const int64_t n_blk = qoff[(size_t)nc] / 4;
    void *bi = nullptr;
    HIP_TRY(d->dp.get(&bi, sizeof(int64_t) * 2 * (size_t)std::max<int64_t>(n_blk, 1)));
    int64_t *brb = (int64_t *)bi, *brs = brb + std::max<int64_t>(n_blk, 1);
    if (n_blk > 0) {
      hipLaunchKernelGGL(block_index, dim3((unsigned)((n_blk + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream, d->d,
                         n_blk, brb, brs);
      HIP_TRY(hipGetLastError());
    }
    d->d.blk_rb = brb;
    d->d.blk_rs = brs;
  }
  // (the column records, the pool's base classes and the projection are derived on first use:
  // ensure_columns / ensure_projection; germline_direct needs none of them)
  HIP_TRY(hipEventRecord(d->tev[1], c->stream));
  d->d.pool_ordered = unordered ? 0 : 1;
  if (lazy) {  // (a re-derivation: the caller's next call goes on behind it on the stream)
    d->pending |= 1;
    return GQ_OK;
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  (void)hipEventElapsedTime(&d->derive_dev_ms, d->tev[0], d->tev[1]);
  return GQ_OK;
}


gq_status gq_reads_upload(gq_ctx *c, const gq_reads *h, gq_dev_reads **out) {
  if (!c || !out) return set_err(GQ_E_ARG, "gq_reads_upload: null argument");
  gq_status st = validate_reads(h);
  if (st) return st;
  HIP_TRY(hipSetDevice(c->device));
  gq_dev_reads *d = new gq_dev_reads();
  d->ctx = c;
  const int64_t n = h->n_reads;
  const auto t0 = std::chrono::steady_clock::now();
  H2DStager stager(c);
  {
    hipError_t e = stager.init();
    if (e != hipSuccess) {
      delete d;
      return set_err(GQ_E_HIP, "upload: pinned staging: %s", hipGetErrorString(e));
    }
  }
  // src_range(out, o, k): bytes [o, o + k) of the array in its device layout
  auto up_from = [&](size_t bytes, void **dst, size_t pad, const auto &src_range) -> hipError_t {
    *dst = nullptr;
    hipError_t e = hipMalloc(dst, std::max(bytes + pad, (size_t)16));
    if (e != hipSuccess) return e;
    d->owned.push_back(*dst);
    if (bytes) e = stager.copy_from(*dst, bytes, src_range);
    if (e == hipSuccess && pad) e = hipMemsetAsync((char *)*dst + bytes, 0, pad, c->stream);
    return e;
  };
  auto up = [&](const void *src, size_t bytes, void **dst, size_t pad) -> hipError_t {
    if (bytes >= (size_t(1) << 20) || (!src && bytes))  // (a null source reads as zeros)
      return up_from(bytes, dst, pad, [src](uint8_t *out, size_t o, size_t k) {
        if (src) memcpy(out, (const uint8_t *)src + o, k);
        else memset(out, 0, k);
      });
    *dst = nullptr;
    hipError_t e = hipMalloc(dst, std::max(bytes + pad, (size_t)16));
    if (e != hipSuccess) return e;
    d->owned.push_back(*dst);
    if (bytes) e = hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && pad) e = hipMemsetAsync((char *)*dst + bytes, 0, pad, c->stream);
    return e;
  };
  void *p;
#define UP_CHECK(field, T, expr)                                                \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      gq_reads_free(d);                                                         \
      return set_err(GQ_E_HIP, "upload %s: %s", #field, hipGetErrorString(_e)); \
    }                                                                           \
    d->d.field = (const T *)p;                                                  \
  } while (0)
#define UP(field, count, T) UP_CHECK(field, T, up(h->field, (size_t)(count) * sizeof(T), &p, pad_##field))
  // the sequence pool gets a zeroed tail so 1 KiB LDS-DMA pieces and 16-byte chunk loads
  // past the last read stay inside the allocation (DevReads::seq_cap)
  enum : size_t { pad_contig_read_begin = 0, pad_start = 0, pad_end = 0, pad_pmax_end = 0, pad_mapq = 0, pad_flags = 0,
                  pad_sample = 0, pad_seq_off = 0, pad_seq_len = 0, pad_cigar_off = 0, pad_n_cigar = 0, pad_md_off = 0,
                  pad_n_md = 0, pad_n_mismatch = 0, pad_seq = kSeqPad, pad_qual = kSeqPad, pad_cigar = 0,
                  pad_md_ev = 0 };
  // HBM layout: the sequence / quality pools in read order (each read's bytes after the
  // previous read's), so a tile's reads are one contiguous byte range for the LDS stage.
  // A host pool in another order is gathered into that order on its way through the pinned
  // staging chunks (the caller's buffers are untouched; no host copy of the pool is made).
  const gq_reads *h0 = h;
  gq_reads hh = *h;
  std::vector<int64_t> off2;
  bool ordered = true;
  for (int64_t r = 1; r < n && ordered; ++r) ordered = h->seq_off[r] >= h->seq_off[r - 1] + h->seq_len[r - 1];
  if (!ordered) {
    off2.resize((size_t)n);
    int64_t o = 0;
    for (int64_t r = 0; r < n; ++r) {
      off2[(size_t)r] = o;
      o += h->seq_len[r];
    }
    hh.seq_off = off2.data();
    hh.seq_bytes = o;
  }
  // pool bytes [o, o + k) in read order, from a caller pool at h0->seq_off
  auto gather = [&](const uint8_t *src) {
    return [&, src](uint8_t *out, size_t o, size_t k) {
      if (!src) {
        memset(out, 0, k);
        return;
      }
      int64_t r = (int64_t)(std::upper_bound(off2.begin(), off2.end(), (int64_t)o) - off2.begin()) - 1;
      size_t done = 0;
      while (done < k) {
        const size_t a = o + done - (size_t)off2[(size_t)r];
        const size_t m = std::min((size_t)h0->seq_len[r] - a, k - done);
        memcpy(out + done, src + h0->seq_off[r] + a, m);
        done += m;
        ++r;
      }
    };
  };
  h = &hh;
  UP(contig_read_begin, h->n_contigs + 1, int64_t);
  UP(start, n, int32_t);
  UP(end, n, int32_t);
  UP(pmax_end, n, int32_t);
  UP(mapq, n, uint8_t);
  UP(flags, n, uint8_t);
  UP(sample, n, uint8_t);
  UP(seq_off, n, int64_t);
  UP(seq_len, n, int32_t);
  UP(cigar_off, n, int64_t);
  UP(n_cigar, n, int32_t);
  UP(md_off, n, int64_t);
  UP(n_md, n, int32_t);
  UP(n_mismatch, n, uint16_t);
  if (ordered) {
    UP(seq, h->seq_bytes, uint8_t);
    UP(qual, h->seq_bytes, uint8_t);
  } else {
    UP_CHECK(seq, uint8_t, up_from((size_t)h->seq_bytes, &p, pad_seq, gather(h0->seq)));
    UP_CHECK(qual, uint8_t, up_from((size_t)h->seq_bytes, &p, pad_qual, gather(h0->qual)));
  }
  UP(cigar, h->cigar_len, uint32_t);
  UP(md_ev, h->md_len, uint32_t);
#undef UP
#undef UP_CHECK
  d->d.n_reads = n;
  d->d.seq_bytes = h->seq_bytes;
  d->d.seq_cap = h->seq_bytes + kSeqPad;
  d->d.cigar_len = h->cigar_len;
  d->d.md_len = h->md_len;
  d->d.n_contigs = h->n_contigs;
  d->d.n_samples = h->n_samples;
  if (h->sample_hash && h->n_samples > 0) {  // a few words: one synchronous copy
    void *sh = nullptr;
    if (hipMalloc(&sh, sizeof(uint32_t) * (size_t)h->n_samples) != hipSuccess ||
        hipMemcpy(sh, h->sample_hash, sizeof(uint32_t) * (size_t)h->n_samples, hipMemcpyHostToDevice) != hipSuccess) {
      if (sh) (void)hipFree(sh);
      gq_reads_free(d);
      return set_err(GQ_E_HIP, "gq_reads_upload: sample hashes");
    }
    d->owned.push_back(sh);
    d->d.sample_hash = (const uint32_t *)sh;
  }
  d->contig_read_begin.assign(h->contig_read_begin, h->contig_read_begin + h->n_contigs + 1);
  d->seq_bytes = h->seq_bytes;
  if (hipStreamSynchronize(c->stream) != hipSuccess) {
    gq_reads_free(d);
    return set_err(GQ_E_HIP, "gq_reads_upload: copies");
  }
  const auto t1 = std::chrono::steady_clock::now();
  d->h2d_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
  gq_status st2 = derive_shape_impl(c, d, h->md_len);
  d->derive_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t1).count();
  if (st2) {
    gq_reads_free(d);
    return st2;
  }
  *out = d;
  return GQ_OK;
}

gq_status gq_reads_wrap_device(gq_ctx *c, const gq_reads *h, gq_dev_reads **out) {
  if (!c || !out) return set_err(GQ_E_ARG, "gq_reads_wrap_device: null argument");
  gq_status st = validate_reads(h);
  if (st) return st;
  gq_dev_reads *d = new gq_dev_reads();
  d->ctx = c;
  d->d.n_reads = h->n_reads;
  d->d.seq_bytes = h->seq_bytes;
  d->d.seq_cap = h->seq_bytes;  // caller-owned buffer: no readable tail assumed
  d->d.cigar_len = h->cigar_len;
  d->d.md_len = h->md_len;
  d->d.n_contigs = h->n_contigs;
  d->d.n_samples = h->n_samples;
  d->d.contig_read_begin = h->contig_read_begin;
  d->d.start = h->start;
  d->d.end = h->end;
  d->d.pmax_end = h->pmax_end;
  d->d.mapq = h->mapq;
  d->d.flags = h->flags;
  d->d.sample = h->sample;
  d->d.seq_off = h->seq_off;
  d->d.seq_len = h->seq_len;
  d->d.cigar_off = h->cigar_off;
  d->d.n_cigar = h->n_cigar;
  d->d.md_off = h->md_off;
  d->d.n_md = h->n_md;
  d->d.n_mismatch = h->n_mismatch;
  d->d.seq = h->seq;
  d->d.qual = h->qual;
  d->d.cigar = h->cigar;
  d->d.md_ev = h->md_ev;
  d->d.sample_hash = h->sample_hash;  // device pointer (or NULL), as every array here
  d->contig_read_begin.resize((size_t)h->n_contigs + 1);
  hipError_t e = hipMemcpy(d->contig_read_begin.data(), h->contig_read_begin,
                           sizeof(int64_t) * ((size_t)h->n_contigs + 1), hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    delete d;
    return set_err(GQ_E_HIP, "wrap: contig_read_begin D2H: %s", hipGetErrorString(e));
  }
  d->seq_bytes = h->seq_bytes;
  const auto t1 = std::chrono::steady_clock::now();
  gq_status st2 = derive_shape_impl(c, d, h->md_len);
  d->derive_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t1).count();
  if (st2) {
    gq_reads_free(d);
    return st2;
  }
  *out = d;
  return GQ_OK;
}

gq_status gq_reads_rederive(gq_ctx *c, gq_dev_reads *d) {
  if (!c || !d) return set_err(GQ_E_ARG, "gq_reads_rederive: null argument");
  if (d->ctx != c) return set_err(GQ_E_ARG, "gq_reads_rederive: the read set belongs to another context");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));  // nothing queued may still read the derived buffers
  HIP_TRY(hipStreamSynchronize(c->side));
  // the previous derivation's figures nobody asked for are dropped (settling them would cost
  // a host round trip per re-derivation)
  d->nok = nullptr;
  d->pending = 0;
  d->dp.release_all();
  DevReads &R = d->d;
  R.lead = nullptr;
  R.ev_rb = R.clean = nullptr;
  R.pool_ordered = 0;
  R.cdesc = nullptr;
  R.cev = nullptr;
  R.caux_off = R.qoff = R.srow = R.pev_off = R.sra = R.soff = R.blk_rb = R.blk_rs = nullptr;
  R.prec = nullptr;
  R.proj = R.pbad = nullptr;
  R.pev = nullptr;
  R.prow = nullptr;
  d->projected = false;
  d->columns = false;
  d->ev_bases = false;
  d->nnb = d->mproj = d->mnb = nullptr;
  d->mproj_mapq = -1;
  d->proj_bytes = d->pev_count = d->proj_reads = d->n_rows = d->n_slices = 0;
  d->proj_ms = d->fill_ms = d->proj_dev_ms = 0;
  const auto t1 = std::chrono::steady_clock::now();
  const gq_status st = derive_shape_impl(c, d, R.md_len, true);
  d->derive_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t1).count();
  return st;
}

gq_status gq_reads_get_info(const gq_dev_reads *dc, gq_reads_info *out) {
  if (!dc || !out) return set_err(GQ_E_ARG, "gq_reads_get_info: null argument");
  gq_dev_reads *d = const_cast<gq_dev_reads *>(dc);  // (settling the pending spans fills cached figures)
  if (d->pending) {
    HIP_TRY(hipSetDevice(d->ctx->device));
    const gq_status s0 = settle_stats(d);
    if (s0) return s0;
  }
  out->n_reads = d->d.n_reads;
  out->seq_bytes = d->seq_bytes;
  out->proj_bytes = d->proj_bytes;
  out->pev_count = d->pev_count;
  out->n_rows = d->n_rows;
  out->proj_reads = d->proj_reads;
  out->h2d_ms = d->h2d_ms;
  out->derive_ms = d->derive_ms;
  out->cigar_len = d->d.cigar_len;
  out->md_len = d->d.md_len;
  out->n_contigs = d->d.n_contigs;
  out->n_samples = d->d.n_samples;
  out->proj_ms = d->proj_ms;
  out->projected = d->projected ? 1 : 0;
  out->fill_ms = d->fill_ms;
  out->proj_dev_ms = d->proj_dev_ms;
  out->derive_dev_ms = d->derive_dev_ms;
  return GQ_OK;
}

void gq_reads_free(gq_dev_reads *d) {
  if (!d) return;
  if (d->ctx) (void)hipSetDevice(d->ctx->device);
  for (hipEvent_t e : d->tev)
    if (e) {
      (void)hipEventSynchronize(e);
      (void)hipEventDestroy(e);
    }
  for (void *p : d->owned) (void)hipFree(p);
  d->dp.free_all();  // every derived structure, margin projection included
  delete d;
}

}  // extern "C"

// ---- shared planning: validate loci, upload ranges, plan tiles -----------------------------
static int gq_dbg() {  // GQ_DBG: diagnostics only (phase clocks, ablations)
  static const int d = getenv("GQ_DBG") ? atoi(getenv("GQ_DBG")) : 0;
  return d;
}

gq_status gq::plan(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, int T, Plan &pl, DevBuf &tiles_buf,
                   int stage_cap, int meta_cap, int ev_cap, bool aligned) {
  if (!loci || loci->n_ranges < 0) return set_err(GQ_E_ARG, "bad loci");
  const int64_t R = loci->n_ranges;
  pl = Plan{};
  pl.T = T;
  pl.aligned = aligned;
  std::vector<int32_t> &rc = pl.rc;
  std::vector<int64_t> &rs = pl.rs, &re = pl.re, &rt = pl.rt, ro;
  int64_t ord = 0, tiles = 0;
  for (int64_t i = 0; i < R; ++i) {
    const int32_t cc = loci->contig[i];
    const int64_t s = loci->start[i], e = loci->end[i];
    if (cc < 0 || cc >= rd->d.n_contigs) return set_err(GQ_E_ARG, "loci range %lld: contig %d out of range", (long long)i, cc);
    if (s < 0 || e < s || e > INT32_MAX) return set_err(GQ_E_ARG, "loci range %lld: bad interval", (long long)i);
    if (e == s) continue;
    const int64_t task = loci->task ? loci->task[i] : 0;
    // a new window at each change of (task, contig); within one, ranges must ascend
    if (pl.wins.empty() || pl.rtask.back() != task || rc.back() != cc) {
      pl.wins.push_back(Plan::Win{cc, (int64_t)rc.size(), (int64_t)rc.size()});
    } else if (s < re.back()) {
      return set_err(GQ_E_ARG, "loci range %lld: ranges of one task and contig must be sorted and disjoint",
                     (long long)i);
    }
    pl.wins.back().r1 = (int64_t)rc.size() + 1;
    pl.rwin.push_back((int32_t)(pl.wins.size() - 1));
    pl.rtask.push_back(task);
    rc.push_back(cc);
    rs.push_back(s);
    re.push_back(e);
    ro.push_back(ord);
    rt.push_back(tiles);
    ord += e - s;
    tiles += aligned ? (e - 1) / T - s / T + 1 : (e - s + T - 1) / T;
  }
  pl.n_tiles = tiles;
  pl.n_loci = ord;
  if (tiles == 0) return GQ_OK;
  const size_t nr = rc.size(), nw = pl.wins.size();
  // device layout: rc | rs re ro rt | w_roff (nw + 1) | rwin | w_contig
  const size_t o_rs = (nr * 4 + 15) & ~(size_t)15, o_wroff = o_rs + 4 * 8 * nr, o_rwin = o_wroff + 8 * (nw + 1),
               o_wc = o_rwin + ((4 * nr + 15) & ~(size_t)15), bytes = o_wc + 4 * nw;
  HIP_TRY(c->ranges.ensure(bytes + 64));
  char *base = (char *)c->ranges.p;
  int32_t *d_rc = (int32_t *)base;
  int64_t *d_rs = (int64_t *)(base + o_rs);
  int64_t *d_re = d_rs + nr, *d_ro = d_re + nr, *d_rt = d_ro + nr;
  {  // one H2D copy from pinned staging (the previous call's copy has completed: every call syncs)
    HIP_TRY(c->pinned(bytes));
    char *hb = (char *)c->pin;
    memcpy(hb, rc.data(), nr * 4);
    memcpy(hb + o_rs, rs.data(), nr * 8);
    memcpy(hb + o_rs + 8 * nr, re.data(), nr * 8);
    memcpy(hb + o_rs + 16 * nr, ro.data(), nr * 8);
    memcpy(hb + o_rs + 24 * nr, rt.data(), nr * 8);
    int64_t *wroff = (int64_t *)(hb + o_wroff);
    int32_t *wc = (int32_t *)(hb + o_wc);
    for (size_t w = 0; w < nw; ++w) {
      wroff[w] = pl.wins[w].r0;
      wc[w] = pl.wins[w].contig;
    }
    wroff[nw] = (int64_t)nr;
    memcpy(hb + o_rwin, pl.rwin.data(), nr * 4);
    HIP_TRY(hipMemcpyAsync(base, hb, bytes, hipMemcpyHostToDevice, c->stream));
  }
  pl.d_rs = d_rs;
  pl.d_re = d_re;
  pl.d_wroff = (const int64_t *)(base + o_wroff);
  pl.d_rwin = (const int32_t *)(base + o_rwin);
  pl.d_wcontig = (const int32_t *)(base + o_wc);
  // aligned 512-locus plans over projected reads carry a TileX per tile after the Tiles
  const bool with_x = aligned && T == 512 && rd->d.srow != nullptr;
  HIP_TRY(tiles_buf.ensure((size_t)tiles * (sizeof(Tile) + (with_x ? sizeof(TileX) : 0))));
  const int nb = (int)((tiles + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(plan_tiles, dim3(nb), dim3(kBlock), 0, c->stream, d_rc, d_rs, d_re, d_ro, d_rt, (int64_t)nr,
                     tiles, T, rd->d, (Tile *)tiles_buf.p, stage_cap, meta_cap, ev_cap, aligned ? 1 : 0,
                     with_x ? (TileX *)((Tile *)tiles_buf.p + tiles) : (TileX *)nullptr);
  HIP_TRY(hipGetLastError());
  return GQ_OK;
}

gq_status gq::check_device_error(gq_ctx *c, const Counters &h) {
  if (h.err == 1 && h.prof[4])  // bucket_count's record past every bucket (an internal fault): its fields
    fprintf(stderr, "gq: record slot %lld (k %llu of %llu): key %llx contig %d pos %d flags/gt %llx\n",
            (long long)h.err_pos, h.prof[3], h.prof[4], h.prof[0], (int)(h.prof[1] >> 32), (int)(uint32_t)h.prof[1],
            h.prof[2]);
  if (h.err) {
    static const char *names[] = {"ok", "assertion", "invalid cigar element", "CIGAR / MD tag mismatch",
                                  "read without MD tag", "multiple reference bases", "unsorted", "argument", "hip",
                                  "nomem", "allele table capacity"};
    const char *nm = (h.err >= 0 && h.err <= 10) ? names[h.err] : "?";
    return set_err((gq_status)h.err, "device error: %s near position %lld", nm, (long long)h.err_pos);
  }
  return GQ_OK;
}

extern "C" {

// The germline pileup kernel of a call: germline_direct (straight from the reads) unless
// GQ_GERM=proj asks for germline_proj over the projection (A/B; the same records).
static bool germline_direct_mode(const DevReads &R) {
  static const char *m = getenv("GQ_GERM");
  static const bool proj = m && strcmp(m, "proj") == 0;
  return !proj && R.seq_cap >= 8;
}

static unsigned germline_grid(gq_ctx *c, int64_t tiles, bool direct) {
  if (c->n_cu <= 0 && hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess)
    c->n_cu = 256;
  // persistent: every resident workgroup (4 waves, a tile per wave at a time) over a contiguous run
  int &per_cu = direct ? c->dir_wg_per_cu : c->proj_wg_per_cu;
  if (per_cu <= 0) {
    int nb = 0;
    const hipError_t e = direct ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, germline_direct<false>, DirCfg::kThreads, 0)
                                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, germline_proj, ProjCfg::kThreads, 0);
    if (e != hipSuccess || nb <= 0) nb = 2;
    per_cu = nb;
  }
  const int64_t want = (tiles + ProjCfg::kWaves - 1) / ProjCfg::kWaves;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>({want, (int64_t)per_cu * c->n_cu, (int64_t)kPartsCols}));
}

static gq_status launch_germline(gq_ctx *c, int64_t tiles, const DevReads &R, const gq_germline_params *p,
                                 CallRec *recs, ComplexItem *cplx, const OutGeom &og, Counters *ctr, bool direct) {
  static const int dbg = getenv("GQ_DBG") ? atoi(getenv("GQ_DBG")) : 0;  // diagnostics only
  HIP_TRY(c->slow.ensure((size_t)tiles * sizeof(int32_t)));
  // germline_proj reads the Tile + TileX arrays through one buffer of 128 B per tile
  if (tiles >= (int64_t)1 << 24) return set_err(GQ_E_ARG, "%lld tiles in one call (at most 2^24)", (long long)tiles);
  if (direct) {
    // the shallow instantiation over every tile, then the deep one over the tiles it listed
    // (read on the device: no host round trip; an empty list sends its waves home at once)
    HIP_TRY(c->deep_tiles.ensure((size_t)tiles * sizeof(int32_t)));
    hipLaunchKernelGGL(germline_direct<false>, dim3((unsigned)og.ncols), dim3(DirCfg::kThreads), 0, c->stream,
                       (const Tile *)c->tiles.p, tiles, R, p->threshold, p->emit_ref, p->emit_no_call, recs, cplx, og, ctr,
                       (int32_t *)c->slow.p, (int32_t *)c->deep_tiles.p, dbg);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(germline_direct<true>, dim3((unsigned)std::min<int64_t>((tiles + DirCfg::kWaves - 1) / DirCfg::kWaves, 512)),
                       dim3(DirCfg::kThreads), 0, c->stream, (const Tile *)c->tiles.p, tiles, R, p->threshold,
                       p->emit_ref, p->emit_no_call, recs, cplx, og, ctr, (int32_t *)c->slow.p,
                       (int32_t *)c->deep_tiles.p, dbg);
  } else {
    hipLaunchKernelGGL(germline_proj, dim3((unsigned)og.ncols), dim3(ProjCfg::kThreads), 0, c->stream,
                       (const Tile *)c->tiles.p, (const TileX *)((const Tile *)c->tiles.p + tiles), tiles, R.proj,
                       R.pev, R.n_samples,
                       p->threshold, p->emit_ref, p->emit_no_call, recs, cplx, og, ctr, (int32_t *)c->slow.p, dbg);
  }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(c->ev[5], c->stream));  // column kernel | walker kernel
  const unsigned wblocks = (unsigned)std::min<int64_t>(tiles, 2048);
  hipLaunchKernelGGL((germline_walk<ProjCfg::kT>), dim3(wblocks), dim3(kBlock), 0, c->stream,
                     (const Tile *)c->tiles.p, (const int32_t *)c->slow.p, R, p->threshold, p->emit_ref,
                     p->emit_no_call, recs, cplx, og, ctr);
  HIP_TRY(hipGetLastError());
  return GQ_OK;
}

// The germline pass.  dev == nullptr: the result image is copied into one host block owned by
// *out.  dev != nullptr: the image stays in HBM (c->image, valid until the next call on c) and
// *out holds device pointers into it (block_ = nullptr).
static gq_status germline_run(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, const gq_germline_params *p,
                              gq_calls **out, gq_calls_device *dev) {
  if (!c || !rd || !loci || !p || !out) return set_err(GQ_E_ARG, "gq_germline_threshold: null argument");
  HIP_TRY(hipSetDevice(c->device));
  const int T = c->germ_tile;
  c->timings = gq_timings{};
  const auto h0 = std::chrono::steady_clock::now();
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  Plan pl;
  const bool direct = germline_direct_mode(rd->d);
  gq_status st = direct ? GQ_OK : ensure_projection(c, rd);  // (derived on first use)
  if (st) return st;
  st = plan(c, rd, loci, T, pl, c->tiles, 0, 0, 0, true);
  if (st) return st;
  HIP_TRY(hipEventRecord(c->ev[1], c->stream));
  gq_calls *res = (gq_calls *)calloc(1, sizeof(gq_calls));
  if (!res) return set_err(GQ_E_NOMEM, "calloc");
  if (pl.n_tiles == 0) {
    *out = res;
    return GQ_OK;
  }
  const int ns = rd->d.n_samples;
  // output partitions: per germline_proj workgroup (capA, its share of the loci) and per
  // walker / complex-kernel wave (capB); grown on overflow
  OutGeom og{};
  og.ncols = (int)germline_grid(c, pl.n_tiles, direct);
  const bool dense = p->emit_ref || p->emit_no_call;
  const unsigned long long wg_loci = (unsigned long long)((pl.n_tiles + og.ncols - 1) / og.ncols) * T;
  og.capA[0] = dense ? 2ull * ns * wg_loci + 64 : wg_loci / 32 + 256;
  og.capA[1] = wg_loci / 32 + 256;
  og.capB[0] = dense ? 2ull * ns * (unsigned long long)pl.n_loci / 8192 + 256 : (unsigned long long)pl.n_loci / 16384 + 256;
  og.capB[1] = (unsigned long long)pl.n_loci / 16384 + 256;
  unsigned long long pool_cap = 1 << 22, amb_cap = 4096;
  unsigned long long gdeep_cap = 1024;  // loci per wide-table hand-off list (grown on overflow)
  Counters hc{};
  // output order: buckets of 2^bshift ordinals (one locus when every locus emits)
  const int bshift = dense ? 0 : 9;
  const uint64_t dead_key = ((uint64_t)pl.n_loci << 12) | 0xFFFu;
  const int64_t nbk = (pl.n_loci >> bshift) + 1;
  size_t scan_tmp = 0;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (int)(nbk + 1), c->stream));
  // ---- the finalize chain (record order, result image), sized from the device: see bucket_count
  auto finalize = [&](Counters *ctr, size_t cap_rec) -> gq_status {
    uint32_t *cnt = (uint32_t *)c->bkt.p, *off = cnt + (nbk + 1), *fill = off + (nbk + 1);
    hipLaunchKernelGGL(zero_u32, dim3((unsigned)std::min<int64_t>((3 * (nbk + 1) + kBlock - 1) / kBlock, 1024)),
                       dim3(kBlock), 0, c->stream, cnt, 3 * (nbk + 1));  // counts, (offsets), fills
    const unsigned gb = (unsigned)std::max<int64_t>(1, std::min<int64_t>(((int64_t)cap_rec + kBlock - 1) / kBlock, kFinBlocks));
    hipLaunchKernelGGL(bucket_count, dim3(gb), dim3(kBlock), 0, c->stream, (const CallRec *)c->recs.p,
                       ctr, og, dead_key, bshift, nbk, (uint64_t *)c->keys.p, (int32_t *)c->idx_sorted.p,
                       (int64_t *)c->idx.p, cnt);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(c->sort_tmp.p, scan_tmp, cnt, off, (int)(nbk + 1), c->stream));
    hipLaunchKernelGGL(bucket_scatter, dim3(gb), dim3(kBlock), 0, c->stream, (const Counters *)ctr,
                       (const int64_t *)c->idx.p, (const uint32_t *)off, fill, (int32_t *)c->keys_sorted.p);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(bucket_rank, dim3(gb), dim3(kBlock), 0, c->stream, nbk, (const uint32_t *)off,
                       (const int32_t *)c->keys_sorted.p, (const uint64_t *)c->keys.p, (const int32_t *)c->idx_sorted.p,
                       (const int64_t *)c->idx.p, (int32_t *)c->recs_sorted.p);
    HIP_TRY(hipGetLastError());
    int64_t *bsum = (int64_t *)c->keys_sorted.p + (cap_rec + 1) / 2 + 1;  // past the members (int32)
    hipLaunchKernelGGL(img_sums, dim3(kImgBlocks), dim3(kBlock), 0, c->stream, (const CallRec *)c->recs.p,
                       (const int32_t *)c->recs_sorted.p, (const uint32_t *)off, nbk, bsum);
    hipLaunchKernelGGL(img_scan, dim3(1), dim3(kImgBlocks), 0, c->stream, bsum);
    hipLaunchKernelGGL(calls_image, dim3(kImgBlocks), dim3(kBlock), 0, c->stream, (const CallRec *)c->recs.p,
                       (const int32_t *)c->recs_sorted.p, (const uint32_t *)off, nbk, (const int64_t *)bsum,
                       (const uint8_t *)c->pool.p, ctr, (uint8_t *)c->image.p);
    HIP_TRY(hipGetLastError());
    return GQ_OK;
  };
  // the counters' head back to the host (one copy, one sync)
  auto read_counters = [&](Counters *ctr) -> gq_status {
    HIP_TRY(c->pinned(kCountersHead));
    HIP_TRY(hipMemcpyAsync(c->pin, ctr, kCountersHead, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    memcpy(&hc, c->pin, kCountersHead);
    return GQ_OK;
  };
  for (int attempt = 0; attempt < 3; ++attempt) {
    HIP_TRY(c->amb.ensure(2 * amb_cap * sizeof(AmbItem)));  // heap-order loci, then order-dependent loci
    const size_t cap_rec = (size_t)og.total(0);
    HIP_TRY(c->recs.ensure(cap_rec * sizeof(CallRec)));
    HIP_TRY(c->cplx.ensure(og.total(1) * sizeof(ComplexItem)));
    HIP_TRY(c->pool.ensure(pool_cap));
    HIP_TRY(c->counters.ensure(sizeof(Counters)));
    // finalize buffers, by the record capacity (the chain never learns the count on the host)
    HIP_TRY(c->keys.ensure((cap_rec + 1) * 8));
    HIP_TRY(c->keys_sorted.ensure((cap_rec + 1) * 4 + 8 * (kImgBlocks + 2) + 16));  // members | chunk sums
    HIP_TRY(c->idx.ensure((cap_rec + 1) * 8));
    HIP_TRY(c->idx_sorted.ensure((cap_rec + 1) * 4));
    HIP_TRY(c->recs_sorted.ensure((cap_rec + 1) * 4));
    HIP_TRY(c->bkt.ensure(sizeof(uint32_t) * (size_t)(3 * (nbk + 1))));
    HIP_TRY(c->sort_tmp.ensure(std::max<size_t>(scan_tmp, 16)));
    HIP_TRY(c->image.ensure(calls_layout((int64_t)cap_rec, (int64_t)pool_cap).bytes));
    Counters *ctr = (Counters *)c->counters.p;
    HIP_TRY(hipMemsetAsync(ctr, 0, sizeof(Counters), c->stream));
    if (attempt == 0) HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    st = launch_germline(c, pl.n_tiles, rd->d, p, (CallRec *)c->recs.p, (ComplexItem *)c->cplx.p, og, ctr, direct);
    if (st) {
      free(res);
      return st;
    }
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
#ifndef GQ_CPLX_BLOCKS
#define GQ_CPLX_BLOCKS 4096
#endif
    const int cblocks = (int)std::min<int64_t>(std::max<int64_t>(pl.n_tiles, 1), GQ_CPLX_BLOCKS);
    // each window's initial-group bound: an order-dependent locus past it needs no re-run
    SomWin wb{};
    st = window_bounds(c, pl, rd, wb);
    if (st) {
      free(res);
      return st;
    }
    hipLaunchKernelGGL(part_scan, dim3(1), dim3(1024), 0, c->stream, ctr, 1, og);
    HIP_TRY(c->deep_list.ensure(3 * sizeof(int64_t) * (size_t)gdeep_cap));
    auto complex_pair = [&](int blocks, int which, AmbItem *amb_out, unsigned long long acap, const AmbItem *amb_in,
                            const uint8_t *amb_ref, int64_t n_amb_in, const SomWin &sw_) -> gq_status {
      // the fast table, then the wide one over the loci it handed over (an empty list: the wide
      // launch's waves read a zero count and leave)
      int64_t *region = (int64_t *)c->deep_list.p + (size_t)which * gdeep_cap;
      const DeepList fast{region, &ctr->n_gdeep[which], nullptr, nullptr, gdeep_cap};
      const DeepList wide{nullptr, nullptr, region, &ctr->n_gdeep[which], gdeep_cap};
      hipLaunchKernelGGL(germline_complex<2>, dim3(blocks), dim3(kBlock), 0, c->stream, (const Tile *)c->tiles.p,
                         (const ComplexItem *)c->cplx.p, rd->d, p->threshold, p->emit_ref, p->emit_no_call,
                         (CallRec *)c->recs.p, og, (uint8_t *)c->pool.p, pool_cap, ctr, amb_out, acap, amb_in, amb_ref,
                         n_amb_in, gq_dbg(), sw_, fast);
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(germline_complex<16>, dim3(64), dim3(kBlock), 0, c->stream, (const Tile *)c->tiles.p,
                         (const ComplexItem *)c->cplx.p, rd->d, p->threshold, p->emit_ref, p->emit_no_call,
                         (CallRec *)c->recs.p, og, (uint8_t *)c->pool.p, pool_cap, ctr, amb_out, acap, amb_in, amb_ref,
                         n_amb_in, gq_dbg(), sw_, wide);
      HIP_TRY(hipGetLastError());
      return GQ_OK;
    };
    st = complex_pair(cblocks, 0, (AmbItem *)c->amb.p, amb_cap, (const AmbItem *)nullptr, (const uint8_t *)nullptr,
                      (int64_t)0, wb);
    if (st) {
      free(res);
      return st;
    }
    hipLaunchKernelGGL(part_scan, dim3(1), dim3(1024), 0, c->stream, ctr, 0, og);
    {  // variant candidates -> records; unused slots get a key behind every ordinal
#ifndef GQ_EXPAND_BLOCKS
#define GQ_EXPAND_BLOCKS 1024  // workgroups of germline_expand (each walks kParts / this many partitions)
#endif
      hipLaunchKernelGGL(germline_expand, dim3(GQ_EXPAND_BLOCKS), dim3(kBlock), 0, c->stream, (CallRec *)c->recs.p, ctr, og,
                         p->threshold, p->emit_ref, p->emit_no_call, dead_key);
      HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(c->ev[3], c->stream));
    // the common case needs no re-run: order the records and build the image right away
    st = finalize(ctr, cap_rec);
    if (st) {
      free(res);
      return st;
    }
    HIP_TRY(hipEventRecord(c->ev[4], c->stream));
    st = read_counters(ctr);
    if (st) {
      free(res);
      return st;
    }
    bool retry = false;
    // part_max = the largest overflow of a partition: grow both capacities by it
    for (int w = 0; w < 2; ++w)
      if (hc.part_max[w]) {
        og.capA[w] += hc.part_max[w] + 64;
        og.capB[w] += hc.part_max[w] + 64;
        retry = true;
      }
    if (hc.pool_used > pool_cap) {
      pool_cap = hc.pool_used + 4096;
      retry = true;
    }
    if (hc.n_amb > amb_cap || hc.n_ord > amb_cap) {
      amb_cap = std::max(hc.n_amb, hc.n_ord) + 1024;
      retry = true;
    }
    if (hc.n_gdeep[0] > gdeep_cap) {
      gdeep_cap = hc.n_gdeep[0] + 1024;
      retry = true;
    }
    // the windows' element order (initial groups in heap order) for the re-runs below: the
    // first occurrences the Scala map orders of those loci depend on
    SomWin sw{};
    const bool rerun = !retry && (hc.n_amb > 0 || hc.n_ord > 0) && !hc.err;
    if (rerun) {
      st = build_somwin(c, pl, rd, rd, sw);
      if (st) {
        free(res);
        return st;
      }
    }
    if (rerun && hc.n_ord > 0) {
      // loci whose output order depends on first occurrences in element order
      const int oblocks = (int)std::min<int64_t>(((int64_t)hc.n_ord + 3) / 4, 4096);
      st = complex_pair(oblocks, 1, (AmbItem *)nullptr, (unsigned long long)0, (const AmbItem *)c->amb.p + amb_cap,
                        (const uint8_t *)nullptr, (int64_t)hc.n_ord, sw);
      if (st) {
        free(res);
        return st;
      }
      hipLaunchKernelGGL(part_scan, dim3(1), dim3(1024), 0, c->stream, ctr, 0, og);
    }
    if (rerun && hc.n_amb > 0) {
      // loci whose reference base depends on heap order: replay the window's queue, then the
      // complex kernel again over just those loci with the resolved base
      std::vector<AmbItem> amb((size_t)hc.n_amb);
      HIP_TRY(hipMemcpyAsync(amb.data(), c->amb.p, amb.size() * sizeof(AmbItem), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(c->amb_ref.ensure(amb.size()));
      st = heap_ref_bases(c, pl, c->tiles, {rd}, amb, (uint8_t *)c->amb_ref.p);
      if (st) {
        free(res);
        return st;
      }
      const int ablocks = (int)std::min<int64_t>(((int64_t)amb.size() + 3) / 4, 4096);
      st = complex_pair(ablocks, 2, (AmbItem *)nullptr, (unsigned long long)0, (const AmbItem *)c->amb.p,
                        (const uint8_t *)c->amb_ref.p, (int64_t)amb.size(), sw);
      if (st) {
        free(res);
        return st;
      }
      hipLaunchKernelGGL(part_scan, dim3(1), dim3(1024), 0, c->stream, ctr, 0, og);
    }
    if (rerun) {  // the re-runs added records: check their capacities, then the chain again
      HIP_TRY(hipEventRecord(c->ev[3], c->stream));
      st = read_counters(ctr);
      if (st) {
        free(res);
        return st;
      }
      if (hc.part_max[0]) {
        og.capA[0] += hc.part_max[0] + 64;
        og.capB[0] += hc.part_max[0] + 64;
        retry = true;
      }
      if (hc.pool_used > pool_cap) {
        pool_cap = hc.pool_used + 4096;
        retry = true;
      }
      if (std::max(hc.n_gdeep[1], hc.n_gdeep[2]) > gdeep_cap) {
        gdeep_cap = std::max(hc.n_gdeep[1], hc.n_gdeep[2]) + 1024;
        retry = true;
      }
      if (!retry) {
        st = finalize(ctr, cap_rec);
        if (!st) {
          HIP_TRY(hipEventRecord(c->ev[4], c->stream));
          st = read_counters(ctr);
        }
        if (st) {
          free(res);
          return st;
        }
      }
    }
    if (!retry) break;
    if (attempt == 2) {
      free(res);
      return set_err(GQ_E_CAPACITY, "output capacity retries exhausted");
    }
  }
  if ((gq_dbg() & 32) && hc.prof[4])
    fprintf(stderr, "gq germline_complex prof (cycles/item/wave): cover %.0f reference-base %.0f elements %.0f "
            "map-order %.0f decision %.0f (%llu items)\n", (double)hc.prof[0] / hc.prof[4],
            (double)hc.prof[1] / hc.prof[4], (double)hc.prof[2] / hc.prof[4], (double)hc.prof[5] / hc.prof[4],
            (double)hc.prof[3] / hc.prof[4], hc.prof[4]);
  if ((gq_dbg() & 16) && hc.prof[5])
    fprintf(stderr,
            "gq prof (cycles/tile/wave): setup %.0f chunks %.0f (runs %.0f [fields %.0f slots %.0f] counting %.0f) "
            "decision %.0f (%llu)\n",
            (double)hc.prof[0] / hc.prof[5], (double)hc.prof[1] / hc.prof[5], (double)hc.prof[2] / hc.prof[5],
            (double)hc.prof[6] / hc.prof[5], (double)hc.prof[7] / hc.prof[5], (double)hc.prof[3] / hc.prof[5],
            (double)hc.prof[4] / hc.prof[5], hc.prof[5]);
  for (int k = 0; k < kSpread; ++k) {
    hc.visited += hc.spread[0][k];
    hc.ambiguous += hc.spread[1][k];
    hc.ties += hc.spread[2][k];
    hc.n_dead += hc.spread[3][k];
  }
  st = check_device_error(c, hc);
  if (st) {
    free(res);
    return st;
  }
  // ---- the image is in HBM (header: pool_len, n); the host block is one D2H copy of it
  const int64_t n = (int64_t)hc.n_out;
  const CallsLayout lay = calls_layout(n, (int64_t)hc.out_pool);
  const int64_t pool_len = (int64_t)hc.out_pool;
  uint8_t *blk = nullptr;
  if (dev) {  // the image stays in HBM
    blk = (uint8_t *)c->image.p;
    dev->image = c->image.p;
    dev->image_bytes = (int64_t)lay.pool + pool_len;
  } else {
    const size_t nbytes = (size_t)lay.pool + (size_t)pool_len;
    blk = (uint8_t *)malloc(std::max<size_t>(nbytes, 64));
    if (!blk) {
      free(res);
      return set_err(GQ_E_NOMEM, "result block of %zu bytes", nbytes);
    }
    HIP_TRY(hipMemcpyAsync(blk, c->image.p, nbytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  // ---- point the result struct into the block (output order)
  const auto h1 = std::chrono::steady_clock::now();
  res->n = n;
  res->block_ = dev ? nullptr : blk;
  res->contig = (int32_t *)(blk + lay.contig);
  res->pos = (int64_t *)(blk + lay.pos);
  res->ref_off = (int64_t *)(blk + lay.ref_off);
  res->alt_off = (int64_t *)(blk + lay.alt_off);
  res->ref_len = (int32_t *)(blk + lay.ref_len);
  res->alt_len = (int32_t *)(blk + lay.alt_len);
  res->sample = blk + lay.sample;
  res->gt0 = blk + lay.gt0;
  res->gt1 = blk + lay.gt1;
  res->flags = blk + lay.flags;
  res->allele_pool = blk + lay.pool;
  res->pool_len = pool_len;
  res->visited_loci = (int64_t)hc.visited;
  res->complex_loci = (int64_t)hc.n_complex;
  res->ambiguous_loci = (int64_t)hc.ambiguous;
  res->tie_loci = (int64_t)hc.ties;
  // timings
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
  c->timings.plan_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[5]);
  c->timings.pileup_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[5], c->ev[2]);
  c->timings.walk_ms = ms;
  c->timings.walk_tiles = (int64_t)hc.n_slow;
  c->timings.order_loci = (int64_t)hc.n_ord;
  (void)hipEventElapsedTime(&ms, c->ev[2], c->ev[3]);
  c->timings.complex_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[3], c->ev[4]);
  c->timings.finalize_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[4]);
  c->timings.total_ms = ms;
  c->timings.pileup_launches = 1;
  c->timings.tiles = pl.n_tiles;
  const auto h2 = std::chrono::steady_clock::now();
  c->timings.host_ms = std::chrono::duration<float, std::milli>(h2 - h0).count();
  c->timings.marshal_ms = std::chrono::duration<float, std::milli>(h2 - h1).count();
  *out = res;
  return GQ_OK;
}

gq_status gq_germline_threshold(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci,
                                const gq_germline_params *p, gq_calls **out) {
  return germline_run(c, rd, loci, p, out, nullptr);
}

gq_status gq_germline_threshold_device(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci,
                                       const gq_germline_params *p, gq_calls_device *out) {
  if (!out) return set_err(GQ_E_ARG, "gq_germline_threshold_device: null argument");
  memset(out, 0, sizeof(*out));
  gq_calls *r = nullptr;
  const gq_status st = germline_run(c, rd, loci, p, &r, out);
  if (st) return st;
  out->calls = *r;
  out->calls.block_ = nullptr;
  free(r);
  return GQ_OK;
}

gq_status gq_write_vcf_germline(const char *path, const char *header, int64_t n, const int32_t *contig,
                                const int64_t *pos, const uint8_t *gt0, const uint8_t *gt1, const int64_t *ref_off,
                                const int32_t *ref_len, const int64_t *alt_off, const int32_t *alt_len,
                                const uint8_t *pool, int32_t n_contigs, const char *const *contig_names) {
  if (!path || !header || (n > 0 && (!contig || !pos || !gt0 || !gt1 || !ref_off || !ref_len || !alt_off || !alt_len ||
                                      !contig_names)))
    return set_err(GQ_E_ARG, "gq_write_vcf_germline: null argument");
  FILE *f = fopen(path, "wb");
  if (!f) return set_err(GQ_E_ARG, "cannot write %s", path);
  std::string buf(header);
  buf.reserve((size_t)n * 48 + buf.size() + 64);
  static const char kGt[4] = {'0', '1', '.', '.'};  // GenotypeAllele Ref, Alt, OtherAlt, NoCall
  std::vector<size_t> clen((size_t)std::max(n_contigs, 0));
  for (int32_t k = 0; k < n_contigs; ++k) clen[(size_t)k] = contig_names[k] ? strlen(contig_names[k]) : 0;
  char num[24];
  bool ok = true;
  for (int64_t i = 0; i < n && ok; ++i) {
    const int32_t c = contig[i];
    if (c < 0 || c >= n_contigs || !contig_names[c]) {
      fclose(f);
      return set_err(GQ_E_ARG, "gq_write_vcf_germline: record %lld has contig %d", (long long)i, c);
    }
    buf.append(contig_names[c], clen[(size_t)c]);
    buf += '\t';
    const int k = snprintf(num, sizeof num, "%lld", (long long)(pos[i] + 1));
    buf.append(num, (size_t)k);
    buf.append("\t.\t", 3);
    buf.append((const char *)pool + ref_off[i], (size_t)ref_len[i]);
    buf += '\t';
    buf.append((const char *)pool + alt_off[i], (size_t)alt_len[i]);
    buf.append("\t.\t.\t.\tGT\t", 10);
    buf += kGt[gt0[i] & 3];
    buf += '/';
    buf += kGt[gt1[i] & 3];
    buf += '\n';
    if (buf.size() > (size_t)(64 << 20)) {  // write in 64 MiB pieces
      ok = fwrite(buf.data(), 1, buf.size(), f) == buf.size();
      buf.clear();
    }
  }
  if (ok && !buf.empty()) ok = fwrite(buf.data(), 1, buf.size(), f) == buf.size();
  if (fclose(f) != 0) ok = false;
  return ok ? GQ_OK : set_err(GQ_E_ARG, "write to %s failed", path);
}

void gq_free_calls(gq_calls *r) {
  if (!r) return;
  free(r->block_);
  free(r);
}

gq_status gq_pileup_counts(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, gq_counts **out) {
  if (!c || !rd || !loci || !out) return set_err(GQ_E_ARG, "gq_pileup_counts: null argument");
  HIP_TRY(hipSetDevice(c->device));
  Plan pl;
  gq_status st = ensure_columns(c, rd);  // (the walker's clean fast path)
  if (st) return st;
  st = plan(c, rd, loci, kCountT, pl, c->tiles);
  if (st) return st;
  gq_counts *res = (gq_counts *)calloc(1, sizeof(gq_counts));
  const int64_t n = pl.n_loci;
  res->n_loci = n;
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  res->depth = (int32_t *)malloc(nn * 4);
  res->pos_depth = (int32_t *)malloc(nn * 4);
  res->base_counts = (int32_t *)malloc(nn * 24);
  res->indel_counts = (int32_t *)malloc(nn * 16);
  res->ref_depth = (int32_t *)malloc(nn * 4);
  res->ref_base = (uint8_t *)malloc(nn);
  res->ambiguous = (uint8_t *)malloc(nn);
  if (n == 0) {
    *out = res;
    return GQ_OK;
  }
  HIP_TRY(c->c_depth.ensure(nn * 4));
  HIP_TRY(c->c_pos.ensure(nn * 4));
  HIP_TRY(c->c_base.ensure(nn * 24));
  HIP_TRY(c->c_indel.ensure(nn * 16));
  HIP_TRY(c->c_ref.ensure(nn * 4));
  HIP_TRY(c->c_rb.ensure(nn));
  HIP_TRY(c->c_amb.ensure(nn));
  HIP_TRY(c->counters.ensure(sizeof(Counters)));
  Counters *ctr = (Counters *)c->counters.p;
  HIP_TRY(hipMemsetAsync(ctr, 0, sizeof(Counters), c->stream));
  hipLaunchKernelGGL((counts_tile<kCountT>), dim3((unsigned)pl.n_tiles), dim3(kBlock), 0, c->stream,
                     (const Tile *)c->tiles.p, rd->d, (int32_t *)c->c_depth.p, (int32_t *)c->c_pos.p,
                     (int32_t *)c->c_base.p, (int32_t *)c->c_indel.p, (int32_t *)c->c_ref.p, (uint8_t *)c->c_rb.p,
                     (uint8_t *)c->c_amb.p, ctr);
  HIP_TRY(hipGetLastError());
  Counters hc{};
  HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(res->depth, c->c_depth.p, nn * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(res->pos_depth, c->c_pos.p, nn * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(res->base_counts, c->c_base.p, nn * 24, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(res->indel_counts, c->c_indel.p, nn * 16, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(res->ref_depth, c->c_ref.p, nn * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(res->ref_base, c->c_rb.p, nn, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(res->ambiguous, c->c_amb.p, nn, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  st = check_device_error(c, hc);
  if (st) {
    gq_free_counts(res);
    return st;
  }
  {  // loci whose reference base depends on the queue's heap order: replayed (gq_replay.h)
    std::vector<AmbItem> amb;
    std::vector<int64_t> ords;
    int64_t o = 0;
    for (size_t r = 0; r < pl.rs.size(); ++r) {
      const int64_t len = pl.re[r] - pl.rs[r];
      for (int64_t i = 0; i < len; ++i)
        if (res->ambiguous[o + i]) {
          amb.push_back(AmbItem{(int32_t)(pl.rt[r] + i / kCountT), (int32_t)(pl.rs[r] + i), (int64_t)amb.size()});
          ords.push_back(o + i);
        }
      o += len;
    }
    if (!amb.empty()) {
      HIP_TRY(c->amb_ref.ensure(amb.size()));
      st = heap_ref_bases(c, pl, c->tiles, {rd}, amb, (uint8_t *)c->amb_ref.p);
      if (st) {
        gq_free_counts(res);
        return st;
      }
      std::vector<uint8_t> rb(amb.size());
      HIP_TRY(hipMemcpy(rb.data(), c->amb_ref.p, rb.size(), hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost));
      st = check_device_error(c, hc);
      if (st) {
        gq_free_counts(res);
        return st;
      }
      for (size_t k = 0; k < amb.size(); ++k) {
        const int64_t x = ords[k];
        const uint8_t b = rb[k];
        const int cat = b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : b == 'T' ? 3 : 4;  // base_counts: A C G T N other
        res->ref_base[x] = b;
        res->ref_depth[x] = res->base_counts[x * 6 + cat];
      }
    }
  }
  *out = res;
  return GQ_OK;
}

gq_status gq_vaf_histogram(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, const gq_vaf_params *p,
                           gq_vaf_hist *out) {
  if (!c || !rd || !loci || !p || !out) return set_err(GQ_E_ARG, "gq_vaf_histogram: null argument");
  if (p->bins < 1 || p->bins > 100) return set_err(GQ_E_ASSERT, "assumption failed: Bins should be between 1 and 100");
  HIP_TRY(hipSetDevice(c->device));
  memset(out, 0, sizeof(*out));
  Plan pl;
  gq_status st = ensure_columns(c, rd);  // (the walker's clean fast path)
  if (st) return st;
  st = plan(c, rd, loci, kCountT, pl, c->tiles);
  if (st) return st;
  if (pl.n_tiles == 0) return GQ_OK;
  unsigned long long amb_cap = 4096;
  Counters hc{};
  for (int attempt = 0;; ++attempt) {
    HIP_TRY(c->counters.ensure(sizeof(Counters)));
    HIP_TRY(c->c_depth.ensure(sizeof(unsigned long long) * 64 * 101));
    HIP_TRY(c->amb.ensure(amb_cap * sizeof(AmbItem)));
    HIP_TRY(c->c_base.ensure(amb_cap * sizeof(VafAmb)));
    Counters *ctr = (Counters *)c->counters.p;
    HIP_TRY(hipMemsetAsync(ctr, 0, sizeof(Counters), c->stream));
    HIP_TRY(hipMemsetAsync(c->c_depth.p, 0, sizeof(unsigned long long) * 64 * 101, c->stream));
    hipLaunchKernelGGL((vaf_tile<kCountT>), dim3((unsigned)pl.n_tiles), dim3(kBlock), 0, c->stream,
                       (const Tile *)c->tiles.p, rd->d, (int)p->bins, (int)p->min_read_depth, (int)p->min_vaf,
                       (unsigned long long *)c->c_depth.p, (AmbItem *)c->amb.p, (VafAmb *)c->c_base.p, amb_cap, ctr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (hc.n_amb <= amb_cap || hc.err) break;
    if (attempt == 2) return set_err(GQ_E_CAPACITY, "vaf-histogram: listed-locus capacity retries exhausted");
    amb_cap = hc.n_amb + 1024;
  }
  st = check_device_error(c, hc);
  if (st) return st;
  std::vector<unsigned long long> h(64 * 101);
  HIP_TRY(hipMemcpy(h.data(), c->c_depth.p, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
  for (int k = 0; k < 64; ++k)
    for (int b = 0; b < 101; ++b) out->counts[b] += (int64_t)h[(size_t)k * 101 + (size_t)b];
  for (int k = 0; k < kSpread; ++k) {
    out->visited_loci += (int64_t)hc.spread[0][k];
    out->variant_loci += (int64_t)hc.spread[1][k];
  }
  if (hc.n_amb > 0) {  // heap-order reference bases (gq_replay.h), binned here as on the device
    std::vector<AmbItem> amb((size_t)hc.n_amb);
    std::vector<VafAmb> cnt((size_t)hc.n_amb);
    HIP_TRY(hipMemcpy(amb.data(), c->amb.p, amb.size() * sizeof(AmbItem), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(cnt.data(), c->c_base.p, cnt.size() * sizeof(VafAmb), hipMemcpyDeviceToHost));
    HIP_TRY(c->amb_ref.ensure(amb.size()));
    st = heap_ref_bases(c, pl, c->tiles, {rd}, amb, (uint8_t *)c->amb_ref.p);
    if (st) return st;
    std::vector<uint8_t> rb(amb.size());
    HIP_TRY(hipMemcpy(rb.data(), c->amb_ref.p, rb.size(), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&hc, c->counters.p, sizeof(Counters), hipMemcpyDeviceToHost));
    st = check_device_error(c, hc);
    if (st) return st;
    const int bin_size = 100 / p->bins;
    for (size_t k = 0; k < amb.size(); ++k) {
      const uint8_t b = rb[k];
      const int cat = b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : b == 'T' ? 3 : b == 'N' ? 4 : 5;
      const int32_t depth = cnt[k].depth, ref = cnt[k].base[cat];
      if (ref == depth) continue;
      const float vaf = (float)(depth - ref) / (float)depth;
      if (!(depth >= p->min_read_depth) || !((double)vaf >= (double)p->min_vaf / 100.0)) continue;
      const int pct = (int)(vaf * 100.0f);
      out->counts[pct - pct % bin_size] += 1;
      out->variant_loci += 1;
    }
  }
  return GQ_OK;
}

void gq_free_counts(gq_counts *r) {
  if (!r) return;
  free(r->depth);
  free(r->pos_depth);
  free(r->base_counts);
  free(r->indel_counts);
  free(r->ref_depth);
  free(r->ref_base);
  free(r->ambiguous);
  free(r);
}



}  // extern "C"

gq_status gq::derive_shape(gq_ctx *c, gq_dev_reads *d, int64_t md_len) { return derive_shape_impl(c, d, md_len); }

// The read base under each MD event (ev_bases), derived on first use by the column records.
gq_status gq::ensure_ev_bases(gq_ctx *c, const gq_dev_reads *cd) {
  gq_dev_reads *d = const_cast<gq_dev_reads *>(cd);
  if (d->ev_bases) return GQ_OK;
  void *q = nullptr;
  HIP_TRY(d->dp.get(&q, (size_t)std::max<int64_t>(d->d.md_len, 16)));
  if (d->d.n_reads > 0) {
    hipLaunchKernelGGL(ev_bases, dim3((unsigned)((d->d.n_reads + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                       d->d, (uint8_t *)q);
    HIP_TRY(hipGetLastError());
  }
  d->d.ev_rb = (const uint8_t *)q;
  d->ev_bases = true;
  return GQ_OK;
}

// The column records of a resident read set, derived on first use by a kernel that reads them
// (the projection's fills and sparse entries, somatic_proj, the walkers' clean fast path):
// clean[r] (every sequenced byte of read r is A C G T N) and its N bytes (pool_clean, or
// read_clean for a pool out of read order), then each read's ColDesc and auxiliary list (MD
// events, a general read's segments).  germline_direct reads none of it.
gq_status gq::ensure_columns(gq_ctx *c, const gq_dev_reads *cd) {
  gq_dev_reads *d = const_cast<gq_dev_reads *>(cd);
  if (d->columns) return GQ_OK;
  {
    const gq_status se = ensure_ev_bases(c, d);  // (col_derive's event words carry them)
    if (se) return se;
  }
  const int64_t n = d->d.n_reads;
  void *cl = nullptr, *nnb = nullptr;
  HIP_TRY(d->dp.get(&cl, (size_t)std::max<int64_t>(n, 1)));
  HIP_TRY(d->dp.get(&nnb, sizeof(uint32_t) * (size_t)std::max<int64_t>(n, 1)));
  HIP_TRY(hipMemsetAsync(nnb, 0, sizeof(uint32_t) * (size_t)std::max<int64_t>(n, 1), c->stream));
  if (n > 0) {
    if (d->d.pool_ordered) {  // the pool in read order: 16-byte chunks, the rare other bytes searched
      HIP_TRY(hipMemsetAsync(cl, 1, (size_t)n, c->stream));
      const int64_t chunks = (d->d.seq_bytes + 15) / 16;
      if (chunks > 0)
        hipLaunchKernelGGL(pool_clean, dim3((unsigned)((chunks + 2 * kBlock - 1) / (2 * kBlock))), dim3(kBlock), 0,
                           c->stream, d->d, (uint8_t *)cl, (uint32_t *)nnb);
    } else {
      hipLaunchKernelGGL(read_clean, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream, d->d,
                         (uint8_t *)cl, (uint32_t *)nnb);
    }
    HIP_TRY(hipGetLastError());
  }
  d->d.clean = (const uint8_t *)cl;
  d->nnb = nnb;  // N bases per read: the projection's sparse entries (ensure_projection)
  // column-kernel records; 1 KiB zeroed tails keep the per-tile LDS-DMA pieces in bounds.  The
  // auxiliary list is sized by its bound (MD events + 6 words per CIGAR op: at most three
  // segments of two words per op, when no two reads share pool words), so no count comes back to
  // the host first; col_derive refuses a read whose list would end past it.
  void *cdp = nullptr, *ce = nullptr, *ao = nullptr, *na = nullptr;
  const size_t ncd = sizeof(ColDesc) * (size_t)std::max<int64_t>(n, 1) + 1024;
  HIP_TRY(d->dp.get(&cdp, ncd));
  HIP_TRY(hipMemsetAsync(cdp, 0, ncd, c->stream));
  HIP_TRY(d->dp.get(&ao, sizeof(int64_t) * (size_t)(n + 1)));
  HIP_TRY(d->dp.get((void **)&na, sizeof(uint32_t) * (size_t)(n + 1)));
  const unsigned nb = (unsigned)((n + 1 + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(col_count, dim3(nb), dim3(kBlock), 0, c->stream, d->d, (uint32_t *)na);
  HIP_TRY(hipGetLastError());
  HIP_TRY(scan_u32_to_i64(d->dp, (const uint32_t *)na, (int64_t *)ao, n + 1, c->stream));
  d->dp.put(na);
  const int64_t aux_bound = std::max<int64_t>(d->d.md_len, 0) + 6 * std::max<int64_t>(d->d.cigar_len, 0);
  const size_t nce = sizeof(uint32_t) * (size_t)std::max<int64_t>(aux_bound, 1) + 1024;
  HIP_TRY(d->dp.get(&ce, nce));
  d->d.cdesc = (const ColDesc *)cdp;
  d->d.cev = (const uint32_t *)ce;
  d->d.caux_off = (const int64_t *)ao;
  if (n > 0) {
    hipLaunchKernelGGL(col_derive, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream, d->d,
                       (const int64_t *)ao, (ColDesc *)cdp, (uint32_t *)ce, aux_bound);
    HIP_TRY(hipGetLastError());
  }
  d->columns = true;
  return GQ_OK;
}

// The projection of a resident read set (ProjRec in gq_kernels.h), derived on first use by a
// kernel that reads it (germline_proj, somatic_proj over the tumor, mproj_fill): records, pbad
// slices, each slice's read window and its pieces' rows (one greedy pass, stored), the rows'
// offsets, the 4-bit code pool, the sparse entries.  A set no such kernel reads (the somatic
// normal) never pays for it.
gq_status gq::ensure_projection(gq_ctx *c, const gq_dev_reads *cd, const MarginReq *mr) {
  gq_dev_reads *d = const_cast<gq_dev_reads *>(cd);
  if (d->projected) return GQ_OK;
  const auto t0 = std::chrono::steady_clock::now();
  const int64_t n = d->d.n_reads;
  const int64_t n_sl = d->n_slices;
  void *pr = nullptr, *sc = nullptr, *sb = nullptr, *br = nullptr, *tmp = nullptr, *pj = nullptr, *ne = nullptr,
       *eo = nullptr, *pe = nullptr, *pbd = nullptr, *sra = nullptr, *scn = nullptr, *so = nullptr, *pw = nullptr;
  HIP_TRY(hipEventRecord(d->tev[2], c->stream));
  {
    const gq_status sc0 = ensure_columns(c, d);
    if (sc0) return sc0;
  }
  HIP_TRY(d->dp.get(&pr, sizeof(ProjRec) * (size_t)(n + 1)));
  const unsigned nb1 = (unsigned)((n + 1 + kBlock - 1) / kBlock);
  // the records, the slices a read the projection cannot take touches (pbad), the sparse entries
  // per read and the reads taken, in one pass
  HIP_TRY(d->dp.get(&pbd, (size_t)n_sl + 16));
  HIP_TRY(hipMemsetAsync(pbd, 0, (size_t)n_sl + 16, c->stream));
  HIP_TRY(d->dp.get((void **)&ne, sizeof(uint32_t) * (size_t)(n + 1)));
  unsigned long long *nok = nullptr;
  HIP_TRY(d->dp.get((void **)&nok, sizeof(unsigned long long) * kOkSpread));
  HIP_TRY(hipMemsetAsync(nok, 0, sizeof(unsigned long long) * kOkSpread, c->stream));
  hipLaunchKernelGGL(proj_prep, dim3(nb1), dim3(kBlock), 0, c->stream, d->d, (const uint32_t *)d->nnb, (ProjRec *)pr,
                     (uint8_t *)pbd, (uint32_t *)ne, nok);
  HIP_TRY(hipGetLastError());
  d->d.prec = (const ProjRec *)pr;
  // each slice's read window and the offsets of its reads' rows
  HIP_TRY(d->dp.get(&sra, sizeof(int64_t) * (size_t)(n_sl + 1)));
  HIP_TRY(d->dp.get((void **)&scn, sizeof(int64_t) * (size_t)(n_sl + 1)));
  HIP_TRY(d->dp.get(&so, sizeof(int64_t) * (size_t)(n_sl + 1)));
  hipLaunchKernelGGL(slice_windows, dim3((unsigned)((n_sl + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                     d->d, n_sl, (int64_t *)sra, (int64_t *)scn);
  HIP_TRY(hipGetLastError());
  {
    size_t tb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (const int64_t *)scn, (int64_t *)so, (int)(n_sl + 1), c->stream));
    HIP_TRY(d->dp.get((void **)&tmp, std::max<size_t>(tb, 16)));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, (const int64_t *)scn, (int64_t *)so, (int)(n_sl + 1), c->stream));
    int64_t tot = 0;
    HIP_TRY(hipMemcpyAsync(&tot, (int64_t *)so + n_sl, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    d->dp.put(tmp);
    d->dp.put(scn);
    HIP_TRY(d->dp.get(&pw, sizeof(uint16_t) * (size_t)std::max<int64_t>(tot, 1)));
  }
  d->d.sra = (const int64_t *)sra;
  d->d.soff = (const int64_t *)so;
  d->d.prow = (const uint16_t *)pw;
  HIP_TRY(d->dp.get((void **)&sc, sizeof(int32_t) * (size_t)std::max<int64_t>(n_sl, 1)));
  HIP_TRY(d->dp.get((void **)&br, sizeof(int64_t) * (size_t)(n_sl + 1)));
  HIP_TRY(d->dp.get(&sb, sizeof(int64_t) * (size_t)(n_sl + 1)));
  if (n_sl > 0) {
    const int64_t blocks = std::min<int64_t>((n_sl + 3) / 4, 1 << 20);
    static const int first_fit = getenv("GQ_ROWS") && strcmp(getenv("GQ_ROWS"), "firstfit") == 0;  // A/B
    hipLaunchKernelGGL(row_count, dim3((unsigned)blocks), dim3(256), 0, c->stream, d->d, n_sl, (uint16_t *)pw,
                       (int32_t *)sc, (uint8_t *)pbd, first_fit);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(rows64, dim3((unsigned)((n_sl + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream, n_sl,
                     (const int32_t *)sc, (int64_t *)br);
  HIP_TRY(hipGetLastError());
  HIP_TRY(d->dp.get(&eo, sizeof(int64_t) * (size_t)(n + 1)));
  size_t tb = 0;
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (const int64_t *)br, (int64_t *)sb, (int)(n_sl + 1), c->stream));
  HIP_TRY(d->dp.get((void **)&tmp, std::max<size_t>(tb, 16)));
  HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb, (const int64_t *)br, (int64_t *)sb, (int)(n_sl + 1), c->stream));
  HIP_TRY(scan_u32_to_i64(d->dp, (const uint32_t *)ne, (int64_t *)eo, n + 1, c->stream));
  int64_t tot[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(&tot[0], (int64_t *)sb + n_sl, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(&tot[1], (int64_t *)eo + n, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  d->dp.put(tmp);
  d->dp.put(sc);
  d->dp.put(br);
  d->dp.put(ne);
  d->d.srow = (const int64_t *)sb;
  d->d.pbad = (const uint8_t *)pbd;
  d->n_rows = tot[0];
  // the pool: rows of 16 words, zero where no piece lies
  const size_t pool_bytes = (size_t)kProjRowBytes * (size_t)tot[0] + 16;
  HIP_TRY(d->dp.get(&pj, pool_bytes));
  const bool cells = fill_pieces();  // the default: every word written, no preset of the pool
  if (cells) HIP_TRY(hipMemsetAsync((uint8_t *)pj + pool_bytes - 16, 0, 16, c->stream));
  else HIP_TRY(hipMemsetAsync(pj, 0, pool_bytes, c->stream));
  HIP_TRY(d->dp.get(&pe, sizeof(uint2) * (size_t)(tot[1] + 1)));
  d->d.proj = (const uint8_t *)pj;
  d->d.pev = (const uint2 *)pe;
  d->d.pev_off = (const int64_t *)eo;
  // the sparse entries on the side stream, beside the pool fill (they read neither the pool nor rows)
  HIP_TRY(hipEventRecord(c->side_ev[2], c->stream));
  HIP_TRY(hipStreamWaitEvent(c->side, c->side_ev[2], 0));
  if (n > 0) {
    hipLaunchKernelGGL(pev_fill, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->side, d->d,
                       (const int64_t *)eo, (uint2 *)pe);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(c->side_ev[3], c->side));
  HIP_TRY(hipEventRecord(d->tev[3], c->stream));
  if (n_sl > 0) {
    static const int fill_u = getenv("GQ_FILL_U") ? atoi(getenv("GQ_FILL_U")) : 0;
    if (cells && fill_mode() == 2) {  // A/B: GQ_FILL=cellsb (a workgroup per slice)
      unsigned long long *nd = nullptr;
      int64_t *dl = nullptr;
      HIP_TRY(d->dp.get((void **)&nd, sizeof(unsigned long long)));
      HIP_TRY(d->dp.get((void **)&dl, sizeof(int64_t) * (size_t)n_sl));
      HIP_TRY(hipMemsetAsync(nd, 0, sizeof(unsigned long long), c->stream));
      const int64_t blocks = std::min<int64_t>(n_sl, 1 << 20);
      hipLaunchKernelGGL(proj_fill_cellsb, dim3((unsigned)blocks), dim3(256), 0, c->stream, d->d, n_sl, (uint8_t *)pj,
                         dl, nd, fill_dbg());
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(proj_fill_deep, dim3((unsigned)std::min<int64_t>(blocks, 2048)), dim3(256), 0, c->stream, d->d,
                         (const int64_t *)dl, (const unsigned long long *)nd, (uint8_t *)pj);
      HIP_TRY(hipGetLastError());
      d->dp.put(nd);
      d->dp.put(dl);
    } else if (cells && fill_mode() == 1) {  // A/B: GQ_FILL=pieces
      const int64_t blocks = std::min<int64_t>((n_sl + 3) / 4, 1 << 20);
      hipLaunchKernelGGL(proj_fill_pieces, dim3((unsigned)blocks), dim3(256), 0, c->stream, d->d, n_sl, (uint8_t *)pj,
                         fill_dbg());
      HIP_TRY(hipGetLastError());
    } else if (cells) {
      unsigned long long *nd = nullptr;
      int64_t *dl = nullptr;
      HIP_TRY(d->dp.get((void **)&nd, sizeof(unsigned long long)));
      HIP_TRY(d->dp.get((void **)&dl, sizeof(int64_t) * (size_t)n_sl));
      HIP_TRY(hipMemsetAsync(nd, 0, sizeof(unsigned long long), c->stream));
      const int64_t blocks = std::min<int64_t>((n_sl + 3) / 4, 1 << 20);
      hipLaunchKernelGGL(fill_u == 8 ? proj_fill_cells<8> : proj_fill_cells<4>, dim3((unsigned)blocks), dim3(256), 0,
                         c->stream, d->d, n_sl, (uint8_t *)pj, dl, nd, fill_dbg());
      HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(proj_fill_deep, dim3((unsigned)std::min<int64_t>(blocks, 2048)), dim3(256), 0, c->stream, d->d,
                         (const int64_t *)dl, (const unsigned long long *)nd, (uint8_t *)pj);
      HIP_TRY(hipGetLastError());
      d->dp.put(nd);
      d->dp.put(dl);
    } else if (fill_slice_major()) {  // A/B: the slice-major fill of round 4 (GQ_FILL=slice)
      const int64_t blocks = std::min<int64_t>((n_sl + 3) / 4, 1 << 20);
      auto kf = fill_u == 4 ? proj_fill<4> : fill_u == 2 ? proj_fill<2> : proj_fill<1>;
      hipLaunchKernelGGL(kf, dim3((unsigned)blocks), dim3(256), 0, c->stream, d->d, n_sl, (uint8_t *)pj);
    } else if (n > 0 && mr && getenv("GQ_FILL_ONE")) {  // A/B: with the margin projection in one pass (measured slower)
      const gq_status st = fused_projection_fill(c, d, (uint8_t *)pj, *mr);
      if (st) return st;
    } else if (n > 0) {
      const int64_t blocks = (std::min<int64_t>((n + 255) / 256, 1 << 20) + 7) & ~(int64_t)7;  // a wave per 64 reads
      static const int fill_w = getenv("GQ_FILL_W") ? atoi(getenv("GQ_FILL_W")) : 1;  // words per lane unit
      auto kf = fill_u == 2 ? proj_fill_rw<2, 1>
                : fill_u == 4 ? proj_fill_rw<4, 1>
                : fill_w == 2 ? proj_fill_rw<1, 2>
                : fill_w == 4 ? proj_fill_rw<1, 4>
                              : proj_fill_rw<1, 1>;
      hipLaunchKernelGGL(kf, dim3((unsigned)blocks), dim3(256), 0, c->stream, d->d, (uint8_t *)pj, fill_dbg());
    }
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(d->tev[4], c->stream));
  HIP_TRY(hipStreamWaitEvent(c->stream, c->side_ev[3], 0));  // (the sparse entries done)
  HIP_TRY(hipEventRecord(d->tev[5], c->stream));
  d->proj_bytes = kProjRowBytes * tot[0];
  d->pev_count = tot[1];
  // the reads the projection takes (proj_prep's counters) and the spans: read when asked for
  // (settle_stats), so the call behind the projection is queued without a host round trip
  d->nok = nok;
  d->pending |= 2;
  d->projected = true;
  d->proj_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return GQ_OK;
}

