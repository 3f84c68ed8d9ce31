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
#include <vector>

#include "../../include/gqpileup.h"
#include "gq_host.h"
#include "gq_alleles.h"

using namespace gq;

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
__global__ void plan_tiles(const int32_t *__restrict__ r_contig, const int64_t *__restrict__ r_start,
                           const int64_t *__restrict__ r_end, const int64_t *__restrict__ r_ord,
                           const int64_t *__restrict__ r_tile0, int64_t n_ranges, int64_t n_tiles, int T,
                           DevReads R, Tile *__restrict__ tiles) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  int64_t lo = 0, hi = n_ranges - 1;  // largest r with r_tile0[r] <= t
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if (r_tile0[mid] <= t) lo = mid;
    else hi = mid - 1;
  }
  const int64_t r = lo;
  const int64_t L0 = r_start[r] + (t - r_tile0[r]) * (int64_t)T;
  const int64_t L1 = min(L0 + (int64_t)T, r_end[r]);
  const int32_t c = r_contig[r];
  int64_t b = R.contig_read_begin[c], e = R.contig_read_begin[c + 1];
  // rb: first read with pmax_end > L0 (pmax_end non-decreasing within the contig)
  int64_t a0 = b, a1 = e;
  while (a0 < a1) {
    int64_t m = (a0 + a1) >> 1;
    if ((int64_t)R.pmax_end[m] > L0) a1 = m;
    else a0 = m + 1;
  }
  const int64_t rb = a0;
  a0 = rb;
  a1 = e;  // re: first read with start >= L1
  while (a0 < a1) {
    int64_t m = (a0 + a1) >> 1;
    if ((int64_t)R.start[m] >= L1) a1 = m;
    else a0 = m + 1;
  }
  Tile tl;
  tl.ordinal0 = r_ord[r] + (L0 - r_start[r]);
  tl.rb = rb;
  tl.re = a0;
  tl.contig = c;
  tl.L0 = (int32_t)L0;
  tl.L1 = (int32_t)L1;
  tl.range = (int32_t)r;
  tiles[t] = tl;
}

// CIGAR shape per read (derived once at upload): leading soft clip if the CIGAR is
// [S|H]* (M|=|X) [S|H]* and the sequence covers it, else -1 (general walker).
__global__ void read_shape(DevReads R, int16_t *__restrict__ lead, uint8_t *__restrict__ ev_rb,
                           uint8_t *__restrict__ clean) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R.n_reads) return;
  {  // every sequenced byte one of A C G T N (the germline fast path's precondition)
    const uint8_t *q = R.seq + R.seq_off[r];
    bool ok = true;
    for (int32_t k = 0; k < R.seq_len[r]; ++k) {
      const uint8_t b = q[k];
      ok = ok && (b == 'A' || b == 'C' || b == 'G' || b == 'T' || b == 'N');
    }
    clean[r] = ok ? 1 : 0;
  }
  const int64_t off = R.cigar_off[r];
  const int32_t n = R.n_cigar[r];
  int32_t ld = 0, mlen = 0;
  int mi = -1;
  bool simple = n > 0;
  for (int k = 0; k < n && simple; ++k) {
    const uint32_t c = R.cigar[off + k];
    const int op = (int)(c & 15u);
    if (op == OP_M || op == OP_EQ || op == OP_X) {
      if (mi >= 0) simple = false;
      mi = k;
      mlen = (int32_t)(c >> 4);
    } else if (op == OP_S) {
      if (mi < 0) ld += (int32_t)(c >> 4);
    } else if (op != OP_H) {
      simple = false;
    }
  }
  if (mi < 0 || ld > 32767 || ld + mlen > R.seq_len[r]) simple = false;
  lead[r] = simple ? (int16_t)ld : (int16_t)-1;
  // sequenced base under each MD event (0 where the event sits on a deletion / outside M)
  const int32_t nmd = R.n_md[r];
  if (nmd <= 0) return;
  const uint32_t *ev = R.md_ev + R.md_off[r];
  uint8_t *rb = ev_rb + R.md_off[r];
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

__device__ __forceinline__ uint64_t pack_inline(uint8_t r0, const uint8_t *alt, int alt_len) {
  uint64_t v = r0;
  for (int i = 0; i < alt_len; ++i) v |= (uint64_t)alt[i] << (8 * (1 + i));
  return v;
}

// ------------------------------------------------------------------------------------------
// germline_tile: LDS histogram + on-device decision for simple loci
// ------------------------------------------------------------------------------------------
#define PUSH_OUT(rec)             \
  do {                            \
    if (nout == 0) out0 = (rec);  \
    else out1 = (rec);            \
    ++nout;                       \
  } while (0)

#include "gq_germline_v2.h"

// ABL (diagnostic builds only, selected by env GQ_ABLATE; results are wrong when != 0):
//   1 = skip the read walk, 2 = skip the decision phase, 4 = base pass without LDS atomics,
//   8 = skip the MD-event pass.
template <int T, int ABL = 0, int STAGE = 0, int CH = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(STAGE ? 4 : T <= 768 ? 8 : T <= 1024 ? (CH ? 5 : 6) : 3))) void germline_tile(const Tile *__restrict__ tiles, DevReads R, int threshold,
                                                        int emit_ref, int emit_no_call, CallRec *__restrict__ recs,
                                                        unsigned long long rec_cap, ComplexItem *__restrict__ cplx,
                                                        unsigned long long cplx_cap, Counters *ctr) {
  constexpr int S = T + 2 * kGuard;
  __shared__ __attribute__((aligned(16))) uint32_t cnt[W_N * S];
  __shared__ __attribute__((aligned(16))) uint4 stage[STAGE ? STAGE / 16 : 1];
  constexpr int NR = (CH && !STAGE) ? kBlock : 1;  // chunk-major walk: one table row per read of a batch
  __shared__ int32_t ch_lo[NR], ch_hi[NR], ch_base[NR];
  __shared__ uint8_t ch_info[NR];
  __shared__ int ch_flag;
  const uint64_t pt0 = (ABL & 32) ? __builtin_readcyclecounter() : 0;
  uint64_t pt1 = 0, pt2 = 0, pt3 = 0;
  const Tile tl = tiles[blockIdx.x];
  const int32_t L0 = tl.L0, L1 = tl.L1;
  // a window of >= 65535 reads could overflow the 16-bit counters: queue every locus of
  // the tile for the exact (32-bit) kernel instead
  const bool wide = (tl.re - tl.rb) >= 65535;
  if (!wide) {
    GermSink<T, (ABL & 31)> sink{cnt, L0, &ctr->err, &ctr->err_pos};
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
    // Reads are walked in batches of up to blockDim.x (one per lane).  A batch's reads
    // sit in one contiguous byte range of the sequence pool (reads are stored in
    // alignment order), which is copied into LDS by LDS-DMA (global_load_lds_dwordx4,
    // 1 KiB per wave-instruction, fully coalesced) while the counters are zeroed; the
    // lanes then read their bases from LDS instead of issuing scattered 16-byte loads.
    for (int64_t r0 = tl.rb; r0 < tl.re || r0 == tl.rb; r0 += blockDim.x) {
      const int64_t nb = min((int64_t)blockDim.x, tl.re - r0);
      int64_t B0 = 0, n1k = 0;
      if (STAGE && nb > 0) {
        B0 = R.seq_off[r0] & ~(int64_t)15;
        const int64_t B1 = R.seq_off[r0 + nb - 1] + R.seq_len[r0 + nb - 1];
        n1k = B1 > B0 ? (B1 - B0 + 1023) >> 10 : 0;
        if (n1k * 1024 > STAGE || B0 + n1k * 1024 > R.seq_cap) n1k = 0;  // not staged: HBM loads
      }
      if (!(ABL & 1))
        for (int64_t q = wave; q < n1k; q += nwaves)
          __builtin_amdgcn_global_load_lds((const void *)(R.seq + B0 + q * 1024 + lane * 16),
                                           (__attribute__((address_space(3))) void *)(stage + q * 64), 16, 0, 0);
      if (r0 == tl.rb) {
        uint4 *c4 = reinterpret_cast<uint4 *>(cnt);
        for (int i = threadIdx.x; i < W_N * S / 4; i += blockDim.x) c4[i] = make_uint4(0u, 0u, 0u, 0u);
      }
      if (STAGE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const StageView sv{stage, B0, B0 + n1k * 1024};
      if ((ABL & 32) && r0 == tl.rb) pt1 = __builtin_readcyclecounter();
      if (CH && !STAGE && nb > 0 && !(ABL & 1)) {
        if (!walk_batch_chunked(R, r0, (int)nb, L0, L1, sink, ChunkRows{ch_lo, ch_hi, ch_base, ch_info}, &ch_flag) &&
            (int64_t)threadIdx.x < nb)
          walk_read_lane(R, r0 + threadIdx.x, L0, L1, sink);  // reads not in pool order: lane per read
      } else if (!(ABL & 1) && (int64_t)threadIdx.x < nb) {
        walk_read_lane(R, r0 + threadIdx.x, L0, L1, sink, sv);
      }
      if (ABL & 32) pt2 = __builtin_readcyclecounter();
      __syncthreads();  // counters complete / stage free for the next batch
      if (nb <= 0) break;
    }
  }
  __syncthreads();
  if (ABL & 32) pt3 = __builtin_readcyclecounter();
  if (ABL & 2) {
    if (threadIdx.x == 0) atomicAdd(&ctr->visited, (unsigned long long)cnt[kGuard + (blockIdx.x & 63)]);
    return;
  }

  const bool multi_sample = R.n_samples > 1;
  unsigned visited = 0, amb = 0, ties = 0;
  const int nloci = L1 - L0;
  // uniform trip count so every wave reaches the wave-level reservations together
  for (int i0 = 0; i0 < nloci; i0 += blockDim.x) {
    const int i = i0 + threadIdx.x;
    CallRec out0, out1;  // named (not an array): no scratch
    unsigned nout = 0;
    bool to_complex = false;
    if (wide && i < nloci) {
      to_complex = true;
    } else if (i < nloci) {
      const uint32_t wac = cnt[W_AC * S + kGuard + i], wtg = cnt[W_TG * S + kGuard + i],
                     wox = cnt[W_OX * S + kGuard + i], wnn = cnt[W_NN * S + kGuard + i];
      const uint32_t c[5] = {wac & 0xFFFFu, wac >> 16, wtg & 0xFFFFu, wtg >> 16, wnn >> 16};  // A C T G N
      const uint32_t cx = (wox & 0xFFFFu) + (wox >> 16);  // other bases + complex elements
      const uint32_t depth = c[0] + c[1] + c[2] + c[3] + c[4] + cx;
      if (depth > 0) {
        ++visited;
        uint32_t mask = cnt[W_MASK * S + kGuard + i] & 0xFu;
        const uint32_t eac = cnt[W_EAC * S + kGuard + i], etg = cnt[W_ETG * S + kGuard + i];
        const uint32_t ev[4] = {eac & 0xFFFFu, eac >> 16, etg & 0xFFFFu, etg >> 16};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (c[k] > ev[k]) mask |= 1u << k;
        const bool ambiguous = __popc(mask) > 1;
        if (ambiguous) ++amb;
        if (ambiguous || cx > 0 || multi_sample) {
          to_complex = true;
        } else {
          // GermlineThresholdCaller.scala:100-177 for a pileup of single-base alleles.
          const uint8_t ref = mask ? bit_base(mask) : (uint8_t)'N';
          const int rc = mask ? (__ffs((int)mask) - 1) : 4;  // select chain: no dynamic register indexing
          const uint32_t c_ref = rc == 0 ? c[0] : rc == 1 ? c[1] : rc == 2 ? c[2] : rc == 3 ? c[3] : c[4];
          if ((long long)(depth - c_ref) * 100 / (long long)depth <= threshold) {
            // fast path: every non-reference allele has count <= depth - c_ref, so none
            // passes the threshold; the call is HomRef if the reference allele passes,
            // else NoCall (same outcome as the general case split below)
            const int32_t pos = L0 + i;
            const bool ref_pass = c_ref > 0 && (long long)c_ref * 100 / (long long)depth > threshold;
            if (ref_pass ? emit_ref : emit_no_call) {
              CallRec rr;
              rr.key = (uint64_t)(tl.ordinal0 + i) << 12;
              rr.contig = tl.contig;
              rr.pos = pos;
              rr.sample = 0;
              rr.gt0 = rr.gt1 = ref_pass ? GQ_GT_REF : GQ_GT_NOCALL;
              rr.flags = 0;
              rr.ref_len = 1;
              rr.alt_len = 5;
              rr.allele = (uint64_t)ref | ((uint64_t)'<' << 8) | ((uint64_t)'A' << 16) | ((uint64_t)'L' << 24) |
                          ((uint64_t)'T' << 32) | ((uint64_t)'>' << 40);
              PUSH_OUT(rr);
            }
          } else {
          // Allele (ref, b) keys: count << 8 | (255 - canonical rank); canonical order of
          // Allele(ref, alt) for one ref is the alt byte order A < C < G < N < T, i.e. the
          // categories 0, 1, 3, 4, 2.  Sorting keys descending = sortBy(-count), ties canonical.
          uint32_t k0 = 0, k1 = 0, k2 = 0;  // top three passing keys
          int npass = 0;
#pragma unroll
          for (int rank = 0; rank < 5; ++rank) {
            const int cat = (0x24310 >> (4 * rank)) & 0xF;
            const uint32_t cc = c[cat];
            if (cc == 0 || (long long)cc * 100 / (long long)depth <= threshold) continue;
            ++npass;
            uint32_t key = (cc << 8) | (uint32_t)(255 - rank);
            // insert into (k0 >= k1 >= k2)
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
          const int32_t pos = L0 + i;
          const uint64_t ord = (uint64_t)(tl.ordinal0 + i);
          auto mk = [&](uint8_t g0, uint8_t g1, uint8_t alt1, bool alt_sym, int sub) {
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
          const uint8_t b0 = key_base(k0), b1 = key_base(k1);
          if (npass == 0) {
            if (emit_no_call) PUSH_OUT(mk(GQ_GT_NOCALL, GQ_GT_NOCALL, 0, true, 0));
          } else if (npass == 1 && b0 == ref) {
            if (emit_ref) PUSH_OUT(mk(GQ_GT_REF, GQ_GT_REF, 0, true, 0));
          } else if (npass == 1) {
            PUSH_OUT(mk(GQ_GT_ALT, GQ_GT_ALT, b0, false, 0));
          } else {
            const bool v1 = b0 != ref, v2 = b1 != ref;
            if (v1 != v2) {
              PUSH_OUT(mk(GQ_GT_REF, GQ_GT_ALT, v1 ? b0 : b1, false, 0));
            } else if (v1 && v2) {
              PUSH_OUT(mk(GQ_GT_ALT, GQ_GT_OTHERALT, b0, false, 0));
              PUSH_OUT(mk(GQ_GT_ALT, GQ_GT_OTHERALT, b1, false, 1));
            }
            // two non-variant single-base alleles cannot occur (all Match alleles share ref)
          }
          }
        }
      }
    }
    // reserve + write records (wave-aggregated)
    const unsigned long long base = wave_reserve(&ctr->n_rec, nout);
    if (nout > 0 && base < rec_cap) recs[base] = out0;
    if (nout > 1 && base + 1 < rec_cap) recs[base + 1] = out1;
    const unsigned long long cb = wave_reserve(&ctr->n_complex, to_complex ? 1u : 0u);
    if (to_complex && cb < cplx_cap) cplx[cb] = ComplexItem{(int32_t)blockIdx.x, L0 + i, wide ? 1 : 0};
  }
  // block-level reduction of run counters
  __shared__ unsigned red[3];
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
  if ((ABL & 32) && (threadIdx.x & 63) == 0) {  // per-wave phase clocks
    const uint64_t pt4 = __builtin_readcyclecounter();
    atomicAdd(&ctr->prof[0], (unsigned long long)(pt1 - pt0));  // tile load + LDS zero + barrier
    atomicAdd(&ctr->prof[1], (unsigned long long)(pt2 - pt1));  // this wave's read walk
    atomicAdd(&ctr->prof[2], (unsigned long long)(pt3 - pt2));  // waiting for the other waves
    atomicAdd(&ctr->prof[3], (unsigned long long)(pt4 - pt3));  // decision + output
    atomicAdd(&ctr->prof[4], 1ull);
  }
}

// ------------------------------------------------------------------------------------------
// germline_complex: exact per-element classification for queued loci (one wave per locus)
// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void germline_complex(const Tile *__restrict__ tiles,
                                                           const ComplexItem *__restrict__ items, DevReads R,
                                                           int threshold, int emit_ref, int emit_no_call,
                                                           CallRec *__restrict__ recs, unsigned long long rec_cap,
                                                           uint8_t *__restrict__ pool, unsigned long long pool_cap,
                                                           unsigned long long cplx_cap, Counters *ctr) {
  const int lane = threadIdx.x & 63;
  const int64_t gwave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves_total = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // items beyond the queue's capacity were never written (the host retries with a larger queue)
  const unsigned long long n_items = ctr->n_complex < cplx_cap ? ctr->n_complex : cplx_cap;
  for (int64_t it = gwave; it < (int64_t)n_items; it += nwaves_total) {
    const ComplexItem item = items[it];
    const Tile tl = tiles[item.tile];
    const int32_t pos = item.pos;
    // ---- pass 1: pileup reference base (Pileup.referenceBaseAtLocus)
    uint32_t mask = 0;
    uint64_t best = ~0ull;  // (end, read) of the heap-root proxy among standard-base reads
    for (int64_t r0 = tl.rb; r0 < tl.re; r0 += 64) {
      const int64_t r = r0 + lane;
      if (r < tl.re && R.start[r] <= pos && pos < R.end[r]) {
        const int v = md_ref_at(R, r, pos);
        if (v < 0) {
          raise_error(&ctr->err, (int64_t *)&ctr->err_pos, v == -4 ? GQ_E_NO_MD : v == -3 ? GQ_E_MD : GQ_E_ASSERT,
                      pos);
        } else if (std_bit((uint8_t)v)) {
          mask |= std_bit((uint8_t)v);
          const uint64_t key = ((uint64_t)(uint32_t)R.end[r] << 32) | (uint64_t)(r - tl.rb);
          best = key < best ? key : best;
        }
      }
    }
    for (int d = 1; d < 64; d <<= 1) {
      mask |= __shfl_xor(mask, d, 64);
      const uint64_t o = __shfl_xor(best, d, 64);
      best = o < best ? o : best;
    }
    const bool ambiguous = __popc(mask) > 1;
    uint8_t refbase = 'N';
    if (ambiguous) {
      const int64_t rr = tl.rb + (int64_t)(best & 0xFFFFFFFFull);
      const int v = md_ref_at(R, rr, pos);
      refbase = (uint8_t)v;
    } else if (mask) {
      refbase = bit_base(mask);
    }
    // ---- pass 2: classify elements, group alleles per (sample, allele) in registers
    uint64_t tlo[kSlots], thi[kSlots];
    uint32_t tcnt[kSlots];
    AlleleDesc tdesc[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      tlo[s] = thi[s] = 0;
      tcnt[s] = 0;
    }
    int nt = 0;  // used slots (uniform)
    bool overflow = false;
    uint32_t sample_total[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t r0 = tl.rb; r0 < tl.re; r0 += 64) {
      const int64_t r = r0 + lane;
      bool act = r < tl.re && R.start[r] <= pos && pos < R.end[r];
      AlleleDesc d;
      Key128 key{0, 0};
      int smp = 0;
      if (act) {
        int errc = 0;
        if (!classify(R, r, pos, refbase, d, &errc)) {
          raise_error(&ctr->err, (int64_t *)&ctr->err_pos, errc, pos);
          act = false;
        } else {
          smp = R.sample[r] & 7;
          key = allele_key(R, d, pos, smp);
        }
      }
      // per-sample totals
      for (int sm = 0; sm < 8; ++sm) {
        const unsigned long long b = __ballot(act && smp == sm);
        sample_total[sm] += (uint32_t)__popcll(b);
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
        for (int s = 0; s < kSlots; ++s) {
          const bool hit = (s * 64 + lane) < nt && tlo[s] == klo && thi[s] == khi;
          const unsigned long long hb = __ballot(hit);
          if (found < 0 && hb) found = s * 64 + (__ffsll((long long)hb) - 1);
        }
        if (found < 0) {
          if (nt >= 64 * kSlots) {
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
            for (int s = 0; s < kSlots; ++s)
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
#pragma unroll
          for (int s = 0; s < kSlots; ++s)
            if (s == sl && lane == owner) tcnt[s] += n;
        }
        pending &= ~mb;
      }
    }
    if (overflow) {
      raise_error(&ctr->err, (int64_t *)&ctr->err_pos, GQ_E_CAPACITY, pos);
      continue;
    }
    if (item.flags & 1) {  // queued from a wide tile: count the visit here
      uint32_t tot = 0;
      for (int sm = 0; sm < 8; ++sm) tot += sample_total[sm];
      if (tot == 0) continue;
      if (lane == 0) {
        atomicAdd(&ctr->visited, 1ull);
        if (ambiguous) atomicAdd(&ctr->ambiguous, 1ull);
      }
    }
    // ---- pass 3: GermlineThreshold decision per sample (uniform serial code)
    const uint64_t ord = (uint64_t)(tl.ordinal0 + (pos - tl.L0));
    for (int sm = 0; sm < 8; ++sm) {
      const uint32_t total = sample_total[sm];
      if (total == 0) continue;
      // select top-3 passing entries by (count desc, allele asc)
      int top[3] = {-1, -1, -1};
      uint32_t topc[3] = {0, 0, 0};
      AlleleDesc topd[3];
      int npass = 0;
      for (int j = 0; j < nt; ++j) {
        const int owner = j & 63, sl = j >> 6;
        uint32_t cj = 0;
        AlleleDesc dj;
#pragma unroll
        for (int s = 0; s < kSlots; ++s)
          if (s == sl) {
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
        ++npass;
        int p = npass - 1 < 3 ? npass - 1 : 3;
        while (p > 0 && (topc[p - 1] < cj || (topc[p - 1] == cj && allele_cmp(R, dj, topd[p - 1], pos) < 0))) {
          if (p < 3) {
            top[p] = top[p - 1];
            topc[p] = topc[p - 1];
            topd[p] = topd[p - 1];
          }
          --p;
        }
        if (p < 3) {
          top[p] = j;
          topc[p] = cj;
          topd[p] = dj;
        }
      }
      const bool tie = npass >= 2 && (topc[0] == topc[1] || (npass >= 3 && topc[1] == topc[2]));
      const uint8_t fl = (tie ? GQ_FLAG_TIE : 0) | (ambiguous ? GQ_FLAG_AMBIGUOUS_REF : 0);
      if (lane == 0 && tie) atomicAdd(&ctr->ties, 1ull);
      // emit helper: alleles from descriptors, or symbolic "<ALT>" with an explicit ref
      auto emit = [&](const AlleleDesc *a, uint8_t sym_ref_kind, const AlleleDesc *ref_src, uint8_t g0, uint8_t g1,
                      int sub) {
        // sym_ref_kind: 0 => allele `a`; 1 => (refbase, <ALT>); 2 => (ref of ref_src, <ALT>)
        int rl, al;
        if (sym_ref_kind == 0) {
          rl = allele_ref_len(*a);
          al = allele_alt_len(*a);
        } else if (sym_ref_kind == 1) {
          rl = 1;
          al = 5;
        } else {
          rl = allele_ref_len(*ref_src);
          al = 5;
        }
        auto byte_at = [&](int which, int i) -> uint8_t {
          if (sym_ref_kind == 0) return allele_byte(R, *a, pos, which, i);
          if (which == 1) return (uint8_t)"<ALT>"[i];
          if (sym_ref_kind == 1) return refbase;
          return allele_byte(R, *ref_src, pos, 0, i);
        };
        CallRec rr;
        rr.key = (ord << 12) | ((uint64_t)sm << 4) | (uint64_t)sub;
        rr.contig = tl.contig;
        rr.pos = pos;
        rr.sample = (uint8_t)sm;
        rr.gt0 = g0;
        rr.gt1 = g1;
        rr.flags = fl;
        rr.ref_len = (uint16_t)rl;
        rr.alt_len = (uint16_t)al;
        if (rl + al <= 8) {
          uint64_t v = 0;
          int j = 0;
          for (int i = 0; i < rl; ++i) v |= (uint64_t)byte_at(0, i) << (8 * j++);
          for (int i = 0; i < al; ++i) v |= (uint64_t)byte_at(1, i) << (8 * j++);
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
          const unsigned long long k = atomicAdd(&ctr->n_rec, 1ull);
          if (k < rec_cap) recs[k] = rr;
        }
      };
      if (npass == 0) {
        if (emit_no_call) emit(nullptr, 1, nullptr, GQ_GT_NOCALL, GQ_GT_NOCALL, 0);
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
          if (emit_ref) emit(nullptr, 1, nullptr, GQ_GT_REF, GQ_GT_REF, 0);
        } else if (npass == 1) {
          emit(&topd[0], 0, nullptr, GQ_GT_ALT, GQ_GT_ALT, 0);
        } else {
          const bool v2 = isvar(topd[1]);
          const bool e1 = allele_alt_len(topd[0]) == 0, e2 = allele_alt_len(topd[1]) == 0;
          if ((!v1 || !v2) && (e1 != e2)) {
            // heterozygous deletion: no call (GermlineThresholdCaller.scala:146-149)
          } else if (v1 != v2) {
            emit(v1 ? &topd[0] : &topd[1], 0, nullptr, GQ_GT_REF, GQ_GT_ALT, 0);
          } else if (v1 && v2) {
            emit(&topd[0], 0, nullptr, GQ_GT_ALT, GQ_GT_OTHERALT, 0);
            emit(&topd[1], 0, nullptr, GQ_GT_ALT, GQ_GT_OTHERALT, 1);
          } else {
            const bool n1 = allele_ref_len(topd[0]) == 1 && allele_byte(R, topd[0], pos, 0, 0) == 'N';
            const bool n2 = allele_ref_len(topd[1]) == 1 && allele_byte(R, topd[1], pos, 0, 0) == 'N';
            if (n1 || n2) emit(nullptr, 2, n1 ? &topd[1] : &topd[0], GQ_GT_REF, GQ_GT_REF, 0);
            else raise_error(&ctr->err, (int64_t *)&ctr->err_pos, GQ_E_MULTI_REF, pos);
          }
        }
      }
    }
  }
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

// ------------------------------------------------------------------------------------------
// Result image: the gq_calls arrays built on device in output order (one D2H copy)
// ------------------------------------------------------------------------------------------
struct CallsLayout {  // byte offsets inside the image; header = int64 pool_len
  size_t contig, pos, ref_off, alt_off, ref_len, alt_len, sample, gt0, gt1, flags, pool, bytes;
};
static CallsLayout calls_layout(int64_t n, int64_t dev_pool_used) {
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

__global__ void iota_i32(int32_t *__restrict__ v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (int32_t)i;
}

__global__ void calls_lengths(const CallRec *__restrict__ recs, const int32_t *__restrict__ order, int64_t n,
                              int64_t *__restrict__ len) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const CallRec r = recs[order[k]];
  len[k] = (int64_t)r.ref_len + (int64_t)r.alt_len;
}

__global__ void calls_image(const CallRec *__restrict__ recs, const int32_t *__restrict__ order,
                            const int64_t *__restrict__ off, const uint8_t *__restrict__ dpool, int64_t n,
                            CallsLayout L, uint8_t *__restrict__ img) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const CallRec r = recs[order[k]];
  const int64_t o = off[k];
  const int tot = (int)r.ref_len + (int)r.alt_len;
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
    for (int i = 0; i < tot; ++i) dst[i] = (uint8_t)(r.allele >> (8 * i));
  } else {
    for (int i = 0; i < tot; ++i) dst[i] = dpool[r.allele + i];
  }
  if (k == n - 1) *reinterpret_cast<int64_t *>(img) = o + tot;  // pool_len
}

}  // namespace

// ==========================================================================================
// Host side: context, resident read sets, entry points
// ==========================================================================================
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
  for (auto &e : c->ev) HIP_TRY(hipEventCreate(&e));
  *out = c;
  return GQ_OK;
}

void gq_close(gq_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (DevBuf *b : {&c->ranges, &c->tiles, &c->recs, &c->recs_sorted, &c->keys, &c->keys_sorted, &c->idx,
                    &c->idx_sorted, &c->cplx, &c->pool, &c->counters, &c->sort_tmp, &c->image, &c->tiles2, &c->srecs, &c->c_depth, &c->c_pos,
                    &c->c_base, &c->c_indel, &c->c_ref, &c->c_rb, &c->c_amb})
    b->release();
  for (auto &e : c->ev) (void)hipEventDestroy(e);
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
  if (t != 512 && t != 768 && t != 1024 && t != 2048) return set_err(GQ_E_ARG, "tile must be 512, 768, 1024 or 2048");
  c->germ_tile = t;
  return GQ_OK;
}

static gq_status validate_reads(const gq_reads *h) {
  if (!h) return set_err(GQ_E_ARG, "null read set");
  if (h->n_reads < 0 || h->n_contigs <= 0) return set_err(GQ_E_ARG, "bad read-set sizes");
  if (h->n_samples < 1 || h->n_samples > 8) return set_err(GQ_E_ARG, "n_samples must be in [1, 8]");
  return GQ_OK;
}

static gq_status derive_shape(gq_ctx *c, gq_dev_reads *d, int64_t md_len) {
  void *p = nullptr, *q = nullptr, *cl = nullptr;
  HIP_TRY(hipMalloc(&p, sizeof(int16_t) * (size_t)std::max<int64_t>(d->d.n_reads, 1)));
  d->owned.push_back(p);
  HIP_TRY(hipMalloc(&cl, (size_t)std::max<int64_t>(d->d.n_reads, 1)));
  d->owned.push_back(cl);
  d->d.clean = (const uint8_t *)cl;
  HIP_TRY(hipMalloc(&q, (size_t)std::max<int64_t>(md_len, 16)));
  d->owned.push_back(q);
  d->d.lead = (const int16_t *)p;
  d->d.ev_rb = (const uint8_t *)q;
  if (d->d.n_reads > 0) {
    const unsigned nb = (unsigned)((d->d.n_reads + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(read_shape, dim3(nb), dim3(kBlock), 0, c->stream, d->d, (int16_t *)p, (uint8_t *)q,
                       (uint8_t *)cl);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
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
  auto up = [&](const void *src, size_t bytes, void **dst, size_t pad) -> hipError_t {
    *dst = nullptr;
    hipError_t e = hipMalloc(dst, std::max(bytes + pad, (size_t)16));
    if (e != hipSuccess) return e;
    d->owned.push_back(*dst);
    if (bytes) e = hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && pad) e = hipMemsetAsync((char *)*dst + bytes, 0, pad, c->stream);
    return e;
  };
  void *p;
#define UP(field, count, T)                                                     \
  do {                                                                          \
    hipError_t _e = up(h->field, (size_t)(count) * sizeof(T), &p, pad_##field); \
    if (_e != hipSuccess) {                                                     \
      gq_reads_free(d);                                                         \
      return set_err(GQ_E_HIP, "upload %s: %s", #field, hipGetErrorString(_e)); \
    }                                                                           \
    d->d.field = (const T *)p;                                                  \
  } while (0)
  // the sequence pool gets a zeroed tail so 1 KiB LDS-DMA pieces and 16-byte chunk loads
  // past the last read stay inside the allocation (DevReads::seq_cap)
  enum : size_t { pad_contig_read_begin = 0, pad_start = 0, pad_end = 0, pad_pmax_end = 0, pad_mapq = 0, pad_flags = 0,
                  pad_sample = 0, pad_seq_off = 0, pad_seq_len = 0, pad_cigar_off = 0, pad_n_cigar = 0, pad_md_off = 0,
                  pad_n_md = 0, pad_n_mismatch = 0, pad_seq = kSeqPad, pad_qual = 0, pad_cigar = 0, pad_md_ev = 0 };
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
  UP(seq, h->seq_bytes, uint8_t);
  UP(qual, h->seq_bytes, uint8_t);
  UP(cigar, h->cigar_len, uint32_t);
  UP(md_ev, h->md_len, uint32_t);
#undef UP
  d->d.n_reads = n;
  d->d.seq_bytes = h->seq_bytes;
  d->d.seq_cap = h->seq_bytes + kSeqPad;
  d->d.n_contigs = h->n_contigs;
  d->d.n_samples = h->n_samples;
  d->contig_read_begin.assign(h->contig_read_begin, h->contig_read_begin + h->n_contigs + 1);
  d->seq_bytes = h->seq_bytes;
  gq_status st2 = derive_shape(c, d, h->md_len);
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
  d->contig_read_begin.resize((size_t)h->n_contigs + 1);
  hipError_t e = hipMemcpy(d->contig_read_begin.data(), h->contig_read_begin,
                           sizeof(int64_t) * ((size_t)h->n_contigs + 1), hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    delete d;
    return set_err(GQ_E_HIP, "wrap: contig_read_begin D2H: %s", hipGetErrorString(e));
  }
  d->seq_bytes = h->seq_bytes;
  gq_status st2 = derive_shape(c, d, h->md_len);
  if (st2) {
    gq_reads_free(d);
    return st2;
  }
  *out = d;
  return GQ_OK;
}

void gq_reads_free(gq_dev_reads *d) {
  if (!d) return;
  for (void *p : d->owned) (void)hipFree(p);
  delete d;
}

}  // extern "C"

// ---- shared planning: validate loci, upload ranges, plan tiles -----------------------------
gq_status gq::plan(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, int T, Plan &pl, DevBuf &tiles_buf) {
  if (!loci || loci->n_ranges < 0) return set_err(GQ_E_ARG, "bad loci");
  const int64_t R = loci->n_ranges;
  std::vector<int32_t> rc;
  std::vector<int64_t> rs, re, ro, rt;
  int64_t ord = 0, tiles = 0;
  for (int64_t i = 0; i < R; ++i) {
    const int32_t cc = loci->contig[i];
    const int64_t s = loci->start[i], e = loci->end[i];
    if (cc < 0 || cc >= rd->d.n_contigs) return set_err(GQ_E_ARG, "loci range %lld: contig %d out of range", (long long)i, cc);
    if (s < 0 || e < s || e > INT32_MAX) return set_err(GQ_E_ARG, "loci range %lld: bad interval", (long long)i);
    if (e == s) continue;
    rc.push_back(cc);
    rs.push_back(s);
    re.push_back(e);
    ro.push_back(ord);
    rt.push_back(tiles);
    ord += e - s;
    tiles += (e - s + T - 1) / T;
  }
  pl.n_tiles = tiles;
  pl.n_loci = ord;
  if (tiles == 0) return GQ_OK;
  const size_t nr = rc.size();
  HIP_TRY(c->ranges.ensure(nr * (4 + 8 * 4) + 64));
  char *base = (char *)c->ranges.p;
  int32_t *d_rc = (int32_t *)base;
  int64_t *d_rs = (int64_t *)(base + ((nr * 4 + 15) & ~(size_t)15));
  int64_t *d_re = d_rs + nr, *d_ro = d_re + nr, *d_rt = d_ro + nr;
  HIP_TRY(c->ranges.ensure((size_t)((char *)(d_rt + nr) - base)));
  HIP_TRY(hipMemcpyAsync(d_rc, rc.data(), nr * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d_rs, rs.data(), nr * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d_re, re.data(), nr * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d_ro, ro.data(), nr * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(d_rt, rt.data(), nr * 8, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(tiles_buf.ensure((size_t)tiles * sizeof(Tile)));
  const int nb = (int)((tiles + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(plan_tiles, dim3(nb), dim3(kBlock), 0, c->stream, d_rc, d_rs, d_re, d_ro, d_rt, (int64_t)nr,
                     tiles, T, rd->d, (Tile *)tiles_buf.p);
  HIP_TRY(hipGetLastError());
  return GQ_OK;
}

gq_status gq::check_device_error(gq_ctx *c, const Counters &h) {
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

extern "C++" template <int T>
static void launch_germline(gq_ctx *c, int64_t tiles, const DevReads &R, const gq_germline_params *p, CallRec *recs,
                            unsigned long long rec_cap, ComplexItem *cplx, unsigned long long cplx_cap,
                            Counters *ctr) {
  static const int abl = getenv("GQ_ABLATE") ? atoi(getenv("GQ_ABLATE")) : 0;
  static const int stg = getenv("GQ_STAGE") ? atoi(getenv("GQ_STAGE")) : 0;
  static const int v2 = getenv("GQ_V2") ? atoi(getenv("GQ_V2")) : 0;
  static const int abl2 = getenv("GQ_V2ABL") ? atoi(getenv("GQ_V2ABL")) : 0;
  if (abl2) {  // diagnostic ablations of the locus-major kernel (results are wrong)
#define GQ_V2A(A)                                                                                                  \
  hipLaunchKernelGGL((germline_tile_v2<T / 256, A>), dim3((unsigned)tiles), dim3(T / 4), 0, c->stream,              \
                     (const Tile *)c->tiles.p, R, p->threshold, p->emit_ref, p->emit_no_call, recs, rec_cap, cplx, \
                     cplx_cap, ctr)
    switch (abl2) {
      case 1: GQ_V2A(1); break;
      case 2: GQ_V2A(2); break;
      case 4: GQ_V2A(4); break;
      case 7: GQ_V2A(7); break;
      default: GQ_V2A(0); break;
    }
#undef GQ_V2A
    return;
  }
  if (v2 && !abl && !stg) {  // locus-major kernel (experimental: more VALU per element than v1)
    hipLaunchKernelGGL((germline_tile_v2<T / 256>), dim3((unsigned)tiles), dim3(T / 4), 0, c->stream,
                       (const Tile *)c->tiles.p, R, p->threshold, p->emit_ref, p->emit_no_call, recs, rec_cap, cplx,
                       cplx_cap, ctr);
    return;
  }
  if (stg == 2) {  // smaller stage (for T = 512 / 768 tiles)
    hipLaunchKernelGGL((germline_tile<T, 0, 24 * 1024>), dim3((unsigned)tiles), dim3(kBlock), 0, c->stream,
                       (const Tile *)c->tiles.p, R, p->threshold, p->emit_ref, p->emit_no_call, recs, rec_cap, cplx,
                       cplx_cap, ctr);
    return;
  }
  if (stg) {
    hipLaunchKernelGGL((germline_tile<T, 0, kStageBytes>), dim3((unsigned)tiles), dim3(kBlock), 0, c->stream,
                       (const Tile *)c->tiles.p, R, p->threshold, p->emit_ref, p->emit_no_call, recs, rec_cap, cplx,
                       cplx_cap, ctr);
    return;
  }
  static const int chunked = getenv("GQ_CHUNKED") ? atoi(getenv("GQ_CHUNKED")) : 0;
  if (chunked) {  // chunk-major walk (experimental: coalesced loads, more VALU per element)
    hipLaunchKernelGGL((germline_tile<T, 0, 0, 1>), dim3((unsigned)tiles), dim3(kBlock), 0, c->stream,
                       (const Tile *)c->tiles.p, R, p->threshold, p->emit_ref, p->emit_no_call, recs, rec_cap, cplx,
                       cplx_cap, ctr);
    return;
  }
#define GQ_LAUNCH(A)                                                                                             \
  hipLaunchKernelGGL((germline_tile<T, A>), dim3((unsigned)tiles), dim3(kBlock), 0, c->stream,                   \
                     (const Tile *)c->tiles.p, R, p->threshold, p->emit_ref, p->emit_no_call, recs, rec_cap, cplx, \
                     cplx_cap, ctr)
  switch (abl) {
    case 1: GQ_LAUNCH(1); break;
    case 2: GQ_LAUNCH(2); break;
    case 4: GQ_LAUNCH(4); break;
    case 8: GQ_LAUNCH(8); break;
    case 12: GQ_LAUNCH(12); break;
    case 14: GQ_LAUNCH(14); break;
    case 32: GQ_LAUNCH(32); break;
    default: GQ_LAUNCH(0); break;
  }
#undef GQ_LAUNCH
}

gq_status gq_germline_threshold(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci,
                                const gq_germline_params *p, gq_calls **out) {
  if (!c || !rd || !loci || !p || !out) return set_err(GQ_E_ARG, "gq_germline_threshold: null argument");
  HIP_TRY(hipSetDevice(c->device));
  const int T = c->germ_tile;
  c->timings = gq_timings{};
  const auto h0 = std::chrono::steady_clock::now();
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  Plan pl;
  gq_status st = plan(c, rd, loci, T, pl, c->tiles);
  if (st) return st;
  HIP_TRY(hipEventRecord(c->ev[1], c->stream));
  gq_calls *res = (gq_calls *)calloc(1, sizeof(gq_calls));
  if (!res) return set_err(GQ_E_NOMEM, "calloc");
  if (pl.n_tiles == 0) {
    *out = res;
    return GQ_OK;
  }
  const int ns = rd->d.n_samples;
  unsigned long long rec_cap = (p->emit_ref || p->emit_no_call) ? (unsigned long long)(2 * ns) * pl.n_loci + 1024
                                                                 : std::max<unsigned long long>(1 << 16, pl.n_loci / 8);
  unsigned long long cplx_cap = std::max<unsigned long long>(1 << 16, pl.n_loci / 8);
  unsigned long long pool_cap = 1 << 22;
  Counters hc{};
  for (int attempt = 0; attempt < 3; ++attempt) {
    HIP_TRY(c->recs.ensure(rec_cap * sizeof(CallRec)));
    HIP_TRY(c->cplx.ensure(cplx_cap * sizeof(ComplexItem)));
    HIP_TRY(c->pool.ensure(pool_cap));
    HIP_TRY(c->counters.ensure(sizeof(Counters)));
    Counters *ctr = (Counters *)c->counters.p;
    HIP_TRY(hipMemsetAsync(ctr, 0, sizeof(Counters), c->stream));
    if (attempt == 0) HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    switch (T) {
      case 512: launch_germline<512>(c, pl.n_tiles, rd->d, p, (CallRec *)c->recs.p, rec_cap, (ComplexItem *)c->cplx.p, cplx_cap, ctr); break;
      case 768: launch_germline<768>(c, pl.n_tiles, rd->d, p, (CallRec *)c->recs.p, rec_cap, (ComplexItem *)c->cplx.p, cplx_cap, ctr); break;
      case 2048: launch_germline<2048>(c, pl.n_tiles, rd->d, p, (CallRec *)c->recs.p, rec_cap, (ComplexItem *)c->cplx.p, cplx_cap, ctr); break;
      default: launch_germline<1024>(c, pl.n_tiles, rd->d, p, (CallRec *)c->recs.p, rec_cap, (ComplexItem *)c->cplx.p, cplx_cap, ctr); break;
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    const int cblocks = (int)std::min<int64_t>(std::max<int64_t>(pl.n_tiles, 1), 4096);
    hipLaunchKernelGGL(germline_complex, dim3(cblocks), dim3(kBlock), 0, c->stream, (const Tile *)c->tiles.p,
                       (const ComplexItem *)c->cplx.p, rd->d, p->threshold, p->emit_ref, p->emit_no_call,
                       (CallRec *)c->recs.p, rec_cap, (uint8_t *)c->pool.p, pool_cap, cplx_cap, ctr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[3], c->stream));
    HIP_TRY(hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    bool retry = false;
    if (hc.n_complex > cplx_cap) {
      cplx_cap = hc.n_complex + 1024;
      retry = true;
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
  if (getenv("GQ_PROF") && hc.prof[4])
    fprintf(stderr, "gq prof (cycles/wave): setup %.0f walk %.0f wait %.0f decide %.0f  (waves %llu)\n",
            (double)hc.prof[0] / hc.prof[4], (double)hc.prof[1] / hc.prof[4], (double)hc.prof[2] / hc.prof[4],
            (double)hc.prof[3] / hc.prof[4], hc.prof[4]);
  for (int k = 0; k < kSpread; ++k) {
    hc.visited += hc.spread[0][k];
    hc.ambiguous += hc.spread[1][k];
    hc.ties += hc.spread[2][k];
  }
  st = check_device_error(c, hc);
  if (st) {
    free(res);
    return st;
  }
  // ---- sort records by key (output order), then build the host result image on device:
  //      one D2H copy of [header | SoA arrays | allele pool] instead of per-record marshalling
  const int64_t n = (int64_t)hc.n_rec;
  const size_t nn = (size_t)std::max<int64_t>(n, 1);
  HIP_TRY(c->keys.ensure(nn * 8));
  HIP_TRY(c->keys_sorted.ensure(nn * 8));
  HIP_TRY(c->idx.ensure(nn * 8));
  HIP_TRY(c->idx_sorted.ensure(nn * 4));
  const CallsLayout lay = calls_layout(n, (int64_t)std::min<unsigned long long>(hc.pool_used, pool_cap));
  HIP_TRY(c->image.ensure(lay.bytes));
  if (n > 0) {
    const unsigned nb = (unsigned)((n + kBlock - 1) / kBlock);
    // keys are the first 8 bytes of each record: strided copy into a dense key array
    HIP_TRY(hipMemcpy2DAsync(c->keys.p, 8, c->recs.p, sizeof(CallRec), 8, (size_t)n, hipMemcpyDeviceToDevice,
                             c->stream));
    hipLaunchKernelGGL(iota_i32, dim3(nb), dim3(kBlock), 0, c->stream, (int32_t *)c->idx.p, n);
    HIP_TRY(hipGetLastError());
    int end_bit = 12;
    while (end_bit < 64 && ((uint64_t)pl.n_loci >> (end_bit - 12)) != 0) ++end_bit;
    size_t tmp = 0, tmp2 = 0;
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const uint64_t *)c->keys.p, (uint64_t *)c->keys_sorted.p,
                                               (const int32_t *)c->idx.p, (int32_t *)c->idx_sorted.p, (int)n, 0,
                                               end_bit, c->stream));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp2, (const int64_t *)c->idx.p, (int64_t *)c->keys.p, (int)n,
                                             c->stream));
    HIP_TRY(c->sort_tmp.ensure(std::max(tmp, tmp2)));
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(c->sort_tmp.p, tmp, (const uint64_t *)c->keys.p,
                                               (uint64_t *)c->keys_sorted.p, (const int32_t *)c->idx.p,
                                               (int32_t *)c->idx_sorted.p, (int)n, 0, end_bit, c->stream));
    // allele byte lengths in output order -> exclusive offsets into the pool
    hipLaunchKernelGGL(calls_lengths, dim3(nb), dim3(kBlock), 0, c->stream, (const CallRec *)c->recs.p,
                       (const int32_t *)c->idx_sorted.p, n, (int64_t *)c->idx.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(c->sort_tmp.p, tmp2, (const int64_t *)c->idx.p, (int64_t *)c->keys.p,
                                             (int)n, c->stream));
    hipLaunchKernelGGL(calls_image, dim3(nb), dim3(kBlock), 0, c->stream, (const CallRec *)c->recs.p,
                       (const int32_t *)c->idx_sorted.p, (const int64_t *)c->keys.p, (const uint8_t *)c->pool.p, n,
                       lay, (uint8_t *)c->image.p);
    HIP_TRY(hipGetLastError());
  } else {
    HIP_TRY(hipMemsetAsync(c->image.p, 0, 64, c->stream));
  }
  uint8_t *blk = (uint8_t *)malloc(lay.bytes);
  if (!blk) {
    free(res);
    return set_err(GQ_E_NOMEM, "result block of %zu bytes", lay.bytes);
  }
  HIP_TRY(hipMemcpyAsync(blk, c->image.p, lay.bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipEventRecord(c->ev[4], c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  // ---- point the result struct into the block (output order)
  const auto h1 = std::chrono::steady_clock::now();
  res->n = n;
  res->block_ = blk;
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
  res->pool_len = *(const int64_t *)blk;
  res->visited_loci = (int64_t)hc.visited;
  res->complex_loci = (int64_t)hc.n_complex;
  res->ambiguous_loci = (int64_t)hc.ambiguous;
  res->tie_loci = (int64_t)hc.ties;
  // timings
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
  c->timings.plan_ms = ms;
  (void)hipEventElapsedTime(&ms, c->ev[1], c->ev[2]);
  c->timings.pileup_ms = ms;
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

void gq_free_calls(gq_calls *r) {
  if (!r) return;
  free(r->block_);
  free(r);
}

gq_status gq_pileup_counts(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, gq_counts **out) {
  if (!c || !rd || !loci || !out) return set_err(GQ_E_ARG, "gq_pileup_counts: null argument");
  HIP_TRY(hipSetDevice(c->device));
  Plan pl;
  gq_status st = plan(c, rd, loci, kCountT, pl, c->tiles);
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
  *out = res;
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
