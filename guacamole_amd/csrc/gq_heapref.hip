// gq_heapref.hip — the pileup reference base at loci where it depends on heap order.
//
// Pileup.referenceBaseAtLocus (pileup/Pileup.scala:157-165) returns the MD-derived base of
// the first read, in SlidingWindow.currentRegions() order (the priority queue's heap array,
// windowing/SlidingWindow.scala:71-73), whose base is A/C/G/T, else N.  When the reads' MD
// tags agree any read gives the same base and the kernels decide alone; where they disagree
// (listed as AmbItems) heap_ref_bases replays the window's queue(s) on the host (gq_replay.h)
// from the last coverage gap and reads the bases in that order on the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "gq_alleles.h"
#include "gq_host.h"
#include "gq_replay.h"

using namespace gq;

namespace {

// One wave per listed locus and read set: reads heap[off[i] .. off[i + 1]) in heap order.
__global__ void heap_refbase(const int64_t *__restrict__ off, const int64_t *__restrict__ heap,
                             const int32_t *__restrict__ pos, int64_t n, int nsets, int set, DevReads R,
                             uint8_t *__restrict__ out, Counters *ctr) {
  const int lane = threadIdx.x & 63;
  const int64_t w = wave_id();
  if (w >= n) return;
  const int32_t p = pos[w];
  const int64_t a = off[w], b = off[w + 1];
  uint8_t base = 'N';
  for (int64_t k0 = a; k0 < b; k0 += 64) {
    const int64_t k = k0 + lane;
    int v = -1;
    if (k < b) {
      v = md_ref_at(R, heap[k], p);
      if (v < 0) raise_error(&ctr->err, (int64_t *)&ctr->err_pos, v == -4 ? GQ_E_NO_MD : v == -3 ? GQ_E_MD : GQ_E_ASSERT, p);
    }
    const unsigned long long m = __ballot(v >= 0 && std_bit((uint8_t)v) != 0);
    if (m) {
      base = (uint8_t)__shfl(v, __ffsll((long long)m) - 1, 64);
      break;
    }
  }
  if (lane == 0) out[w * nsets + set] = base;
}

// Read bounds of a set's contig for the replay: q.x = first read of [cb, ce) with pmax_end >
// x (upper_bound on the prefix max), else the first read with start >= x (lower_bound).  One
// thread per query.
struct BoundQ {
  int64_t cb, ce;
  int32_t x, by_pmax;
};
__global__ void read_bounds(const BoundQ *__restrict__ q, int64_t n, DevReads R, int64_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const BoundQ b = q[i];
  int64_t lo = b.cb, hi = b.ce;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    const bool right = b.by_pmax ? R.pmax_end[m] > b.x : R.start[m] >= b.x;
    if (right) hi = m;
    else lo = m + 1;
  }
  out[i] = lo;
}

}  // namespace

gq_status gq::heap_ref_bases(gq_ctx *c, const Plan &pl, const DevBuf &tiles_buf,
                             const std::vector<const gq_dev_reads *> &sets, const std::vector<AmbItem> &items,
                             uint8_t *out_ref) {
  const int64_t n = (int64_t)items.size();
  if (n == 0) return GQ_OK;
  const int ns = (int)sets.size();
  // items by window, then locus
  std::vector<int64_t> order((size_t)n), win((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    order[(size_t)i] = i;
    const int64_t r = pl.range_of_tile(items[(size_t)i].tile);
    if (r < 0 || r >= (int64_t)pl.rwin.size()) return set_err(GQ_E_ASSERT, "heap_ref_bases: tile outside the plan");
    win[(size_t)i] = pl.rwin[(size_t)r];
  }
  std::sort(order.begin(), order.end(), [&](int64_t x, int64_t y) {
    return win[(size_t)x] != win[(size_t)y] ? win[(size_t)x] < win[(size_t)y] : items[(size_t)x].pos < items[(size_t)y].pos;
  });
  // The replay of a window needs, per set, the reads that can overlap the window's loci up to
  // its last listed locus: pmax_end > the window's first start, start <= that locus.  Those
  // bounds come from a device search (one thread per bound), and each (set, contig) is copied
  // to the host ONCE per call, as the one slice covering every listed window on the contig.
  std::vector<int64_t> gw;  // the listed windows, in order, and their last listed locus
  std::vector<int32_t> glast;
  for (size_t g = 0; g < order.size(); ++g) {
    const int64_t w = win[(size_t)order[g]];
    if (gw.empty() || gw.back() != w) {
      gw.push_back(w);
      glast.push_back(items[(size_t)order[g]].pos);
    } else {
      glast.back() = std::max(glast.back(), items[(size_t)order[g]].pos);
    }
  }
  const int64_t nw = (int64_t)gw.size();
  std::vector<int64_t> blo((size_t)(nw * ns)), bhi((size_t)(nw * ns));
  for (int k = 0; k < ns; ++k) {
    const gq_dev_reads *d = sets[(size_t)k];
    std::vector<BoundQ> q((size_t)(2 * nw));
    for (int64_t j = 0; j < nw; ++j) {
      const Plan::Win &W = pl.wins[(size_t)gw[(size_t)j]];
      const int64_t cb = d->contig_read_begin[(size_t)W.contig], ce = d->contig_read_begin[(size_t)W.contig + 1];
      q[(size_t)(2 * j)] = BoundQ{cb, ce, (int32_t)pl.rs[(size_t)W.r0], 1};
      q[(size_t)(2 * j + 1)] = BoundQ{cb, ce, glast[(size_t)j] + 1, 0};
    }
    HIP_TRY(c->heap_off.ensure(sizeof(BoundQ) * q.size() + sizeof(int64_t) * q.size() + 64));
    BoundQ *d_q = (BoundQ *)c->heap_off.p;
    int64_t *d_b = (int64_t *)(d_q + q.size());
    std::vector<int64_t> b(q.size());
    HIP_TRY(hipMemcpyAsync(d_q, q.data(), sizeof(BoundQ) * q.size(), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(read_bounds, dim3((unsigned)((q.size() + 255) / 256)), dim3(256), 0, c->stream, (const BoundQ *)d_q,
                       (int64_t)q.size(), d->d, d_b);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(b.data(), d_b, sizeof(int64_t) * b.size(), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int64_t j = 0; j < nw; ++j) {
      blo[(size_t)(j * ns + k)] = b[(size_t)(2 * j)];
      bhi[(size_t)(j * ns + k)] = std::max(b[(size_t)(2 * j)], b[(size_t)(2 * j + 1)]);
    }
  }
  // one host slice per (set, contig): the union of its windows' bounds
  struct Slice {
    int64_t lo = 0, hi = 0;
    std::vector<int32_t> start, end, pmax;
  };
  std::vector<std::vector<Slice>> slices((size_t)ns);  // [set][contig]
  for (int k = 0; k < ns; ++k) {
    const gq_dev_reads *d = sets[(size_t)k];
    const size_t nc = d->contig_read_begin.size() > 0 ? d->contig_read_begin.size() - 1 : 0;
    slices[(size_t)k].resize(nc);
    std::vector<char> seen(nc, 0);
    for (int64_t j = 0; j < nw; ++j) {
      const size_t ci = (size_t)pl.wins[(size_t)gw[(size_t)j]].contig;
      Slice &S = slices[(size_t)k][ci];
      const int64_t lo = blo[(size_t)(j * ns + k)], hi = bhi[(size_t)(j * ns + k)];
      if (!seen[ci]) S.lo = lo, S.hi = hi, seen[ci] = 1;
      else S.lo = std::min(S.lo, lo), S.hi = std::max(S.hi, hi);
    }
    for (size_t ci = 0; ci < nc; ++ci) {
      Slice &S = slices[(size_t)k][ci];
      if (!seen[ci] || S.hi <= S.lo) continue;
      const size_t m = (size_t)(S.hi - S.lo);
      S.start.resize(m), S.end.resize(m), S.pmax.resize(m);
      HIP_TRY(hipMemcpyAsync(S.start.data(), d->d.start + S.lo, sizeof(int32_t) * m, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipMemcpyAsync(S.end.data(), d->d.end + S.lo, sizeof(int32_t) * m, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipMemcpyAsync(S.pmax.data(), d->d.pmax_end + S.lo, sizeof(int32_t) * m, hipMemcpyDeviceToHost, c->stream));
    }
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  std::vector<std::vector<std::vector<int64_t>>> heaps((size_t)n, std::vector<std::vector<int64_t>>((size_t)ns));
  for (size_t g0 = 0, j = 0; g0 < order.size(); ++j) {
    size_t g1 = g0;
    const int64_t w = win[(size_t)order[g0]];
    while (g1 < order.size() && win[(size_t)order[g1]] == w) ++g1;
    const Plan::Win &W = pl.wins[(size_t)w];
    std::vector<int64_t> rs(pl.rs.begin() + W.r0, pl.rs.begin() + W.r1), re(pl.re.begin() + W.r0, pl.re.begin() + W.r1);
    std::vector<ReplaySet> rsets((size_t)ns);
    for (int k = 0; k < ns; ++k) {
      const Slice &S = slices[(size_t)k][(size_t)W.contig];
      const int64_t lo = blo[(size_t)(j * ns + k)], hi = bhi[(size_t)(j * ns + k)];
      ReplaySet &R = rsets[(size_t)k];
      R.lo = lo;
      if (hi > lo) {
        R.start.assign(S.start.begin() + (lo - S.lo), S.start.begin() + (hi - S.lo));
        R.end.assign(S.end.begin() + (lo - S.lo), S.end.begin() + (hi - S.lo));
        R.pmax.assign(S.pmax.begin() + (lo - S.lo), S.pmax.begin() + (hi - S.lo));
      }
    }
    std::vector<ReplayQuery> qs;
    for (size_t g = g0; g < g1; ++g) qs.push_back(ReplayQuery{items[(size_t)order[g]].pos, (int32_t)order[g]});
    replay_heaps(rs, re, rsets, qs, [&](int32_t id, int k, const int64_t *h, int64_t nh) {
      heaps[(size_t)id][(size_t)k].assign(h, h + nh);
    });
    g0 = g1;
  }
  (void)tiles_buf;
  // flatten per set, read the bases on the device
  std::vector<int32_t> pos((size_t)n);
  for (int64_t i = 0; i < n; ++i) pos[(size_t)i] = items[(size_t)i].pos;
  for (int k = 0; k < ns; ++k) {
    std::vector<int64_t> off((size_t)n + 1, 0), flat;
    for (int64_t i = 0; i < n; ++i) {
      const auto &h = heaps[(size_t)i][(size_t)k];
      flat.insert(flat.end(), h.begin(), h.end());
      off[(size_t)i + 1] = (int64_t)flat.size();
    }
    HIP_TRY(c->heap_off.ensure(sizeof(int64_t) * (off.size() + 1) + sizeof(int32_t) * pos.size() + 64));
    HIP_TRY(c->heap_reads.ensure(sizeof(int64_t) * std::max<size_t>(flat.size(), 1)));
    int64_t *d_off = (int64_t *)c->heap_off.p;
    int32_t *d_pos = (int32_t *)(d_off + off.size() + 1);
    HIP_TRY(hipMemcpyAsync(d_off, off.data(), sizeof(int64_t) * off.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_pos, pos.data(), sizeof(int32_t) * pos.size(), hipMemcpyHostToDevice, c->stream));
    if (!flat.empty())
      HIP_TRY(hipMemcpyAsync(c->heap_reads.p, flat.data(), sizeof(int64_t) * flat.size(), hipMemcpyHostToDevice, c->stream));
    const unsigned nb = (unsigned)((n * 64 + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(heap_refbase, dim3(nb), dim3(kBlock), 0, c->stream, (const int64_t *)d_off,
                       (const int64_t *)c->heap_reads.p, (const int32_t *)d_pos, n, ns, k, sets[(size_t)k]->d, out_ref,
                       (Counters *)c->counters.p);
    HIP_TRY(hipGetLastError());
    // the host vectors must outlive the async copies
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  return GQ_OK;
}

gq_status gq::reads_overlap(gq_ctx *c, const gq_dev_reads *set, int32_t contig,
                            const std::vector<std::pair<int64_t, int64_t>> &ranges, std::vector<char> &out) {
  out.assign(ranges.size(), 0);
  if (ranges.empty()) return GQ_OK;
  const int64_t cb = set->contig_read_begin[(size_t)contig], ce = set->contig_read_begin[(size_t)contig + 1];
  if (ce <= cb) return GQ_OK;
  std::vector<BoundQ> q(ranges.size());
  for (size_t i = 0; i < ranges.size(); ++i)
    q[i] = BoundQ{cb, ce, (int32_t)std::min<int64_t>(std::max<int64_t>(ranges[i].first, INT32_MIN), INT32_MAX), 1};
  HIP_TRY(c->heap_off.ensure(sizeof(BoundQ) * q.size() + sizeof(int64_t) * q.size() + 64));
  BoundQ *d_q = (BoundQ *)c->heap_off.p;
  int64_t *d_b = (int64_t *)(d_q + q.size());
  std::vector<int64_t> first(q.size());
  HIP_TRY(hipMemcpyAsync(d_q, q.data(), sizeof(BoundQ) * q.size(), hipMemcpyHostToDevice, c->stream));
  hipLaunchKernelGGL(read_bounds, dim3((unsigned)((q.size() + 255) / 256)), dim3(256), 0, c->stream, (const BoundQ *)d_q,
                     (int64_t)q.size(), set->d, d_b);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(first.data(), d_b, sizeof(int64_t) * first.size(), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  // the starts of those first reads
  std::vector<int32_t> st(first.size(), INT32_MAX);
  for (size_t i = 0; i < first.size(); ++i)
    if (first[i] < ce) HIP_TRY(hipMemcpyAsync(&st[i], set->d.start + first[i], sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < ranges.size(); ++i)
    out[i] = (first[i] < ce && (int64_t)st[i] < ranges[i].second && ranges[i].first < ranges[i].second) ? 1 : 0;
  return GQ_OK;
}

namespace {
__global__ void warm_k() {}
}  // namespace
hipError_t gq::warm_heapref(hipStream_t s) {
  hipLaunchKernelGGL(warm_k, dim3(1), dim3(64), 0, s);
  return hipGetLastError();
}
