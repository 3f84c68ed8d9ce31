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
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
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
  std::vector<std::vector<std::vector<int64_t>>> heaps((size_t)n, std::vector<std::vector<int64_t>>((size_t)ns));
  for (size_t g0 = 0; g0 < order.size();) {
    size_t g1 = g0;
    const int64_t w = win[(size_t)order[g0]];
    while (g1 < order.size() && win[(size_t)order[g1]] == w) ++g1;
    const Plan::Win &W = pl.wins[(size_t)w];
    std::vector<int64_t> rs(pl.rs.begin() + W.r0, pl.rs.begin() + W.r1), re(pl.re.begin() + W.r0, pl.re.begin() + W.r1);
    // each set's read window over the whole window: the first tile's rb .. the last tile's re
    // (the tiles were planned over this set's reads only for sets[0]; the others are searched
    // on the host copy of their contig's start / pmax_end)
    std::vector<ReplaySet> rsets((size_t)ns);
    for (int k = 0; k < ns; ++k) {
      const gq_dev_reads *d = sets[(size_t)k];
      const int64_t cb = d->contig_read_begin[(size_t)W.contig], ce = d->contig_read_begin[(size_t)W.contig + 1];
      // the contig's start / pmax_end come over PCIe in one piece; rare path (MD tags disagree)
      std::vector<int32_t> st((size_t)(ce - cb)), pm((size_t)(ce - cb)), en((size_t)(ce - cb));
      if (ce > cb) {
        HIP_TRY(hipMemcpyAsync(st.data(), d->d.start + cb, sizeof(int32_t) * (size_t)(ce - cb), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(pm.data(), d->d.pmax_end + cb, sizeof(int32_t) * (size_t)(ce - cb), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(en.data(), d->d.end + cb, sizeof(int32_t) * (size_t)(ce - cb), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
      }
      // reads that can overlap the window: pmax_end > first start, start < last end
      const int64_t lo = (int64_t)(std::upper_bound(pm.begin(), pm.end(), (int32_t)rs.front()) - pm.begin());
      const int64_t hi = (int64_t)(std::lower_bound(st.begin(), st.end(), (int32_t)re.back()) - st.begin());
      ReplaySet &S = rsets[(size_t)k];
      S.lo = cb + lo;
      if (hi > lo) {
        S.start.assign(st.begin() + lo, st.begin() + hi);
        S.end.assign(en.begin() + lo, en.begin() + hi);
        S.pmax.assign(pm.begin() + lo, pm.begin() + hi);
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
