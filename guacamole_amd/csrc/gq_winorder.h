// gq_winorder.h — the pileup element order of each task window (included inside the
// anonymous namespace of each translation unit that needs it).
#pragma once

// ------------------------------------------------------------------------------------------
// Pileup element order.  Pileup.atGreaterLocus (Pileup.scala:103-132) keeps the surviving
// elements in order and appends new reads in start order, and the first pileup of a window
// (one per task and contig) takes the reads in SlidingWindow.currentRegions() order: the
// priority queue's heap array after enqueueing, in start order, the reads that overlap the
// window's first visited locus F (DistributedUtil.scala:260-274).  So at any locus the
// elements are the reads of that initial group still covering it, in heap order, then the
// other covering reads in read order.  The order matters for the FP sums (Likelihood,
// AlleleEvidence mean); it is restored here from the per-window initial ranks.
// ------------------------------------------------------------------------------------------
struct WinInit {
  int32_t F;    // first visited locus of the window (INT32_MAX: none)
  int32_t E;    // largest end of this set's initial-group reads (loci >= E hold none of them)
  int64_t off;  // the group's reads (ascending) and heap ranks at init_reads / init_rank [off, off + n)
  int32_t n, cap;
};

// F of each window over both read sets (the first locus of its ranges covered by a read of
// either set), and each set's candidate reads for the group (prefix-max end past F, start at
// or before F): their count is the group's capacity.  One wave per window: every search is a
// 64-way wave_first_true (a few dependent loads over a whole contig, not ~24).
__global__ void window_first(const int32_t *__restrict__ w_contig, const int64_t *__restrict__ w_roff,
                             const int64_t *__restrict__ r_s, const int64_t *__restrict__ r_e, int64_t n_win,
                             DevReads RT, DevReads RN, WinInit *__restrict__ wi, int64_t *__restrict__ wi_lo) {
  const int64_t w = wave_id();
  if (w >= n_win) return;  // wave-uniform
  const int lane = threadIdx.x & 63;
  const int32_t c = w_contig[w];
  int64_t F = INT32_MAX;
  for (int s = 0; s < 2; ++s) {
    const DevReads &R = s ? RN : RT;
    const int64_t cb = R.contig_read_begin[c], ce = R.contig_read_begin[c + 1];
    for (int64_t k = w_roff[w]; k < w_roff[w + 1]; ++k) {
      const int64_t a = r_s[k];
      if (a >= F) break;
      // the first read with pmax_end > a covers max(a, its start)
      const int64_t lo = wave_first_true(cb, ce, [&](int64_t m) { return (int64_t)R.pmax_end[m] > a; });
      if (lo < ce) {
        const int64_t f = max(a, (int64_t)R.start[lo]);
        if (f < r_e[k]) {
          F = min(F, f);
          break;
        }
      }
    }
  }
  for (int s = 0; s < 2; ++s) {
    const DevReads &R = s ? RN : RT;
    WinInit x{(int32_t)F, INT32_MIN, 0, 0, 0};
    int64_t lo = 0;
    if (F < INT32_MAX) {
      const int64_t cb = R.contig_read_begin[c], ce = R.contig_read_begin[c + 1];
      lo = wave_first_true(cb, ce, [&](int64_t m) { return (int64_t)R.pmax_end[m] > F; });
      const int64_t a = wave_first_true(lo, ce, [&](int64_t m) { return (int64_t)R.start[m] > F; });
      x.cap = (int32_t)min<int64_t>(a - lo, INT32_MAX);
      // a bound on the group's largest end until window_group sets it exactly: the prefix
      // max of end over the reads starting at or before F
      if (a > lo) x.E = R.pmax_end[a - 1];
    }
    if (lane == 0) {
      wi[2 * w + s] = x;
      wi_lo[2 * w + s] = lo;
    }
  }
}

// The initial group of each (window, set): reads [lo, lo + cap) that overlap F, enqueued in
// read order into an empty Scala PriorityQueue (fixUp while the parent's end is larger,
// SlidingWindow.scala:62-68); rank = position in the heap array.  One thread per (window, set).
__global__ void window_group(WinInit *__restrict__ wi, const int64_t *__restrict__ wi_lo, int64_t n,
                             DevReads RT, DevReads RN, int64_t *__restrict__ init_reads,
                             int32_t *__restrict__ init_rank, int32_t *__restrict__ heap) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  WinInit x = wi[k];
  const DevReads &R = (k & 1) ? RN : RT;
  int64_t *rd = init_reads + x.off;
  int32_t *rk = init_rank + x.off;
  int32_t *h = heap + x.off;  // heap of group positions, 0-based (h[i] <-> Scala index i + 1)
  int32_t m = 0;
  int32_t E = INT32_MIN;
  for (int64_t i = 0; i < x.cap; ++i) {
    const int64_t r = wi_lo[k] + i;
    if (R.end[r] <= x.F) continue;
    rd[m] = r;
    E = max(E, R.end[r]);
    int32_t q = m++;
    h[q] = q;
    while (q > 0) {
      const int32_t p = (q + 1) / 2 - 1;
      if (!(R.end[rd[h[q]]] < R.end[rd[h[p]]])) break;
      const int32_t t = h[q];
      h[q] = h[p];
      h[p] = t;
      q = p;
    }
  }
  for (int32_t i = 0; i < m; ++i) rk[h[i]] = i;
  x.n = m;
  x.E = E;
  wi[k] = x;
}

// Per-window data of the element order (window_first / window_group), by tile range.
struct SomWin {
  const int32_t *range_win;  // plan range -> window
  const WinInit *wi;         // [window * 2 + set]
  const int64_t *init_reads;
  const int32_t *init_rank;
};

// Window bounds only (germline first pass): window_first over the plan's device copies of its
// ranges (valid until the next plan() on the context), no host round trip.  SomWin without
// init_reads: every WinInit has n = 0 (element order = read order) and E = an upper bound on
// the initial group's ends, so a locus at or past E is known to have read-order elements.
gq_status window_bounds(gq_ctx *c, const Plan &pl, const gq_dev_reads *t, SomWin &sw) {
  const int64_t nw = (int64_t)pl.wins.size();
  if (nw == 0 || !pl.d_rwin) {
    sw = SomWin{};
    return GQ_OK;
  }
  HIP_TRY(c->win_bound.ensure((size_t)nw * (2 * sizeof(WinInit) + 2 * sizeof(int64_t)) + 64));
  WinInit *d_wi = (WinInit *)c->win_bound.p;
  int64_t *d_lo = (int64_t *)(d_wi + 2 * nw);
  hipLaunchKernelGGL(window_first, dim3((unsigned)((nw * 64 + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                     pl.d_wcontig, pl.d_wroff, pl.d_rs, pl.d_re, nw, t->d, t->d, d_wi, d_lo);
  HIP_TRY(hipGetLastError());
  sw = SomWin{pl.d_rwin, d_wi, nullptr, nullptr};
  return GQ_OK;
}

// The pileup element order of a plan's windows (SomWin): each window's first visited locus and
// its initial (heap-ordered) group of reads, for the two read sets t and n.
gq_status build_somwin(gq_ctx *c, const Plan &pt, const gq_dev_reads *t, const gq_dev_reads *n, SomWin &sw) {
  {
    const int64_t nw = (int64_t)pt.wins.size(), nr = (int64_t)pt.rs.size();
    std::vector<int32_t> w_contig((size_t)nw);
    std::vector<int64_t> w_roff((size_t)nw + 1);
    for (int64_t w = 0; w < nw; ++w) {
      w_contig[(size_t)w] = pt.wins[(size_t)w].contig;
      w_roff[(size_t)w] = pt.wins[(size_t)w].r0;
    }
    w_roff[(size_t)nw] = nr;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_roff = al(4 * (size_t)nw), o_rs = o_roff + al(8 * ((size_t)nw + 1)), o_re = o_rs + al(8 * (size_t)nr),
                 o_rw = o_re + al(8 * (size_t)nr), o_wi = o_rw + al(4 * (size_t)nr),
                 o_lo = o_wi + al(sizeof(WinInit) * 2 * (size_t)nw), o_end = o_lo + al(8 * 2 * (size_t)nw);
    HIP_TRY(c->win_meta.ensure(o_end));
    char *b = (char *)c->win_meta.p;
    HIP_TRY(hipMemcpyAsync(b, w_contig.data(), 4 * (size_t)nw, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(b + o_roff, w_roff.data(), 8 * ((size_t)nw + 1), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(b + o_rs, pt.rs.data(), 8 * (size_t)nr, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(b + o_re, pt.re.data(), 8 * (size_t)nr, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(b + o_rw, pt.rwin.data(), 4 * (size_t)nr, hipMemcpyHostToDevice, c->stream));
    WinInit *d_wi = (WinInit *)(b + o_wi);
    int64_t *d_lo = (int64_t *)(b + o_lo);
    hipLaunchKernelGGL(window_first, dim3((unsigned)((nw * 64 + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                       (const int32_t *)b, (const int64_t *)(b + o_roff), (const int64_t *)(b + o_rs),
                       (const int64_t *)(b + o_re), nw, t->d, n->d, d_wi, d_lo);
    HIP_TRY(hipGetLastError());
    std::vector<WinInit> wi((size_t)(2 * nw));
    HIP_TRY(hipMemcpyAsync(wi.data(), d_wi, sizeof(WinInit) * wi.size(), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    int64_t tot = 0;
    for (WinInit &x : wi) {
      x.off = tot;
      tot += x.cap;
    }
    HIP_TRY(hipMemcpyAsync(d_wi, wi.data(), sizeof(WinInit) * wi.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c->win_grp.ensure((size_t)std::max<int64_t>(tot, 1) * 16));
    int64_t *d_reads = (int64_t *)c->win_grp.p;
    int32_t *d_rank = (int32_t *)(d_reads + std::max<int64_t>(tot, 1));
    int32_t *d_heap = d_rank + std::max<int64_t>(tot, 1);
    hipLaunchKernelGGL(window_group, dim3((unsigned)((2 * nw + kBlock - 1) / kBlock)), dim3(kBlock), 0, c->stream,
                       d_wi, (const int64_t *)d_lo, 2 * nw, t->d, n->d, d_reads, d_rank, d_heap);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(c->stream));  // wi (host) outlives its copy
    sw = SomWin{(const int32_t *)(b + o_rw), d_wi, d_reads, d_rank};
  }
  return GQ_OK;
}


// Element-order key of read r (index in its set) covering pos: the initial group's reads still
// covering pos come first, by heap rank; every other read after them, by read index.  Without
// window data (w.n == 0) the read index alone.  Monotone in pileup element order.
__device__ __forceinline__ int64_t element_order_key(const DevReads &R, int64_t r, int32_t pos, const WinInit &w,
                                                     const int64_t *__restrict__ init_reads,
                                                     const int32_t *__restrict__ init_rank) {
  if (w.n > 0 && pos < w.E && R.start[r] <= w.F) {
    int lo = 0, hi = w.n;  // r in the group's ascending read list
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (init_reads[w.off + m] < r) lo = m + 1;
      else hi = m;
    }
    if (lo < w.n && init_reads[w.off + lo] == r) return (int64_t)init_rank[w.off + lo];
  }
  return (1ll << 40) + r;
}
