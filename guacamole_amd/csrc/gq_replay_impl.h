// gq_replay_impl.h — implementation of replay_heaps (see gq_replay.h).  Host code.
#pragma once
#include <algorithm>
#include <climits>
#include <utility>
#include <vector>

namespace gq {
namespace replay_detail {

// One window's queue over one read set: the Scala 2.10 mutable.PriorityQueue with
// SlidingWindow's ordering (compare(a, b) = b.end compare a.end, SlidingWindow.scala:62-68):
// heap array from index 1, the root holds the smallest end.
//   enqueue: append, fixUp (swap with the parent while the parent's end is larger)
//   dequeue: swap root and last, fixDown over the rest (descend to the child with the
//            smaller end, the left one on ties, while it is smaller than the node), pop
struct Queue {
  const ReplaySet *S = nullptr;
  std::vector<int64_t> h{0};  // local read indices, h[0] unused
  int32_t max_end = INT32_MIN;
  int64_t nxt = 0;            // next pending (relevant) read
  size_t rp = 0;              // first window range whose end is past the pending read's start

  int32_t end_of(int64_t i) const { return S->end[(size_t)i]; }
  int64_t n() const { return (int64_t)S->start.size(); }
  bool empty() const { return h.size() < 2; }
  int32_t head_end() const { return end_of(h[1]); }

  void enqueue(int64_t i) {
    h.push_back(i);
    size_t k = h.size() - 1;
    while (k > 1 && end_of(h[k]) < end_of(h[k / 2])) {
      std::swap(h[k], h[k / 2]);
      k /= 2;
    }
    max_end = std::max(max_end, end_of(i));
  }
  void dequeue() {
    const size_t last = h.size() - 1;
    std::swap(h[1], h[last]);
    const size_t n = last - 1;  // heap size after removal
    size_t k = 1;
    while (n >= 2 * k) {
      size_t j = 2 * k;
      if (j < n && end_of(h[j + 1]) < end_of(h[j])) ++j;
      if (end_of(h[k]) <= end_of(h[j])) break;
      std::swap(h[k], h[j]);
      k = j;
    }
    h.pop_back();
    if (empty()) max_end = INT32_MIN;
  }
  // skip pending reads that overlap none of the window's ranges (not in the task)
  void settle(const std::vector<int64_t> &rs, const std::vector<int64_t> &re) {
    while (nxt < n()) {
      const int32_t s = S->start[(size_t)nxt], e = S->end[(size_t)nxt];
      while (rp < re.size() && re[rp] <= s) ++rp;
      if (rp < re.size() && rs[rp] < e) return;
      ++nxt;
    }
  }
  int64_t next_start() const { return nxt < n() ? (int64_t)S->start[(size_t)nxt] : LLONG_MAX; }
  // setCurrentLocus(locus) (SlidingWindow.scala:83-110), halfWindowSize = 0
  void call(int64_t locus, const std::vector<int64_t> &rs, const std::vector<int64_t> &re) {
    while (!empty() && head_end() <= locus) dequeue();
    settle(rs, re);
    while (nxt < n() && S->start[(size_t)nxt] <= locus) {
      if (S->end[(size_t)nxt] > locus) enqueue(nxt);
      ++nxt;
      settle(rs, re);
    }
  }
  // largest x <= hi with no read of this set starting before x covering x, or LLONG_MIN
  // when there is none above `floor` (pmax is the contig-wide prefix max of end)
  int64_t gap_at_or_below(int64_t hi, int64_t floor) const {
    const auto &st = S->start;
    int64_t j = (int64_t)(std::upper_bound(st.begin(), st.end(), (int32_t)std::min<int64_t>(hi, INT32_MAX)) - st.begin());
    int64_t upper = hi;  // candidates (start[j - 1], upper]: the first read starting at or after them is j
    while (upper > floor) {
      if (j == 0) return upper;  // reads before the slice end at or before the window start
      if ((int64_t)S->pmax[(size_t)(j - 1)] <= upper) return upper;
      upper = st[(size_t)(j - 1)];
      --j;
      while (j > 0 && st[(size_t)(j - 1)] == upper) --j;  // equal starts: empty candidate range
    }
    return LLONG_MIN;
  }
  void reset_to(int64_t x) {
    h.assign(1, 0);
    max_end = INT32_MIN;
    const auto &st = S->start;
    const int64_t j = (int64_t)(std::lower_bound(st.begin(), st.end(), (int32_t)std::min<int64_t>(x, INT32_MAX)) - st.begin());
    if (j > nxt) nxt = j;
  }
};

}  // namespace replay_detail

template <class Emit>
void replay_heaps(const std::vector<int64_t> &rs, const std::vector<int64_t> &re, const std::vector<ReplaySet> &sets,
                  const std::vector<ReplayQuery> &queries, Emit emit) {
  using replay_detail::Queue;
  std::vector<Queue> qs(sets.size());
  for (size_t k = 0; k < sets.size(); ++k) {
    qs[k].S = &sets[k];
    qs[k].settle(rs, re);
  }
  size_t rng = 0;  // first range whose end is past the last call
  // first locus of the window's loci >= x (LociSet iterator skipTo + next), or LLONG_MAX
  auto first_locus = [&](int64_t x) -> int64_t {
    while (rng < re.size() && re[rng] <= x) ++rng;
    if (rng >= re.size()) return LLONG_MAX;
    return std::max(x, rs[rng]);
  };
  int64_t last = LLONG_MIN;  // locus of the last call
  auto snapshot = [&](const ReplayQuery &q) {
    for (size_t k = 0; k < qs.size(); ++k) {
      std::vector<int64_t> heap(qs[k].h.size() - 1);
      for (size_t i = 1; i < qs[k].h.size(); ++i) heap[i - 1] = sets[k].lo + qs[k].h[i];
      emit(q.id, (int)k, heap.data(), (int64_t)heap.size());
    }
  };
  size_t qi = 0;
  while (qi < queries.size()) {
    const int64_t target = queries[qi].pos;
    // restart from empty queues at the last coverage gap of every set before the target
    {
      const int64_t floor = last == LLONG_MIN ? LLONG_MIN + 1 : last;
      int64_t x = target;
      for (int guard = 0; guard < 64 && x > floor; ++guard) {
        int64_t y = x;
        for (auto &q : qs) y = std::min(y, q.gap_at_or_below(y, floor));
        if (y == x || y <= floor) {
          x = y;
          break;
        }
        x = y;
      }
      bool joint = x > floor;
      for (auto &q : qs) joint = joint && q.gap_at_or_below(x, floor) == x;
      if (joint && x > floor && (last == LLONG_MIN || x > last)) {
        for (auto &q : qs) {
          q.reset_to(x);
          q.settle(rs, re);
        }
        last = x - 1;
      }
    }
    // event-driven calls up to the target: the next call that changes a queue is at the first
    // locus >= min(smallest end in any queue, next pending start) (calls in between dequeue and
    // add nothing; a queue that would drain there drains whether or not the call is merged
    // with the next one)
    for (;;) {
      int64_t e = LLONG_MAX;
      for (auto &q : qs) {
        if (!q.empty()) e = std::min<int64_t>(e, q.head_end());
        e = std::min(e, q.next_start());
      }
      if (e == LLONG_MAX) break;
      const int64_t c = first_locus(std::max<int64_t>(e, last == LLONG_MIN ? e : last + 1));
      if (c == LLONG_MAX || c > target) break;
      for (auto &q : qs) q.call(c, rs, re);
      last = c;
    }
    while (qi < queries.size() && queries[qi].pos <= target) snapshot(queries[qi++]);
  }
}

}  // namespace gq
