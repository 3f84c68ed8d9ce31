// gq_replay.h — host replay of SlidingWindow's priority queue for heap-order-dependent loci.
//
// Pileup.referenceBaseAtLocus (pileup/Pileup.scala:157-165) takes the MD-derived base of the
// first read, in currentRegions() order, whose base is standard.  currentRegions() is the
// Scala 2.10 mutable.PriorityQueue's heap array (windowing/SlidingWindow.scala:62-73), whose
// layout depends on every enqueue / dequeue since the window (one per task and contig,
// DistributedUtil.scala:473-486) began.  Where the overlapping reads' MD tags disagree
// (GQ_FLAG_AMBIGUOUS_REF loci, rare) the kernels list the locus and this module replays the
// window's queue(s) on the host to recover the heap array at that locus.
//
// The replay is event-driven: calls of setCurrentLocus that neither dequeue nor add reads
// leave the heap unchanged and are skipped, and the replay restarts from an empty queue at
// the last coverage gap before a queried locus (no read starting before x covers x, so every
// queue drains at the first call >= x).  Cost: O(reads between the gap and the locus x log D).
#pragma once
#include <stdint.h>

#include <vector>

namespace gq {

// Host copy of reads [lo, lo + n) of one contig of a resident read set (index order).
struct ReplaySet {
  int64_t lo = 0;
  std::vector<int32_t> start, end, pmax;  // pmax = prefix max of end over the whole contig
};

struct ReplayQuery {
  int32_t pos;  // a visited locus of the window
  int32_t id;   // caller's tag
};

// Replays the queues of one window (its sorted, disjoint loci ranges [rs[i], re[i])) over
// the read sets `sets` (one queue per set, advanced together as advanceMultipleWindows does,
// SlidingWindow.scala:149-187, skipEmpty = true) and calls emit(id, set, heap, n) with each
// set's heap array (absolute read indices, root first) at every queried locus.  Queries must
// be sorted by pos.  Reads that overlap none of the ranges are not part of the window (they
// are not shuffled to the task, DistributedUtil.scala:584-597).
template <class Emit>
void replay_heaps(const std::vector<int64_t> &rs, const std::vector<int64_t> &re, const std::vector<ReplaySet> &sets,
                  const std::vector<ReplayQuery> &queries, Emit emit);

}  // namespace gq

#include "gq_replay_impl.h"
