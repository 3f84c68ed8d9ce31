"""LociSet / LociMap and loci partitioning — host side of the pileup path.

Restates (paths relative to /root/reference/src/main/scala/org/hammerlab/guacamole/):

* ``LociSet.Builder.putExpression`` / ``result``        LociSet.scala:118-217
  - ``"all"`` => every contig ``[0, length - 1)``     (LociSet.scala:205-207, quirk)
  - bare ``contig`` => ``[0, length)``                 (LociSet.scala:209-213)
* ``LociMap.Builder.result`` range coalescing          LociMap.scala:186-235
* contigs iterate lexicographically                    LociMap.scala:39-42
* ``LociMap.take`` / ``asInverseMap``                    LociMap.scala:51-62, 110-146
* ``DistributedUtil.partitionLociUniformly``           DistributedUtil.scala:83-108
* ``DistributedUtil.partitionLociByApproximateDepth``  DistributedUtil.scala:162-251

Everything here is O(ranges) / O(reads) integer bookkeeping on the host: it
decides *which* loci each GPU / task owns; the per-locus work runs on the GPU.
"""
from __future__ import annotations

import bisect
import math
import re
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np


def _java_round(x: float) -> int:
    """java.lang.Math.round(double) (used via scala.math.round)."""
    if math.isnan(x):
        return 0
    return int(math.floor(x + 0.5))


class _RangeMap:
    """Guava TreeRangeMap<Long, T> restricted to what LociMap uses: closed-open
    ranges, put() overwrites the covered part of existing entries."""

    def __init__(self) -> None:
        self.starts: List[int] = []
        self.ends: List[int] = []
        self.values: List[object] = []

    def get_entry(self, locus: int):
        i = bisect.bisect_right(self.starts, locus) - 1
        if i >= 0 and self.starts[i] <= locus < self.ends[i]:
            return self.starts[i], self.ends[i], self.values[i]
        return None

    def put(self, start: int, end: int, value) -> None:
        if end <= start:
            return
        new_s, new_e, new_v = [], [], []
        for s, e, v in zip(self.starts, self.ends, self.values):
            if e <= start or s >= end:
                new_s.append(s), new_e.append(e), new_v.append(v)
                continue
            if s < start:
                new_s.append(s), new_e.append(start), new_v.append(v)
            if e > end:
                new_s.append(end), new_e.append(e), new_v.append(v)
        new_s.append(start), new_e.append(end), new_v.append(value)
        order = sorted(range(len(new_s)), key=lambda k: new_s[k])
        self.starts = [new_s[k] for k in order]
        self.ends = [new_e[k] for k in order]
        self.values = [new_v[k] for k in order]

    def items(self):
        return list(zip(self.starts, self.ends, self.values))


class LociMapSingleContig:
    def __init__(self, contig: str, entries: Sequence[Tuple[int, int, object]]):
        self.contig = contig
        self.entries = sorted(entries)
        self._starts = [e[0] for e in self.entries]

    def get(self, locus: int):
        i = bisect.bisect_right(self._starts, locus) - 1
        if i >= 0 and self.entries[i][0] <= locus < self.entries[i][1]:
            return self.entries[i][2]
        return None

    def get_all(self, start: int, end: int) -> set:
        """SingleContig.getAll: values of ranges intersecting [start, end)."""
        if end <= start:
            return set()
        out = set()
        i = max(0, bisect.bisect_right(self._starts, start) - 1)
        while i < len(self.entries) and self.entries[i][0] < end:
            s, e, v = self.entries[i]
            if e > start:
                out.add(v)
            i += 1
        return out

    def intersects(self, start: int, end: int) -> bool:
        return bool(self.get_all(start, end))

    @property
    def ranges(self) -> List[Tuple[int, int]]:
        return [(s, e) for s, e, _ in self.entries]

    @property
    def count(self) -> int:
        return sum(e - s for s, e, _ in self.entries)


class LociMap:
    """LociMap[T]: per-contig range -> value map (LociMap.scala:37-341)."""

    def __init__(self, by_contig: Optional[Dict[str, LociMapSingleContig]] = None):
        self.by_contig = {k: v for k, v in (by_contig or {}).items() if v.entries}

    @property
    def contigs(self) -> List[str]:
        return sorted(self.by_contig)  # TreeMap of contig names: lexicographic

    def on_contig(self, contig: str) -> LociMapSingleContig:
        return self.by_contig.get(contig) or LociMapSingleContig(contig, [])

    @property
    def count(self) -> int:
        return sum(c.count for c in self.by_contig.values())

    def entries(self) -> List[Tuple[str, int, int, object]]:
        return [(c, s, e, v) for c in self.contigs for (s, e, v) in self.on_contig(c).entries]

    def as_inverse_map(self) -> Dict[object, "LociSet"]:
        builders: Dict[object, LociMapBuilder] = {}
        for c, s, e, v in self.entries():
            builders.setdefault(v, LociMapBuilder()).put(c, s, e, 0)
        return {v: LociSet(b.result()) for v, b in builders.items()}

    def take(self, n: int) -> Tuple["LociMap", "LociMap"]:
        assert n <= self.count, "Can't take %d loci from a map of size %d." % (n, self.count)
        if n == 0:
            return LociMap(), self
        if n == self.count:
            return self, LociMap()
        first, second = LociMapBuilder(), LociMapBuilder()
        remaining, done = n, False
        for c, s, e, v in self.entries():
            if done:
                second.put(c, s, e, v)
            elif remaining >= e - s:
                first.put(c, s, e, v)
                remaining -= e - s
            else:
                first.put(c, s, s + remaining, v)
                second.put(c, s + remaining, e, v)
                done = True
        return first.result(), second.result()

    def __eq__(self, other) -> bool:
        return isinstance(other, LociMap) and self.entries() == other.entries()

    def __str__(self) -> str:
        return ",".join("%s:%d-%d=%s" % (c, s, e, v) for c, s, e, v in self.entries())

    __repr__ = __str__


class LociMapBuilder:
    """LociMap.Builder (LociMap.scala:186-235), including its coalescing rule."""

    def __init__(self) -> None:
        self.data: Dict[str, List[Tuple[int, int, object]]] = {}

    def put(self, contig: str, start: int, end: int, value) -> "LociMapBuilder":
        assert end >= start
        if end > start:
            self.data.setdefault(contig, []).append((start, end, value))
        return self

    def put_set(self, loci: "LociSet", value) -> "LociMapBuilder":
        for c in loci.contigs:
            for s, e in loci.on_contig(c).ranges:
                self.put(c, s, e, value)
        return self

    def result(self) -> LociMap:
        out = {}
        for contig, items in self.data.items():
            rm = _RangeMap()
            for start, end, value in items:
                ex = rm.get_entry(start - 1)
                if ex is not None and ex[2] == value:
                    start = ex[0]
                ex = rm.get_entry(end)
                if ex is not None and ex[2] == value:
                    end = ex[1]
                rm.put(start, end, value)
            out[contig] = LociMapSingleContig(contig, rm.items())
        return LociMap(out)


class LociSet:
    """LociSet (LociSet.scala:39-353), a LociMap[Long] with all values 0."""

    def __init__(self, m: Optional[LociMap] = None):
        self.map = m or LociMap()

    @property
    def contigs(self) -> List[str]:
        return self.map.contigs

    def on_contig(self, contig: str) -> LociMapSingleContig:
        return self.map.on_contig(contig)

    @property
    def count(self) -> int:
        return self.map.count

    def ranges(self) -> List[Tuple[str, int, int]]:
        return [(c, s, e) for c, s, e, _ in self.map.entries()]

    def take(self, n: int) -> Tuple["LociSet", "LociSet"]:
        if n == 0:
            return LociSet(), self
        if n == self.count:
            return self, LociSet()
        a, b = self.map.take(n)
        return LociSet(a), LociSet(b)

    def union(self, other: "LociSet") -> "LociSet":
        b = LociMapBuilder()
        for c, s, e in self.ranges() + other.ranges():
            b.put(c, s, e, 0)
        return LociSet(b.result())

    def is_empty(self) -> bool:
        return self.count == 0

    def __eq__(self, other) -> bool:
        return isinstance(other, LociSet) and self.map == other.map

    def __str__(self) -> str:
        return ",".join("%s:%d-%d" % r for r in self.ranges())

    __repr__ = __str__

    @staticmethod
    def parse(expr: str) -> "LociSetBuilder":
        return LociSetBuilder().put_expression(expr)


_CONTIG_AND_LOCI = re.compile(r"([\w.]+):(\d+)-(\d+)", re.UNICODE)
_CONTIG_ONLY = re.compile(r"([\w.]+)", re.UNICODE)


class LociSetBuilder:
    """LociSet.Builder (LociSet.scala:118-217)."""

    def __init__(self) -> None:
        self.fully_resolved = True
        self.contains_all = False
        self._ranges: List[Tuple[str, int, Optional[int]]] = []

    def put_all_contigs(self) -> "LociSetBuilder":
        self.contains_all = True
        self.fully_resolved = False
        return self

    def put(self, contig: str, start: int = 0, end: Optional[int] = None) -> "LociSetBuilder":
        assert start >= 0
        assert end is None or end >= start
        if not self.contains_all:
            self._ranges.append((contig, start, end))
            if end is None:
                self.fully_resolved = False
        return self

    def put_expression(self, loci: str) -> "LociSetBuilder":
        if loci == "all":
            return self.put_all_contigs()
        # Scala Regex extractors require a full match (Regex.unapplySeq).
        for piece in re.sub(r"\s", "", loci).split(","):
            if piece == "":
                continue
            m = _CONTIG_AND_LOCI.fullmatch(piece)
            if m:
                self.put(m.group(1), int(m.group(2)), int(m.group(3)))
                continue
            if _CONTIG_ONLY.fullmatch(piece):
                self.put(piece)
                continue
            raise ValueError("Couldn't parse loci range: %s" % piece)
        return self

    def result(self, contig_lengths: Optional[Dict[str, int]] = None) -> LociSet:
        assert contig_lengths is not None or self.fully_resolved
        if contig_lengths is not None:
            for contig, start, end in self._ranges:
                if contig not in contig_lengths:
                    raise ValueError("No such contig: %s" % contig)
                if end is not None and end > contig_lengths[contig]:
                    raise ValueError("Invalid range %d-%d for contig '%s' which has length %d"
                                     % (start, end, contig, contig_lengths[contig]))
        b = LociMapBuilder()
        if self.contains_all:
            for contig, length in contig_lengths.items():
                b.put(contig, 0, length - 1, 0)  # LociSet.scala:205-207: "all" drops the last base
        else:
            for contig, start, end in self._ranges:
                b.put(contig, start, contig_lengths[contig] if end is None else end, 0)
        return LociSet(b.result())


def partition_loci_uniformly(tasks: int, loci: LociSet) -> LociMap:
    """DistributedUtil.partitionLociUniformly (DistributedUtil.scala:83-108)."""
    assert tasks >= 1, "`tasks` (--parallelism) should be >= 1"
    loci_per_task = max(1.0, loci.count / float(tasks))
    b = LociMapBuilder()
    assigned = 0
    task = 0

    def remaining() -> int:
        return _java_round((task + 1) * loci_per_task - assigned)

    for contig in loci.contigs:
        for start, end in loci.on_contig(contig).ranges:
            while start < end:
                length = min(remaining(), end - start)
                b.put(contig, start, start + length, task)
                start += length
                assigned += length
                if remaining() == 0:
                    task += 1
    result = b.result()
    assert assigned == loci.count
    return result


def _region_counts(micro: LociMap, regions: Iterable[Tuple[str, np.ndarray, np.ndarray]],
                   n_micro: int) -> np.ndarray:
    """countByValue of getAll(region.start, region.end) over micro partitions
    (DistributedUtil.scala:181-189), vectorised per contig."""
    counts = np.zeros(n_micro, dtype=np.int64)
    for contig, starts, ends in regions:
        sc = micro.on_contig(contig)
        if not sc.entries or len(starts) == 0:
            continue
        rs = np.array([e[0] for e in sc.entries], dtype=np.int64)
        re_ = np.array([e[1] for e in sc.entries], dtype=np.int64)
        rv = np.array([e[2] for e in sc.entries], dtype=np.int64)
        # collapse consecutive entries with the same value into runs (getAll is a Set)
        run_id = np.concatenate([[0], np.cumsum(rv[1:] != rv[:-1])])
        run_val = rv[np.concatenate([[0], np.nonzero(rv[1:] != rv[:-1])[0] + 1])]
        starts = np.asarray(starts, dtype=np.int64)
        ends = np.asarray(ends, dtype=np.int64)
        ok = ends > starts
        starts, ends = starts[ok], ends[ok]
        first = np.searchsorted(re_, starts, side="right")     # first entry with end > start
        last = np.searchsorted(rs, ends, side="left") - 1       # last entry with start < end
        hit = first <= last
        first, last = first[hit], last[hit]
        nr = len(run_val) + 1
        diff = (np.bincount(run_id[first], minlength=nr) - np.bincount(run_id[last] + 1, minlength=nr)).astype(np.int64)
        counts_runs = np.cumsum(diff)[:-1]
        np.add.at(counts, run_val, counts_runs)
    return counts


def partition_loci_by_approximate_depth(tasks: int, loci_used: LociSet, accuracy: int,
                                        *region_sets) -> LociMap:
    """DistributedUtil.partitionLociByApproximateDepth (DistributedUtil.scala:162-251).

    ``region_sets``: each an iterable of (contig, starts, ends) arrays."""
    assert tasks >= 1
    assert loci_used.count > 0
    assert len(region_sets) > 0
    n_micro = micro_partition_count(tasks, loci_used, accuracy)
    micro = partition_loci_uniformly(n_micro, loci_used)
    counts = np.zeros(n_micro, dtype=np.int64)
    for rs in region_sets:
        counts += _region_counts(micro, rs, n_micro)
    return partition_loci_by_counts(tasks, loci_used, micro, counts)


def micro_partition_count(tasks: int, loci_used: LociSet, accuracy: int) -> int:
    """numMicroPartitions (DistributedUtil.scala:172-173)."""
    return accuracy * tasks if accuracy * tasks < loci_used.count else loci_used.count


def partition_loci_by_counts(tasks: int, loci_used: LociSet, micro: LociMap, counts: np.ndarray) -> LociMap:
    """The second half of partitionLociByApproximateDepth (DistributedUtil.scala:191-251): the
    greedy proportional take over micro partitions, from their region counts (computed in one
    process, or summed over ranks that each counted their own micro partitions)."""
    n_micro = len(counts)
    total = int(counts.sum())
    regions_per_task = max(1.0, total / float(tasks))
    inverse = micro.as_inverse_map()
    b = LociMapBuilder()
    regions_assigned = 0.0
    task = 0

    def remaining_for_task() -> int:
        return _java_round((task + 1) * regions_per_task - regions_assigned)

    for micro_task in range(n_micro):
        s = inverse[micro_task]
        in_set = int(counts[micro_task])
        while not s.is_empty():
            if in_set == 0:
                b.put_set(s, task)
                s = LociSet()
            else:
                if remaining_for_task() == 0:
                    task += 1
                assert remaining_for_task() > 0
                assert task < tasks
                fraction = min(1.0, remaining_for_task() / float(in_set))
                loci_to_take = max(1, int(fraction * s.count))
                regions_to_take = int(fraction * in_set)
                cur, s = s.take(loci_to_take)
                b.put_set(cur, task)
                regions_assigned += regions_to_take
                in_set -= regions_to_take
    result = b.result()
    assert result.count == loci_used.count
    return result


def flatten_partitions(partitions: LociMap, contig_index: Dict[str, int]):
    """LociMap[Long] -> flat (contig_id, start, end, task) arrays in the order the
    reference emits results: task ascending, contigs lexicographic, start ascending."""
    rows = sorted(((v, c, s, e) for c, s, e, v in partitions.entries()), key=lambda r: (r[0], r[1], r[2]))
    contig = np.array([contig_index[r[1]] for r in rows], dtype=np.int32)
    start = np.array([r[2] for r in rows], dtype=np.int64)
    end = np.array([r[3] for r in rows], dtype=np.int64)
    task = np.array([r[0] for r in rows], dtype=np.int64)
    return contig, start, end, task
