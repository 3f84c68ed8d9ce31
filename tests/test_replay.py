"""Heap-order replay (guacamole_amd/csrc/gq_replay.h, built here for the host) against the
oracle's restatement of SlidingWindow's Scala 2.10 PriorityQueue (SlidingWindow.scala:45-187,
advanceMultipleWindows with skipEmpty).  The product resolves the pileup reference base at
loci where the reads' MD tags disagree from this heap array (Pileup.scala:157-165); the replay
skips calls that change no queue and restarts at coverage gaps, so it is checked here against
the oracle's locus-by-locus queue on random read sets: one and two sets (the somatic caller
advances two windows together), several tasks, ranges with holes, dense and sparse queries."""
import ctypes as C
import os
import subprocess
import types

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def rp(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("rp") / "librp.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", so,
                           os.path.join(ROOT, "tests", "native", "replay_check.cpp")])
    lib = C.CDLL(so)
    lib.rp_replay.restype = C.c_int
    return lib


def _reads(rng, length, n, clustered):
    if clustered:  # clusters separated by coverage gaps
        centers = rng.integers(0, length, size=max(1, n // 40))
        starts = np.clip(rng.choice(centers, size=n) + rng.integers(-150, 150, size=n), 0, length - 1)
    else:
        starts = rng.integers(0, length, size=n)
    starts = np.sort(starts).astype(np.int64)
    spans = rng.choice([1, 5, 30, 76, 100, 100, 100, 101, 150, 150, 300], size=n).astype(np.int64)
    ends = np.minimum(starts + spans, length)
    spans = np.maximum(ends - starts, 1)
    lens = spans.astype(np.int32)
    cig = (lens.astype(np.uint32) << 4)  # <len>M
    md = "".join(str(int(x)) for x in lens).encode()
    md_len = np.array([len(str(int(x))) for x in lens], np.int32)
    md_off = np.concatenate([[0], np.cumsum(md_len)[:-1]]).astype(np.int64)
    seq_off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    rs = types.SimpleNamespace(
        n=n, contig=np.zeros(n, np.int32), start=starts, mapq=np.full(n, 60, np.uint8), flags=np.zeros(n, np.uint8),
        sample=np.zeros(n, np.int32), seq_off=seq_off, seq_len=lens, seq=np.full(int(lens.sum()), ord("A"), np.uint8),
        qual=np.full(int(lens.sum()), 30, np.uint8), cigar_off=np.arange(n, dtype=np.int64),
        n_cigar=np.ones(n, np.int32), cigar=cig, md_off=md_off, md_len=md_len, md=np.frombuffer(md, np.uint8),
        contig_names=["chr1"])
    return rs, starts.astype(np.int32), (starts + spans).astype(np.int32)


def _product(lib, sets, ranges, queries):
    """sets: [(start, end)] per set; ranges: the window's [(s, e)]; queries: sorted loci."""
    keep, ns, st_p, en_p, pm_p, los = [], [], [], [], [], []
    r0, r1 = ranges[0][0], ranges[-1][1]
    for start, end in sets:
        pmax = np.maximum.accumulate(end).astype(np.int32)
        lo = int(np.searchsorted(pmax, r0, side="right"))
        hi = int(np.searchsorted(start, r1, side="left"))
        hi = max(hi, lo)
        a, b, c = (np.ascontiguousarray(x[lo:hi], np.int32) for x in (start, end, pmax))
        keep += [a, b, c]
        ns.append(hi - lo)
        los.append(lo)
        st_p.append(a.ctypes.data_as(C.POINTER(C.c_int32)))
        en_p.append(b.ctypes.data_as(C.POINTER(C.c_int32)))
        pm_p.append(c.ctypes.data_as(C.POINTER(C.c_int32)))
    k = len(sets)
    rs = np.array([r[0] for r in ranges], np.int64)
    re = np.array([r[1] for r in ranges], np.int64)
    q = np.array(queries, np.int32)
    out, n = C.c_char_p(), C.c_int64()
    rc = lib.rp_replay(C.c_int(k), (C.c_int64 * k)(*ns), (C.POINTER(C.c_int32) * k)(*st_p),
                       (C.POINTER(C.c_int32) * k)(*en_p), (C.POINTER(C.c_int32) * k)(*pm_p), (C.c_int64 * k)(*los),
                       C.c_int64(len(ranges)), rs.ctypes.data_as(C.c_void_p), re.ctypes.data_as(C.c_void_p),
                       C.c_int64(len(q)), q.ctypes.data_as(C.c_void_p), C.byref(out), C.byref(n))
    assert rc == 0
    text = C.string_at(out, n.value).decode()
    lib.rp_free(out)
    res = {}
    for line in text.splitlines():
        f = line.split("\t")
        res.setdefault(int(f[0]), [None] * k)[int(f[1])] = [int(x) for x in f[2].split(",")] if f[2] else []
    return res


@pytest.mark.parametrize("seed", range(12))
def test_replay_matches_oracle_heap(rp, seed):
    rng = np.random.default_rng(20261016 + seed)
    length = 12000
    n_sets = 1 + (seed % 2)
    clustered = seed % 3 != 0
    data = [_reads(rng, length, int(rng.integers(300, 900)), clustered) for _ in range(n_sets)]
    # tasks: contiguous pieces, some with holes (several ranges in one window)
    cuts = sorted(set(int(x) for x in rng.integers(1, length - 1, size=int(rng.integers(0, 4)))))
    bounds = [0] + cuts + [length]
    ranges, tasks = [], []
    for t in range(len(bounds) - 1):
        a, b = bounds[t], bounds[t + 1]
        if seed % 4 == 1 and b - a > 400:  # a hole inside the task's loci
            h0 = int(rng.integers(a + 100, b - 200))
            pieces = [(a, h0), (h0 + int(rng.integers(1, 150)), b)]
        else:
            pieces = [(a, b)]
        for p in pieces:
            if p[1] > p[0]:
                ranges.append(p)
                tasks.append(t)
    loci = (np.zeros(len(ranges), np.int32), np.array([r[0] for r in ranges]), np.array([r[1] for r in ranges]),
            np.array(tasks, np.int64))
    want = O.heap_orders([d[0] for d in data], loci)
    assert want, "no visited loci"
    for t in sorted(set(tasks)):
        wr = [r for r, tt in zip(ranges, tasks) if tt == t]
        visited = sorted(l for (_, l) in want if any(a <= l < b for a, b in wr))
        if not visited:
            continue
        sparse = sorted(rng.choice(visited, size=max(1, len(visited) // 40), replace=False).tolist())
        for qset in (visited, sparse, [visited[-1]]):
            got = _product(rp, [(d[1], d[2]) for d in data], wr, qset)
            for l in qset:
                assert got[l] == want[(0, l)], "task %d locus %d: heap arrays differ" % (t, l)
