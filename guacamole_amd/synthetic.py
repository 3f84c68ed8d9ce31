"""Synthetic coordinate-sorted reads with consistent CIGAR / MD.

Reference: i.i.d. bases, GC = 0.41.  Two haplotypes carry germline het SNVs
(rate 1e-3, VAF 0.5), hom-alt SNVs (5e-4) and indels (1e-4, 1-10 bp, 2/3 het);
an optional "tumor" layer adds somatic SNVs at VAF U(0.1, 0.5).  Reads: length
L, uniform starts (Poisson depth), 50 % reverse strand, mapq 60 (2 % uniform
0-59), base qualities from an Illumina-like mixture on 2..41 (mean ~33.5), and
substitution errors with probability 10^(-q/10).

Output is the device SoA of soa.assemble (MD already as events), so large
configurations never materialise MD strings; `to_read_set(sel)` builds the
raw ReadSet (MD strings) for any subset, which is what the CPU oracle consumes.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from .reads import OP_D, OP_I, OP_M, ReadSet
from .soa import assemble

_BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
SEED = 20261015


@dataclass
class Variants:
    snv_pos: np.ndarray      # sorted positions
    snv_alt: np.ndarray      # alt base (uint8)
    snv_haps: np.ndarray     # bitmask of haplotypes carrying it (1, 2 or 3)
    indels: List[Tuple[int, int, bytes, int]]  # (anchor pos, del_len, ins_bases, hap mask)


def random_reference(n: int, rng: np.random.Generator, gc: float = 0.41) -> np.ndarray:
    p = np.array([(1 - gc) / 2, gc / 2, gc / 2, (1 - gc) / 2])  # A C G T
    return _BASES[rng.choice(4, size=n, p=p).astype(np.uint8)]


def make_variants(ref: np.ndarray, rng: np.random.Generator, het=1e-3, hom=5e-4, indel=1e-4, L: int = 150,
                  somatic: float = 0.0) -> Variants:
    n = len(ref)
    k_het = rng.binomial(n, het)
    k_hom = rng.binomial(n, hom)
    pos = np.unique(rng.integers(0, n, size=k_het + k_hom))
    haps = np.where(rng.random(len(pos)) < het / (het + hom), rng.integers(1, 3, size=len(pos)), 3).astype(np.uint8)
    alt = _BASES[(np.searchsorted(_BASES, ref[pos]) + rng.integers(1, 4, size=len(pos))) % 4]
    indels = []
    k_ind = rng.binomial(n, indel)
    for p in np.sort(rng.integers(L, max(L + 1, n - L - 20), size=k_ind)):
        ln = int(rng.integers(1, 11))
        hm = int(rng.integers(1, 3)) if rng.random() < 2 / 3 else 3
        if rng.random() < 0.5:
            indels.append((int(p), ln, b"", hm))
        else:
            indels.append((int(p), 0, _BASES[rng.integers(0, 4, size=ln)].tobytes(), hm))
    # drop SNVs inside / adjacent to indels on the same locus to keep alignments canonical
    if indels:
        blocked = np.zeros(n + 1, dtype=bool)
        for p, dl, ins, hm in indels:
            blocked[max(0, p - 1):min(n, p + dl + 2)] = True
        keep = ~blocked[pos]
        pos, haps, alt = pos[keep], haps[keep], alt[keep]
        # indels must not overlap each other
        clean, last_end = [], -10
        for iv in indels:
            if iv[0] > last_end + 2:
                clean.append(iv)
                last_end = iv[0] + iv[1] + 1
        indels = clean
    return Variants(pos, alt, haps, indels)


def _quals(rng: np.random.Generator, n: int) -> np.ndarray:
    u = rng.random(n, dtype=np.float32)
    q = np.empty(n, dtype=np.uint8)
    a = u < 0.75
    b = (u >= 0.75) & (u < 0.95)
    c = u >= 0.95
    q[a] = rng.integers(33, 42, size=int(a.sum()), dtype=np.uint8)
    q[b] = rng.integers(20, 33, size=int(b.sum()), dtype=np.uint8)
    q[c] = rng.integers(2, 20, size=int(c.sum()), dtype=np.uint8)
    return q


_ERR_THRESH = np.array([min(65535, int(round(65536 * 10 ** (-q / 10.0)))) for q in range(256)], dtype=np.uint32)


@dataclass
class SyntheticReads:
    contig_names: List[str]
    contig_lengths: List[int]
    arrays: Dict[str, np.ndarray]   # soa.assemble layout
    ref: np.ndarray                 # reference of contig 0
    variants: Variants

    @property
    def n(self) -> int:
        return int(self.arrays["start"].shape[0])

    def to_read_set(self, sel: Optional[np.ndarray] = None) -> ReadSet:
        """Raw ReadSet (MD strings) for the reads `sel` (default: all) — oracle input."""
        a = self.arrays
        idx = np.arange(self.n) if sel is None else np.asarray(sel)
        seqs, quals, cigs, mds = [], [], [], []
        for i in idx:
            so, sl = int(a["seq_off"][i]), int(a["seq_len"][i])
            seqs.append(a["seq"][so:so + sl])
            quals.append(a["qual"][so:so + sl])
            co, nc = int(a["cigar_off"][i]), int(a["n_cigar"][i])
            cig = a["cigar"][co:co + nc]
            cigs.append(cig)
            mo, nm = int(a["md_off"][i]), int(a["n_md"][i])
            mds.append(md_string(cig, a["md_ev"][mo:mo + nm]))
        n = len(idx)
        seq_len = np.array([len(s) for s in seqs], dtype=np.int32)
        seq_off = np.zeros(n, np.int64)
        if n:
            seq_off[1:] = np.cumsum(seq_len)[:-1]
        n_cigar = np.array([len(c) for c in cigs], dtype=np.int32)
        cigar_off = np.zeros(n, np.int64)
        if n:
            cigar_off[1:] = np.cumsum(n_cigar)[:-1]
        md_b = [m.encode() for m in mds]
        md_len = np.array([len(m) for m in md_b], dtype=np.int32)
        md_off = np.zeros(n, np.int64)
        if n:
            md_off[1:] = np.cumsum(md_len)[:-1]
        cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
        return ReadSet(contig_names=list(self.contig_names), contig_lengths=list(self.contig_lengths),
                       sample_names=["synthetic"], contig=np.zeros(n, np.int32),
                       start=a["start"][idx].astype(np.int64), end=a["end"][idx].astype(np.int64),
                       mapq=a["mapq"][idx].copy(), flags=a["flags"][idx].copy(),
                       sample=a["sample"][idx].astype(np.int32), seq_off=seq_off, seq_len=seq_len,
                       seq=cat(seqs, np.uint8), qual=cat(quals, np.uint8), cigar_off=cigar_off, n_cigar=n_cigar,
                       cigar=cat(cigs, np.uint32), md_off=md_off, md_len=md_len,
                       md=np.frombuffer(b"".join(md_b), dtype=np.uint8).copy())


def md_string(cigar: np.ndarray, events: np.ndarray) -> str:
    """MD string for a read from its CIGAR and MD events (offset << 8 | ref base)."""
    ev = {int(e) >> 8: chr(int(e) & 0xFF) for e in events}
    out, run, ref = [], 0, 0
    for c in cigar:
        op, ln = int(c) & 15, int(c) >> 4
        if op in (0, 7, 8):
            for j in range(ln):
                b = ev.get(ref + j)
                if b is None:
                    run += 1
                else:
                    out.append(str(run))
                    out.append(b)
                    run = 0
            ref += ln
        elif op == OP_D:
            out.append(str(run))
            out.append("^" + "".join(ev.get(ref + j, "N") for j in range(ln)))
            run = 0
            ref += ln
        elif op == 3:
            ref += ln
    out.append(str(run))
    return "".join(out)


def generate(length: int, depth: float, seed: int = SEED, L: int = 150, contig: str = "20",
             somatic_rate: float = 0.0, chunk_reads: int = 1 << 20, variants: Optional[Variants] = None,
             ref: Optional[np.ndarray] = None, indel_rate: float = 1e-4) -> SyntheticReads:
    """Generate reads for one contig of `length` loci at mean `depth`."""
    rng = np.random.default_rng(seed)
    if ref is None:
        ref = random_reference(length, rng)
    if variants is None:
        variants = make_variants(ref, rng, L=L, indel=indel_rate)
    # haplotype sequences (SNVs only; indels handled per read)
    haps = [ref.copy(), ref.copy()]
    for h in range(2):
        m = (variants.snv_haps & (1 << h)) != 0
        haps[h][variants.snv_pos[m]] = variants.snv_alt[m]
    # optional somatic layer (tumor): SNVs on a random subset of reads, VAF U(0.1, 0.5)
    som_pos = som_alt = som_vaf = None
    if somatic_rate > 0:
        k = rng.binomial(length, somatic_rate)
        som_pos = np.unique(rng.integers(L, length - L, size=k))
        som_alt = _BASES[(np.searchsorted(_BASES, ref[som_pos]) + rng.integers(1, 4, size=len(som_pos))) % 4]
        som_vaf = rng.uniform(0.1, 0.5, size=len(som_pos))
    n_reads = int(round(depth * length / L))
    starts = np.sort(rng.integers(0, length - L, size=n_reads)).astype(np.int64)
    hap_of = rng.integers(0, 2, size=n_reads).astype(np.uint8)
    rev = (rng.random(n_reads) < 0.5).astype(np.uint8)
    mapq = np.full(n_reads, 60, np.uint8)
    low = rng.random(n_reads) < 0.02
    mapq[low] = rng.integers(0, 60, size=int(low.sum()), dtype=np.uint8)
    # which reads touch an indel on their haplotype: handled by the slow path
    special = np.zeros(n_reads, dtype=bool)
    if variants.indels:
        ip = np.array([iv[0] for iv in variants.indels], dtype=np.int64)
        ie = np.array([iv[0] + iv[1] + 1 for iv in variants.indels], dtype=np.int64)
        ih = np.array([iv[3] for iv in variants.indels], dtype=np.uint8)
        # reads with start <= anchor + del_len and start + L > anchor can see the indel
        lo = np.searchsorted(ip, starts - 0, side="left")
        hi = np.searchsorted(ip, starts + L + 12, side="right")
        for k in np.nonzero(hi > lo)[0]:
            for j in range(lo[k], hi[k]):
                if (ih[j] >> hap_of[k]) & 1 and starts[k] <= ie[j] and starts[k] + L > ip[j]:
                    special[k] = True
                    break
    seqs = np.empty(n_reads * L, dtype=np.uint8)
    quals = np.empty(n_reads * L, dtype=np.uint8)
    ar = np.arange(L, dtype=np.int64)
    for c0 in range(0, n_reads, chunk_reads):
        c1 = min(n_reads, c0 + chunk_reads)
        pos = starts[c0:c1, None] + ar[None, :]
        hp = hap_of[c0:c1, None]
        s = np.where(hp == 0, haps[0][pos], haps[1][pos])
        if som_pos is not None and len(som_pos):
            # a read carries the somatic allele with probability VAF
            li = np.searchsorted(som_pos, starts[c0:c1], side="left")
            ri = np.searchsorted(som_pos, starts[c0:c1] + L, side="left")
            for k in np.nonzero(ri > li)[0]:
                for j in range(li[k], ri[k]):
                    if rng.random() < som_vaf[j]:
                        s[k, som_pos[j] - starts[c0 + k]] = som_alt[j]
        q = _quals(rng, (c1 - c0) * L).reshape(c1 - c0, L)
        err = rng.integers(0, 65536, size=(c1 - c0) * L, dtype=np.uint32).reshape(c1 - c0, L) < _ERR_THRESH[q]
        if err.any():
            ei = np.nonzero(err)
            cur = np.searchsorted(_BASES, s[ei])
            s[ei] = _BASES[(cur + rng.integers(1, 4, size=len(cur))) % 4]
        seqs[c0 * L:c1 * L] = s.reshape(-1)
        quals[c0 * L:c1 * L] = q.reshape(-1)
    # simple reads: 150M, MD events = positions where read != reference
    cig_simple = np.uint32((L << 4) | OP_M)
    read_cigs: Dict[int, np.ndarray] = {}
    read_events: Dict[int, np.ndarray] = {}
    read_start = starts.copy()
    read_end = starts + L
    for k in np.nonzero(special)[0]:
        st, cig, sq, ev = _indel_read(ref, haps[hap_of[k]], variants.indels, int(starts[k]), L, int(hap_of[k]),
                                      seqs[k * L:(k + 1) * L])
        read_start[k] = st
        read_cigs[k] = cig
        read_events[k] = ev
        seqs[k * L:(k + 1) * L] = sq
        span = sum(int(c) >> 4 for c in cig if (int(c) & 15) in (0, 2, 3, 7, 8))
        read_end[k] = st + span
    # events for simple reads, vectorised in chunks
    ev_parts, n_md = [], np.zeros(n_reads, np.int32)
    n_mm = np.zeros(n_reads, np.uint16)
    for c0 in range(0, n_reads, chunk_reads):
        c1 = min(n_reads, c0 + chunk_reads)
        pos = starts[c0:c1, None] + ar[None, :]
        s = seqs[c0 * L:c1 * L].reshape(c1 - c0, L)
        mm = s != ref[pos]
        sp = special[c0:c1]
        mm[sp] = False
        ri, ci = np.nonzero(mm)
        evs = (ci.astype(np.uint32) << 8) | ref[pos[ri, ci]].astype(np.uint32)
        counts = np.bincount(ri, minlength=c1 - c0).astype(np.int32)
        # splice in special reads' events at their positions
        if sp.any():
            parts, pos_in = [], 0
            offs = np.concatenate([[0], np.cumsum(counts)])
            for k in range(c1 - c0):
                if sp[k]:
                    e = read_events[c0 + k]
                    parts.append(e)
                    counts[k] = len(e)
                else:
                    parts.append(evs[offs[k]:offs[k + 1]])
            evs = np.concatenate(parts) if parts else evs
        n_md[c0:c1] = counts
        ev_parts.append(evs.astype(np.uint32))
    md_ev = np.concatenate(ev_parts) if ev_parts else np.zeros(0, np.uint32)
    md_off = np.zeros(n_reads, np.int64)
    if n_reads:
        md_off[1:] = np.cumsum(n_md.astype(np.int64))[:-1]
    # mismatch counts (events on M positions): simple reads = all events
    n_mm[:] = np.minimum(n_md, 65535)
    for k, cig in read_cigs.items():
        n_mm[k] = _count_mismatches(cig, read_events[k])
    # CIGAR pool
    n_cigar = np.ones(n_reads, np.int32)
    for k, cig in read_cigs.items():
        n_cigar[k] = len(cig)
    cigar_off = np.zeros(n_reads, np.int64)
    if n_reads:
        cigar_off[1:] = np.cumsum(n_cigar.astype(np.int64))[:-1]
    cigar = np.full(int(n_cigar.sum()), cig_simple, dtype=np.uint32)
    for k, cig in read_cigs.items():
        cigar[cigar_off[k]:cigar_off[k] + len(cig)] = cig
    seq_off = np.arange(n_reads, dtype=np.int64) * L
    seq_len = np.full(n_reads, L, np.int32)
    # re-sort by start (indel reads may have moved); stable
    order = np.argsort(read_start, kind="stable")
    if not np.all(order == np.arange(n_reads)):
        seq_off, seq_len = seq_off[order], seq_len[order]
        n_cigar, cigar_off = n_cigar[order], cigar_off[order]
        n_md, md_off, n_mm = n_md[order], md_off[order], n_mm[order]
        read_start, read_end = read_start[order], read_end[order]
        mapq, rev = mapq[order], rev[order]
    arrays = assemble(np.zeros(n_reads, np.int32), read_start, read_end, mapq, rev, np.zeros(n_reads, np.uint8),
                      seq_off, seq_len, seqs, quals, cigar_off, n_cigar, cigar, md_off, n_md, n_mm, md_ev, 1, 1)
    return SyntheticReads([contig], [length], arrays, ref, variants)


def _count_mismatches(cig, events) -> int:
    mpos = set()
    ref = 0
    for c in cig:
        op, ln = int(c) & 15, int(c) >> 4
        if op in (0, 7, 8):
            mpos.update(range(ref, ref + ln))
        if op in (0, 2, 3, 7, 8):
            ref += ln
    return sum(1 for e in events if (int(e) >> 8) in mpos)


def _indel_read(ref, hap, indels, start, L, h, seq_noisy):
    """Build one read from haplotype `h` starting at reference `start` through any indels
    (error-free bases; an insertion that would not be followed by a matched base is
    left out).  Returns (start, cigar u32 array, sequence, md events)."""
    ind = {iv[0]: iv for iv in indels if (iv[3] >> h) & 1}
    for p, dl, ins, hm in ind.values():  # a start inside a deleted run moves past it
        if dl and p < start <= p + dl:
            start = p + dl + 1
    ops: List[List[int]] = []

    def push(op, n):
        if ops and ops[-1][0] == op:
            ops[-1][1] += n
        else:
            ops.append([op, n])

    seq = bytearray()
    events = []
    p, i = start, 0
    while i < L:
        b = int(hap[p])
        seq.append(b)
        push(OP_M, 1)
        if b != int(ref[p]):
            events.append(((p - start) << 8) | int(ref[p]))
        i += 1
        if p in ind and i < L:
            _, dl, ins, _ = ind[p]
            if dl:
                push(OP_D, dl)
                for j in range(1, dl + 1):
                    events.append(((p + j - start) << 8) | int(ref[p + j]))
                p += dl
            elif ins and i + len(ins) < L:
                push(OP_I, len(ins))
                seq.extend(ins)
                i += len(ins)
        p += 1
    cig = np.array([(n << 4) | op for op, n in ops], dtype=np.uint32)
    events.sort()
    return start, cig, np.frombuffer(bytes(seq), dtype=np.uint8), np.array(events, dtype=np.uint32)
