"""ReadSet -> device SoA layout consumed by libgqpileup (include/gqpileup.h: gq_reads).

The MD tag is parsed here into *events* — (offset from read start) << 8 | base —
for mismatching reference bases on M/=/X positions and deleted reference bases
on D positions, with N (skipped-region) gaps advancing the reference position.
This restates ADAM MdTag(md, start, cigar) as used by MappedRead.apply
(reads/MappedRead.scala:114-131, MDTagUtils.scala:23-78): digits = matches,
letters = mismatches, '^' + letters = deletions.  Pinned by MDTagUtilsSuite
cases in tests/test_soa.py.

Layout in HBM (one buffer per field, reads sorted by (contig, start)):
  start/end/pmax_end i32, mapq/flags/sample u8, seq_off i64, seq_len i32,
  cigar_off i64, n_cigar i32, md_off i64, n_md i32, n_mismatch u16,
  pools: seq u8, qual u8, cigar u32, md_ev u32.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from .reads import OP_D, OP_EQ, OP_M, OP_N, OP_X, ReadSet

_MD_CONSUMED = (OP_M, OP_EQ, OP_X, OP_D)
_REF_CONSUMING = (OP_M, OP_D, OP_N, OP_EQ, OP_X)


class MdParseError(ValueError):
    pass


def md_events(md: bytes, start: int, cigar_ops: List[Tuple[int, int]]) -> Tuple[List[int], int]:
    """-> (sorted events (offset << 8 | base), number of mismatches)."""
    # reference offsets (relative to start) consumed by MD, N gaps skipped
    offs: List[int] = []
    ref = 0
    for op, ln in cigar_ops:
        if op in _MD_CONSUMED:
            offs.extend(range(ref, ref + ln))
        if op in _REF_CONSUMING:
            ref += ln

    def at(k: int) -> int:
        if k < len(offs):
            return offs[k]
        return (offs[-1] if offs else -1) + (k - len(offs) + 1)

    s = md.upper()
    i, k, n = 0, 0, len(s)
    ev: Dict[int, int] = {}
    mism = 0

    def digits():
        nonlocal i, k
        j = i
        while j < n and 48 <= s[j] <= 57:
            j += 1
        if j == i:
            raise MdParseError("MdTag %r: digit expected at %d" % (md, i))
        k += int(s[i:j])
        i = j

    if n == 0:
        return [], 0
    digits()
    while i < n:
        if s[i] == ord("^"):
            i += 1
            while i < n and 65 <= s[i] <= 90:
                ev[at(k)] = s[i]
                k += 1
                i += 1
        elif 65 <= s[i] <= 90:
            while i < n and 65 <= s[i] <= 90:
                ev[at(k)] = s[i]
                mism += 1
                k += 1
                i += 1
        else:
            raise MdParseError("MdTag %r: invalid character" % md)
        digits()
    out = [(o << 8) | b for o, b in sorted(ev.items()) if o >= 0]
    return out, mism


def pack(rs: ReadSet) -> Dict[str, np.ndarray]:
    """Build the gq_reads host arrays for a ReadSet (cached on the ReadSet).  MD events come
    from libgqingest (gq_md_count / gq_md_fill); md_events above is their Python statement,
    the checker in tests/test_ingest.py."""
    if rs._gq is not None:
        return rs._gq
    from .ingest import md_events as native_md_events  # libgqingest; raises if not built
    n_md, n_mm, md_off, md_ev = native_md_events(rs.cigar_off, rs.n_cigar, rs.cigar, rs.md_off, rs.md_len, rs.md)
    out = assemble(rs.contig, rs.start, rs.end, rs.mapq, rs.flags, rs.sample, rs.seq_off, rs.seq_len, rs.seq,
                   rs.qual, rs.cigar_off, rs.n_cigar, rs.cigar, md_off, n_md, n_mm, md_ev, len(rs.contig_names),
                   max(1, len(rs.sample_names)))
    out["sample_hash"] = sample_hashes(rs.sample_names, int(out["n_samples"]))
    rs._gq = out
    return out


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode (over UTF-16 code units), as an unsigned 32-bit value."""
    h = 0
    u = s.encode("utf-16-be")
    for i in range(0, len(u), 2):
        h = (31 * h + ((u[i] << 8) | u[i + 1])) & 0xFFFFFFFF
    return h


def sample_hashes(sample_names, n_samples: int) -> np.ndarray:
    """gq_reads.sample_hash: the Scala ## (String.hashCode) of each sample slot's name; a slot
    past the names is the reference's "default" sample (Pileup.scala:58)."""
    names = list(sample_names)
    return np.array([java_string_hash(names[k] if k < len(names) else "default") for k in range(n_samples)],
                    np.uint32)


def assemble(contig, start, end, mapq, flags, sample, seq_off, seq_len, seq, qual, cigar_off, n_cigar, cigar,
             md_off, n_md, n_mismatch, md_ev, n_contigs: int, n_samples: int) -> Dict[str, np.ndarray]:
    contig = np.asarray(contig, np.int32)
    begin = np.searchsorted(contig, np.arange(n_contigs + 1), side="left").astype(np.int64)
    start32 = np.asarray(start, np.int32)
    end32 = np.asarray(end, np.int32)
    pmax = np.empty_like(end32)
    for c in range(n_contigs):
        b, e = begin[c], begin[c + 1]
        if e > b:
            pmax[b:e] = np.maximum.accumulate(end32[b:e])
    return dict(contig_read_begin=begin, start=start32, end=end32, pmax_end=pmax,
                mapq=np.asarray(mapq, np.uint8), flags=np.asarray(flags, np.uint8),
                sample=np.asarray(sample, np.uint8), seq_off=np.asarray(seq_off, np.int64),
                seq_len=np.asarray(seq_len, np.int32), cigar_off=np.asarray(cigar_off, np.int64),
                n_cigar=np.asarray(n_cigar, np.int32), md_off=np.asarray(md_off, np.int64),
                n_md=np.asarray(n_md, np.int32), n_mismatch=np.asarray(n_mismatch, np.uint16),
                seq=np.asarray(seq, np.uint8), qual=np.asarray(qual, np.uint8),
                cigar=np.asarray(cigar, np.uint32), md_ev=np.asarray(md_ev, np.uint32),
                n_contigs=np.int64(n_contigs), n_samples=np.int64(n_samples))
