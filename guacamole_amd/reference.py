"""Reference genome input (`--reference-fasta`) and MD tags rebuilt from it.

Restates (paths relative to /root/reference/src/main/scala/org/hammerlab/guacamole/):
  * FASTA -> per-contig unmasked bytes   reference/ReferenceBroadcast.scala:39-55 (htsjdk
    FastaSequenceFile with truncateNamesAtWhitespace = true), Bases.unmaskBases Bases.scala:115-125
  * contig lookup / ContigNotFound       reference/ReferenceBroadcast.scala:26-37, :57-58
  * MD built from the reference          reference/ReferenceGenome.scala:41-47 -> ADAM's
    MdTag(readSequence, referenceSequence, cigar, start) (adam-core 0.18.x, a dependency absent
    from /root/reference; its published algorithm is restated in `md_from_reference`)
  * when the MD is built                 reads/Read.scala:217-250: a mapped read keeps its own MD
    unless it has none or --recompute-md-tags; --recompute-md-tags without a reference is an error
  * the pileup's reference base          DistributedUtil.scala:266-268: with a reference every
    pileup takes the FASTA base (somatic-standard only: SomaticStandardCaller.scala:57, :75, :118)

The device side is `gq_reference_upload` (include/gqpileup.h): the contigs of a read set's contig
list in HBM, consulted by gq_somatic_standard_ref for every pileup's reference base.
"""
from __future__ import annotations

import gzip
from dataclasses import replace
from typing import Tuple, Dict, Iterable, List, Optional

import numpy as np

from .reads import CIGAR_OPS, ReadSet

# CIGAR op codes (BAM numbering) that consume query / reference bases
_OP_M, _OP_I, _OP_D, _OP_N, _OP_S, _OP_H, _OP_P, _OP_EQ, _OP_X = range(9)
_CONSUMES_READ = {_OP_M, _OP_I, _OP_S, _OP_EQ, _OP_X}
_CONSUMES_REF = {_OP_M, _OP_D, _OP_N, _OP_EQ, _OP_X}

# Bases.unmaskBases: a c g t n -> upper case, any other byte `toChar.toUpper`
_UNMASK = bytes(range(256)).upper()


class ContigNotFound(KeyError):
    """ReferenceBroadcast.scala:57-58."""

    def __init__(self, contig: str, available: Iterable[str]):
        self.msg = "Contig %s does not exist in the current reference. Available contigs are %s" % (
            contig, ",".join(available))
        super().__init__(self.msg)

    def __str__(self) -> str:
        return self.msg


class ReferenceGenome:
    """Contig name -> unmasked bases (uint8).  ReferenceBroadcast without the Spark broadcast."""

    def __init__(self, contigs: Dict[str, np.ndarray]):
        self.contigs = {k: np.ascontiguousarray(v, np.uint8) for k, v in contigs.items()}

    @classmethod
    def load_fasta(cls, path: str) -> "ReferenceGenome":
        """ReferenceBroadcast.apply (ReferenceBroadcast.scala:39-55): every record of the FASTA,
        name truncated at the first whitespace, sequence lines joined and unmasked.  A gzip
        FASTA is read through gzip (htsjdk opens .gz the same way)."""
        with open(path, "rb") as fh:
            magic = fh.read(2)
        opener = gzip.open if magic == b"\x1f\x8b" else open
        with opener(path, "rb") as fh:
            data = fh.read()
        contigs: Dict[str, np.ndarray] = {}
        pos = data.find(b">")
        if pos < 0 and data.strip():
            raise ValueError("%s: not a FASTA file (no '>' header line)" % path)
        while pos >= 0:
            nl = data.find(b"\n", pos)
            header = data[pos + 1:(len(data) if nl < 0 else nl)].decode("latin-1").strip()
            nxt = data.find(b"\n>", nl) if nl >= 0 else -1
            body = data[(len(data) if nl < 0 else nl + 1):(len(data) if nxt < 0 else nxt + 1)]
            name = header.split()[0] if header.split() else ""
            if name in contigs:
                raise ValueError("%s: duplicate FASTA record %r" % (path, name))
            seq = body.translate(_UNMASK, b" \t\r\n")
            contigs[name] = np.frombuffer(seq, dtype=np.uint8).copy()
            pos = -1 if nxt < 0 else nxt + 1
        return cls(contigs)

    def names(self) -> List[str]:
        return list(self.contigs)

    def get_contig(self, name: str) -> np.ndarray:
        try:
            return self.contigs[name]
        except KeyError:
            raise ContigNotFound(name, self.contigs.keys()) from None

    def get_reference_base(self, name: str, locus: int) -> int:
        return int(self.get_contig(name)[locus])

    def get_reference_sequence(self, name: str, start: int, end: int) -> np.ndarray:
        """Array.slice semantics: clamped to the contig (ReferenceBroadcast.scala:32-34)."""
        c = self.get_contig(name)
        return c[max(start, 0):max(min(end, len(c)), 0)]

    def build_md_tag(self, read_seq: np.ndarray, contig: str, start: int, cigar: np.ndarray) -> str:
        """ReferenceGenome.buildMdTag (ReferenceGenome.scala:41-47)."""
        ref_len = sum(int(c) >> 4 for c in cigar if int(c) & 15 in _CONSUMES_REF)
        return md_from_reference(read_seq, self.get_reference_sequence(contig, start, start + ref_len), cigar)

    def for_contigs(self, contig_names: List[str]) -> List[Optional[np.ndarray]]:
        """The reference's bytes for each name of a read set's contig list (None where absent)."""
        return [self.contigs.get(n) for n in contig_names]


def md_from_reference(read_seq: np.ndarray, ref_seq: np.ndarray, cigar: np.ndarray) -> str:
    """ADAM MdTag.apply(read, reference, cigar, start) (adam-core 0.18.x), restated:
    M / = / X: each base either extends the match run or closes it with the reference base
    (a mismatch); D: the first deleted base of a run opens "<run>^", every deleted base appends
    its reference base (the deletion run is only closed by an aligned base, as in ADAM); other
    read-consuming ops skip read bases; any other reference-consuming op (N) is refused; the
    final run is appended.  The string is then parsed into mismatches / deletions (MdTag.apply
    (string, start, cigar)), so only its events matter downstream."""
    read = np.asarray(read_seq, np.uint8)
    ref = np.asarray(ref_seq, np.uint8)
    out: List[str] = []
    run = 0
    in_del = False
    rp = fp = 0
    for c in cigar:
        op, ln = int(c) & 15, int(c) >> 4
        if op in (_OP_M, _OP_EQ, _OP_X):
            if fp + ln > len(ref) or rp + ln > len(read):
                raise IndexError("MD rebuild: alignment runs past the end of the reference or read sequence")
            diff = np.flatnonzero(read[rp:rp + ln] != ref[fp:fp + ln])
            last = 0
            for d in diff:
                d = int(d)
                out.append(str(run + d - last))
                out.append(chr(int(ref[fp + d])))
                run = 0
                last = d + 1
            run += ln - last
            if ln:
                in_del = False
            rp += ln
            fp += ln
        elif op == _OP_D:
            if fp + ln > len(ref):
                raise IndexError("MD rebuild: deletion runs past the end of the reference sequence")
            for j in range(ln):
                if not in_del:
                    out.append(str(run) + "^")
                out.append(chr(int(ref[fp + j])))
                run = 0
                in_del = True
            fp += ln
        else:
            if op in _CONSUMES_READ:
                rp += ln
            if op in _CONSUMES_REF:
                raise ValueError("Cannot handle operator: %s" % CIGAR_OPS[op])
    out.append(str(run))
    return "".join(out)


def rebuild_md_tags(rs: ReadSet, reference: Optional[ReferenceGenome], recompute: bool = False) -> ReadSet:
    """Read.fromSAMRecord's MD choice (Read.scala:223-247) over a loaded read set: reads without
    an MD tag (md_len < 0), or every read when `recompute`, get the MD built from the reference.
    Without a reference, `recompute` is refused and reads keep what they have."""
    if recompute and reference is None:
        raise ValueError("To recompute MD tags, a reference genome fasta must be provided.")
    if reference is None or rs.n == 0:
        return rs
    todo = np.arange(rs.n) if recompute else np.flatnonzero(rs.md_len < 0)
    if len(todo) == 0:
        return rs
    new_md = [reference.build_md_tag(rs.seq[int(rs.seq_off[i]):int(rs.seq_off[i]) + int(rs.seq_len[i])],
                                     rs.contig_names[int(rs.contig[i])], int(rs.start[i]),
                                     rs.cigar[int(rs.cigar_off[i]):int(rs.cigar_off[i]) + int(rs.n_cigar[i])]).encode()
              for i in todo]
    md_off, lens, md = repack_md(rs.md, np.asarray(rs.md_off, np.int64), np.asarray(rs.md_len, np.int32), todo, new_md)
    out = replace(rs, md_off=md_off, md_len=lens, md=md)
    out._gq = None
    return out


def repack_md(pool: np.ndarray, md_off: np.ndarray, md_len: np.ndarray, todo: np.ndarray,
              new_md: List[bytes]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """The MD pool with the reads `todo` given the strings `new_md`, packed in read order, in
    vectorised numpy (no per-read Python work for the reads that keep their tag): each read's
    bytes are gathered from the old pool or from the new strings appended behind it."""
    n = len(md_len)
    todo = np.asarray(todo, np.int64)
    new_lens = np.fromiter((len(m) for m in new_md), np.int64, len(new_md))
    src_off = np.asarray(md_off, np.int64).copy()
    lens = np.asarray(md_len, np.int64).copy()
    base = len(pool)
    if len(todo):
        noff = np.zeros(len(todo), np.int64)
        noff[1:] = np.cumsum(new_lens)[:-1]
        src_off[todo] = base + noff
        lens[todo] = new_lens
    src = np.concatenate([np.asarray(pool, np.uint8), np.frombuffer(b"".join(new_md), np.uint8)])
    take = np.maximum(lens, 0)
    out_off = np.zeros(n, np.int64)
    if n:
        out_off[1:] = np.cumsum(take)[:-1]
    total = int(take.sum())
    # byte k of read i comes from src[src_off[i] + k]
    idx = np.repeat(src_off - out_off, take) + np.arange(total, dtype=np.int64)
    return out_off, lens.astype(np.int32), src[idx].copy()
