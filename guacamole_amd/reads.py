"""Read ingest: SAM / BAM -> structure-of-arrays ReadSet.

Host side of the path; restates the reference's loading + filtering semantics
(paths relative to /root/reference/src/main/scala/org/hammerlab/guacamole/):

* ``Read.InputFilters`` (mapped / overlapsLoci / nonDuplicate /
  passedVendorQualityChecks / isPaired / hasMdTag)       reads/Read.scala:95-152
* samtools loading path and its per-record filters       reads/Read.scala:382-430
* ``Read.fromSAMRecord`` (isMapped, sample name, start)   reads/Read.scala:217-291
* ``ReadSet.mappedReads``                                ReadSet.scala:47-53
* ``MappedRead.end = start + paddedReferenceLength``      reads/MappedRead.scala:87

BAM input goes through the native loader (``ingest.load_bam``, libgqingest: parallel
BGZF inflate + record decode).  ``_load_bam_py`` states the same
rules in Python and is the checker of the native loader in tests/test_ingest.py.
"""
from __future__ import annotations

import gzip
import io
import os
import struct
import zlib
from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional

import numpy as np

from .loci import LociSet, LociSetBuilder

CIGAR_OPS = "MIDNSHP=X"
OP_M, OP_I, OP_D, OP_N, OP_S, OP_H, OP_P, OP_EQ, OP_X = range(9)
_CONSUMES_REF = {OP_M, OP_D, OP_N, OP_EQ, OP_X}
_BAM_SEQ = "=ACMGRSVTWYHKDBN"

FLAG_PAIRED = 0x1
FLAG_UNMAPPED = 0x4
FLAG_REVERSE = 0x10
FLAG_QCFAIL = 0x200
FLAG_DUP = 0x400


class ReadLoadError(ValueError):
    pass


@dataclass
class InputFilters:
    """Read.InputFilters (reads/Read.scala:95-122)."""
    overlaps_loci: Optional[LociSetBuilder] = None
    non_duplicate: bool = False
    passed_vendor_quality_checks: bool = False
    is_paired: bool = False
    has_md_tag: bool = False

    @staticmethod
    def make(mapped: bool = False, overlaps_loci: Optional[LociSetBuilder] = None, non_duplicate: bool = False,
             passed_vendor_quality_checks: bool = False, is_paired: bool = False,
             has_md_tag: bool = False) -> "InputFilters":
        if overlaps_loci is None and mapped:
            overlaps_loci = LociSetBuilder().put_all_contigs()
        return InputFilters(overlaps_loci, non_duplicate, passed_vendor_quality_checks, is_paired, has_md_tag)


@dataclass
class ReadSet:
    """Mapped reads of one input file, SoA, sorted by (contig, start) with ties in
    file order (the TaskPosition sort of DistributedUtil.scala:515-530 is stable)."""
    contig_names: List[str]
    contig_lengths: List[int]
    sample_names: List[str]
    contig: np.ndarray       # int32
    start: np.ndarray        # int64, 0-based
    end: np.ndarray          # int64
    mapq: np.ndarray         # uint8
    flags: np.ndarray        # uint8: bit0 reverse
    sample: np.ndarray       # int32
    seq_off: np.ndarray      # int64
    seq_len: np.ndarray      # int32
    seq: np.ndarray          # uint8 pool (ASCII)
    qual: np.ndarray         # uint8 pool (phred)
    cigar_off: np.ndarray    # int64
    n_cigar: np.ndarray      # int32
    cigar: np.ndarray        # uint32 pool: len << 4 | op
    md_off: np.ndarray       # int64
    md_len: np.ndarray       # int32, -1 => no MD tag
    md: np.ndarray           # uint8 pool (MD strings)
    names: Optional[List[str]] = None
    _gq: Optional[dict] = field(default=None, repr=False)

    @property
    def n(self) -> int:
        return int(self.contig.shape[0])

    @property
    def contig_lengths_map(self) -> Dict[str, int]:
        return dict(zip(self.contig_names, self.contig_lengths))

    def contig_index(self) -> Dict[str, int]:
        return {c: i for i, c in enumerate(self.contig_names)}

    def regions(self):
        """(contig name, starts, ends) per contig, for partitionLociByApproximateDepth."""
        out = []
        c = self.contig
        if len(c) and bool(np.all(c[1:] >= c[:-1])):  # sorted by contig (the loaders' order): slices, no copies
            bounds = np.searchsorted(c, np.arange(len(self.contig_names) + 1), side="left")
            for ci, name in enumerate(self.contig_names):
                a, b = int(bounds[ci]), int(bounds[ci + 1])
                if b > a:
                    out.append((name, self.start[a:b], self.end[a:b]))
            return out
        for ci, name in enumerate(self.contig_names):
            m = c == ci
            if m.any():
                out.append((name, self.start[m], self.end[m]))
        return out

    def subset(self, idx) -> "ReadSet":
        """ReadSet of the reads `idx` (kept in the given order; pools re-packed)."""
        idx = np.asarray(idx, dtype=np.int64)

        def pool(off, ln, data):
            lens = np.maximum(ln[idx], 0).astype(np.int64)
            new_off = np.zeros(len(idx), np.int64)
            if len(idx):
                new_off[1:] = np.cumsum(lens)[:-1]
            parts = [data[off[i]:off[i] + max(int(ln[i]), 0)] for i in idx]
            return new_off, (np.concatenate(parts) if parts else data[:0].copy())

        seq_off, seq = pool(self.seq_off, self.seq_len, self.seq)
        _, qual = pool(self.seq_off, self.seq_len, self.qual)
        cigar_off, cigar = pool(self.cigar_off, self.n_cigar, self.cigar)
        md_off, md = pool(self.md_off, self.md_len, self.md)
        return ReadSet(self.contig_names, self.contig_lengths, self.sample_names, self.contig[idx].copy(),
                       self.start[idx].copy(), self.end[idx].copy(), self.mapq[idx].copy(), self.flags[idx].copy(),
                       self.sample[idx].copy(), seq_off, self.seq_len[idx].copy(), seq, qual, cigar_off,
                       self.n_cigar[idx].copy(), cigar, md_off, self.md_len[idx].copy(), md,
                       None if self.names is None else [self.names[i] for i in idx])

    def cigar_string(self, i: int) -> str:
        ops = self.cigar[self.cigar_off[i]:self.cigar_off[i] + self.n_cigar[i]]
        return "".join("%d%s" % (int(c) >> 4, CIGAR_OPS[int(c) & 15]) for c in ops)


def parse_cigar(s: str) -> List[int]:
    if s == "*" or s == "":
        return []
    out, num = [], ""
    for ch in s:
        if ch.isdigit():
            num += ch
        else:
            op = CIGAR_OPS.find(ch)
            if op < 0 or not num:
                raise ReadLoadError("bad CIGAR %r" % s)
            out.append((int(num) << 4) | op)
            num = ""
    if num:
        raise ReadLoadError("bad CIGAR %r" % s)
    return out


def reference_length(cigar: List[int]) -> int:
    """htsjdk Cigar.getReferenceLength (M, D, N, =, X)."""
    return sum(c >> 4 for c in cigar if (c & 15) in _CONSUMES_REF)


def padded_reference_length(cigar: List[int]) -> int:
    """htsjdk Cigar.getPaddedReferenceLength (also counts P)."""
    return sum(c >> 4 for c in cigar if (c & 15) in _CONSUMES_REF or (c & 15) == OP_P)


class _Builder:
    def __init__(self) -> None:
        self.contig, self.start, self.mapq, self.flags, self.sample = [], [], [], [], []
        self.seqs, self.quals, self.cigars, self.mds, self.names = [], [], [], [], []

    def add(self, name, contig, start, mapq, reverse, sample, seq: bytes, qual: bytes, cigar, md):
        if len(qual) != len(seq):  # MappedRead.scala:50-51
            raise ReadLoadError("Base qualities have length %d but sequence has length %d" % (len(qual), len(seq)))
        self.names.append(name)
        self.contig.append(contig)
        self.start.append(start)
        self.mapq.append(mapq)
        self.flags.append(1 if reverse else 0)
        self.sample.append(sample)
        self.seqs.append(seq)
        self.quals.append(qual)
        self.cigars.append(cigar)
        self.mds.append(md)

    def build(self, contig_names, contig_lengths, sample_names) -> ReadSet:
        n = len(self.contig)
        contig = np.array(self.contig, dtype=np.int32)
        start = np.array(self.start, dtype=np.int64)
        order = np.lexsort((np.arange(n), start, contig)) if n else np.zeros(0, dtype=np.int64)
        seq_len = np.array([len(s) for s in self.seqs], dtype=np.int32)[order]
        seq_off = np.zeros(n, dtype=np.int64)
        if n:
            seq_off[1:] = np.cumsum(seq_len)[:-1]
        seq = np.frombuffer(b"".join(self.seqs[i] for i in order), dtype=np.uint8).copy()
        qual = np.frombuffer(b"".join(self.quals[i] for i in order), dtype=np.uint8).copy()
        n_cigar = np.array([len(self.cigars[i]) for i in order], dtype=np.int32)
        cigar_off = np.zeros(n, dtype=np.int64)
        if n:
            cigar_off[1:] = np.cumsum(n_cigar)[:-1]
        cigar = np.array([c for i in order for c in self.cigars[i]], dtype=np.uint32)
        md_len = np.array([-1 if self.mds[i] is None else len(self.mds[i]) for i in order], dtype=np.int32)
        md_off = np.zeros(n, dtype=np.int64)
        if n:
            md_off[1:] = np.cumsum(np.maximum(md_len, 0))[:-1]
        md = np.frombuffer(b"".join(self.mds[i] or b"" for i in order), dtype=np.uint8).copy()
        end = start[order] + np.array([padded_reference_length(self.cigars[i]) for i in order], dtype=np.int64)
        return ReadSet(contig_names=list(contig_names), contig_lengths=list(contig_lengths),
                       sample_names=list(sample_names), contig=contig[order], start=start[order], end=end,
                       mapq=np.array(self.mapq, dtype=np.uint8)[order], flags=np.array(self.flags, dtype=np.uint8)[order],
                       sample=np.array(self.sample, dtype=np.int32)[order], seq_off=seq_off, seq_len=seq_len,
                       seq=seq, qual=qual, cigar_off=cigar_off, n_cigar=n_cigar, cigar=cigar, md_off=md_off,
                       md_len=md_len, md=md, names=[self.names[i] for i in order])


def _record_filter(filters: InputFilters, loci: Optional[LociSet], unmapped: bool, contig_name: Optional[str],
                   start0: int, cigar: List[int], flag: int) -> bool:
    """The raw-record filters of Read.scala:411-418.  True => keep."""
    if filters.overlaps_loci is not None and unmapped:
        return False
    if loci is not None and not unmapped:
        # record.getStart - 1 .. record.getEnd (1-based inclusive alignment end)
        if contig_name is None or not loci.on_contig(contig_name).intersects(start0, start0 + reference_length(cigar)):
            return False
    if filters.non_duplicate and flag & FLAG_DUP:
        return False
    if filters.passed_vendor_quality_checks and flag & FLAG_QCFAIL:
        return False
    if filters.is_paired and not flag & FLAG_PAIRED:
        return False
    return True


def _sample_of(rg: Optional[str], rg_samples: Dict[str, str]) -> str:
    """Read.scala:233-237: read group's SM, else "default"."""
    if rg is not None and rg in rg_samples and rg_samples[rg] is not None:
        return rg_samples[rg]
    return "default"


def _header_read_groups(text: str) -> Dict[str, str]:
    out = {}
    for line in text.splitlines():
        if line.startswith("@RG"):
            f = dict(x.split(":", 1) for x in line.split("\t")[1:] if ":" in x)
            if "ID" in f:
                out[f["ID"]] = f.get("SM")
    return out


def load_reads(path: str, filters: InputFilters = InputFilters(), reference=None, recompute_md: bool = False,
               contig_lengths_from_dictionary: bool = True) -> ReadSet:
    """Load mapped reads of a SAM/BAM file (Read.loadReadRDDAndSequenceDictionaryFromBAM,
    samtools path, then ReadSet.mappedReads).  `reference` (reference.ReferenceGenome) supplies
    MD tags for reads without one, or for every read with `recompute_md` (Read.scala:223-247);
    the hasMdTag filter then sees the rebuilt tags (Read.scala:422).  With
    `contig_lengths_from_dictionary` False (--no-sequence-dictionary) contig lengths are the
    largest read end per contig, and contigs without reads are dropped (ReadSet.scala:69-80)."""
    if recompute_md and reference is None:
        raise ValueError("To recompute MD tags, a reference genome fasta must be provided.")
    if reference is not None:
        from .reference import rebuild_md_tags
        rs = load_reads(path, replace(filters, has_md_tag=False), None, False, contig_lengths_from_dictionary)
        rs = rebuild_md_tags(rs, reference, recompute_md)
        if filters.has_md_tag and (rs.md_len < 0).any():
            rs = rs.subset(np.flatnonzero(rs.md_len >= 0))
        return rs
    if not contig_lengths_from_dictionary:
        return contig_lengths_from_reads(load_reads(path, filters))
    from .adam import is_sam_or_bam
    if not is_sam_or_bam(path):  # Read.scala:345-364: every other name is ADAM AlignmentRecord Parquet
        from .adam import load_adam
        return load_adam(path, filters)[0]
    if is_bam(path):
        from .ingest import load_bam  # native (libgqingest); raises if not built
        return load_bam(path, filters)
    return _load_sam(path, filters)


def is_bam(path: str) -> bool:
    """A BGZF/gzip stream holding BAM (a damaged first block counts: the BAM decoder names
    the fault); anything else is read as SAM text."""
    if os.path.isdir(path):  # (an ADAM directory)
        return False
    with open(path, "rb") as fh:
        head = fh.read(2)
    if head != b"\x1f\x8b":
        return False
    try:
        with gzip.open(path, "rb") as fh:
            return fh.read(4) == b"BAM\x01"
    except (OSError, EOFError, zlib.error):
        return True


def contig_lengths_from_reads(rs: ReadSet) -> ReadSet:
    """ReadSet.contigLengths with contigLengthsFromDictionary = false (ReadSet.scala:75-79):
    contig -> max read end over the mapped reads; contigs without reads are absent."""
    if rs.n == 0:
        raise ValueError("no mapped reads to take contig lengths from (--no-sequence-dictionary)")
    keep = sorted(set(int(c) for c in np.unique(rs.contig)))
    remap = np.full(len(rs.contig_names), -1, np.int32)
    remap[keep] = np.arange(len(keep), dtype=np.int32)
    lengths = [int(rs.end[rs.contig == c].max()) for c in keep]
    return replace(rs, contig_names=[rs.contig_names[c] for c in keep], contig_lengths=lengths,
                   contig=remap[rs.contig].astype(np.int32), _gq=None)


def _finish(b: _Builder, contig_names, contig_lengths, samples: List[str]) -> ReadSet:
    return b.build(contig_names, contig_lengths, samples)


def _load_sam(path: str, filters: InputFilters) -> ReadSet:
    opener = gzip.open if path.endswith(".gz") else open
    contig_names, contig_lengths, header = [], [], []
    b = _Builder()
    samples: List[str] = []
    loci = None
    rg_samples: Dict[str, str] = {}
    with opener(path, "rt") as fh:
        for line in fh:
            line = line.rstrip("\n").rstrip("\r")
            if not line:
                continue
            if line.startswith("@"):
                header.append(line)
                if line.startswith("@SQ"):
                    f = dict(x.split(":", 1) for x in line.split("\t")[1:] if ":" in x)
                    contig_names.append(f["SN"])
                    contig_lengths.append(int(f["LN"]))
                continue
            if loci is None and filters.overlaps_loci is not None:
                loci = filters.overlaps_loci.result(dict(zip(contig_names, contig_lengths)))
                rg_samples = _header_read_groups("\n".join(header))
            elif not rg_samples:
                rg_samples = _header_read_groups("\n".join(header))
            t = line.split("\t")
            qname, flag, rname, pos, mapq, cigar_s = t[0], int(t[1]), t[2], int(t[3]), int(t[4]), t[5]
            seq_s, qual_s = t[9], t[10]
            tags = {}
            for x in t[11:]:
                k, ty, v = x.split(":", 2)
                tags[k] = v
            cigar = parse_cigar(cigar_s)
            unmapped = bool(flag & FLAG_UNMAPPED) or rname == "*"
            if not _record_filter(filters, loci, unmapped, None if rname == "*" else rname, pos - 1, cigar, flag):
                continue
            is_mapped = (not unmapped) and pos - 1 >= 0
            md = tags.get("MD")
            if filters.has_md_tag and (not is_mapped or md is None):
                continue
            if not is_mapped:
                continue
            if rname not in contig_names:
                raise ReadLoadError("read on unknown contig %s" % rname)
            sname = _sample_of(tags.get("RG"), rg_samples)
            if sname not in samples:
                samples.append(sname)
            seq = b"*" if seq_s == "*" else seq_s.encode()
            qual = b"" if qual_s == "*" else bytes(ord(c) - 33 for c in qual_s)
            b.add(qname, contig_names.index(rname), pos - 1, mapq, flag & FLAG_REVERSE, samples.index(sname), seq, qual,
                  cigar, None if md is None else md.encode())
    return _finish(b, contig_names, contig_lengths, samples)


def _load_bam_py(path: str, filters: InputFilters) -> ReadSet:
    """The same BAM rules in Python: the checker of the native loader (tests/test_ingest.py)."""
    with gzip.open(path, "rb") as fh:
        data = fh.read()
    if data[:4] != b"BAM\x01":
        raise ReadLoadError("not a BAM file: %s" % path)
    off = 4
    (l_text,) = struct.unpack_from("<i", data, off)
    off += 4
    text = data[off:off + l_text].decode("utf-8", "replace").rstrip("\x00")
    off += l_text
    (n_ref,) = struct.unpack_from("<i", data, off)
    off += 4
    contig_names, contig_lengths = [], []
    for _ in range(n_ref):
        (l_name,) = struct.unpack_from("<i", data, off)
        off += 4
        contig_names.append(data[off:off + l_name - 1].decode())
        off += l_name
        (l_ref,) = struct.unpack_from("<i", data, off)
        off += 4
        contig_lengths.append(l_ref)
    loci = filters.overlaps_loci.result(dict(zip(contig_names, contig_lengths))) if filters.overlaps_loci else None
    rg_samples = _header_read_groups(text)
    samples: List[str] = []
    b = _Builder()
    n = len(data)
    while off < n:
        (block_size,) = struct.unpack_from("<i", data, off)
        rec = off + 4
        off = rec + block_size
        ref_id, pos, l_read_name, mapq, _bin, n_cigar, flag, l_seq, _nr, _np, _tl = struct.unpack_from(
            "<iiBBHHHiiii", data, rec)
        p = rec + 32
        qname = data[p:p + l_read_name - 1].decode()
        p += l_read_name
        cigar = list(struct.unpack_from("<%dI" % n_cigar, data, p))
        p += 4 * n_cigar
        packed = data[p:p + (l_seq + 1) // 2]
        p += (l_seq + 1) // 2
        qual = data[p:p + l_seq]
        p += l_seq
        md = None
        rg = None
        while p < off:
            tag = data[p:p + 2]
            ty = chr(data[p + 2])
            p += 3
            if ty in "AcC":
                p += 1
            elif ty in "sS":
                p += 2
            elif ty in "iIf":
                p += 4
            elif ty in "ZH":
                e = data.index(b"\x00", p)
                val = data[p:e]
                if tag == b"MD":
                    md = val
                elif tag == b"RG":
                    rg = val.decode()
                p = e + 1
            elif ty == "B":
                sub = chr(data[p])
                (cnt,) = struct.unpack_from("<i", data, p + 1)
                q = p + 5 + cnt * {"c": 1, "C": 1, "s": 2, "S": 2, "i": 4, "I": 4, "f": 4}[sub]
                if cnt < 0 or q > off:
                    raise ReadLoadError("truncated aux array in BAM record")
                p = q
            else:
                raise ReadLoadError("bad aux type %r" % ty)
        unmapped = bool(flag & FLAG_UNMAPPED) or ref_id < 0
        cname = contig_names[ref_id] if ref_id >= 0 else None
        if not _record_filter(filters, loci, unmapped, cname, pos, cigar, flag):
            continue
        is_mapped = (not unmapped) and pos >= 0
        if filters.has_md_tag and (not is_mapped or md is None):
            continue
        if not is_mapped:
            continue
        seq = bytes(_BAM_SEQ[(packed[i >> 1] >> (4 * (1 - (i & 1)))) & 15].encode()[0] for i in range(l_seq))
        if l_seq and qual[0] == 0xFF:
            qual = b""  # htsjdk: missing qualities -> empty array -> MappedRead assertion
        sname = _sample_of(rg, rg_samples)
        if sname not in samples:
            samples.append(sname)
        b.add(qname, ref_id, pos, mapq, flag & FLAG_REVERSE, samples.index(sname), seq, bytes(qual), cigar, md)
    return _finish(b, contig_names, contig_lengths, samples)


def make_read_set(reads, contig_names=("chr1",), contig_lengths=None, sample_names=("default",)) -> ReadSet:
    """Build a ReadSet from in-memory records, mirroring TestUtil.makeRead
    (src/test/.../util/TestUtil.scala:65-89): default quals '@' (phred 31),
    mapq 30, positive strand.  ``reads``: dicts with sequence, cigar, mdtag,
    start, chr, quals (list or None), mapq, reverse, sample."""
    contig_names = list(contig_names)
    if contig_lengths is None:
        contig_lengths = [1 << 30] * len(contig_names)
    b = _Builder()
    for i, r in enumerate(reads):
        seq = r["sequence"].encode()
        quals = r.get("quals")
        qual = bytes([31] * len(seq)) if quals is None else bytes(quals)
        chr_ = r.get("chr", "chr1")
        if chr_ not in contig_names:
            contig_names.append(chr_)
            contig_lengths.append(1 << 30)
        md = r.get("mdtag")
        b.add("r%d" % i, contig_names.index(chr_), int(r.get("start", 1)), int(r.get("mapq", 30)),
              bool(r.get("reverse", False)), int(r.get("sample", 0)), seq, qual, parse_cigar(r["cigar"]),
              None if md is None else md.encode())
    return b.build(contig_names, contig_lengths, list(sample_names))


def make_read(sequence: str, cigar: str, mdtag: Optional[str], start: int = 1, chr: str = "chr1",
              quals=None, mapq: int = 30, reverse: bool = False, sample: int = 0) -> dict:
    return dict(sequence=sequence, cigar=cigar, mdtag=mdtag, start=start, chr=chr, quals=quals, mapq=mapq,
                reverse=reverse, sample=sample)

