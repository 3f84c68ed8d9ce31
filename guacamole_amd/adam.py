"""ADAM AlignmentRecord input: `--reads` / `--tumor-reads` / `--normal-reads` that are not SAM/BAM.

Restates the reference's ADAM read path (paths relative to
/root/reference/src/main/scala/org/hammerlab/guacamole/):

* ``Read.loadReadRDDAndSequenceDictionary`` sends every filename not ending in .bam / .sam to
  ``loadReadRDDAndSequenceDictionaryFromADAM`` (reads/Read.scala:338-364, 454-474): ADAM's
  ``loadAlignments`` over the Parquet files, the sequence dictionary from the records' contigs,
  ``fromADAMRecord`` per record, then ``InputFilters.filterRDD`` (reads/Read.scala:131-151).
* ``Read.fromADAMRecord`` (reads/Read.scala:484-539): bases upper-cased
  (``Bases.stringToBases``, Bases.scala:87-89), qualities ``baseQualityStringToArray`` (all 0 when
  the string is empty, else phred + 33: Read.scala:201-209), the sample from
  ``recordGroupSample.toString`` (a record without one fails there, as in the reference), MD from
  ``mismatchingPositions``, ``start`` as stored (ADAM positions are 0-based), the strand from
  ``readNegativeStrand``; a record with ``readMapped`` false is an UnmappedRead.
* ``ReadSet.mappedReads`` (ReadSet.scala:47-53): the mapped reads, in (contig, start) order with
  ties in record order, as the other loaders keep them.

The records' schema is bdg-formats 0.6.1's ``AlignmentRecord`` (pom.xml:287-291), a dependency
absent from /root/reference: its field list is restated in ``output.ALIGNMENT_RECORD_SCHEMA`` and
is parity unpinned, as is the byte layout of ADAM's Parquet files.  ``sam_to_alignment_records``
restates ADAM 0.18's SAM -> AlignmentRecord conversion (``SAMRecordConverter``; the reference's
test converts ``mdtagissue.sam`` that way, ReadSetSuite.scala:88-109) so that an ADAM directory
can be written here from a SAM file (``write_alignment_parquet``) — also parity unpinned.
"""
from __future__ import annotations

import gzip
import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from .loci import LociSet
from .reads import (FLAG_DUP, FLAG_PAIRED, FLAG_QCFAIL, FLAG_REVERSE, FLAG_UNMAPPED, InputFilters, ReadLoadError,
                    ReadSet, _Builder, parse_cigar, reference_length)

FLAG_PROPER = 0x2
FLAG_MATE_UNMAPPED = 0x8
FLAG_MATE_REVERSE = 0x20
FLAG_FIRST = 0x40
FLAG_SECOND = 0x80
FLAG_SECONDARY = 0x100
FLAG_SUPPLEMENTARY = 0x800


def is_sam_or_bam(path: str) -> bool:
    """The reference's test for its BAM/SAM path (Read.scala:345): the name ends in .bam or .sam
    (here also .sam.gz, the gzip-compressed SAM this repository's fixtures are kept as)."""
    return path.endswith(".bam") or path.endswith(".sam") or path.endswith(".sam.gz")


# ---- SAM -> AlignmentRecord (ADAM 0.18 SAMRecordConverter, restated) ----------------------
def _sam_header(lines: List[str]):
    contigs: List[Dict] = []
    rgs: Dict[str, Dict[str, str]] = {}
    for line in lines:
        f = dict(x.split(":", 1) for x in line.split("\t")[1:] if ":" in x)
        if line.startswith("@SQ"):
            contigs.append({"contigName": f["SN"], "contigLength": int(f["LN"]), "contigMD5": f.get("M5"),
                            "referenceURL": f.get("UR"), "assembly": f.get("AS"), "species": f.get("SP"),
                            "referenceIndex": len(contigs)})
        elif line.startswith("@RG") and "ID" in f:
            rgs[f["ID"]] = f
    return contigs, rgs


def sam_to_alignment_records(path: str) -> List[Dict]:
    """Every record of a SAM file (plain or gzip) as an AlignmentRecord dict, in file order: read
    name, sequence, CIGAR, qualities (unset for "*"), hard-clip trims; contig / start (0-based) /
    end / mapq for an aligned read; the mate's contig and 0-based start; the flags; MD as
    mismatchingPositions, OQ as origQual, the other tags as attributes (TAG:TYPE:VALUE, tab
    separated, in reverse order as ADAM's list prepends them); the read group's name and its
    fields."""
    opener = gzip.open if path.endswith(".gz") else open
    header: List[str] = []
    out: List[Dict] = []
    contigs: List[Dict] = []
    by_name: Dict[str, Dict] = {}
    rgs: Dict[str, Dict[str, str]] = {}
    with opener(path, "rt") as fh:
        for line in fh:
            line = line.rstrip("\n").rstrip("\r")
            if not line:
                continue
            if line.startswith("@"):
                header.append(line)
                continue
            if not by_name and header:
                contigs, rgs = _sam_header(header)
                by_name = {c["contigName"]: c for c in contigs}
            t = line.split("\t")
            qname, flag, rname, pos, mapq, cigar = t[0], int(t[1]), t[2], int(t[3]), int(t[4]), t[5]
            rnext, pnext, tlen, seq, qual = t[6], int(t[7]), int(t[8]), t[9], t[10]
            r: Dict = {"readName": qname, "sequence": seq, "cigar": cigar}
            lead = cigar[:len(cigar) - len(cigar.lstrip("0123456789"))]
            r["basesTrimmedFromStart"] = int(lead) if cigar != "*" and cigar[len(lead)] == "H" else 0
            if cigar.endswith("H"):
                body = cigar[:-1]
                r["basesTrimmedFromEnd"] = int(body[len(body.rstrip("0123456789")):])
            else:
                r["basesTrimmedFromEnd"] = 0
            if qual != "*":
                r["qual"] = qual
            if rname != "*":
                if rname not in by_name:
                    raise ReadLoadError("record %s on contig %s, not in the header" % (qname, rname))
                r["contig"] = dict(by_name[rname])
                if pos != 0:
                    r["start"] = pos - 1
                    r["end"] = pos - 1 + (reference_length(parse_cigar(cigar)) if cigar != "*" else 0)
                if mapq != 255:
                    r["mapq"] = mapq
            mate = rname if rnext == "=" else rnext
            if mate != "*" and mate in by_name:
                r["mateContig"] = dict(by_name[mate])
                if pnext > 0:
                    r["mateAlignmentStart"] = pnext - 1
            if flag & FLAG_PAIRED:
                r["readPaired"] = True
                r["mateNegativeStrand"] = bool(flag & FLAG_MATE_REVERSE)
                r["mateMapped"] = not flag & FLAG_MATE_UNMAPPED
                r["properPair"] = bool(flag & FLAG_PROPER)
                if flag & FLAG_FIRST:
                    r["readNum"] = 0
                if flag & FLAG_SECOND:
                    r["readNum"] = 1
            r["duplicateRead"] = bool(flag & FLAG_DUP)
            r["readNegativeStrand"] = bool(flag & FLAG_REVERSE)
            r["primaryAlignment"] = not flag & FLAG_SECONDARY
            r["secondaryAlignment"] = bool(flag & FLAG_SECONDARY)
            r["supplementaryAlignment"] = bool(flag & FLAG_SUPPLEMENTARY)
            r["failedVendorQualityChecks"] = bool(flag & FLAG_QCFAIL)
            r["readMapped"] = not flag & FLAG_UNMAPPED
            if tlen != 0:
                r["inferredInsertSize"] = tlen
            tags = []
            rg = None
            for x in t[11:]:
                k, ty, v = x.split(":", 2)
                if k == "MD":
                    r["mismatchingPositions"] = v
                elif k == "OQ":
                    r["origQual"] = v
                else:
                    tags.insert(0, x)
                    if k == "RG":
                        rg = v
            r["attributes"] = "\t".join(tags)
            if rg is not None and rg in rgs:
                g = rgs[rg]
                r["recordGroupName"] = rg
                r["recordGroupSample"] = g.get("SM")
                r["recordGroupSequencingCenter"] = g.get("CN")
                r["recordGroupDescription"] = g.get("DS")
                r["recordGroupFlowOrder"] = g.get("FO")
                r["recordGroupKeySequence"] = g.get("KS")
                r["recordGroupLibrary"] = g.get("LB")
                if "PI" in g:
                    r["recordGroupPredictedMedianInsertSize"] = int(g["PI"])
                r["recordGroupPlatform"] = g.get("PL")
                r["recordGroupPlatformUnit"] = g.get("PU")
            out.append(r)
    return out


def write_alignment_parquet(path: str, records: List[Dict], codec: str = "GZIP") -> List[str]:
    """adamParquetSave of AlignmentRecords: a Hadoop output directory with one part file (the
    Parquet layout of output.write_parquet_dir, the AlignmentRecord schema in the footer)."""
    from .output import write_parquet_dir
    return write_parquet_dir(path, records, codec=codec, record="AlignmentRecord")


# ---- AlignmentRecord Parquet -> ReadSet ---------------------------------------------------
def read_alignment_records(path: str) -> List[Dict]:
    """The AlignmentRecords of an ADAM Parquet path: a directory of part files (taken in name
    order; ADAM loads a directory's parts the same way) or one Parquet file."""
    import glob
    import pyarrow.parquet as pq
    if os.path.isdir(path):
        files = sorted(f for f in glob.glob(os.path.join(path, "*.parquet")) if not os.path.basename(f).startswith("."))
        if not files:
            raise ReadLoadError("%s: no Parquet part files (an ADAM AlignmentRecord directory was expected)" % path)
    elif os.path.isfile(path):
        with open(path, "rb") as fh:
            if fh.read(4) != b"PAR1":
                raise ReadLoadError("%s is neither SAM / BAM (by name) nor ADAM Parquet" % path)
        files = [path]
    else:
        raise ReadLoadError("%s: no such file or directory" % path)
    out: List[Dict] = []
    for f in files:
        out.extend(pq.read_table(f).to_pylist())
    return out


def _sequence_dictionary(records: List[Dict]) -> Tuple[List[str], List[int]]:
    """ADAMSpecificRecordSequenceDictionaryRDDAggregator.adamGetSequenceDictionary: the distinct
    contigs of the records (their own and their mates'), by referenceIndex where set, else in
    order of first appearance."""
    seen: Dict[str, Tuple[int, int, int]] = {}
    for i, r in enumerate(records):
        for key in ("contig", "mateContig"):
            c = r.get(key)
            if c and c.get("contigName") is not None and c["contigName"] not in seen:
                ri = c.get("referenceIndex")
                seen[c["contigName"]] = (ri if ri is not None else 1 << 40, len(seen), int(c.get("contigLength") or 0))
    names = sorted(seen, key=lambda n: seen[n][:2])
    return names, [seen[n][2] for n in names]


def load_adam(path: str, filters: InputFilters = InputFilters()) -> Tuple[ReadSet, int]:
    """loadReadRDDAndSequenceDictionaryFromADAM + ReadSet.mappedReads: (the mapped reads passing
    the filters, the number of reads of either kind passing them — the RDD's count)."""
    return alignment_records_to_reads(read_alignment_records(path), filters)


def alignment_records_to_reads(records: List[Dict], filters: InputFilters = InputFilters()) -> Tuple[ReadSet, int]:
    names, lengths = _sequence_dictionary(records)
    index = {n: i for i, n in enumerate(names)}
    loci: Optional[LociSet] = filters.overlaps_loci.result(dict(zip(names, lengths))) if filters.overlaps_loci else None
    b = _Builder()
    samples: List[str] = []
    kept = 0
    for r in records:
        # fromADAMRecord (Read.scala:484-539)
        seq = (r.get("sequence") or "").upper().encode()
        qs = r.get("qual")
        if qs is None:
            raise ReadLoadError("record %s: no qual (Read.scala:487 calls toString on it)" % r.get("readName"))
        qual = bytes(len(seq)) if qs == "" else bytes((ord(ch) - 33) & 0xFF for ch in qs)
        sample = r.get("recordGroupSample")
        if sample is None:
            raise ReadLoadError("record %s: no recordGroupSample (Read.scala:498 calls toString on it)"
                                % r.get("readName"))
        mapped = bool(r.get("readMapped"))
        md = r.get("mismatchingPositions")
        # InputFilters.filterRDD (Read.scala:131-151)
        if loci is not None:
            if not mapped:
                continue
            c = (r.get("contig") or {}).get("contigName")
            cig = parse_cigar(r["cigar"])
            s0 = int(r["start"])
            if c is None or not loci.on_contig(c).intersects(s0, s0 + reference_length(cig)):
                continue
        if filters.non_duplicate and r.get("duplicateRead"):
            continue
        if filters.passed_vendor_quality_checks and r.get("failedVendorQualityChecks"):
            continue
        if filters.is_paired and not r.get("readPaired"):
            continue
        if filters.has_md_tag and not (mapped and md is not None):
            continue
        kept += 1
        if not mapped:  # ReadSet.mappedReads
            continue
        contig = (r.get("contig") or {}).get("contigName")
        if contig not in index:
            raise ReadLoadError("record %s: mapped without a contig" % r.get("readName"))
        if sample not in samples:
            samples.append(sample)
        mapq, start = r.get("mapq"), r.get("start")
        if mapq is None or start is None:  # (getMapq / getStart unboxed in Read.scala:502, 505)
            raise ReadLoadError("record %s: mapped without %s" % (r.get("readName"), "mapq" if mapq is None else "start"))
        b.add(r.get("readName"), index[contig], int(start), int(mapq),
              bool(r.get("readNegativeStrand")), samples.index(sample), seq, qual, parse_cigar(r["cigar"]),
              None if md is None else md.encode())
    return b.build(names, lengths, samples), kept
