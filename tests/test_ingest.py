"""Native read ingest (libgqingest, include/gqingest.h) against its Python statement.

* BAM -> ReadSet: guacamole_amd.ingest.load_bam (parallel BGZF inflate + record decode) must
  give arrays identical to reads._load_bam_py (Read.scala:368-451 filters, Read.fromSAMRecord
  sample / start rules, MappedRead end) on the reference's chrM.sorted.bam under every filter
  combination the callers use, and on written BAMs that exercise what chrM does not: read
  groups, unmapped / duplicate / QC-fail / unpaired reads, unsorted input, every aux type,
  records split across BGZF blocks, a plain-gzip BAM, and the error cases.
* MD tags -> MD events: ingest.md_events (gq_md_count / gq_md_fill) against soa.md_events
  (ADAM MdTag as MappedRead.apply builds it; pinned by MDTagUtilsSuite cases in test_host.py).
"""
import os
import random

import numpy as np
import pytest

from guacamole_amd import ingest, soa
from guacamole_amd.build import build_ingest
from guacamole_amd.loci import LociSet
from guacamole_amd.reads import InputFilters, ReadLoadError, _load_bam_py, load_reads, make_read, make_read_set
from tests import bam_writer as bw
from tests.conftest import fixture

FIELDS = ["contig", "start", "end", "mapq", "flags", "sample", "seq_off", "seq_len", "seq", "qual", "cigar_off",
          "n_cigar", "cigar", "md_off", "md_len", "md"]


@pytest.fixture(scope="module", autouse=True)
def _built():
    build_ingest()


def same(a, b):
    assert a.contig_names == b.contig_names and a.contig_lengths == b.contig_lengths
    assert a.sample_names == b.sample_names
    for f in FIELDS:
        x, y = getattr(a, f), getattr(b, f)
        assert x.dtype == y.dtype, f
        assert np.array_equal(x, y), f
    assert list(a.names) == list(b.names)


CHRM_FILTERS = [
    InputFilters(),
    InputFilters.make(mapped=True),
    InputFilters.make(overlaps_loci=LociSet.parse("chrM:1000-2000,chrM:9000-9001"), non_duplicate=True,
                      has_md_tag=True),
    InputFilters.make(overlaps_loci=LociSet.parse("all"), passed_vendor_quality_checks=True,
                      non_duplicate=True, has_md_tag=True),
]


@pytest.mark.parametrize("k", range(len(CHRM_FILTERS)))
def test_chrm_bam_native_equals_python(k):
    p = fixture("chrM.sorted.bam")
    f = CHRM_FILTERS[k]
    same(load_reads(p, f), _load_bam_py(p, f))


def _records(rng, n, contigs, unsorted=False):
    recs = []
    bases = "ACGTN"
    for i in range(n):
        ref_id = rng.randrange(len(contigs)) if unsorted else min(i * len(contigs) // n, len(contigs) - 1)
        pos = rng.randrange(0, 5000) if unsorted else (i * 37) % 5000
        cig = rng.choice(["50M", "10M2D40M", "5S40M5S", "20M3I27M", "10M100N40M", "25M1P25M", "50="])
        ops = bw.cigar_ops(cig)
        l_seq = sum(c >> 4 for c in ops if (c & 15) in (0, 1, 4, 7, 8))
        seq = "".join(rng.choice(bases) for _ in range(l_seq))
        qual = [rng.randrange(2, 41) for _ in range(l_seq)]
        flag = rng.choice([0, 0, 0, 16, 1, 17, 0x400, 0x200, 0x401, 4])
        tags = b""
        if rng.random() < 0.9:
            tags += bw.tag_z("MD", rng.choice(["50", "10A39", "10^AC40", "0C49", "25^T0G24", "50"]))
        r = rng.random()
        if r < 0.4:
            tags += bw.tag_z("RG", "rg1")
        elif r < 0.6:
            tags += bw.tag_z("RG", "rg2")
        elif r < 0.7:
            tags += bw.tag_z("RG", "rg_nosm")
        tags += bw.tag_i("NM", 1) + bw.tag_b("ZB", rng.choice("cCsSiIf"), [1, 2, 3]) + b"XAA!" + b"XCc\x05" + \
            b"XSs\x01\x00" + b"XFf\x00\x00\x80\x3f" + b"XHH0A0B\x00"
        ref = ref_id if flag != 4 else rng.choice([ref_id, -1])
        recs.append(bw.record(ref, pos if ref >= 0 else -1, "q%d" % i, cig if ref >= 0 else "*", seq, qual,
                              mapq=rng.randrange(0, 61), flag=flag, tags=tags))
    return recs


HEADER = "@HD\tVN:1.6\n@RG\tID:rg1\tSM:alice\n@RG\tID:rg2\tSM:bob\n@RG\tID:rg_nosm\tPL:x\n"
CONTIGS = [("chr2", 100000), ("chr10", 50000), ("chrX", 20000)]


@pytest.mark.parametrize("unsorted", [False, True])
@pytest.mark.parametrize("block", [65280, 1000])
def test_written_bam_native_equals_python(tmp_path, unsorted, block):
    rng = random.Random(7 + unsorted + block)
    p = str(tmp_path / "x.bam")
    bw.write_bam(p, HEADER, CONTIGS, _records(rng, 1500, CONTIGS, unsorted), block=block)
    for f in [InputFilters(), InputFilters.make(mapped=True, non_duplicate=True),
              InputFilters.make(overlaps_loci=LociSet.parse("chr10:100-3000,chrX"), is_paired=True),
              InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True,
                                passed_vendor_quality_checks=True, has_md_tag=True)]:
        a, b = load_reads(p, f), _load_bam_py(p, f)
        same(a, b)
        assert a.n > 0
    assert load_reads(p).sample_names == _load_bam_py(p, InputFilters()).sample_names
    assert set(load_reads(p).sample_names) == {"alice", "bob", "default"}


def test_plain_gzip_bam(tmp_path):
    rng = random.Random(3)
    p = str(tmp_path / "g.bam")
    bw.write_bam(p, HEADER, CONTIGS, _records(rng, 300, CONTIGS), plain_gzip=True)
    same(load_reads(p), _load_bam_py(p, InputFilters()))


def test_empty_bam(tmp_path):
    p = str(tmp_path / "e.bam")
    bw.write_bam(p, "", CONTIGS, [])
    a = load_reads(p)
    same(a, _load_bam_py(p, InputFilters()))
    assert a.n == 0 and a.sample_names == []


def test_missing_quals_error(tmp_path):  # MappedRead.scala:50-51 via htsjdk's empty quality array
    p = str(tmp_path / "q.bam")
    bw.write_bam(p, "", CONTIGS, [bw.record(0, 10, "a", "4M", "ACGT", None, tags=bw.tag_z("MD", "4"))])
    with pytest.raises(ReadLoadError, match="Base qualities have length 0 but sequence has length 4"):
        _load_bam_py(p, InputFilters())
    with pytest.raises(ReadLoadError, match="Base qualities have length 0 but sequence has length 4"):
        load_reads(p)


def test_bad_aux_type_error(tmp_path):
    p = str(tmp_path / "a.bam")
    bw.write_bam(p, "", CONTIGS, [bw.record(0, 10, "a", "4M", "ACGT", [30] * 4, tags=b"XYq\x00")])
    with pytest.raises(ReadLoadError, match="bad aux type 'q'"):
        _load_bam_py(p, InputFilters())
    with pytest.raises(ReadLoadError, match="bad aux type 'q'"):
        load_reads(p)


def test_corrupt_block_is_an_error(tmp_path):
    p = str(tmp_path / "c.bam")
    bw.write_bam(p, "", CONTIGS, [bw.record(0, 10, "a", "4M", "ACGT", [30] * 4)])
    raw = bytearray(open(p, "rb").read())
    raw[30] ^= 0xFF  # inside the first block's deflate payload
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ReadLoadError):
        load_reads(p)


# ---- MD events --------------------------------------------------------------------------
def _py_events(rs):
    n_md, n_mm, ev = np.zeros(rs.n, np.int32), np.zeros(rs.n, np.uint16), []
    for i in range(rs.n):
        if rs.md_len[i] < 0:
            n_md[i] = -1
            continue
        ops = [(int(c) & 15, int(c) >> 4) for c in rs.cigar[rs.cigar_off[i]:rs.cigar_off[i] + rs.n_cigar[i]]]
        e, mm = soa.md_events(rs.md[rs.md_off[i]:rs.md_off[i] + rs.md_len[i]].tobytes(), int(rs.start[i]), ops)
        n_md[i], n_mm[i] = len(e), min(mm, 65535)
        ev.extend(e)
    return n_md, n_mm, np.array(ev, np.uint32)


def _check_events(rs):
    n_md, n_mm, off, ev = ingest.md_events(rs.cigar_off, rs.n_cigar, rs.cigar, rs.md_off, rs.md_len, rs.md)
    p_md, p_mm, p_ev = _py_events(rs)
    assert np.array_equal(n_md, p_md) and np.array_equal(n_mm, p_mm) and np.array_equal(ev, p_ev)
    assert np.array_equal(off[1:], np.cumsum(np.maximum(p_md, 0))[:-1])


def test_md_events_chrm():
    _check_events(load_reads(fixture("chrM.sorted.bam")))


def test_md_events_reference_sams():
    for name in ["same_start_reads.sam", "different_start_reads.sam", "testrna.sam",
                 "synthetic.challenge.set1.normal.v2.withMDTags.chr2.syn1fp.sam", "tumor.chr20.tough.sam"]:
        _check_events(load_reads(fixture(name)))


def test_md_events_edge_cases():
    reads = [
        make_read("TCGATCGA", "8M", "8"),
        make_read("TCGATCGA", "8M", "0G7"),
        make_read("TCGATCGA", "8M", "3a4"),              # lower case
        make_read("TCGACGA", "3M1D4M", "3^T4"),
        make_read("TCGACGA", "3M1D4M", "3^t4"),
        make_read("TCGACGA", "3M2N4M", "1C5"),           # N gap skipped
        make_read("TCGACGA", "2S5M", "1^AC0G3"),         # MD longer than the CIGAR
        make_read("TCGACGAAA", "3M2I4M", "0AC5"),
        make_read("TCGA", "4M", ""),                     # empty MD
        make_read("TCGA", "4M", None),                   # no MD
        make_read("TCGA", "2M1P2M", "1T0T1"),
        make_read("TCGA", "4=", "4"),
        make_read("TCGA", "4X", "0A0C0G0T0"),
    ]
    _check_events(make_read_set(reads))


@pytest.mark.parametrize("md", ["A4", "4^", "4%2", "x"])
def test_md_events_errors(md):
    rs = make_read_set([make_read("TCGA", "4M", md)])
    py_err = None
    try:
        _py_events(rs)
    except soa.MdParseError as e:
        py_err = e
    if py_err is None:  # the Python statement accepts it: so must the native parser
        _check_events(rs)
        return
    with pytest.raises(soa.MdParseError):
        ingest.md_events(rs.cigar_off, rs.n_cigar, rs.cigar, rs.md_off, rs.md_len, rs.md)


def test_md_events_random():
    rng = random.Random(11)
    reads = []
    for i in range(3000):
        ops, md, seq = [], "", ""
        nm = 0
        for _ in range(rng.randrange(1, 6)):
            op = rng.choice("MMMDIN=XS")
            ln = rng.randrange(1, 6)
            ops.append("%d%s" % (ln, op))
            if op in "MI=XS":
                seq += "".join(rng.choice("ACGT") for _ in range(ln))
        # MD string of random matches / mismatches / deletions (need not agree with the CIGAR)
        parts = [str(rng.randrange(0, 6))]
        for _ in range(rng.randrange(0, 5)):
            if rng.random() < 0.5:
                parts.append("".join(rng.choice("ACGTacgtN") for _ in range(rng.randrange(1, 3))))
            else:
                parts.append("^" + "".join(rng.choice("ACGT") for _ in range(rng.randrange(1, 4))))
            parts.append(str(rng.randrange(0, 6)))
        reads.append(make_read(seq or "A", "".join(ops) if seq else "1M", "".join(parts), start=1 + i))
    _check_events(make_read_set(reads))


def test_pack_uses_native_events():
    rs = load_reads(fixture("chrM.sorted.bam"))
    p = soa.pack(rs)
    n_md, n_mm, ev = _py_events(rs)
    assert np.array_equal(p["n_md"], n_md) and np.array_equal(p["md_ev"], ev)
    assert np.array_equal(p["n_mismatch"], n_mm)


# ---- larger files: several record-boundary segments, both inflate backends ----------------
def _synthetic_bam(tmp_path, length=100_000):
    from guacamole_amd import synthetic
    g = synthetic.generate(length, 30.0)
    p = str(tmp_path / "syn.bam")
    g.write_bam(p)
    return g, p


def test_synthetic_bam_roundtrip_and_python_statement(tmp_path):
    """Generator arrays -> BAM -> native loader: identical reads and MD events (the bench's
    round trip), and identical to the Python statement of the loader."""
    g, p = _synthetic_bam(tmp_path)
    assert os.path.getsize(p) > 1 << 20  # > 2 MiB inflated: several boundary segments
    rs = load_reads(p)
    a = g.arrays
    assert rs.n == g.n
    assert np.array_equal(rs.start, a["start"].astype(np.int64)) and np.array_equal(rs.end, a["end"].astype(np.int64))
    n_md, n_mm, off, ev = ingest.md_events(rs.cigar_off, rs.n_cigar, rs.cigar, rs.md_off, rs.md_len, rs.md)
    assert np.array_equal(n_md, a["n_md"]) and np.array_equal(n_mm, a["n_mismatch"])
    ref_ev = np.concatenate([a["md_ev"][a["md_off"][i]:a["md_off"][i] + a["n_md"][i]] for i in range(g.n)])
    assert np.array_equal(ev, ref_ev)
    same(rs, _load_bam_py(p, InputFilters()))


def test_zlib_backend_matches(tmp_path):
    """The zlib inflate path (GQ_INGEST_ZLIB) decodes the same bytes as libdeflate's."""
    import subprocess
    import sys
    _, p = _synthetic_bam(tmp_path, 50_000)
    code = ("import sys, hashlib; sys.path.insert(0, %r)\n"
            "from guacamole_amd.reads import load_reads\n"
            "r = load_reads(%r); h = hashlib.sha1()\n"
            "[h.update(getattr(r, f).tobytes()) for f in %r]\n"
            "print(h.hexdigest())" % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), p, FIELDS))
    outs = []
    for env in ({}, {"GQ_INGEST_ZLIB": "1"}):
        e = dict(os.environ, **env)
        outs.append(subprocess.check_output([sys.executable, "-c", code], env=e).strip())
    assert outs[0] == outs[1]
