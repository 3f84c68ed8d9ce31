"""CPU tests of the reference-genome input (guacamole_amd/reference.py) and of the oracle's
--reference-fasta mode.

Pinned by ReferenceBroadcastSuite (test/.../reference/ReferenceBroadcastSuite.scala:11-50) on the
reference's own sample.fasta; the MD rebuild (ADAM MdTag.apply, restated) is checked by a round
trip over every fixture read that carries an MD tag: the reference segment the tag describes,
handed back to the rebuild, must give the same MD events."""
import numpy as np
import pytest

from conftest import fixture
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.reads import InputFilters, load_reads, make_read as mr, make_read_set
from guacamole_amd.reference import ContigNotFound, ReferenceGenome, md_from_reference, rebuild_md_tags
from guacamole_amd.soa import md_events
from oracle import oracle as O
from reference_helpers import assembled_reference, own_reference

TN_FILTERS = InputFilters.make(mapped=True, non_duplicate=True, passed_vendor_quality_checks=True, has_md_tag=True)


def _loci(rs):
    ls = LociSet.parse("all").result(rs.contig_lengths_map)
    return flatten_partitions(partition_loci_uniformly(1, ls), rs.contig_index())


def test_reference_broadcast_suite_kats():
    """ReferenceBroadcastSuite.scala:11-50."""
    r = ReferenceGenome.load_fasta(fixture("sample.fasta"))
    assert sorted(r.names()) == ["1", "2"]
    b = lambda c, l: chr(r.get_reference_base(c, l))
    assert [b("1", x) for x in (0, 80, 160, 240, 320)] == ["N", "C", "T", "G", "A"]
    assert [b("2", x) for x in (0, 80, 160, 240)] == ["N", "T", "C", "G"]
    s = lambda c, a, e: r.get_reference_sequence(c, a, e).tobytes().decode()
    assert s("1", 80, 160) == "CATCAAAATACCACCATCATTCTTCACAGAACTAGAAAAAACAAGGCTAAAATTCACATGGAACCAAAAAAGAGCCCACA"
    assert s("2", 240, 320) == "GACGTTCATTCAGAATGCCACCTAACTAGGCCAGTTTTTGGACTGTATGCCAGCCTCTTTCTGCGGGATGTAATCTCAAT"
    assert s("2", 720, 800) == "CTGATGATCGCACCTGCATAACTGCTACCAGACCTGCTAAGGGGGAGCCTGGCCCAGCCATCTCTTCTTTGTGGTCACAA"
    with pytest.raises(ContigNotFound, match="Contig 3 does not exist in the current reference"):
        r.get_contig("3")


def test_soft_masked_fasta_is_unmasked():
    """Bases.unmaskBases (Bases.scala:115-125) on the reference's soft-masked chrMT fixture."""
    r = ReferenceGenome.load_fasta(fixture("human_GRCh37_75_dna_chrMT.fasta"))
    mt = r.get_contig("MT")
    assert len(mt) == 16569
    assert set(mt.tobytes()) <= set(b"ACGTN")


def test_md_rebuild_cases():
    A = lambda s: np.frombuffer(s.encode(), np.uint8)
    C = lambda *ops: np.array([(ln << 4) | op for op, ln in ops], np.uint32)
    assert md_from_reference(A("TCGATCGA"), A("TCGATCGA"), C((0, 8))) == "8"
    assert md_from_reference(A("TCGGTCGA"), A("TCGATCGA"), C((0, 8))) == "3A4"
    assert md_from_reference(A("TCGTCGA"), A("TCGATCGA"), C((0, 3), (2, 1), (0, 4))) == "3^A4"
    assert md_from_reference(A("AATCGA"), A("TCGA"), C((4, 2), (0, 4))) == "4"
    assert md_from_reference(A("GTCGA"), A("TCGA"), C((0, 1), (1, 1), (0, 3))) == "0T3"
    # a deletion run is closed only by an aligned base (ADAM's delCount), even across an insertion
    assert md_from_reference(A("TCCTT"), A("TCGATT"), C((0, 2), (2, 1), (1, 1), (2, 1), (0, 2))) == "2^GA2"
    with pytest.raises(ValueError, match="Cannot handle operator: N"):
        md_from_reference(A("TCGA"), A("TCGAAAAA"), C((0, 2), (3, 4), (0, 2)))


@pytest.mark.parametrize("name", ["tumor.chr20.tough.sam", "normal.chr20.tough.sam", "mdtagissue.sam",
                                  "synthetic.challenge.set1.tumor.v2.withMDTags.chr2.complexvar.sam"])
def test_md_rebuild_round_trip(name):
    rs = load_reads(fixture(name))
    checked = 0
    for i in range(rs.n):
        seg = own_reference(rs, i)
        if seg is None:
            continue
        co, nc = int(rs.cigar_off[i]), int(rs.n_cigar[i])
        cig = rs.cigar[co:co + nc]
        so = int(rs.seq_off[i])
        rebuilt = md_from_reference(rs.seq[so:so + int(rs.seq_len[i])], seg, cig).encode()
        ops = [(int(c) & 15, int(c) >> 4) for c in cig]
        orig = rs.md[int(rs.md_off[i]):int(rs.md_off[i]) + int(rs.md_len[i])].tobytes()
        # events equal up to mismatches whose MD base equals the read base (the rebuild cannot see those)
        e_new, _ = md_events(rebuilt, 0, ops)
        e_old, _ = md_events(orig, 0, ops)
        assert set(e_new) <= set(e_old), (name, i, orig, rebuilt)
        checked += 1
    assert checked > 0


def test_load_without_md_tags():
    """Read.scala:223-247 / :422 on the reference's MD-less fixtures: without a reference the
    hasMdTag filter drops every read; with one every read gets a rebuilt tag."""
    path = fixture("tumor_without_mdtag.sam")
    assert load_reads(path, TN_FILTERS).n == 0
    mt = ReferenceGenome.load_fasta(fixture("human_GRCh37_75_dna_chrMT.fasta")).get_contig("MT")
    ref = ReferenceGenome({"chrM": mt})
    rs = load_reads(path, TN_FILTERS, reference=ref)
    assert rs.n == 50 and (rs.md_len > 0).all()
    with pytest.raises(ValueError, match="To recompute MD tags, a reference genome fasta must be provided."):
        load_reads(path, TN_FILTERS, recompute_md=True)
    with pytest.raises(ContigNotFound):
        load_reads(path, TN_FILTERS, reference=ReferenceGenome({"MT": mt}))


def test_recompute_replaces_existing_tags():
    rs = make_read_set([mr("TCGGTCGA", "8M", "8", 0)])  # the tag claims a match at the G
    ref = ReferenceGenome({"chr1": np.frombuffer(b"TCGATCGAAAAA", np.uint8)})
    kept = rebuild_md_tags(rs, ref, recompute=False)
    assert kept.md.tobytes() == b"8"
    redone = rebuild_md_tags(rs, ref, recompute=True)
    assert redone.md.tobytes() == b"3A4"


def test_no_sequence_dictionary_lengths():
    """ReadSet.contigLengths from the reads (ReadSet.scala:75-79)."""
    rs = load_reads(fixture("tumor.chr20.tough.sam"), contig_lengths_from_dictionary=False)
    full = load_reads(fixture("tumor.chr20.tough.sam"))
    assert rs.contig_names == sorted(set(full.contig_names[c] for c in np.unique(full.contig)), key=full.contig_names.index)
    assert rs.contig_lengths == [int(full.end[full.contig == full.contig_names.index(c)].max()) for c in rs.contig_names]


def test_oracle_reference_matches_md_reference_where_unambiguous():
    """With a FASTA equal to the reads' MD-derived reference, the oracle's --reference-fasta mode
    gives the MD mode's calls at every locus whose MD bases agree (flags 0)."""
    t = load_reads(fixture("tumor.chr20.tough.sam"), TN_FILTERS)
    n = load_reads(fixture("normal.chr20.tough.sam"), TN_FILTERS)
    ref = ReferenceGenome(assembled_reference(t, n))
    loci = _loci(t)
    want = [r for r in O.somatic_standard(t, n, loci, apply_filters=0) if r["flags"] & 3 == 0]
    got = O.somatic_standard(t, n, loci, reference=ref, apply_filters=0)
    gk = {(r["locus"], r["ref"], r["alt"]): r for r in got}
    for w in want:
        g = gk.get((w["locus"], w["ref"], w["alt"]))
        assert g is not None and g["log_odds"] == w["log_odds"] and g["tumor"] == w["tumor"], w
    assert all(r["flags"] & 3 == 0 for r in got)


def test_oracle_reference_changes_calls():
    """The tumor reads show G at locus 2 and their MD says G is the reference; the normal reads
    show A.  From the MD every tumor element is a Match (no call); with a FASTA whose base is A
    the tumor elements are Mismatches and the normal's Matches: a G somatic call."""
    t = make_read_set([mr("TCGATCGA", "8M", "8", 0)] * 4)
    n = make_read_set([mr("TCAATCGA", "8M", "8", 0)] * 4)
    loci = (np.array([0], np.int32), np.array([2], np.int64), np.array([3], np.int64), np.array([0], np.int64))
    assert O.somatic_standard(t, n, loci, odds=2, apply_filters=0) == []
    ref = ReferenceGenome({t.contig_names[0]: np.frombuffer(b"TCAATCGAAAAA", np.uint8)})
    rows = O.somatic_standard(t, n, loci, reference=ref, odds=2, apply_filters=0)
    assert [(r["locus"], r["ref"], r["alt"]) for r in rows] == [(2, "A", "G")]
    with pytest.raises(O.OracleError, match="does not exist in the current reference"):
        O.somatic_standard(t, n, loci, reference=ReferenceGenome({"other": ref.get_contig(t.contig_names[0])}),
                           apply_filters=0)


def test_repack_md_matches_the_per_read_layout():
    """repack_md (vectorised) = the straightforward per-read repack: reads keep their MD bytes
    unless listed, listed reads take the new strings, MD-less reads (length -1) stay MD-less."""
    import numpy as np
    from guacamole_amd.reference import repack_md
    rng = np.random.default_rng(5)
    n = 200
    lens = rng.integers(-1, 9, n).astype(np.int32)
    off = np.zeros(n, np.int64)
    off[1:] = np.cumsum(np.maximum(lens, 0))[:-1]
    pool = rng.integers(48, 58, int(np.maximum(lens, 0).sum())).astype(np.uint8)
    todo = np.sort(rng.choice(n, 37, replace=False))
    new = [bytes(rng.integers(65, 70, int(k))) for k in rng.integers(0, 7, len(todo))]
    got_off, got_len, got = repack_md(pool, off, lens, todo, new)
    want = []
    want_len = []
    nm = dict(zip(todo.tolist(), new))
    for i in range(n):
        m = nm.get(i)
        if m is None:
            m = pool[off[i]:off[i] + lens[i]].tobytes() if lens[i] >= 0 else None
        want_len.append(-1 if m is None else len(m))
        want.append(m or b"")
    assert got_len.tolist() == want_len and got.tobytes() == b"".join(want)
    assert all(got[got_off[i]:got_off[i] + max(got_len[i], 0)].tobytes() == want[i] for i in range(n))
