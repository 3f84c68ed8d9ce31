"""Known-answer tests that pin the CPU oracle (oracle/oracle.cpp) to the reference's own suites.

Each test transcribes the inputs and expected values of one reference test (file:line under
/root/reference/src/test/scala/org/hammerlab/guacamole/).  Reads are built like
TestUtil.makeRead (util/TestUtil.scala:65-89: quals '@' = phred 31, mapq 30, positive strand);
fixtures are the reference's SAM/BAM test resources (tests/golden/reference_fixtures/).
The oracle is test infrastructure only; these tests never touch the product path.
"""
import math

import pytest

from oracle import oracle as O
from guacamole_amd.reads import InputFilters, load_reads, make_read, make_read_set
from tests.conftest import fixture

R = make_read


def rs(*reads, **kw):
    return make_read_set(list(reads), **kw)


def alleles(els):
    return [(e["kind"], e["ref"], e["alt"]) for e in els]


# ------------------------------------------------------------------------------------------
# PileupSuite (pileup/PileupSuite.scala)
# ------------------------------------------------------------------------------------------
LONG_INSERT = [R("TCGATCGA", "8M", "8", 1), R("TCGATCGA", "8M", "8", 1), R("TCGACCCTCGA", "4M3I4M", "8", 1)]
Q8 = [10, 15, 20, 25, 10, 15, 20, 25]
Q11 = [10, 15, 20, 25, 5, 5, 5, 10, 15, 20, 25]
LONG_INSERT_Q = [R("TCGATCGA", "8M", "8", 1, quals=Q8), R("TCGATCGA", "8M", "8", 1, quals=Q8),
                 R("TCGACCCTCGA", "4M3I4M", "8", 1, quals=Q11)]


def test_long_insert_reads():  # PileupSuite.scala:51-69
    s = rs(*LONG_INSERT)
    assert O.elements_at(s, "chr1", 0)[1] == []
    _, els = O.elements_at(s, "chr1", 1)
    assert all(e["kind"] == "Match" and e["quality"] == 31 for e in els)
    _, els = O.elements_at(s, "chr1", 4)
    assert alleles(els) == [("Match", "A", "A"), ("Match", "A", "A"), ("Insertion", "A", "ACCC")]
    assert all(e["quality"] == 31 for e in els)


def test_long_insert_qualities():  # PileupSuite.scala:71-87 (insertion quality = min over its bases)
    _, els = O.elements_at(rs(*LONG_INSERT_Q), "chr1", 4)
    assert [e["kind"] for e in els] == ["Match", "Match", "Insertion"]
    assert [e["quality"] for e in els] == [25, 25, 5]


def test_long_insert_after():  # PileupSuite.scala:89-103, 105-114, 116-129
    s = rs(*LONG_INSERT_Q)
    _, els = O.elements_at(s, "chr1", 5)
    assert all(e["kind"] == "Match" and e["quality"] == 10 for e in els)
    _, els = O.elements_at(rs(*LONG_INSERT), "chr1", 7)
    assert all(e["kind"] == "Match" and e["alt"] == "G" for e in els)
    _, els = O.elements_at(s, "chr1", 8)
    assert all(e["kind"] == "Match" and e["alt"] == "A" and e["quality"] == 25 for e in els)


def test_same_start_reads():  # PileupSuite.scala:131-158, 221-245
    s = load_reads(fixture("same_start_reads.sam"))
    c = s.contig_names[0]
    assert len(O.elements_at(s, c, 0)[1]) == 10
    for i in range(1, 60):
        assert len(O.elements_at(s, c, i)[1]) == 10
    _, els = O.elements_at(s, c, 9)
    dels = [e for e in els if e["kind"] == "Deletion"]
    assert len(dels) == 5 and all(e["ref"] == "AAAAAAAAAAA" for e in dels)
    for i in range(10, 20):
        assert sum(e["kind"] == "MidDeletion" for e in O.elements_at(s, c, i)[1]) == 5
    for i in range(60, 70):
        assert len(O.elements_at(s, c, i)[1]) == 5


def test_element_index_within_cigar():  # PileupSuite.scala:144-171
    s = rs(R("AATTG", "5M", "5", 0))
    for locus in range(3):
        (e,) = O.elements_at(s, "chr1", locus, own_ref=True)[1]
        assert e["kind"] == "Match" and e["indexWithin"] == locus
    s = rs(R("AAATTT", "3M3M", "6", 0))
    assert O.elements_at(s, "chr1", 3, own_ref=True)[1][0]["indexWithin"] == 0
    assert O.elements_at(s, "chr1", 4, own_ref=True)[1][0]["indexWithin"] == 1


def test_insertion_at_contig_start():  # PileupSuite.scala:173-177
    (e,) = O.elements_at(rs(R("AAAAAACGT", "5I4M", "4", 0)), "chr1", 0, own_ref=True)[1]
    assert (e["kind"], e["ref"], e["alt"]) == ("Insertion", "A", "AAAAAA")


def test_deletion_elements():  # PileupSuite.scala:194-219
    s = rs(R("AATTGAATTG", "5M1D5M", "5^C5", 0))
    e = O.elements_at(s, "chr1", 0, own_ref=True)[1][0]
    assert e["kind"] == "Match" and e["indexWithin"] == 0
    e = O.elements_at(s, "chr1", 4, own_ref=True)[1][0]
    assert (e["kind"], e["ref"], e["alt"], e["quality"], e["indexWithin"]) == ("Deletion", "GC", "G", 31, 4)
    e = O.elements_at(s, "chr1", 5, own_ref=True)[1][0]
    assert e["kind"] == "MidDeletion" and e["indexWithin"] == 0
    e = O.elements_at(s, "chr1", 6, own_ref=True)[1][0]
    assert e["kind"] == "Match" and e["indexWithin"] == 0
    e = O.elements_at(s, "chr1", 9, own_ref=True)[1][0]
    assert e["kind"] == "Match" and e["indexWithin"] == 3


def _decadent():
    return load_reads(fixture("different_start_reads.sam"))


def _one(s, name):
    """ReadSet holding only the named read (testAdamRecords(i) is file order: read1..read7)."""
    return s.subset([s.names.index(name)])


def test_decadent_read1():  # PileupSuite.scala:247-305 (29M10D31M at 0-based 5)
    r1 = _one(_decadent(), "read1")
    c = r1.contig_names[0]
    assert O.elements_at(r1, c, 4)[1] == []
    assert O.elements_at(r1, c, 75)[1] == []
    e = O.elements_at(r1, c, 5, own_ref=True)[1][0]
    assert e["alt"] == "A"
    assert O.elements_at(r1, c, 74, own_ref=True)[1]
    e = O.elements_at(r1, c, 5 + 28, own_ref=True)[1][0]
    assert (e["kind"], e["ref"]) == ("Deletion", "AGGGGGGGGGG")
    for locus in (5 + 29, 5 + 38):
        assert O.elements_at(r1, c, locus, own_ref=True)[1][0]["kind"] == "MidDeletion"
    assert O.elements_at(r1, c, 5 + 39, own_ref=True)[1][0]["alt"] == "A"
    r3 = _one(_decadent(), "read3")
    got = [O.elements_at(r3, c, l, own_ref=True)[1][0]["alt"] for l in (15, 16, 17, 18)]
    assert got == ["A", "T", "C", "G"]


def test_decadent_read4():  # PileupSuite.scala:307-324 (10M10I10D40M, ACGT x15)
    r4 = _one(_decadent(), "read4")
    c = r4.contig_names[0]
    for i in range(2):
        got = [O.elements_at(r4, c, 20 + i * 4 + k, own_ref=True)[1][0]["alt"][0] for k in range(4)]
        assert got == list("ACGT")
    e = O.elements_at(r4, c, 29, own_ref=True)[1][0]
    assert e["kind"] == "Insertion" and e["alt"] == "CGTACGTACGT"


def test_decadent_read5_to_7():  # PileupSuite.scala:326-383 (=, X, N, S, H)
    s = _decadent()
    c = s.contig_names[0]
    r5 = _one(s, "read5")
    exp5 = {10: "A", 14: "A", 18: "A", 19: "C", 20: "G", 21: "T", 22: "A", 24: "G"}
    for l, b in exp5.items():
        assert O.elements_at(r5, c, l, own_ref=True)[1][0]["alt"] == b
    for name in ("read6", "read7"):  # the fixture's CIGARs are 4=1D4=4S / 4=1D4=4H
        r = _one(s, name)
        exp = {40: "A", 41: "C", 42: "G", 43: "T", 44: "", 45: "A", 48: "T"}
        for l, b in exp.items():
            assert O.elements_at(r, c, l, own_ref=True)[1][0]["alt"] == b
        assert O.elements_at(r, c, 49)[1] == []


RNA = R("CCCCAGCCTAGGCCTTCGACACTGGGGGGCTGAGGGAAGGGGCACCTGCC", "7M191084N43M", "9T24T7G7", 229538779)


def test_rna_read():  # PileupSuite.scala:385-405
    s = rs(RNA)
    exp = {229538780: "C", 229538781: "C", 229539779: "", 229729912: "C"}
    for l, b in exp.items():
        assert O.elements_at(s, "chr1", l, own_ref=True)[1][0]["alt"] == b


def test_rna_pileup_depth():  # PileupSuite.scala:407-418
    s = load_reads(fixture("testrna.sam"))
    c = s.contig_names[0]
    assert len(O.elements_at(s, c, 229580594)[1]) == 94
    assert len(O.elements_at(s, c, 229580706)[1]) == 4
    assert len(O.elements_at(s, c, 229580707)[1]) == 1


def test_pileup_in_deletion():  # PileupSuite.scala:420-432
    s = rs(*[R("TCGAAAAGCT", "5M6D5M", "5^GCTTCG5", 0)] * 3)
    assert {(e["ref"], e["alt"]) for e in O.elements_at(s, "chr1", 4)[1]} == {("AGCTTCG", "A")}
    assert {(e["ref"], e["alt"]) for e in O.elements_at(s, "chr1", 5)[1]} == {("G", "")}


# ------------------------------------------------------------------------------------------
# GermlineThresholdCallerSuite (commands/GermlineThresholdCallerSuite.scala:30-113)
# ------------------------------------------------------------------------------------------
REF3 = [R("TCGATCGA", "8M", "8", 1)] * 3
HET = [R("TCGATCGA", "8M", "8", 1)] * 2 + [R("GCGATCGA", "8M", "0T7", 1)]
HOM = [R("TCGATCGA", "8M", "8", 1)] + [R("GCGATCGA", "8M", "0T7", 1)] * 2


@pytest.mark.parametrize("reads,threshold,gt", [
    (REF3, 0, ("Ref", "Ref")),
    (HET, 0, ("Ref", "Alt")),
    (HET, 30, ("Ref", "Alt")),
    (HET, 50, ("Ref", "Ref")),
])
def test_germline_threshold_kats(reads, threshold, gt):
    calls = O.germline_at(rs(*reads), "chr1", 1, threshold)
    assert calls and all(c["gt"] == gt for c in calls)


def test_germline_hom_alt():  # :78-92
    calls = O.germline_at(rs(*HOM), "chr1", 1, 50, emit_ref=False)
    assert calls == [dict(locus=1, gt=("Alt", "Alt"), ref="T", alt="G")]


def test_germline_hom_alt_no_ref_bases():  # :94-107
    calls = O.germline_at(rs(*[R("TGGATCGA", "8M", "1C6", 1)] * 3), "chr1", 2, 50, emit_ref=False)
    assert calls == [dict(locus=2, gt=("Alt", "Alt"), ref="C", alt="G")]


def test_germline_heterozygous_deletion():  # :110-121
    s = load_reads(fixture("synthetic.challenge.set1.normal.v2.withMDTags.chr2.syn1fp.sam"),
                   InputFilters.make(mapped=True, non_duplicate=True, passed_vendor_quality_checks=True))
    assert O.germline_at(s, "2", 16050070, 8, emit_ref=False, emit_no_call=False) == []


# ------------------------------------------------------------------------------------------
# LikelihoodSuite (likelihood/LikelihoodSuite.scala:58-210), tolerance 1e-12
# ------------------------------------------------------------------------------------------
def _err(q):  # PhredUtils.phredToErrorProbability
    return 10 ** (-q / 10)


E30, E40 = _err(30), _err(40)


def ref_read(q):
    return R("C", "1M", "1", 1, quals=[q])


def alt_read(q):
    return R("A", "1M", "0C0", 1, quals=[q])


def G(a, b):
    return (("C", a), ("C", b))


@pytest.mark.parametrize("reads,expect", [
    ((ref_read(30), ref_read(40), ref_read(30)),
     {("C", "C"): (1 - E30) * (1 - E40) * (1 - E30), ("C", "A"): 1 / 8, ("A", "C"): 1 / 8,
      ("A", "A"): E30 * E40 * E30, ("A", "T"): E30 * E40 * E30}),
    ((ref_read(30), ref_read(40), alt_read(30)),
     {("C", "C"): (1 - E30) * (1 - E40) * E30, ("C", "A"): 1 / 8, ("A", "C"): 1 / 8,
      ("A", "A"): E30 * E40 * (1 - E30), ("A", "T"): E30 * E40 / 2, ("T", "T"): E30 * E40 * E30}),
    ((ref_read(30), alt_read(40), alt_read(30)),
     {("C", "C"): (1 - E30) * E40 * E30, ("C", "A"): 1 / 8, ("A", "C"): 1 / 8,
      ("A", "A"): E30 * (1 - E40) * (1 - E30), ("A", "T"): E30 / 4, ("T", "T"): E30 * E40 * E30}),
    ((alt_read(30), alt_read(40), alt_read(30)),
     {("C", "C"): E30 * E40 * E30, ("C", "A"): 1 / 8, ("A", "C"): 1 / 8,
      ("A", "A"): (1 - E30) * (1 - E40) * (1 - E30), ("A", "T"): 1 / 8, ("T", "T"): E30 * E40 * E30}),
])
def test_genotype_likelihoods(reads, expect):  # :58-110
    gts = [G(a, b) for a, b in expect]
    got = O.likelihoods_at(rs(*reads), "chr1", 1, genotypes=gts)
    assert len(got) == len(gts)
    for (g, v), e in zip(got, expect.values()):
        assert abs(v - e) < 1e-12


@pytest.mark.parametrize("log_space", [False, True])
@pytest.mark.parametrize("reads,expect", [
    ((ref_read(30), ref_read(40), ref_read(30)), {("C", "C"): (1 - E30) * (1 - E40) * (1 - E30)}),
    ((ref_read(30), ref_read(40), alt_read(30)),
     {("C", "C"): (1 - E30) * (1 - E40) * E30, ("A", "C"): 1 / 8, ("A", "A"): E30 * E40 * (1 - E30)}),
    ((alt_read(30), alt_read(40), alt_read(30)), {("A", "A"): (1 - E30) * (1 - E40) * (1 - E30)}),
])
def test_all_possible_genotypes(reads, expect, log_space):  # :112-210
    got = {tuple(sorted(x[1] for x in g)): v
           for g, v in O.likelihoods_at(rs(*reads), "chr1", 1, log_space=log_space)}
    want = {tuple(sorted(k)): (math.log(v) if log_space else v) for k, v in expect.items()}
    assert set(got) == set(want)
    for k in want:
        assert abs(got[k] - want[k]) < 1e-12


# ------------------------------------------------------------------------------------------
# AlleleEvidenceSuite (variants/AlleleEvidenceSuite.scala:9-61)
# ------------------------------------------------------------------------------------------
def test_allele_evidence_all_support():
    s = rs(R("TCGATCGA", "8M", "1A6", 1, mapq=30), R("TCGATCGA", "8M", "1A6", 1, mapq=30),
           R("TCGACCCTCGA", "4M3I4M", "1A6", 1, mapq=60))
    ev = O.allele_evidence_at(s, "chr1", 2, 0.5, "A", "C")
    assert ev["meanMappingQuality"] == 40.0 and ev["medianMappingQuality"] == 30
    assert ev["medianMismatchesPerRead"] == 1


def test_allele_evidence_one_supports():
    s = rs(R("TAGATCGA", "8M", "8", 1, mapq=30), R("TCGATCGA", "8M", "1A6", 1, mapq=60),
           R("TAGACCCTCGA", "4M3I4M", "8", 1, mapq=60))
    ev = O.allele_evidence_at(s, "chr1", 2, 0.5, "A", "C")
    assert ev["meanMappingQuality"] == 60.0 and ev["medianMappingQuality"] == 60
    assert ev["medianMismatchesPerRead"] == 1


def test_allele_evidence_none_supports():
    s = rs(R("TAGATCGA", "8M", "8", 1, mapq=30), R("TAGATCGA", "8M", "8", 1, mapq=60),
           R("TAGACCCTCGA", "4M3I4M", "8", 1, mapq=60))
    ev = O.allele_evidence_at(s, "chr1", 2, 0.5, "A", "C")
    for k in ("meanMappingQuality", "medianMappingQuality", "medianMismatchesPerRead"):
        assert math.isnan(ev[k])


# ------------------------------------------------------------------------------------------
# MDTagUtilsSuite (reads/MDTagUtilsSuite.scala:9-241): MD-derived reference per locus
# ------------------------------------------------------------------------------------------
def own_reference(read_set, start, end):
    """Reference bases a single read reconstructs from its MD tag (MDTagUtils.getReference)."""
    return "".join(O.elements_at(read_set, "chr1", l, own_ref=True)[0] for l in range(start, end))


@pytest.mark.parametrize("seq,cigar,md,ref", [
    ("GATGATTCGA", "10M", "10", "GATGATTCGA"),
    ("GATGATTCGA", "10M", "0CC8", "CCTGATTCGA"),
    ("GATGACCCTTCGA", "5M3I5M", "10", "GATGATTCGA"),
    ("GATA", "3M6D1M", "3^GATTCG1", "GATGATTCGA"),
    ("TCGATCGA", "8M", "1A6", "TAGATCGA"),
])
def test_md_reference_single_read(seq, cigar, md, ref):  # :11-38, 233-240
    assert own_reference(rs(R(seq, cigar, md, 0)), 0, len(ref)) == ref


def pileup_reference(read_set, start, end):
    """Pileup.referenceBaseAtLocus over [start, end); 'N' where no read covers."""
    return "".join(O.elements_at(read_set, "chr1", l)[0] for l in range(start, end))


REF18 = "AAATTGATACTCGAACGA"


@pytest.mark.parametrize("reads,start,end,ref", [
    ([R(REF18[0:10], "10M", "10", 0), R(REF18[5:15], "10M", "10", 5), R(REF18[8:18], "10M", "10", 8)], 0, 18, REF18),
    ([R(REF18[0:10], "10M", "10", 0), R("GCTACTCGAA", "10M", "1A9", 5), R(REF18[8:18], "10M", "10", 8)], 0, 18, REF18),
    ([R(REF18[0:10], "10M", "10", 0), R("GCTACTCAAA", "10M", "1A5G2", 5), R(REF18[8:18], "10M", "10", 8)], 0, 18,
     REF18),
    ([R(REF18[0:10], "10M", "10", 0), R("GCTACTCAAA", "10M", "1A5G2", 5), R(REF18[8:18], "10M", "10", 8)], 5, 12,
     "GATACTC"),
    ([R(REF18[0:10], "10M", "10", 0), R("GAGGGTACTCGAA", "2M3I8M", "10", 5), R(REF18[8:18], "10M", "10", 8)], 0, 18,
     REF18),
    ([R(REF18[0:10], "10M", "10", 0), R("GCGGGTACTCGAA", "2M3I8M", "1A5G2", 5), R("ACTCGAATTA", "10M", "7CG1", 8)],
     0, 18, REF18),
    ([R(REF18[0:10], "10M", "10", 0), R("GAGAA", "2M5D3M", "2^TACTC3", 5), R(REF18[8:18], "10M", "10", 8)], 0, 18,
     REF18),
    ([R(REF18[0:10], "10M", "10", 0), R("GAGAA", "2M5D3M", "2^TACTC3", 5), R("ACTCGA", "5M4D1M", "5^AACG1", 8)], 0,
     18, REF18),
    ([R(REF18[0:7], "7M", "7", 0), R(REF18[11:18], "7M", "7", 11)], 0, 18, "AAATTGANNNNCGAACGA"),
    ([R(REF18[3:7], "4M", "4", 3), R(REF18[11:18], "7M", "7", 11)], 0, 18, "NNNTTGANNNNCGAACGA"),
    ([R(REF18[0:7], "7M", "7", 0), R(REF18[11:14], "3M", "3", 11)], 0, 18, "AAATTGANNNNCGANNNN"),
])
def test_md_reference_multi_read(reads, start, end, ref):  # :40-211
    assert pileup_reference(rs(*reads), start, end) == ref


def test_md_reference_rna():  # :213-231
    s = rs(RNA)
    assert own_reference(s, 229538779, 229538779 + 7) == "CCCCAGC"
    end = 229538779 + 7 + 191084 + 43
    assert own_reference(s, end - 43, end) == "CTTGGCCTTCGACACTGGGGGGCTGAGTGAAGGGGGACCTGCC"
    assert O.elements_at(s, "chr1", 229538779 + 100, own_ref=True)[1][0]["kind"] == "Clipped"


# ------------------------------------------------------------------------------------------
# SomaticStandardCallerSuite (commands/SomaticStandardCallerSuite.scala:37-262)
# ------------------------------------------------------------------------------------------
SUITE_PARAMS = dict(odds=120, min_mapq=1, filter_multi_allelic=0, min_tumor_read_depth=8, max_tumor_read_depth=200,
                    min_normal_read_depth=4, min_tumor_alternate_read_depth=3, min_likelihood=70, min_vaf=5,
                    apply_filters=2)
TN_FILTERS = dict(mapped=True, non_duplicate=True, passed_vendor_quality_checks=True)  # TestUtil.scala:178-183


def _tn(tumor, normal):
    f = InputFilters.make(**TN_FILTERS)
    return load_reads(fixture(tumor), f), load_reads(fixture(normal), f)


SOMATIC_CASES = [
    ("tumor.chr20.tough.sam", "normal.chr20.tough.sam", "20", True,
     [42999694, 25031215, 44061033, 45175149, 755754, 1843813, 3555766, 3868620, 9896926, 14017900, 17054263,
      35951019, 50472935, 51858471, 58201903, 7087895, 19772181, 30430960, 32150541, 42186626, 44973412, 46814443,
      52311925, 53774355, 57280858, 62262870]),
    ("synthetic.challenge.set1.tumor.v2.withMDTags.chr2.syn1fp.sam",
     "synthetic.challenge.set1.normal.v2.withMDTags.chr2.syn1fp.sam", "2", False,
     [216094721, 3529313, 8789794, 104043280, 104175801, 126651101, 241901237, 57270796, 120757852]),
    ("synthetic.challenge.set1.tumor.v2.withMDTags.chr2.complexvar.sam",
     "synthetic.challenge.set1.normal.v2.withMDTags.chr2.complexvar.sam", "2", False,
     [148487667, 134307261, 90376213, 3638733, 109347468]),
    ("synthetic.challenge.set1.tumor.v2.withMDTags.chr2.complexvar.sam",
     "synthetic.challenge.set1.normal.v2.withMDTags.chr2.complexvar.sam", "2", True, [82949713, 130919744]),
    ("tumor.chr20.simplefp.sam", "normal.chr20.simplefp.sam", "20", False,
     [26211835, 29652479, 54495768, 13046318, 25939088]),
]


@pytest.mark.parametrize("tumor,normal,contig,positive,loci", SOMATIC_CASES,
                         ids=["tough+", "syn1fp-", "complexvar-", "complexvar+", "simplefp-"])
def test_somatic_real_data(tumor, normal, contig, positive, loci):  # :82-115
    t, n = _tn(tumor, normal)
    for locus in loci:
        found = len(O.somatic_at(t, n, contig, locus, **SUITE_PARAMS)) > 0
        assert found == positive, (contig, locus)


NORMAL8 = [R("TCGATCGA", "8M", "8", 0)] * 3


@pytest.mark.parametrize("tumor,normal,locus,ref,alt", [
    ([R("TCGGTCGA", "8M", "3G4", 0)] * 3, NORMAL8, 2, None, None),  # :117-133 no indels
    ([R("TCGTCGA", "3M1D4M", "3^A4", 0)] * 3, NORMAL8, 2, "GA", "G"),  # :135-153
    ([R("TCGAAAAGCT", "5M6D5M", "5^GCTTCG5", 0)] * 3, [R("TCGAAGCTTCGAAGCT", "16M", "16", 0)] * 3, 4, "AGCTTCG",
     "A"),  # :155-175
    ([R("TCGAGTCGA", "4M1I4M", "8", 0)] * 3, NORMAL8, 3, "A", "AG"),  # :177-197
    ([R("TCGAGGTCTCGA", "4M4I4M", "8", 0)] * 3, NORMAL8, 3, "A", "AGGTC"),  # :199-218
])
def test_somatic_synthetic_indels(tumor, normal, locus, ref, alt):
    got = O.somatic_at(rs(*tumor), rs(*normal), "chr1", locus, odds=2, apply_filters=0)
    if ref is None:
        assert got == []
    else:
        assert [(g["ref"], g["alt"]) for g in got] == [(ref, alt)]


@pytest.mark.parametrize("locus,ref,alt", [(11, "CGA", "C"), (14, "A", "ATC"), (16, "C", "CAAAA"), (18, "ATC", "A")])
def test_somatic_insertions_and_deletions(locus, ref, alt):  # :220-262
    normal = [R("TCGAATCGATCGATCGA", "17M", "17", 10)] * 3
    tumor = [R("TCATCTCAAAAGAGATCGA", "2M2D1M2I2M4I2M2D6M", "2^GA5^TC6", 10)] * 3
    got = O.somatic_at(rs(*tumor), rs(*normal), "chr1", locus, odds=2, apply_filters=0)
    assert [(g["ref"], g["alt"]) for g in got] == [(ref, alt)]


# ------------------------------------------------------------------------------------------
# ReadSetSuite counts (reads/ReadSetSuite.scala:32-52)
# ------------------------------------------------------------------------------------------
def test_read_set_filter_counts():
    import gzip
    p = fixture("mdtagissue.sam")
    with gzip.open(p, "rt") as fh:  # all records (8), incl. unmapped ones the MappedRead SoA never holds
        assert sum(1 for line in fh if not line.startswith("@")) == 8
    assert load_reads(p, InputFilters.make(mapped=True)).n == 5
    assert load_reads(p, InputFilters.make(mapped=True, non_duplicate=True)).n == 3
