"""GPU parity at the three sites where the reference's output depends on Scala 2.10 hash-map
iteration order (restated in gq_scala_order.h / the oracle's scala_order, parity unpinned: no
JVM here), each locus built so that the order decides the output:

* count ties among passing germline alleles (GermlineThresholdCaller.scala:103-104): the SNV
  path (germline_expand) with up to four and with five alleles; the (C, G) / (C, N) pair that
  shares a mutable.HashMap bucket, where the first occurrence in pileup element order decides
  (heap order of the window's initial group: germline_complex re-run with the element order);
* the per-sample record order of Pileup.bySample (Pileup.scala:57-61) with 3 and 5 samples;
* the somatic normal variant mass summed in HashTrieMap order (three normal alleles: six
  genotypes, SomaticStandardCaller.scala:206-217).
Rows are compared with the oracle in order; tests/scala_order_py.py (an independent Python
statement) says what the order must pick."""
import numpy as np
import pytest

import scala_order_py as S
from guacamole_amd.commands import germline_threshold_reads, somatic_standard_reads
from guacamole_amd.reads import make_read as mr, make_read_set
from oracle import oracle as O
from test_gpu_somatic import assert_rows_match

pytestmark = pytest.mark.gpu


def _one_locus(pos, contig=0):
    return (np.array([contig], np.int32), np.array([pos], np.int64), np.array([pos + 1], np.int64),
            np.array([0], np.int64))


def _snv_reads(ref, counts, length=10, pos=5, start=0, sample=0, mapq=30):
    """Reads over [start, start + length) of a poly-`ref` contig with base b at `pos`, counts[b] of each."""
    reads = []
    for b, n in counts:
        seq = ref * (pos - start) + b + ref * (start + length - pos - 1)
        md = "%d" % length if b == ref else "%d%s%d" % (pos - start, ref, start + length - pos - 1)
        reads += [mr(seq, "%dM" % length, md, start, sample=sample, mapq=mapq)] * n
    return reads


def _expected_snv_order(ref, present):
    hs = [S.allele_hash(ref, b) for b in present]
    return [present[k] for k in S.group_by_order(hs)]


def test_three_way_tie_snv(gpu_ctx):
    """4 A / 4 C / 4 G at ref A: the top two come from the counts map's order (G, A, C), so the
    call is A>G (het), not the A>C an Allele-order tie-break would give."""
    rs = make_read_set(_snv_reads("A", [("A", 4), ("C", 4), ("G", 4)]))
    got = germline_threshold_reads(gpu_ctx, rs, _one_locus(5), 8)
    assert got == O.germline_threshold(rs, _one_locus(5), 8)
    assert _expected_snv_order("A", ["A", "C", "G"])[:2] == ["G", "A"]
    assert [(r[4], r[5], r[3]) for r in got] == [("A", "G", ("Ref", "Alt"))]


def test_compound_alt_tie_order(gpu_ctx):
    rs = make_read_set(_snv_reads("A", [("C", 5), ("G", 5)]))
    got = germline_threshold_reads(gpu_ctx, rs, _one_locus(5), 8)
    assert got == O.germline_threshold(rs, _one_locus(5), 8)
    order = _expected_snv_order("A", ["C", "G"])
    assert [r[5] for r in got] == order and all(r[3] == ("Alt", "OtherAlt") for r in got)


@pytest.mark.parametrize("ref", list("ACGT"))
def test_five_alleles_trie_order(gpu_ctx, ref):
    """Five distinct alleles (A C G T N, 3 reads each): a HashTrieMap orders the counts map."""
    rs = make_read_set(_snv_reads(ref, [(b, 3) for b in "ACGTN"]))
    for t in (8, 0):
        got = germline_threshold_reads(gpu_ctx, rs, _one_locus(5), t, True, True)
        assert got == O.germline_threshold(rs, _one_locus(5), t, True, True), t


@pytest.mark.parametrize("g_first", [True, False])
def test_shared_bucket_decided_by_element_order(gpu_ctx, g_first):
    """ref C with 4 G, 4 N and 4 C reads: (C, G) and (C, N) share a mutable.HashMap bucket, so
    the newest first occurrence comes first.  The reads all start at 0 and end differently, so
    the window's initial heap-ordered group puts the shorter reads first in the pileup: element
    order, not read order, decides."""
    g = _snv_reads("C", [("G", 4)], length=12)
    n = _snv_reads("C", [("N", 4)], length=10)
    c = _snv_reads("C", [("C", 4)], length=14)
    rs = make_read_set((g + n if g_first else n + g) + c)
    for locus in (_one_locus(5), (np.array([0], np.int32), np.array([0], np.int64), np.array([14], np.int64),
                                  np.array([0], np.int64))):
        got = germline_threshold_reads(gpu_ctx, rs, locus, 8, True, False)
        assert got == O.germline_threshold(rs, locus, 8, True, False)
    assert S.mutable_bucket(S.allele_hash("C", "G")) == S.mutable_bucket(S.allele_hash("C", "N"))


@pytest.mark.parametrize("names", [["tumor", "normal", "blood"], ["s0", "s1", "s2", "s3", "s4"],
                                   ["NA12878", "NA12891", "NA12892"]])
def test_samples_in_by_sample_order(gpu_ctx, names):
    """One call per sample at a locus, in Pileup.bySample's Map order over the sample names."""
    reads = []
    for k in range(len(names)):
        reads += _snv_reads("A", [("A", 3), ("T", 3 + k)], sample=k)
    rs = make_read_set(reads, sample_names=names)
    got = germline_threshold_reads(gpu_ctx, rs, _one_locus(5), 8)
    want = O.germline_threshold(rs, _one_locus(5), 8)
    assert got == want
    order = [names[k] for k in S.group_by_order([S.java_string_hash(n) for n in names])]
    assert [names[r[2]] for r in got] == order


def test_normal_variant_mass_trie_order(gpu_ctx, monkeypatch):
    """Three normal alleles at the locus: six genotypes, so the variant genotypes' likelihoods
    are added in HashTrieMap order; checked on the fast and the deep caller."""
    quals = [20 + (i * 7) % 17 for i in range(10)]
    tumor = []
    for i, (b, n) in enumerate([("A", 12), ("C", 12), ("G", 2)]):
        for k in range(n):
            r = _snv_reads("A", [(b, 1)], mapq=40 + k % 20)[0]
            r["quals"] = [quals[(k + i) % 10]] * 10
            tumor.append(r)
    normal = []
    for i, (b, n) in enumerate([("A", 9), ("C", 7), ("G", 3)]):
        for k in range(n):
            r = _snv_reads("A", [(b, 1)])[0]
            r["quals"] = [quals[(3 * k + i) % 10]] * 10
            normal.append(r)
    t, n = make_read_set(tumor), make_read_set(normal)
    for dbg in ("0", "64"):
        monkeypatch.setenv("GQ_DBG", dbg)
        for params in (dict(odds=1, apply_filters=0), dict(odds=1, apply_filters=1, min_lod=-100)):
            got = somatic_standard_reads(gpu_ctx, t, n, _one_locus(5), **params)
            assert_rows_match(got, O.somatic_standard(t, n, _one_locus(5), **params))
