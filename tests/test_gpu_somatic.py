"""GPU parity: somatic-standard (HIP, gfx950) vs the CPU oracle.

Every row compared bit for bit: loci, alleles, depths, flags, and the FP64 log-odds,
likelihoods and evidence means / medians (NaN == NaN).  The kernel sums the per-element
log terms in the reference's Colt order (last element first) over the pileup element order,
with java.lang.StrictMath's log / exp / log10 (fdlibm), as the oracle does, so rows whose
decision lands within an ulp of a threshold (GQ_FLAG_KNIFE_EDGE) are compared like any other.
BASELINE.json's tolerance for log-likelihoods (1e-6) is therefore not needed here."""
import math

import numpy as np
import pytest

from conftest import fixture
from guacamole_amd import native
from guacamole_amd.commands import somatic_standard_reads
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.reads import InputFilters, load_reads, make_read as mr, make_read_set
from guacamole_amd.synthetic import generate
from oracle import oracle as O

pytestmark = pytest.mark.gpu

# SomaticStandard.Caller.run input filters (SomaticStandardCaller.scala:69-73)
TN_FILTERS = InputFilters.make(mapped=True, non_duplicate=True, passed_vendor_quality_checks=True, has_md_tag=True)
PAIRS = [("tumor.chr20.tough.sam", "normal.chr20.tough.sam"),
         ("tumor.chr20.simplefp.sam", "normal.chr20.simplefp.sam"),
         ("synthetic.challenge.set1.tumor.v2.withMDTags.chr2.syn1fp.sam",
          "synthetic.challenge.set1.normal.v2.withMDTags.chr2.syn1fp.sam"),
         ("synthetic.challenge.set1.tumor.v2.withMDTags.chr2.complexvar.sam",
          "synthetic.challenge.set1.normal.v2.withMDTags.chr2.complexvar.sam")]
SUITE = dict(odds=120, min_mapq=1, min_tumor_read_depth=8, max_tumor_read_depth=200, min_normal_read_depth=4,
             min_tumor_alternate_read_depth=3, min_likelihood=70, min_vaf=5)


def _loci(rs, expr="all"):
    ls = LociSet.parse(expr).result(rs.contig_lengths_map)
    return flatten_partitions(partition_loci_uniformly(1, ls), rs.contig_index())


def _same(a, b):
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b


def assert_rows_match(got, want):
    """Strict comparison of every row, knife-edge ones included."""
    key = lambda r: (r["contig"], r["locus"], r["ref"], r["alt"])
    assert [key(r) for r in got] == [key(r) for r in want]
    for g, w in zip(got, want):
        assert g["log_odds"] == w["log_odds"], (key(g), g["log_odds"], w["log_odds"])
        assert g["gq"] == w["gq"], (key(g), g["gq"], w["gq"])
        for side in ("tumor", "normal"):
            gv, wv = g[side], w[side]
            assert all(_same(x, y) for x, y in zip(gv, wv)), (key(g), side, gv, wv)
        assert g["flags"] == w["flags"], (key(g), g["flags"], w["flags"])


@pytest.mark.parametrize("tumor,normal", PAIRS, ids=["tough", "simplefp", "syn1fp", "complexvar"])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_fixture_pairs_match_oracle(gpu_ctx, tumor, normal, mode):
    t = load_reads(fixture(tumor), TN_FILTERS)
    n = load_reads(fixture(normal), TN_FILTERS)
    loci = _loci(t)
    params = dict(SUITE, apply_filters=mode) if mode else dict(apply_filters=0)
    got = somatic_standard_reads(gpu_ctx, t, n, loci, **params)
    want = O.somatic_standard(t, n, loci, **params)
    assert len(want) > 0 or mode == 2
    assert_rows_match(got, want)


def test_suite_positive_loci_are_called(gpu_ctx):
    """SomaticStandardCallerSuite.scala:82-89 positives, through the GPU path."""
    t = load_reads(fixture("tumor.chr20.tough.sam"), TN_FILTERS)
    n = load_reads(fixture("normal.chr20.tough.sam"), TN_FILTERS)
    got = somatic_standard_reads(gpu_ctx, t, n, _loci(t), **dict(SUITE, apply_filters=2))
    called = {r["locus"] for r in got}
    for locus in (42999694, 25031215, 44061033, 45175149, 755754, 1843813, 3555766, 3868620, 9896926, 14017900):
        assert locus in called


NORMAL8 = [mr("TCGATCGA", "8M", "8", 0)] * 3


@pytest.mark.parametrize("tumor,normal,locus,expect", [
    ([mr("TCGGTCGA", "8M", "3G4", 0)] * 3, NORMAL8, 2, None),
    ([mr("TCGTCGA", "3M1D4M", "3^A4", 0)] * 3, NORMAL8, 2, ("GA", "G")),
    ([mr("TCGAAAAGCT", "5M6D5M", "5^GCTTCG5", 0)] * 3, [mr("TCGAAGCTTCGAAGCT", "16M", "16", 0)] * 3, 4,
     ("AGCTTCG", "A")),
    ([mr("TCGAGTCGA", "4M1I4M", "8", 0)] * 3, NORMAL8, 3, ("A", "AG")),
    ([mr("TCGAGGTCTCGA", "4M4I4M", "8", 0)] * 3, NORMAL8, 3, ("A", "AGGTC")),
])
def test_synthetic_indels(gpu_ctx, tumor, normal, locus, expect):  # SomaticStandardCallerSuite.scala:117-218
    t, n = make_read_set(tumor), make_read_set(normal)
    loci = (np.array([0], np.int32), np.array([locus], np.int64), np.array([locus + 1], np.int64),
            np.array([0], np.int64))
    got = somatic_standard_reads(gpu_ctx, t, n, loci, odds=2, apply_filters=0)
    assert [(r["ref"], r["alt"]) for r in got] == ([] if expect is None else [expect])
    assert_rows_match(got, O.somatic_standard(t, n, loci, odds=2, apply_filters=0))


def test_synthetic_tumor_normal_window(gpu_ctx):
    """Generator tumor (60x, somatic SNVs) / normal (30x) over a 300 kb contig: every locus."""
    L = 300_000
    tg = generate(L, 60.0, seed=20261015 + 3, somatic_rate=2e-4, tumor=True, read_seed=11)
    ng = generate(L, 30.0, seed=20261015 + 3, somatic_rate=2e-4, tumor=False, read_seed=12)
    t, n = tg.to_read_set(), ng.to_read_set()
    loci = _loci(t)
    for params in (dict(apply_filters=0), dict(apply_filters=1), dict(SUITE, apply_filters=1)):
        got = somatic_standard_reads(gpu_ctx, t, n, loci, **params)
        want = O.somatic_standard(t, n, loci, **params)
        assert_rows_match(got, want)


def test_deep_panel_500x_tumor_normal(gpu_ctx):
    """BASELINE configs[4]: 500x tumor / 500x normal over a panel-sized region (deep-pileup LDS
    stress; tiles of ~7000 reads per sample), every locus, three parameter sets.  The candidate
    pass stays on somatic_proj (~550 projection rows a block, 16-bit counts, 32-bit margin
    sums): no tile goes to the walker."""
    L = 12_000
    tg = generate(L, 500.0, seed=20261015 + 5, somatic_rate=1e-3, tumor=True, read_seed=21)
    ng = generate(L, 500.0, seed=20261015 + 5, somatic_rate=1e-3, tumor=False, read_seed=22)
    t, n = tg.to_read_set(), ng.to_read_set()
    loci = _loci(t)
    for params in (dict(apply_filters=0), dict(apply_filters=1), dict(SUITE, apply_filters=1, max_tumor_read_depth=5000)):
        got = somatic_standard_reads(gpu_ctx, t, n, loci, **params)
        assert gpu_ctx.timings()["walk_tiles"] == 0
        want = O.somatic_standard(t, n, loci, **params)
        assert_rows_match(got, want)
    assert len(want) > 0


@pytest.fixture
def deep_everywhere(monkeypatch):
    """GQ_DBG=64: the fast caller hands every candidate to the deep caller (global-memory
    element records, no depth limit), so the deep kernel runs over every ordinary case too."""
    monkeypatch.setenv("GQ_DBG", "64")
    yield


@pytest.mark.parametrize("tumor,normal", PAIRS, ids=["tough", "simplefp", "syn1fp", "complexvar"])
def test_deep_caller_on_fixture_pairs(gpu_ctx, deep_everywhere, tumor, normal):
    t = load_reads(fixture(tumor), TN_FILTERS)
    n = load_reads(fixture(normal), TN_FILTERS)
    loci = _loci(t)
    for params in (dict(apply_filters=0), dict(SUITE, apply_filters=1)):
        got = somatic_standard_reads(gpu_ctx, t, n, loci, **params)
        assert_rows_match(got, O.somatic_standard(t, n, loci, **params))


def test_deep_caller_on_synthetic_window(gpu_ctx, deep_everywhere):
    L = 60_000
    tg = generate(L, 60.0, seed=20261015 + 3, somatic_rate=1e-3, tumor=True, read_seed=31)
    ng = generate(L, 30.0, seed=20261015 + 3, somatic_rate=1e-3, tumor=False, read_seed=32)
    t, n = tg.to_read_set(), ng.to_read_set()
    loci = _loci(t)
    got = somatic_standard_reads(gpu_ctx, t, n, loci, apply_filters=1)
    want = O.somatic_standard(t, n, loci, apply_filters=1)
    assert len(want) > 0
    assert_rows_match(got, want)


def test_1000x_panel_over_several_tasks(gpu_ctx):
    """1000x tumor / 1000x normal over 3 kb split into 4 tasks: every task's first pileup is a
    heap-ordered group of ~1000 reads per sample (no capacity limit: the deep caller), and the
    likelihood normalisation underflows as the reference's does (Likelihood.scala:191-193,
    SURVEY Appendix A #15)."""
    L = 3_000
    tg = generate(L, 1000.0, seed=20261015 + 5, somatic_rate=2e-3, tumor=True, read_seed=41)
    ng = generate(L, 1000.0, seed=20261015 + 5, somatic_rate=2e-3, tumor=False, read_seed=42)
    t, n = tg.to_read_set(), ng.to_read_set()
    ls = LociSet.parse("all").result(t.contig_lengths_map)
    loci = flatten_partitions(partition_loci_uniformly(4, ls), t.contig_index())
    for params in (dict(apply_filters=0), dict(apply_filters=1, max_tumor_read_depth=100000)):
        got = somatic_standard_reads(gpu_ctx, t, n, loci, **params)
        want = O.somatic_standard(t, n, loci, **params)
        assert_rows_match(got, want)


def _insertion_sample(n_distinct, n_alt, n_ref, start=100, n_md_conflict=0):
    """n_distinct reads of distinct 6-base insertions (base quality 2, so the pileup's genotype
    likelihoods stay above FP64 underflow), n_alt reads of one 7-base insertion and n_ref
    reference reads: 10M kI 10M over a 20-base reference.  n_md_conflict more reads whose MD tag
    puts a G at the insertions' anchor locus (offset 9, a C in the others' MD-derived reference):
    the pileup reference base there depends on heap order (Pileup.scala:157-165)."""
    ref = "ACGTTGCAACGGTACCATGA"
    reads = [mr(ref[:9] + "T" + ref[10:], "20M", "9G10", start, mapq=60)] * n_md_conflict
    for i in range(n_distinct):
        ins = "".join("ACGT"[(i >> (2 * k)) & 3] for k in range(6))
        reads.append(mr(ref[:10] + ins + ref[10:], "10M6I10M", "20", start, quals=[2] * 26, mapq=60))
    reads += [mr(ref[:10] + "TTTTTTT" + ref[10:], "10M7I10M", "20", start, mapq=60)] * n_alt
    reads += [mr(ref, "20M", "20", start, mapq=60)] * n_ref
    reads.sort(key=lambda r: r["start"])
    return make_read_set(reads)


@pytest.mark.parametrize("n_tumor,n_normal", [(200, 0), (20, 20), (100, 40), (700, 0)])
def test_more_alleles_than_the_deep_table(gpu_ctx, n_tumor, n_normal):
    """Tumor pileups with 200 and 700 distinct insertion alleles (more than the deep kernel's
    128-allele table), and normals with 21-41 eligible alleles (more genotypes than its
    128-genotype scratch: the variant mass in HashTrieMap order over the wide kernel's scratch):
    the wide kernel (somatic_call_k, 1024 alleles per sample) calls them; rows equal the oracle's."""
    t = _insertion_sample(n_tumor, 40, 100)
    n = _insertion_sample(n_normal, 0, 60)
    loci = _loci(t, "chr1:90-130")
    for mode in (0, 1):
        params = dict(apply_filters=mode)
        got = somatic_standard_reads(gpu_ctx, t, n, loci, **params)
        want = O.somatic_standard(t, n, loci, **params)
        assert len(want) > 0
        assert_rows_match(got, want)


def test_wide_candidate_at_a_heap_order_locus(gpu_ctx):
    """A tumor locus with more distinct insertion alleles than the deep table (the wide kernel's)
    whose reference base depends on heap order (the reads' MD tags disagree there): the
    heap-order replay hands it to the wide kernel with the resolved base instead of raising a
    capacity error; rows equal the oracle's."""
    t = _insertion_sample(200, 40, 100, n_md_conflict=30)
    n = _insertion_sample(0, 0, 60)
    loci = _loci(t, "chr1:90-130")
    for mode in (0, 1):
        got = somatic_standard_reads(gpu_ctx, t, n, loci, apply_filters=mode)
        want = O.somatic_standard(t, n, loci, apply_filters=mode)
        assert_rows_match(got, want)


def test_reads_sharing_pool_words(gpu_ctx):
    """Wrapped device reads whose MD events and CIGAR share pool words (a deduplicated pool):
    the column records' auxiliary list is sized from the pools, so it cannot hold every read's
    events; the reads past its allocation get no list and their tiles go to the walkers instead
    of being written past its end.  Somatic rows equal the unshared upload's and the oracle's."""
    from guacamole_amd import soa
    from test_gpu_germline import _DeviceArray
    ref = "ACGTTGCAACGGTACCATGACCGTAGGTCA"
    alt = ref[:5] + "T" + ref[6:]  # read base T where the MD tag says G
    t = make_read_set([mr(alt, "30M", "5G24", 100, mapq=60)] * 300 + [mr(ref, "30M", "30", 100, mapq=60)] * 100)
    n = make_read_set([mr(ref, "30M", "30", 100, mapq=60)] * 60)
    loci = _loci(t, "chr1:90-140")
    a = soa.pack(t)
    ev = a["n_md"] > 0
    shared = dict(a, cigar=a["cigar"][:1].copy(), cigar_off=np.zeros_like(a["cigar_off"]),
                  md_ev=a["md_ev"][a["md_off"][ev][:1]].copy(), md_off=np.zeros_like(a["md_off"]))
    assert int(a["n_md"].sum()) > int(shared["md_ev"].shape[0]) + 6 * int(shared["cigar"].shape[0])
    dev = {k: (_DeviceArray(v) if np.ndim(v) else v) for k, v in shared.items()}
    tw = gpu_ctx.wrap_device(dev)
    tu = gpu_ctx.upload(a)
    nd = gpu_ctx.upload(soa.pack(n))
    for mode in (0, 1):
        got = gpu_ctx.somatic_standard(tw, nd, loci, apply_filters=mode).rows
        assert got == gpu_ctx.somatic_standard(tu, nd, loci, apply_filters=mode).rows
        got = [dict(r, contig=t.contig_names[r["contig"]]) for r in got]
        want = O.somatic_standard(t, n, loci, apply_filters=mode)
        assert len(want) == 1
        assert_rows_match(got, want)
