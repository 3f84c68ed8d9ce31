"""GPU parity for branches the first round left untested, each against the CPU oracle:

* several samples (read groups) through germline-threshold: Pileup.bySample
  (pileup/Pileup.scala:57-61), per-sample decisions in the general-allele kernel;
* the somatic pileup filters: --filter-multi-allelic (filters/PileupFilter.scala:29-44) and
  --min-mapq 0 / 20 (filters/PileupElementsFilter.scala:25-36);
* several contigs with b37 names: contigs are iterated lexicographically (LociMap.scala:39-42),
  so "10" comes before "2" in the output;
* many tasks: one SlidingWindow (and one initial heap-ordered pileup) per task and contig
  (DistributedUtil.scala:473-486), so somatic FP sums see many window starts;
* heap-order reference bases in somatic-standard (both samples' queues replayed);
* knife-edge somatic rows, compared bit for bit;
* the error paths: a read without MD tag (ReferenceWithoutMDTagException, MappedRead.scala:141),
  "Multiple reference bases found" (GermlineThresholdCaller.scala:171-174), unsorted reads
  ("Regions must be sorted", SlidingWindow.scala:55-56) and out-of-pool offsets at upload.
"""
import dataclasses

import numpy as np
import pytest

from conftest import fixture
from guacamole_amd import native, soa
from guacamole_amd.commands import germline_threshold_reads, somatic_standard_reads
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.reads import InputFilters, ReadSet, load_reads, make_read as mr, make_read_set
from guacamole_amd.synthetic import generate
from oracle import oracle as O
from test_gpu_somatic import TN_FILTERS, assert_rows_match

pytestmark = pytest.mark.gpu


def _loci(rs, expr="all", tasks=1):
    ls = LociSet.parse(expr).result(rs.contig_lengths_map)
    return flatten_partitions(partition_loci_uniformly(tasks, ls), rs.contig_index())


@pytest.fixture(scope="module")
def chrm():
    return load_reads(fixture("chrM.sorted.bam"),
                      InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True))


def _with_samples(rs: ReadSet, k: int) -> ReadSet:
    """The same reads spread over k samples (read r -> sample r % k)."""
    return dataclasses.replace(rs, sample=(np.arange(rs.n) % k).astype(np.int32),
                               sample_names=["s%d" % i for i in range(k)], _gq=None)


@pytest.mark.parametrize("k", [2, 3])
def test_multi_sample_germline_chrm(gpu_ctx, chrm, k):
    rs = _with_samples(chrm, k)
    loci = _loci(rs)
    for args in ((8, False, False), (30, True, True)):
        got = germline_threshold_reads(gpu_ctx, rs, loci, *args)
        want = O.germline_threshold(rs, loci, *args)
        assert got == want, args
        assert {r[2] for r in want} == set(range(k))  # every sample calls somewhere


def test_multi_sample_germline_synthetic(gpu_ctx):
    g = generate(60_000, 30, seed=31, indel_rate=3e-4)
    rs = _with_samples(g.to_read_set(), 2)
    loci = _loci(rs)
    got = germline_threshold_reads(gpu_ctx, rs, loci, 8, True, False)
    want = O.germline_threshold(rs, loci, 8, True, False)
    assert got == want
    assert any(r[2] == 1 for r in want)


@pytest.mark.parametrize("params", [dict(filter_multi_allelic=1), dict(min_mapq=0), dict(min_mapq=20),
                                    dict(filter_multi_allelic=1, min_mapq=20)],
                         ids=["multi_allelic", "mapq0", "mapq20", "both"])
def test_somatic_pileup_filters(gpu_ctx, params):
    for tumor, normal in (("tumor.chr20.tough.sam", "normal.chr20.tough.sam"),
                          ("synthetic.challenge.set1.tumor.v2.withMDTags.chr2.syn1fp.sam",
                           "synthetic.challenge.set1.normal.v2.withMDTags.chr2.syn1fp.sam")):
        t = load_reads(fixture(tumor), TN_FILTERS)
        n = load_reads(fixture(normal), TN_FILTERS)
        loci = _loci(t)
        for mode in (0, 1):
            got = somatic_standard_reads(gpu_ctx, t, n, loci, apply_filters=mode, **params)
            want = O.somatic_standard(t, n, loci, apply_filters=mode, **params)
            assert_rows_match(got, want)


@pytest.fixture(scope="module")
def tn200k():
    L = 200_000
    tg = generate(L, 60.0, seed=20261015 + 3, somatic_rate=2e-4, tumor=True, read_seed=41)
    ng = generate(L, 30.0, seed=20261015 + 3, somatic_rate=2e-4, tumor=False, read_seed=42)
    return tg.to_read_set(), ng.to_read_set()


@pytest.mark.parametrize("params", [dict(filter_multi_allelic=1), dict(min_mapq=20), dict(min_mapq=0, apply_filters=0)],
                         ids=["multi_allelic", "mapq20", "mapq0_raw"])
def test_somatic_filters_synthetic(gpu_ctx, tn200k, params):
    t, n = tn200k
    loci = _loci(t)
    got = somatic_standard_reads(gpu_ctx, t, n, loci, **params)
    want = O.somatic_standard(t, n, loci, **params)
    assert_rows_match(got, want)
    assert want


def _merge(sets, names):
    """One ReadSet over several single-contig ReadSets (contig i = sets[i]), pools concatenated."""
    def cat(key, dt):
        return np.concatenate([np.asarray(getattr(s, key), dt) for s in sets])

    def offs(key, pool):
        out, base = [], 0
        for s in sets:
            out.append(np.asarray(getattr(s, key), np.int64) + base)
            base += len(getattr(s, pool))
        return np.concatenate(out)

    return ReadSet(contig_names=list(names), contig_lengths=[s.contig_lengths[0] for s in sets],
                   sample_names=list(sets[0].sample_names),
                   contig=np.concatenate([np.full(s.n, i, np.int32) for i, s in enumerate(sets)]),
                   start=cat("start", np.int64), end=cat("end", np.int64), mapq=cat("mapq", np.uint8),
                   flags=cat("flags", np.uint8), sample=cat("sample", np.int32), seq_off=offs("seq_off", "seq"),
                   seq_len=cat("seq_len", np.int32), seq=cat("seq", np.uint8), qual=cat("qual", np.uint8),
                   cigar_off=offs("cigar_off", "cigar"), n_cigar=cat("n_cigar", np.int32),
                   cigar=cat("cigar", np.uint32), md_off=offs("md_off", "md"), md_len=cat("md_len", np.int32),
                   md=cat("md", np.uint8))


B37 = ["1", "2", "10", "X"]  # sequence-dictionary order; lexicographic output order is 1, 10, 2, X


def test_multi_contig_b37_germline(gpu_ctx):
    rs = _merge([generate(30_000, 30, seed=50 + i, indel_rate=3e-4).to_read_set() for i in range(4)], B37)
    for tasks in (1, 3):
        loci = _loci(rs, tasks=tasks)
        got = germline_threshold_reads(gpu_ctx, rs, loci, 8)
        want = O.germline_threshold(rs, loci, 8)
        assert got == want
        order = [c for i, c in enumerate(r[0] for r in got) if i == 0 or c != got[i - 1][0]]
        assert order == sorted(B37), order  # "1" < "10" < "2" < "X"


def test_multi_contig_b37_somatic(gpu_ctx):
    t = _merge([generate(40_000, 60.0, seed=60 + i, somatic_rate=1e-3, tumor=True, read_seed=70 + i).to_read_set()
                for i in range(4)], B37)
    n = _merge([generate(40_000, 30.0, seed=60 + i, somatic_rate=1e-3, tumor=False, read_seed=80 + i).to_read_set()
                for i in range(4)], B37)
    loci = _loci(t)
    got = somatic_standard_reads(gpu_ctx, t, n, loci, apply_filters=0)
    want = O.somatic_standard(t, n, loci, apply_filters=0)
    assert_rows_match(got, want)
    assert [c for c in dict.fromkeys(r["contig"] for r in want)] == sorted(B37)


@pytest.mark.parametrize("tasks", [7, 97])
def test_somatic_many_tasks(gpu_ctx, tasks):
    """A window per task and contig: the first pileup of each takes the queue's heap order, so
    the per-element FP sums near every window start follow it (DistributedUtil.scala:260-274)."""
    t = load_reads(fixture("tumor.chr20.tough.sam"), TN_FILTERS)
    n = load_reads(fixture("normal.chr20.tough.sam"), TN_FILTERS)
    loci = _loci(t, tasks=tasks)
    got = somatic_standard_reads(gpu_ctx, t, n, loci, apply_filters=0, odds=2)
    want = O.somatic_standard(t, n, loci, apply_filters=0, odds=2)
    assert_rows_match(got, want)
    g = generate(100_000, 60.0, seed=91, somatic_rate=5e-4, tumor=True, read_seed=92).to_read_set()
    h = generate(100_000, 30.0, seed=91, somatic_rate=5e-4, tumor=False, read_seed=93).to_read_set()
    loci = _loci(g, tasks=tasks)
    got = somatic_standard_reads(gpu_ctx, g, h, loci, apply_filters=0, odds=2)
    want = O.somatic_standard(g, h, loci, apply_filters=0, odds=2)
    assert_rows_match(got, want)


def test_somatic_heap_order_reference_bases(gpu_ctx, chrm):
    """chrM's reads disagree on the MD-derived base at a few loci: tumor = every read, normal =
    every other read; both windows' queues are replayed where either sample is ambiguous."""
    normal = chrm.subset(np.arange(0, chrm.n, 2))
    loci = _loci(chrm)
    for params in (dict(apply_filters=0, odds=1), dict(apply_filters=0, odds=1, min_mapq=0)):
        got = somatic_standard_reads(gpu_ctx, chrm, normal, loci, **params)
        want = O.somatic_standard(chrm, normal, loci, **params)
        assert_rows_match(got, want)
    assert any(r["flags"] & 3 for r in want), "a call at a heap-order-dependent locus"


def test_knife_edge_rows_compared(gpu_ctx):
    """Calls whose odds test lands within an ulp of its threshold (germline hets: odds = 1 +- ulp
    against --min-lod 0) are present and identical on both sides."""
    L = 300_000
    tg = generate(L, 60.0, seed=20261015 + 3, somatic_rate=2e-4, tumor=True, read_seed=11)
    ng = generate(L, 30.0, seed=20261015 + 3, somatic_rate=2e-4, tumor=False, read_seed=12)
    t, n = tg.to_read_set(), ng.to_read_set()
    loci = _loci(t)
    got = somatic_standard_reads(gpu_ctx, t, n, loci, apply_filters=1)
    want = O.somatic_standard(t, n, loci, apply_filters=1)
    assert_rows_match(got, want)
    assert any(r["flags"] & native.FLAG_KNIFE_EDGE for r in want)


def _err_code(fn):
    with pytest.raises(native.GQError) as e:
        fn()
    return e.value.code


def test_error_read_without_md(gpu_ctx):
    reads = [mr("TCGATCGA", "8M", "8", 1), mr("TCGATCGA", "8M", None, 1), mr("TCGATCGA", "8M", "8", 1)]
    rs = make_read_set(reads)
    loci = _loci(rs, "chr1:0-20")
    assert _err_code(lambda: germline_threshold_reads(gpu_ctx, rs, loci, 8)) == 4  # GQ_E_NO_MD
    with pytest.raises(O.OracleError) as e:
        O.germline_threshold(rs, loci, 8)
    assert e.value.code == 4


def test_error_multiple_reference_bases(gpu_ctx):
    """Two non-variant alleles with different bases pass the threshold: (A, A) Match elements and
    (G, G) 'insertions' of reads whose sequence stops at the anchor (4M2I over 4 bases)."""
    reads = [mr("TCGA", "4M", "4", 1)] * 2 + [mr("TCGG", "4M2I", "3A0", 1)] * 2
    rs = make_read_set(reads)
    loci = _loci(rs, "chr1:0-20")
    assert _err_code(lambda: germline_threshold_reads(gpu_ctx, rs, loci, 8)) == 5  # GQ_E_MULTI_REF
    with pytest.raises(O.OracleError) as e:
        O.germline_threshold(rs, loci, 8)
    assert e.value.code == 5


def test_error_unsorted_and_bad_offsets(gpu_ctx):
    g = generate(20_000, 10, seed=97)
    a = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) and v.ndim else v) for k, v in g.arrays.items()}
    ok = gpu_ctx.upload(a)  # the generator's arrays are valid
    ok.free()
    s = dict(a)
    s["start"] = a["start"].copy()
    s["start"][10], s["start"][11] = a["start"][11] + 5, a["start"][10]  # two reads out of order
    assert _err_code(lambda: gpu_ctx.upload(s)) == 6  # GQ_E_UNSORTED
    p = dict(a)
    p["pmax_end"] = a["pmax_end"].copy()
    p["pmax_end"][100] -= 1  # not the running maximum
    assert _err_code(lambda: gpu_ctx.upload(p)) == 6
    o = dict(a)
    o["seq_off"] = a["seq_off"].copy()
    o["seq_off"][-1] = int(a["seq"].shape[0])  # past the pool
    assert _err_code(lambda: gpu_ctx.upload(o)) == 7  # GQ_E_ARG
