"""GPU parity: germline-standard (gq_germline_standard, HIP) vs the CPU oracle
(GermlineStandard.Caller.callVariantsAtLocus + GenotypeFilter,
commands/GermlineStandardCaller.scala:63-124): every CalledAllele row — locus, sample, ref,
alt, likelihood, evidence — identical."""
import os
from dataclasses import replace

import numpy as np
import pytest

from conftest import fixture
from guacamole_amd.commands import germline_standard_reads, main
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.output import read_avro_json
from guacamole_amd.reads import InputFilters, load_reads
from guacamole_amd.synthetic import generate
from oracle import oracle as O

from test_gpu_somatic import _same

pytestmark = pytest.mark.gpu

# GermlineStandard.Caller.run input filters (GermlineStandardCaller.scala:53-54)
FILTERS = InputFilters.make(mapped=True, non_duplicate=True, has_md_tag=True)


def _loci(rs, expr="all", tasks=1):
    ls = LociSet.parse(expr).result(rs.contig_lengths_map)
    return flatten_partitions(partition_loci_uniformly(tasks, ls), rs.contig_index())


def assert_rows_match(got, want):
    key = lambda r: (r["contig"], r["locus"], r["sample"], r["ref"], r["alt"])
    assert [key(r) for r in got] == [key(r) for r in want]
    for g, w in zip(got, want):
        assert g["log_odds"] == w["log_odds"], (key(g), g["log_odds"], w["log_odds"])
        assert g["gq"] == w["gq"], (key(g), g["gq"], w["gq"])
        assert all(_same(x, y) for x, y in zip(g["tumor"], w["tumor"])), (key(g), g["tumor"], w["tumor"])
        assert g["flags"] == w["flags"], key(g)


@pytest.mark.parametrize("params", [dict(), dict(min_mapq=20), dict(min_mapq=0),
                                    dict(min_read_depth=20, min_alternate_read_depth=4, min_likelihood=40,
                                         apply_filters=1)],
                         ids=["default", "mapq20", "mapq0", "filters"])
def test_chrm_matches_oracle(gpu_ctx, params):
    rs = load_reads(fixture("chrM.sorted.bam"), FILTERS)
    loci = _loci(rs, "chrM:0-16571", 3)
    got = germline_standard_reads(gpu_ctx, rs, loci, **params)
    want = O.germline_standard(rs, loci, **params)
    assert len(want) > 10
    assert_rows_match(got, want)
    if not params:
        assert any(r["flags"] & 1 for r in want)  # heap-order reference bases exercised


@pytest.mark.parametrize("name", ["tumor.chr20.tough.sam", "normal.chr20.simplefp.sam",
                                  "synthetic.challenge.set1.tumor.v2.withMDTags.chr2.complexvar.sam"])
def test_fixtures_match_oracle(gpu_ctx, name):
    rs = load_reads(fixture(name), FILTERS)
    loci = _loci(rs)
    assert_rows_match(germline_standard_reads(gpu_ctx, rs, loci), O.germline_standard(rs, loci))


def test_synthetic_indels_match_oracle(gpu_ctx):
    rs = generate(40_000, 30, seed=13, indel_rate=1e-3).to_read_set()
    loci = _loci(rs, "20:0-40000", 2)
    got = germline_standard_reads(gpu_ctx, rs, loci)
    want = O.germline_standard(rs, loci)
    assert len(want) > 20 and any(len(r["ref"]) > 1 or len(r["alt"]) > 1 for r in want)
    assert_rows_match(got, want)


def test_two_samples_match_oracle(gpu_ctx):
    """Reads of two samples: one genotype per sample per locus (GermlineStandardCaller.scala:96-99)."""
    rs = generate(30_000, 40, seed=17, indel_rate=5e-4).to_read_set()
    rs = replace(rs, sample=(np.arange(len(rs.sample)) % 2).astype(np.int32), sample_names=["s0", "s1"])
    loci = _loci(rs, "20:0-30000", 2)
    got = germline_standard_reads(gpu_ctx, rs, loci)
    want = O.germline_standard(rs, loci)
    assert {r["sample"] for r in want} == {0, 1}
    assert_rows_match(got, want)


def test_cli_germline_standard(tmp_path):
    out = tmp_path / "g.json"
    bam = fixture("chrM.sorted.bam")
    assert main(["germline-standard", "--reads", bam, "--out", str(out), "--loci", "chrM:0-6000",
                 "--min-read-depth", "10"]) == 0
    recs = [r["variant"]["org.bdgenomics.formats.avro.Variant"] if "org.bdgenomics.formats.avro.Variant" in r["variant"]
            else r["variant"]["Variant"] for r in read_avro_json(open(out).read())]
    rs = load_reads(bam, FILTERS)
    want = O.germline_standard(rs, _loci(rs, "chrM:0-6000"), min_read_depth=10, apply_filters=1)
    assert len(want) > 5
    assert [(v["start"]["long"], v["alternateAllele"]["string"]) for v in recs] == [(w["locus"], w["alt"]) for w in want]
    assert all(v["end"]["long"] == v["start"]["long"] + 1 for v in recs)


def test_deep_pileups_match_oracle(gpu_ctx):
    """1500x with the window's initial group deeper than the LDS cover list (768 reads), and a
    locus with 200 distinct insertion alleles (past the fast allele table and genotype array):
    both handed to the deep instantiation, no capacity error (the reference has no depth limit)."""
    from test_gpu_germline import _many_insertions
    rs = generate(3_000, 1500, seed=19, indel_rate=1e-3).to_read_set()
    loci = _loci(rs, "20:200-2800", 2)
    got = germline_standard_reads(gpu_ctx, rs, loci)
    want = O.germline_standard(rs, loci)
    assert len(want) > 0
    assert_rows_match(got, want)
    rs = _many_insertions(200, n_ref=60, n_alt=120, singleton_qual=5)  # (low: no likelihood underflow)
    loci = _loci(rs, "chr1:90-130")
    want = O.germline_standard(rs, loci)
    assert any(len(r["alt"]) > 1 for r in want)
    assert_rows_match(germline_standard_reads(gpu_ctx, rs, loci), want)
