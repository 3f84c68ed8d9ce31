"""GPU parity: variant-support (gq_variant_support, HIP) vs the CPU oracle
(VariantSupport.pileupToAlleleCounts, commands/VariantSupport.scala:110-118): every row —
sample, locus, ref, alt, count, flags — identical, heap-order reference bases included."""
import os

import numpy as np
import pytest

from conftest import fixture
from guacamole_amd.commands import main, variant_support_reads
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.reads import InputFilters, load_reads
from guacamole_amd.synthetic import generate
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _loci(rs, expr, tasks=1):
    ls = LociSet.parse(expr).result(rs.contig_lengths_map)
    return flatten_partitions(partition_loci_uniformly(tasks, ls), rs.contig_index())


def _oracle(rs, loci):
    return [(rs.sample_names[s], c, l, ref, alt, n, f) for s, c, l, ref, alt, n, f in O.variant_support(rs, loci)]


@pytest.mark.parametrize("nondup", [False, True])
def test_gatk_region_matches_oracle(gpu_ctx, nondup):
    rs = load_reads(fixture("gatk_mini_bundle_extract.bam"),
                    InputFilters.make(mapped=True, non_duplicate=nondup, has_md_tag=True))
    for expr, tasks in (("20:9999900-10010100", 1), ("20:10007000-10009100", 3), ("20:10007174-10007175", 1)):
        loci = _loci(rs, expr, tasks)
        got = variant_support_reads(gpu_ctx, rs, loci)
        assert got == _oracle(rs, loci), expr
    got = variant_support_reads(gpu_ctx, rs, _loci(rs, "20:10008920-10008921"))
    if nondup:
        assert {r[4]: r[5] for r in got} == {"C": 2, "CA": 1, "CAA": 1}


def test_chrm_matches_oracle_with_heap_order_bases(gpu_ctx):
    rs = load_reads(fixture("chrM.sorted.bam"), InputFilters.make(mapped=True, has_md_tag=True))
    loci = _loci(rs, "chrM:0-16571", 4)
    got = variant_support_reads(gpu_ctx, rs, loci)
    want = _oracle(rs, loci)
    assert got == want
    assert any(r[6] & 1 for r in want)  # heap-order reference bases exercised


def test_synthetic_indels_match_oracle(gpu_ctx):
    g = generate(40_000, 30, seed=11, indel_rate=1e-3)
    rs = g.to_read_set()
    loci = _loci(rs, "20:0-40000", 2)
    got = variant_support_reads(gpu_ctx, rs, loci)
    assert got == _oracle(rs, loci)
    assert any(len(r[3]) > 1 or len(r[4]) > 1 for r in got)


def test_cli_variant_support(tmp_path):
    v = tmp_path / "v.vcf"
    v.write_text("##fileformat=VCFv4.1\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n"
                 "20\t10007175\t.\tC\tT\t.\t.\t.\n20\t10008921\t.\tCAA\tC,CA\t.\t.\t.\n20\t10009054\t.\tT\tA\t.\t.\t.\n")
    out = tmp_path / "out"
    bam = fixture("gatk_mini_bundle_extract.bam")
    assert main(["variant-support", "-v", str(v), "-o", str(out), "--parallelism", "2", bam, bam]) == 0
    parts = sorted(p for p in os.listdir(out) if p.startswith("part-"))
    assert parts == ["part-%05d" % i for i in range(4)] and os.path.exists(out / "_SUCCESS")
    lines = [l.rstrip("\n") for p in parts for l in open(out / p)]
    rs = load_reads(bam)
    ls = LociSet.parse("20:10007174-10007175,20:10008920-10008923,20:10009053-10009054").result()
    want = ["%s, %s, %d, %s, %s, %d" % r[:6] for r in _oracle(rs, flatten_partitions(
        partition_loci_uniformly(2, ls), rs.contig_index()))]
    assert lines == want + want


def test_deep_pileups_match_oracle(gpu_ctx):
    """1500x, and a locus with 200 distinct insertion alleles (past the fast table of 128):
    the deep instantiation, no capacity error."""
    from test_gpu_germline import _many_insertions
    rs = generate(3_000, 1500, seed=23, indel_rate=1e-3).to_read_set()
    loci = _loci(rs, "20:200-2800", 2)
    assert variant_support_reads(gpu_ctx, rs, loci) == _oracle(rs, loci)
    rs = _many_insertions(200, n_ref=60, n_alt=120, singleton_qual=5)  # (low: no likelihood underflow)
    loci = _loci(rs, "chr1:90-130")
    got = variant_support_reads(gpu_ctx, rs, loci)
    assert got == _oracle(rs, loci) and len({r[4] for r in got if r[2] == 109}) > 200
