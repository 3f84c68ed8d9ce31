"""GPU parity: vaf-histogram (gq_vaf_histogram, HIP) vs the CPU oracle (VAFHistogram.scala:
31-37, 188-229): every bin count identical, heap-order reference bases included (chrM)."""
import numpy as np
import pytest

from conftest import fixture
from guacamole_amd.commands import main, vaf_histogram_reads
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.reads import InputFilters, load_reads
from guacamole_amd.synthetic import generate
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _loci(rs, expr="all", tasks=1):
    ls = LociSet.parse(expr).result(rs.contig_lengths_map)
    return flatten_partitions(partition_loci_uniformly(tasks, ls), rs.contig_index())


@pytest.mark.parametrize("bins,min_depth,min_vaf,tasks", [(20, 0, 0, 1), (7, 50, 5, 3), (100, 0, 30, 800), (1, 0, 0, 1)])
def test_chrm_matches_oracle(gpu_ctx, bins, min_depth, min_vaf, tasks):
    rs = load_reads(fixture("chrM.sorted.bam"), InputFilters())
    loci = _loci(rs, "chrM:0-16571", tasks)
    got = vaf_histogram_reads(gpu_ctx, rs, loci, bins, min_depth, min_vaf)
    want_h, want_n = O.vaf_histogram(rs, loci, bins, min_depth, min_vaf)
    assert got["histogram"] == want_h and got["variant_loci"] == want_n
    assert want_n > 0


def test_synthetic_matches_oracle(gpu_ctx):
    g = generate(200_000, 30, seed=9, indel_rate=3e-4)
    rs = g.to_read_set()
    loci = _loci(rs)
    got = vaf_histogram_reads(gpu_ctx, rs, loci, 20, 10, 0)
    assert (got["histogram"], got["variant_loci"]) == O.vaf_histogram(rs, loci, 20, 10, 0)


def test_cli_vaf_histogram(tmp_path):
    out = tmp_path / "h.csv"
    bam = fixture("chrM.sorted.bam")
    assert main(["vaf-histogram", "--local-out", str(out), "--bins", "10", "--loci", "chrM", bam]) == 0
    lines = open(out).read().splitlines()
    assert lines[0] == "Filename, SampleName, BinStart, BinEnd, Size"
    rs = load_reads(bam, InputFilters())
    want_h, _ = O.vaf_histogram(rs, _loci(rs, "chrM"), 10)
    sample = rs.sample_names[int(rs.sample[0])]
    assert lines[1:] == ["%s, %s, %d, %d, %d" % (bam, sample, b, min(b + 10, 100), n) for b, n in sorted(want_h.items())]


@pytest.mark.parametrize("bins", [10, 20, 100])
def test_vaf_histogram_suite_gpu(gpu_ctx, bins):
    """VAFHistogramSuite.scala:8-43 through the device binning."""
    from test_vaf_histogram import SUITE_HIST, suite_reads
    rs = suite_reads()
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([8], np.int64), np.array([0], np.int64))
    got = vaf_histogram_reads(gpu_ctx, rs, loci, bins)
    assert got["histogram"] == SUITE_HIST[bins] and got["variant_loci"] == 5
