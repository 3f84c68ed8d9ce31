"""CPU tests of vaf-histogram's oracle (VAFHistogram.scala:31-37, 188-229): the histogram
against one built from the oracle's raw per-locus pileup counts (depth, Match elements), and a
small KAT."""
import numpy as np
import pytest

from conftest import fixture
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.reads import InputFilters, load_reads, make_read as mr, make_read_set
from oracle import oracle as O


def _loci(rs, expr="all", tasks=1):
    ls = LociSet.parse(expr).result(rs.contig_lengths_map)
    return flatten_partitions(partition_loci_uniformly(tasks, ls), rs.contig_index())


def _from_stats(rows, bins, min_depth, min_vaf):
    hist, variant = {}, 0
    size = 100 // bins
    for r in rows:
        depth, ref = r[3], r[7]
        if ref == depth:
            continue
        vaf = np.float32(depth - ref) / np.float32(depth)
        if not (depth >= min_depth and float(vaf) >= min_vaf / 100.0):
            continue
        pct = int(vaf * np.float32(100))
        hist[pct - pct % size] = hist.get(pct - pct % size, 0) + 1
        variant += 1
    return hist, variant


@pytest.mark.parametrize("bins,min_depth,min_vaf", [(20, 0, 0), (7, 50, 5), (100, 0, 30)])
def test_chrm_histogram_matches_counts(bins, min_depth, min_vaf):
    rs = load_reads(fixture("chrM.sorted.bam"), InputFilters())
    loci = _loci(rs, "chrM:0-16571", 3)
    want = _from_stats(O.pileup_stats(rs, loci), bins, min_depth, min_vaf)
    assert O.vaf_histogram(rs, loci, bins, min_depth, min_vaf) == want
    assert want[1] > 0


def test_kat_vaf():  # noqa: D103
    # 4 reads, one with a mismatch at locus 3: VAF 0.25 -> bin 25 (bins 20: width 5)
    reads = [mr("TCGATCGA", "8M", "8", 0)] * 3 + [mr("TCGGTCGA", "8M", "3A4", 0)]
    rs = make_read_set(reads)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([8], np.int64), np.array([0], np.int64))
    assert O.vaf_histogram(rs, loci, 20) == ({25: 1}, 1)
    assert O.vaf_histogram(rs, loci, 20, 5) == ({}, 0)       # depth 4 < 5
    assert O.vaf_histogram(rs, loci, 20, 0, 26) == ({}, 0)   # 0.25 < 0.26
    with pytest.raises(O.OracleError, match="Bins should be between 1 and 100"):
        O.vaf_histogram(rs, loci, 0)


def suite_reads():
    """20 reads over loci 0-7 (reference A) whose mismatch counts give VAFs 0.25, 0.35, 0.4,
    0.5, 0.55 at loci 1-5 (VAFHistogramSuite's loci, built as pileups)."""
    mism = {1: 5, 2: 7, 3: 8, 4: 10, 5: 11}
    reads = []
    for i in range(20):
        seq, md, run = [], [], 0
        for l in range(8):
            if l in mism and i < mism[l]:
                seq.append("C")
                md.append("%dA" % run)
                run = 0
            else:
                seq.append("A")
                run += 1
        reads.append(mr("".join(seq), "8M", "".join(md) + str(run), 0))
    return make_read_set(reads)


SUITE_HIST = {10: {20: 1, 30: 1, 40: 1, 50: 2}, 20: {25: 1, 35: 1, 40: 1, 50: 1, 55: 1},
              100: {25: 1, 35: 1, 40: 1, 50: 1, 55: 1}}


@pytest.mark.parametrize("bins", [10, 20, 100])
def test_vaf_histogram_suite(bins):
    """VAFHistogramSuite.scala:8-43 (generateVAFHistogram at 10 / 20 / 100 bins)."""
    rs = suite_reads()
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([8], np.int64), np.array([0], np.int64))
    assert O.vaf_histogram(rs, loci, bins) == (SUITE_HIST[bins], 5)
