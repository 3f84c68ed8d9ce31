"""CPU tests of germline-standard's oracle (GermlineStandardCaller.scala:90-124): built from the
Likelihood / AlleleEvidence restatements the KAT suites pin (LikelihoodSuite,
AlleleEvidenceSuite); here the caller's own rules on small pileups."""
import numpy as np

from guacamole_amd.reads import make_read as mr, make_read_set
from oracle import oracle as O

LOCI = (np.array([0], np.int32), np.array([0], np.int64), np.array([8], np.int64), np.array([0], np.int64))


def test_hom_alt_emits_the_allele_twice():
    """Genotype.getNonReferenceAlleles keeps both alleles of a hom-alt genotype
    (variants/Genotype.scala:46-48): two CalledAlleles."""
    rs = make_read_set([mr("TCGGTCGA", "8M", "3A4", 0)] * 6)
    rows = [(r["locus"], r["ref"], r["alt"]) for r in O.germline_standard(rs, LOCI)]
    assert rows == [(3, "A", "G"), (3, "A", "G")]


def test_het_and_hom_ref():
    rs = make_read_set([mr("TCGATCGA", "8M", "8", 0)] * 5 + [mr("TCGGTCGA", "8M", "3A4", 0)] * 5)
    rows = O.germline_standard(rs, LOCI)
    assert [(r["locus"], r["ref"], r["alt"]) for r in rows] == [(3, "A", "G")]
    ev = rows[0]["tumor"]
    assert ev[1] == 10 and ev[2] == 5  # readDepth, alleleReadDepth over the sample's pileup
    assert O.germline_standard(make_read_set([mr("TCGATCGA", "8M", "8", 0)] * 5), LOCI) == []


def test_mapq_filter_and_genotype_filters():
    reads = [mr("TCGATCGA", "8M", "8", 0, mapq=30)] * 5 + [mr("TCGGTCGA", "8M", "3A4", 0, mapq=5)] * 5
    rs = make_read_set(reads)
    assert O.germline_standard(rs, LOCI, min_mapq=10) == []     # the G reads are filtered out
    assert len(O.germline_standard(rs, LOCI, min_mapq=1)) == 1
    assert O.germline_standard(rs, LOCI, min_read_depth=11) == []
    assert O.germline_standard(rs, LOCI, min_alternate_read_depth=6) == []
    assert len(O.germline_standard(rs, LOCI, min_alternate_read_depth=5)) == 1
