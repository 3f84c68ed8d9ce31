"""GPU parity: somatic-standard with --reference-fasta (gq_somatic_standard_ref) vs the CPU oracle.

Every pileup's reference base is the reference genome's (DistributedUtil.scala:266-268).  Inputs:
  * the reference's MD-less fixtures (tumor/normal_without_mdtag.sam) with MD rebuilt from the
    reference's soft-masked chrMT FASTA (Read.scala:241-247), contig renamed to the reads' chrM;
  * tumor/normal.chr20.tough with a FASTA cut from the fixture's MD-reconstructed reference, once
    as is and once with every 37th covered base changed (the FASTA then disagrees with the reads'
    MD, so the candidate kernels must hand those loci to the exact caller).
Rows compared bit for bit as in test_gpu_somatic.py."""
import numpy as np
import pytest

from conftest import fixture
from guacamole_amd import native
from guacamole_amd.commands import somatic_standard_reads
from guacamole_amd.reads import InputFilters, load_reads, make_read as mr, make_read_set
from guacamole_amd.reference import ReferenceGenome
from oracle import oracle as O
from reference_helpers import assembled_reference
from test_gpu_somatic import SUITE, _loci, assert_rows_match

pytestmark = pytest.mark.gpu

TN_FILTERS = InputFilters.make(mapped=True, non_duplicate=True, passed_vendor_quality_checks=True, has_md_tag=True)


def _mt_reference():
    mt = ReferenceGenome.load_fasta(fixture("human_GRCh37_75_dna_chrMT.fasta")).get_contig("MT")
    return ReferenceGenome({"chrM": mt})


@pytest.mark.parametrize("mode", [0, 1])
def test_mdless_fixtures_with_reference(gpu_ctx, mode):
    ref = _mt_reference()
    t = load_reads(fixture("tumor_without_mdtag.sam"), TN_FILTERS, reference=ref)
    n = load_reads(fixture("normal_without_mdtag.sam"), TN_FILTERS, reference=ref)
    assert t.n == 50 and n.n == 50
    loci = _loci(t)
    params = dict(apply_filters=mode)
    got = somatic_standard_reads(gpu_ctx, t, n, loci, reference=ref, **params)
    want = O.somatic_standard(t, n, loci, reference=ref, **params)
    assert len(want) > 0
    assert_rows_match(got, want)


@pytest.fixture(scope="module")
def tough():
    t = load_reads(fixture("tumor.chr20.tough.sam"), TN_FILTERS)
    n = load_reads(fixture("normal.chr20.tough.sam"), TN_FILTERS)
    return t, n


@pytest.mark.parametrize("modify_every", [0, 37], ids=["md_reference", "modified"])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_tough_with_reference(gpu_ctx, tough, modify_every, mode):
    t, n = tough
    ref = ReferenceGenome(assembled_reference(t, n, modify_every=modify_every))
    loci = _loci(t)
    params = dict(SUITE, apply_filters=mode) if mode else dict(apply_filters=0)
    got = somatic_standard_reads(gpu_ctx, t, n, loci, reference=ref, **params)
    want = O.somatic_standard(t, n, loci, reference=ref, **params)
    assert len(want) > 0 or mode == 2
    assert_rows_match(got, want)
    assert all(r["flags"] & 3 == 0 for r in got)


def test_reference_base_decides_call(gpu_ctx):
    """test_reference.test_oracle_reference_changes_calls through the GPU path."""
    t = make_read_set([mr("TCGATCGA", "8M", "8", 0)] * 4)
    n = make_read_set([mr("TCAATCGA", "8M", "8", 0)] * 4)
    loci = (np.array([0], np.int32), np.array([2], np.int64), np.array([3], np.int64), np.array([0], np.int64))
    assert somatic_standard_reads(gpu_ctx, t, n, loci, odds=2, apply_filters=0) == []
    ref = ReferenceGenome({t.contig_names[0]: np.frombuffer(b"TCAATCGAAAAA", np.uint8)})
    got = somatic_standard_reads(gpu_ctx, t, n, loci, reference=ref, odds=2, apply_filters=0)
    assert [(r["locus"], r["ref"], r["alt"]) for r in got] == [(2, "A", "G")]
    assert_rows_match(got, O.somatic_standard(t, n, loci, reference=ref, odds=2, apply_filters=0))


def test_reference_errors(gpu_ctx):
    """ContigNotFound where reads cover a contig the reference lacks; a locus past the reference
    contig's end where a read covers it; loci no read reaches are not looked up."""
    t = make_read_set([mr("TCGATCGA", "8M", "8", 0)] * 2)
    n = make_read_set([mr("TCGATCGA", "8M", "8", 0)] * 2)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([8], np.int64), np.array([0], np.int64))
    with pytest.raises(native.GQError, match="does not exist in the current reference"):
        somatic_standard_reads(gpu_ctx, t, n, loci, reference=ReferenceGenome({"other": np.zeros(8, np.uint8)}))
    short = ReferenceGenome({t.contig_names[0]: np.frombuffer(b"TCGAT", np.uint8)})
    with pytest.raises(native.GQError, match="past the end of the reference contig"):
        somatic_standard_reads(gpu_ctx, t, n, loci, reference=short)
    far = (np.array([0], np.int32), np.array([0], np.int64), np.array([400], np.int64), np.array([0], np.int64))
    full = ReferenceGenome({t.contig_names[0]: np.frombuffer(b"TCGATCGA" + b"A" * 100, np.uint8)})
    assert somatic_standard_reads(gpu_ctx, t, n, far, reference=full) == []


def test_read_past_the_range_is_not_looked_up(gpu_ctx):
    """A read beyond the FASTA contig's end but outside the loci range forms no pileup in the
    range, so nothing fails (getReferenceBase is only called at visited loci of the range,
    ReferenceBroadcast.scala:26-30); the same read inside the range does fail."""
    reads = [mr("TCGATCGA", "8M", "8", 0)] * 2 + [mr("AAAAAAAA", "8M", "8", 200)]
    t, n = make_read_set(reads), make_read_set(reads)
    ref = ReferenceGenome({t.contig_names[0]: np.frombuffer(b"TCGATCGA" + b"A" * 92, np.uint8)})  # length 100
    inside = (np.array([0], np.int32), np.array([0], np.int64), np.array([150], np.int64), np.array([0], np.int64))
    assert somatic_standard_reads(gpu_ctx, t, n, inside, reference=ref) == O.somatic_standard(
        t, n, inside, reference=ref)
    reach = (np.array([0], np.int32), np.array([0], np.int64), np.array([205], np.int64), np.array([0], np.int64))
    with pytest.raises(native.GQError, match="past the end of the reference contig"):
        somatic_standard_reads(gpu_ctx, t, n, reach, reference=ref)
