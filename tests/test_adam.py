"""ADAM AlignmentRecord read input (guacamole_amd/adam.py): Read.loadReadRDDAndSequenceDictionary
sends every --reads that is not .bam / .sam to loadReadRDDAndSequenceDictionaryFromADAM
(reads/Read.scala:345-364, 454-539).

The reference pins the path with ReadSetSuite "load read from ADAM"
(src/test/scala/org/hammerlab/guacamole/reads/ReadSetSuite.scala:88-109): mdtagissue.sam
converted to ADAM Parquet and loaded back gives 8 reads, 3 after InputFilters(mapped,
nonDuplicate).  The conversion here is the repository's own restatement of ADAM's
(adam.sam_to_alignment_records + write_alignment_parquet): byte parity with ADAM's Parquet files
is unpinned (no ADAM output exists in the reference's fixtures), so the read sets are compared
with the SAM loader's instead, array for array."""
import numpy as np
import pytest

from conftest import fixture
from guacamole_amd.adam import load_adam, sam_to_alignment_records, write_alignment_parquet
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.reads import InputFilters, ReadLoadError, load_reads
from oracle import oracle as O


def _adam(tmp_path, name):
    out = str(tmp_path / (name.split(".")[0] + ".adam"))
    write_alignment_parquet(out, sam_to_alignment_records(fixture(name)))
    return out


def _same(a, b):
    """Read for read; the contigs by name (ADAM's sequence dictionary holds only the records'
    contigs, ADAMSpecificRecordSequenceDictionaryRDDAggregator, where the SAM header lists all)."""
    la, lb = a.contig_lengths_map, b.contig_lengths_map
    assert all(lb[c] == n for c, n in la.items())
    assert [a.contig_names[i] for i in a.contig] == [b.contig_names[i] for i in b.contig]
    assert a.sample_names == b.sample_names
    for k in ("start", "end", "mapq", "flags", "sample", "seq_off", "seq_len", "seq", "qual", "cigar_off",
              "n_cigar", "cigar", "md_off", "md_len", "md"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert a.names == b.names


def test_read_set_suite_load_read_from_adam(tmp_path):
    """ReadSetSuite.scala:88-109: 8 reads from the ADAM copy of mdtagissue.sam, 3 mapped and not
    duplicates; the mapped reads are the SAM loader's."""
    p = _adam(tmp_path, "mdtagissue.sam")
    rs, count = load_adam(p)
    assert count == 8
    f = InputFilters.make(mapped=True, non_duplicate=True)
    rs, count = load_adam(p, f)
    assert count == 3 and rs.n == 3
    _same(rs, load_reads(fixture("mdtagissue.sam"), f))
    # the load_reads route (any name but .bam / .sam) gives the same set
    _same(load_reads(p, f), rs)


@pytest.mark.parametrize("name", ["tumor.chr20.tough.sam", "normal.chr20.tough.sam",
                                  "synthetic.challenge.set1.tumor.v2.withMDTags.chr2.syn1fp.sam"])
def test_adam_reads_equal_the_sam_reads(tmp_path, name):
    """The callers' filters (GermlineThresholdCaller.scala:61-63, SomaticStandardCaller.scala:
    69-73) over the ADAM copy keep the SAM loader's reads, field for field, and the germline
    oracle calls the same records from them."""
    p = _adam(tmp_path, name)
    for f in (InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True),
              InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True,
                                passed_vendor_quality_checks=True)):
        a, b = load_reads(p, f), load_reads(fixture(name), f)
        _same(a, b)
    f = InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True)
    a, b = load_reads(p, f), load_reads(fixture(name), f)

    def loci(rs):
        return flatten_partitions(partition_loci_uniformly(1, LociSet.parse("all").result(rs.contig_lengths_map)),
                                  rs.contig_index())
    assert O.germline_threshold(a, loci(a), 8) == O.germline_threshold(b, loci(b), 8)


def test_adam_record_without_sample_fails(tmp_path):
    """fromADAMRecord calls recordGroupSample.toString (Read.scala:498): a record without a read
    group sample fails the load, as the reference's NullPointerException does."""
    recs = sam_to_alignment_records(fixture("mdtagissue.sam"))
    for r in recs:
        r.pop("recordGroupSample", None)
    out = str(tmp_path / "nosample.adam")
    write_alignment_parquet(out, recs)
    with pytest.raises(ReadLoadError, match="recordGroupSample"):
        load_adam(out)


def test_not_parquet_is_an_error(tmp_path):
    p = tmp_path / "reads.txt"
    p.write_text("not parquet\n")
    with pytest.raises(ReadLoadError, match="neither SAM / BAM"):
        load_reads(str(p))
