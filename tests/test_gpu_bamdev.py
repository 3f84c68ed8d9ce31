"""BAM decoded on the GPU (bamdev.load_reads_device, gqpileup.h gq_bam_dev_*) against the host
loader (ingest.load_bam + soa.pack, itself pinned by tests/test_ingest.py against the Python
statement of Read.scala's rules): every SoA array of the resident read set, copied back
(gq_reads_download), must equal what the host path uploads — on the reference's chrM BAM
under the callers' filters, on written BAMs with read groups / every aux type / unmapped,
duplicate, QC-fail and unpaired reads / records split across 1000-byte BGZF blocks, on the
native generator's 30x shard, and through the germline-threshold and somatic-standard CLIs
(device ingest vs GQ_INGEST=host, identical output files).  Errors raise the host loader's
classes; unsorted and plain-gzip BAMs go back to the host loader (None)."""
import os
import random

import numpy as np
import pytest

from guacamole_amd import bamdev, soa, synthetic
from guacamole_amd.loci import LociSet
from guacamole_amd.reads import InputFilters, ReadLoadError, load_reads
from tests import bam_writer as bw
from tests.conftest import fixture
from tests.test_ingest import CHRM_FILTERS, CONTIGS, HEADER, _records

pytestmark = pytest.mark.gpu

KEYS = ["contig_read_begin", "start", "end", "pmax_end", "mapq", "flags", "sample", "seq_off", "seq_len", "cigar_off",
        "n_cigar", "md_off", "n_md", "n_mismatch", "seq", "qual", "cigar", "md_ev", "sample_hash"]


def _sorted(recs):
    """Records in (contig, start) order (unmapped ones last), ties in their order: the
    writer's bytes are block_size, refID, pos, ..."""
    def key(r):
        ref, pos = int.from_bytes(r[4:8], "little", signed=True), int.from_bytes(r[8:12], "little", signed=True)
        return (ref if ref >= 0 else 1 << 40, pos)
    return sorted(recs, key=key)


def compare(ctx, path, f):
    host = load_reads(path, f)
    want = soa.pack(host)
    dev = bamdev.load_reads_device(ctx, path, f)
    assert dev is not None
    assert dev.contig_names == host.contig_names and dev.contig_lengths == host.contig_lengths
    assert dev.sample_names == host.sample_names and dev.n == host.n
    got = bamdev.download(dev.reads)
    for k in KEYS:
        assert got[k].dtype == np.asarray(want[k]).dtype, k
        assert np.array_equal(got[k], want[k]), k
    assert int(got["n_samples"]) == int(want["n_samples"])
    begin, start, end = dev.positions()
    for (n1, s1, e1), (n2, s2, e2) in zip(dev.regions(), host.regions()):
        assert n1 == n2 and np.array_equal(s1, s2) and np.array_equal(e1, e2)
    return dev


@pytest.mark.parametrize("k", range(len(CHRM_FILTERS)))
def test_chrm_device_equals_host(gpu_ctx, k):
    compare(gpu_ctx, fixture("chrM.sorted.bam"), CHRM_FILTERS[k])


def test_gatk_bundle_device_equals_host(gpu_ctx):
    p = fixture("gatk_mini_bundle_extract.bam")
    for f in (InputFilters(), InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True,
                                                  passed_vendor_quality_checks=True, has_md_tag=True)):
        compare(gpu_ctx, p, f)


@pytest.mark.parametrize("block", [65280, 1000])
def test_written_bam_device_equals_host(gpu_ctx, tmp_path, block):
    rng = random.Random(11 + block)
    p = str(tmp_path / "x.bam")
    bw.write_bam(p, HEADER, CONTIGS, _sorted(_records(rng, 3000, CONTIGS)), block=block)
    for f in [InputFilters(), InputFilters.make(mapped=True, non_duplicate=True),
              InputFilters.make(overlaps_loci=LociSet.parse("chr10:100-3000,chrX"), is_paired=True),
              InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True,
                                passed_vendor_quality_checks=True, has_md_tag=True)]:
        d = compare(gpu_ctx, p, f)
        assert d.n > 0
    assert set(compare(gpu_ctx, p, InputFilters()).sample_names) == {"alice", "bob", "default"}


def test_synthetic_shard_device_equals_host(gpu_ctx, tmp_path):
    g = synthetic.generate(400_000, 30.0, seed=synthetic.SEED + 5)
    p = str(tmp_path / "s.bam")
    g.write_bam(p)
    d = compare(gpu_ctx, p, InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True,
                                               has_md_tag=True))
    assert d.n > 70_000 and d.timings["blocks"] > 100


def test_unsorted_and_plain_gzip_go_to_the_host_loader(gpu_ctx, tmp_path):
    rng = random.Random(5)
    p = str(tmp_path / "u.bam")
    bw.write_bam(p, HEADER, CONTIGS, _records(rng, 500, CONTIGS, unsorted=True))
    assert bamdev.load_reads_device(gpu_ctx, p, InputFilters()) is None
    q = str(tmp_path / "g.bam")
    bw.write_bam(q, HEADER, CONTIGS, _records(rng, 300, CONTIGS), plain_gzip=True)
    assert bamdev.load_reads_device(gpu_ctx, q, InputFilters()) is None


def test_empty_bam(gpu_ctx, tmp_path):
    p = str(tmp_path / "e.bam")
    bw.write_bam(p, "", CONTIGS, [])
    d = compare(gpu_ctx, p, InputFilters())
    assert d.n == 0 and d.sample_names == []


def test_errors_are_the_host_loaders(gpu_ctx, tmp_path):
    p = str(tmp_path / "q.bam")
    bw.write_bam(p, "", CONTIGS, [bw.record(0, 10, "a", "4M", "ACGT", None, tags=bw.tag_z("MD", "4"))])
    with pytest.raises(ReadLoadError, match="Base qualities have length 0 but sequence has length 4"):
        bamdev.load_reads_device(gpu_ctx, p, InputFilters())
    a = str(tmp_path / "a.bam")
    bw.write_bam(a, "", CONTIGS, [bw.record(0, 10, "a", "4M", "ACGT", [30] * 4, tags=b"XYq\x00")])
    with pytest.raises(ReadLoadError, match="bad aux type 'q'"):
        bamdev.load_reads_device(gpu_ctx, a, InputFilters())
    c = str(tmp_path / "c.bam")
    bw.write_bam(c, "", CONTIGS, [bw.record(0, 10, "a", "4M", "ACGT", [30] * 4)])
    raw = bytearray(open(c, "rb").read())
    raw[30] ^= 0xFF  # inside the first block's deflate payload
    open(c, "wb").write(bytes(raw))
    with pytest.raises(ReadLoadError):
        bamdev.load_reads_device(gpu_ctx, c, InputFilters())
    m = str(tmp_path / "m.bam")
    bw.write_bam(m, "", CONTIGS, [bw.record(0, 10, "a", "4M", "ACGT", [30] * 4, tags=bw.tag_z("MD", "2X"))])
    with pytest.raises(soa.MdParseError):
        soa.pack(load_reads(m))
    with pytest.raises(soa.MdParseError):
        bamdev.load_reads_device(gpu_ctx, m, InputFilters())


def _run(env_ingest, argv):
    from guacamole_amd.commands import main
    old = os.environ.get("GQ_INGEST")
    os.environ["GQ_INGEST"] = env_ingest
    try:
        assert main(argv) == 0
    finally:
        if old is None:
            os.environ.pop("GQ_INGEST", None)
        else:
            os.environ["GQ_INGEST"] = old


def test_cli_device_ingest_equals_host(tmp_path):
    g = synthetic.generate(200_000, 30.0, seed=synthetic.SEED + 6)
    bam = str(tmp_path / "s.bam")
    g.write_bam(bam)
    outs = {}
    for mode in ("device", "host"):
        out = tmp_path / ("g_%s.vcf" % mode)
        _run(mode, ["germline-threshold", "--reads", bam, "--out", str(out), "--parallelism", "3"])
        outs[mode] = (out / "part-r-00000").read_text()
    assert outs["device"] == outs["host"] and outs["device"].count("\n") > 50
    t = synthetic.generate(200_000, 40.0, seed=synthetic.SEED + 7)
    tb = str(tmp_path / "t.bam")
    t.write_bam(tb)
    for mode in ("device", "host"):
        out = tmp_path / ("s_%s.json" % mode)
        _run(mode, ["somatic-standard", "--tumor-reads", tb, "--normal-reads", bam, "--loci", "20:0-150000",
                    "--out", str(out)])
        outs[mode] = out.read_text()
    assert outs["device"] == outs["host"]


# ---- region-restricted loads (the multi-GPU ingest, gq_bam_dev_plan) ------------------------
def compare_region(ctx, path, f, region, halo=bamdev.DEFAULT_HALO):
    """A planned device load of `region` against the host loader's reads overlapping it."""
    from guacamole_amd.distributed import reads_overlapping
    host = load_reads(path, f)
    idx = host.contig_index()
    rng = [(idx[c], s, e) for c, s, e in region.ranges()]
    sub = host.subset(reads_overlapping(host, *[np.asarray(a) for a in zip(*rng)])) if rng else host.subset([])
    want = soa.pack(sub)
    dev = bamdev.load_reads_device(ctx, path, f, region=region, halo=halo)
    assert dev is not None and dev.n == sub.n
    got = bamdev.download(dev.reads)
    for k in KEYS:
        assert np.array_equal(got[k], want[k]), k
    return dev


@pytest.mark.parametrize("index", [False, True])
def test_region_load_equals_host_subset(gpu_ctx, tmp_path, index):
    from tests.test_region_plan import CONTIGS as RC, HEADER as RH, _records as region_records
    rng = random.Random(21 + index)
    p = str(tmp_path / "r.bam")
    bw.write_bam(p, RH, RC, region_records(rng, 4000, long_every=40), block=4000, index=index)
    f = InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True)
    lengths = dict(RC)
    for expr in ("c2:100000-100500", "c1:0-50000,c10:150000-200000", "c1:200000-210000,c1:230000-240000", "c2"):
        dev = compare_region(gpu_ctx, p, f, LociSet.parse(expr).result(lengths))
        plan = dev.timings["plan"]
        assert plan is not None and plan["used_index"] == int(index)
        assert dev.timings["blocks"] < 0.8 * 440  # a part of the ~440-block file
    # a halo shorter than the 3 kb reads: without an index the load plans again from the span it saw
    dev = compare_region(gpu_ctx, p, f, LociSet.parse("c1:100000-100100").result(lengths), halo=500)
    assert dev.timings["replans"] == (0 if index else 1)


def test_region_load_gatk_bundle(gpu_ctx):
    p = fixture("gatk_mini_bundle_extract.bam")
    f = InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, passed_vendor_quality_checks=True,
                          has_md_tag=True)
    host = load_reads(p, f)
    c = host.contig_names[int(host.contig[0])]
    s0, s1 = int(host.start[0]), int(host.start[-1])
    region = LociSet.parse("%s:%d-%d" % (c, (s0 + s1) // 2, (s0 + s1) // 2 + 200)).result(host.contig_lengths_map)
    compare_region(gpu_ctx, p, f, region)


def test_region_load_without_sort_order_reads_everything(gpu_ctx, tmp_path):
    """No SO:coordinate: no plan, the whole file decoded and filtered to the region."""
    from tests.test_region_plan import CONTIGS as RC, _records as region_records
    p = str(tmp_path / "n.bam")
    bw.write_bam(p, "@HD\tVN:1.6\n", RC, region_records(random.Random(3), 500))
    dev = compare_region(gpu_ctx, p, InputFilters(), LociSet.parse("c2:1000-40000").result(dict(RC)))
    assert dev.timings["plan"] is None


@pytest.mark.parametrize("level,strategy", [(0, 0), (6, 4)])  # stored blocks; fixed Huffman codes (Z_FIXED)
def test_stored_and_fixed_huffman_blocks(gpu_ctx, tmp_path, level, strategy):
    rng = random.Random(31 + level)
    p = str(tmp_path / "z.bam")
    bw.write_bam(p, HEADER, CONTIGS, _sorted(_records(rng, 1500, CONTIGS)), level=level, strategy=strategy)
    compare(gpu_ctx, p, InputFilters())


def test_malformed_aux_array(gpu_ctx, tmp_path):
    """A B array whose count is negative (or runs past the record) is a truncated aux array, on
    the device as on the host loader (it must not walk the aux scan backwards)."""
    bad = b"ZBB" + b"i" + (-2).to_bytes(4, "little", signed=True) + b"\0" * 8
    p = str(tmp_path / "b.bam")
    bw.write_bam(p, "", CONTIGS, [bw.record(0, 10, "a", "4M", "ACGT", [30] * 4, tags=bad)])
    with pytest.raises(ReadLoadError, match="truncated aux array"):
        load_reads(p)
    with pytest.raises(ReadLoadError, match="truncated aux array"):
        bamdev.load_reads_device(gpu_ctx, p, InputFilters())
    long_arr = b"ZBB" + b"C" + (1000).to_bytes(4, "little") + b"\0" * 4
    q = str(tmp_path / "c.bam")
    bw.write_bam(q, "", CONTIGS, [bw.record(0, 10, "a", "4M", "ACGT", [30] * 4, tags=long_arr)])
    with pytest.raises(ReadLoadError, match="truncated aux array"):
        bamdev.load_reads_device(gpu_ctx, q, InputFilters())
