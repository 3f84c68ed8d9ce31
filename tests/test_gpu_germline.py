"""GPU parity: libgqpileup (HIP, gfx950) vs the CPU oracle, germline-threshold path."""
import numpy as np
import pytest

from conftest import fixture
from guacamole_amd import native
from guacamole_amd.commands import germline_threshold_reads
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.reads import InputFilters, load_reads, make_read as mr, make_read_set
from guacamole_amd.synthetic import generate
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _loci(rs, expr="all", tasks=1):
    ls = LociSet.parse(expr).result(rs.contig_lengths_map)
    return flatten_partitions(partition_loci_uniformly(tasks, ls), rs.contig_index())


def _ambiguous(rows):
    return [r for r in rows if r[6] & native.FLAG_AMBIGUOUS_REF]


@pytest.fixture(scope="module")
def chrm():
    return load_reads(fixture("chrM.sorted.bam"),
                      InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True))


@pytest.mark.parametrize("threshold,emit_ref,emit_no_call", [(8, False, False), (0, False, False), (30, True, True)])
def test_chrm_germline_matches_oracle(gpu_ctx, chrm, threshold, emit_ref, emit_no_call):
    loci = _loci(chrm)
    got = germline_threshold_reads(gpu_ctx, chrm, loci, threshold, emit_ref, emit_no_call)
    want = O.germline_threshold(chrm, loci, threshold, emit_ref, emit_no_call)
    # every record, including those at loci whose reference base the reference takes from the
    # SlidingWindow queue's heap order (the reads' MD tags disagree there: replayed on the host)
    assert got == want
    assert _ambiguous(want), "chrM holds heap-order-dependent loci"


def test_chrm_counts_match_oracle(gpu_ctx, chrm):
    loci = _loci(chrm)
    from guacamole_amd.commands import device_reads
    c = gpu_ctx.pileup_counts(device_reads(gpu_ctx, chrm), loci)
    stats = O.pileup_stats(chrm, loci)
    start = int(loci[1][0])
    visited = np.nonzero(c["depth"] > 0)[0]
    assert len(visited) == len(stats) == 15904
    for row in stats:
        i = row[1] - start
        assert c["depth"][i] == row[3]
        assert c["pos_depth"][i] == row[4]
        assert tuple(c["base_counts"][i]) == row[5]
        assert tuple(c["indel_counts"][i]) == row[6]
        assert c["ambiguous"][i] == row[8]
        assert chr(c["ref_base"][i]) == row[2]
        assert c["ref_depth"][i] == row[7]
    assert any(row[8] for row in stats)


def test_parallelism_partitions_agree(gpu_ctx, chrm):
    """DistributedUtilSuite (1 vs 5 vs 800 tasks): identical calls wherever the reads' MD tags
    agree; at heap-order-dependent loci each split gives what the reference gives for that
    split (each task starts its own SlidingWindow queue)."""
    base = germline_threshold_reads(gpu_ctx, chrm, _loci(chrm, tasks=1), 8)
    firm = lambda rows: [r for r in rows if not (r[6] & native.FLAG_AMBIGUOUS_REF)]
    for tasks in (5, 800):
        loci = _loci(chrm, tasks=tasks)
        got = germline_threshold_reads(gpu_ctx, chrm, loci, 8)
        assert firm(got) == firm(base)
        assert got == O.germline_threshold(chrm, loci, 8)


@pytest.mark.parametrize("seed", [1, 2])
def test_synthetic_germline_matches_oracle(gpu_ctx, seed):
    g = generate(150_000, 30, seed=seed, indel_rate=5e-4)
    rs = g.to_read_set()
    loci = _loci(rs)
    got = germline_threshold_reads(gpu_ctx, rs, loci, 8)
    want = O.germline_threshold(rs, loci, 8)
    assert got == want
    assert any(len(r[4]) > 1 or len(r[5]) > 1 for r in want)  # indels exercised


def test_kat_pileups(gpu_ctx):
    """Small KAT read sets (DistributedUtilSuite / GermlineThresholdCallerSuite shapes)."""
    cases = [
        [mr("TCGATCGA", "8M", "8", 1), mr("TCGGTCGA", "8M", "3A4", 1), mr("TCGGTCGA", "8M", "3A4", 1)],
        [mr("CCGATCGA", "8M", "0T7", 1)] * 3,
        [mr("TCGATCGA", "8M", "8", 1), mr("TCGATCGA", "8M", "8", 1), mr("TCGACCCTCGA", "4M3I4M", "8", 1)],
        [mr("TCGAAAAGCT", "5M6D5M", "5^GCTTCG5", 0)] * 3,
        [mr("TCATCTCAAAAGAGATCGA", "2M2D1M2I2M4I2M2D6M", "2^GA5^TC6", 10)] * 3,
        [mr("AAAAAACGT", "5I4M", "4", 0), mr("ACGT", "4M", "4", 0)],
        [mr("CCCCAGCCTAGGCCTTCGACACTGGGGGGCTGAGGGAAGGGGCACCTGCC", "7M191084N43M", "9T24T7G7", 229538779)],
    ]
    for reads in cases:
        rs = make_read_set(reads)
        for expr in ("chr1:0-100", "chr1:0-300", "chr1:229538770-229729950"):
            loci = flatten_partitions(partition_loci_uniformly(1, LociSet.parse(expr).result()), rs.contig_index())
            for t in (0, 8, 50):
                got = germline_threshold_reads(gpu_ctx, rs, loci, t, True, True)
                want = O.germline_threshold(rs, loci, t, True, True)
                assert got == want, (reads, expr, t)


def test_cli_germline_vcf_and_somatic_json(tmp_path):
    """End-to-end CLI (python -m guacamole_amd ...) writes the callers' outputs."""
    from guacamole_amd.commands import main
    vcf = str(tmp_path / "g.vcf")
    assert main(["germline-threshold", "--reads", fixture("chrM.sorted.bam"), "--loci", "chrM:0-16570",
                 "--out", vcf]) == 0
    # saveAsVcf's Hadoop layout: a directory with one part file (Common.scala:290-293)
    import os
    assert sorted(os.listdir(vcf)) == ["_SUCCESS", "part-r-00000"]
    lines = [l for l in open(os.path.join(vcf, "part-r-00000")) if not l.startswith("#")]
    assert len(lines) > 100 and all(l.split("\t")[0] == "chrM" for l in lines)
    js = str(tmp_path / "s.json")
    assert main(["somatic-standard", "--tumor-reads", fixture("tumor.chr20.tough.sam"), "--normal-reads",
                 fixture("normal.chr20.tough.sam"), "--out", js, "--min-tumor-read-depth", "8"]) == 0
    from guacamole_amd.output import read_avro_json
    rows = read_avro_json(open(js).read())
    assert rows and all(r["alleles"] == ["Ref", "Alt"] and r["readDepth"]["int"] >= 8 for r in rows)


def test_cli_parquet_equals_json(tmp_path):
    """--out X.adam (adamParquetSave, Common.scala:294-302): the CLI's Parquet directory holds one
    part per loci task and its rows equal the Avro-JSON output's records, for both callers."""
    import os
    from guacamole_amd.commands import main
    from guacamole_amd.output import read_avro_json, read_parquet_dir, unwrap_avro_json
    for cmd in (["germline-threshold", "--reads", fixture("chrM.sorted.bam"), "--parallelism", "3"],
                ["somatic-standard", "--tumor-reads", fixture("tumor.chr20.tough.sam"), "--normal-reads",
                 fixture("normal.chr20.tough.sam"), "--parallelism", "2"]):
        js, pq = str(tmp_path / (cmd[0] + ".json")), str(tmp_path / (cmd[0] + ".adam"))
        assert main(cmd + ["--out", js]) == 0
        assert main(cmd + ["--out", pq]) == 0
        parts = sorted(f for f in os.listdir(pq) if f.startswith("part-r-"))
        assert len(parts) == int(cmd[-1])
        want = [unwrap_avro_json("Genotype", r) for r in read_avro_json(open(js).read())]
        got = read_parquet_dir(pq)
        assert len(got) == len(want) > 0
        for x, y in zip(got, want):
            if y["expectedAlleleDosage"] is not None:
                assert np.float32(x.pop("expectedAlleleDosage")) == np.float32(y.pop("expectedAlleleDosage"))
            assert x == y


def test_cli_adam_read_input_equals_sam(tmp_path):
    """--reads / --tumor-reads / --normal-reads naming ADAM AlignmentRecord Parquet (any name but
    .bam / .sam: Read.scala:345-364, 454-539): both callers write the records they write from the
    SAM files the ADAM directories were converted from (adam.sam_to_alignment_records)."""
    from guacamole_amd.adam import sam_to_alignment_records, write_alignment_parquet
    from guacamole_amd.commands import main
    ad = {}
    for name in ("tumor.chr20.tough.sam", "normal.chr20.tough.sam"):
        ad[name] = str(tmp_path / name.replace(".sam", ".adam"))
        write_alignment_parquet(ad[name], sam_to_alignment_records(fixture(name)))
    for cmd, swap in ((["germline-threshold", "--reads", "tumor.chr20.tough.sam", "--threshold", "5"], (2,)),
                      (["somatic-standard", "--tumor-reads", "tumor.chr20.tough.sam", "--normal-reads",
                        "normal.chr20.tough.sam", "--min-tumor-read-depth", "8"], (2, 4))):
        outs = []
        for src in ("sam", "adam"):
            c = list(cmd)
            for k in swap:
                c[k] = fixture(c[k]) if src == "sam" else ad[c[k]]
            js = str(tmp_path / ("%s_%s.json" % (cmd[0], src)))
            assert main(c + ["--out", js]) == 0
            outs.append(open(js).read())
        assert outs[0] == outs[1] and len(outs[0]) > 100, cmd[0]


def test_synthetic_column_path_dense_outputs(gpu_ctx):
    """emit_ref / emit_no_call through the column kernel (HomRef / NoCall rows inline,
    variant candidates through germline_expand); the column kernel keeps nearly every tile."""
    g = generate(60_000, 30, seed=7, indel_rate=3e-4)
    rs = g.to_read_set()
    loci = _loci(rs)
    for t, er, enc in ((8, True, False), (30, False, True), (0, True, True)):
        got = germline_threshold_reads(gpu_ctx, rs, loci, t, er, enc)
        want = O.germline_threshold(rs, loci, t, er, enc)
        assert got == want, (t, er, enc)
        tm = gpu_ctx.timings()
        assert tm["walk_tiles"] <= 0.05 * tm["tiles"], tm


def test_chrm_subsampled_column_path(gpu_ctx, chrm):
    """Real reads (29-80 bp, real MD tags) at a depth whose tiles fit the column kernel's stage
    (every 8th read of chrM.sorted.bam: about 18x)."""
    from guacamole_amd.reads import ReadSet
    sub = chrm.subset(np.arange(0, chrm.n, 8))
    loci = _loci(sub)
    for t, er, enc in ((8, False, False), (0, True, True)):
        got = germline_threshold_reads(gpu_ctx, sub, loci, t, er, enc)
        want = O.germline_threshold(sub, loci, t, er, enc)
        assert got == want
    tm = gpu_ctx.timings()
    assert tm["walk_tiles"] < tm["tiles"] // 2, tm  # most tiles through the column kernel


class _DeviceArray:
    """A numpy array copied to device memory with the HIP runtime the library links (hipMalloc /
    hipMemcpy through ctypes), exposing what native._ptr needs."""
    _hip = None

    def __init__(self, a):
        import ctypes as C
        if _DeviceArray._hip is None:
            _DeviceArray._hip = C.CDLL("libamdhip64.so.7")  # by SONAME: the runtime libgqpileup.so already uses
        a = np.ascontiguousarray(a)
        self.shape, self.dtype, self.nbytes = a.shape, a.dtype, max(a.nbytes, 16)
        self.ptr = C.c_void_p()
        assert _DeviceArray._hip.hipMalloc(C.byref(self.ptr), C.c_size_t(self.nbytes)) == 0
        assert _DeviceArray._hip.hipMemcpy(self.ptr, a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes), 1) == 0

    def data_ptr(self):
        return self.ptr.value

    def __del__(self):
        if self.ptr and _DeviceArray._hip is not None:
            _DeviceArray._hip.hipFree(self.ptr)


def test_wrapped_device_reads_unordered_pool(gpu_ctx):
    """gq_reads_wrap_device over device buffers whose sequence pool is NOT in read order: the
    column kernel's per-read stage check sends such reads' tiles to the walker, results equal."""
    g = generate(40_000, 30, seed=11, indel_rate=3e-4)
    a = {k: np.asarray(v) for k, v in g.arrays.items()}
    n = a["start"].shape[0]
    # reverse the pool: read r's bytes move to the mirrored offset
    L = a["seq_len"].astype(np.int64)
    total = int(a["seq"].shape[0])
    new_off = total - a["seq_off"] - L
    seq2 = np.empty_like(a["seq"])
    qual2 = np.empty_like(a["qual"])
    for r in range(n):
        o, no, l = int(a["seq_off"][r]), int(new_off[r]), int(L[r])
        seq2[no:no + l] = a["seq"][o:o + l]
        qual2[no:no + l] = a["qual"][o:o + l]
    host = dict(a, seq=seq2, qual=qual2, seq_off=new_off.astype(np.int64))
    dev = {k: (_DeviceArray(v) if v.ndim else int(v)) for k, v in host.items()}
    dr = gpu_ctx.wrap_device(dev)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([39_999], np.int64), np.array([0], np.int64))
    got = gpu_ctx.germline_threshold(dr, loci, 8)
    ref = gpu_ctx.germline_threshold(gpu_ctx.upload(a), loci, 8)
    assert got.tuples(g.contig_names) == ref.tuples(g.contig_names)
    want = O.germline_threshold(g.to_read_set(), loci, 8)
    assert ref.tuples(g.contig_names) == want


def test_deep_panel_500x_germline(gpu_ctx):
    """BASELINE configs[4] depth (500x, a targeted-panel region): blocks of ~550 projection rows
    (16-bit counts past 240 rows) stay on germline_proj, none goes to the walker; calls
    identical to the oracle."""
    g = generate(12_000, 500.0, seed=5, indel_rate=3e-4)
    rs = g.to_read_set()
    loci = _loci(rs)
    for t in (2, 8):
        got = germline_threshold_reads(gpu_ctx, rs, loci, t)
        assert gpu_ctx.timings()["walk_tiles"] == 0
        want = O.germline_threshold(rs, loci, t)
        assert got == want
        assert len(want) > 10


def test_device_results_equal_host_results(gpu_ctx, chrm):
    """gq_germline_threshold_device leaves the same records in HBM as gq_germline_threshold
    copies to the host (the bench's timed path vs the API the parity tests use)."""
    from guacamole_amd.commands import device_reads
    g = generate(80_000, 30, seed=3, indel_rate=3e-4)
    for rs in (chrm, g.to_read_set()):
        d = device_reads(gpu_ctx, rs)
        loci = _loci(rs)
        for args in ((8, False, False), (0, True, True), (25, False, True)):
            h = gpu_ctx.germline_threshold(d, loci, *args)
            dv = gpu_ctx.germline_threshold_device(d, loci, *args)
            assert len(dv) == len(h) and dv.visited_loci == h.visited_loci
            x = dv.to_host()
            for k in h.a:
                assert np.array_equal(x.a[k], h.a[k]), k
            assert x.pool == h.pool
            assert x.tuples(rs.contig_names) == h.tuples(rs.contig_names)


def _many_insertions(n_distinct, n_ref=100, n_alt=40, start=100, singleton_qual=31):
    """A locus holding `n_distinct` distinct insertion alleles (one read each, base quality
    singleton_qual), n_alt reads of one more insertion and n_ref reference reads: 10M kI 10M over
    a 20-base reference."""
    ref = "ACGTTGCAACGGTACCATGA"
    reads = []
    for i in range(n_distinct):
        ins = "".join("ACGT"[(i >> (2 * k)) & 3] for k in range(6))
        reads.append(mr(ref[:10] + ins + ref[10:], "10M6I10M", "20", start, quals=[singleton_qual] * 26))
    reads += [mr(ref[:10] + "TTTTTTT" + ref[10:], "10M7I10M", "20", start)] * n_alt
    reads += [mr(ref, "20M", "20", start)] * n_ref
    reads.sort(key=lambda r: r["start"])
    return make_read_set(reads)


@pytest.mark.parametrize("n_distinct", [100, 200, 700])
def test_more_distinct_alleles_than_the_fast_table(gpu_ctx, n_distinct):
    """germline_complex keeps 128 (sample, allele) keys in registers; a locus with more goes to
    the wide instantiation (1024 keys) instead of a capacity error (Pileup.scala:37-146 has no
    limit): records equal the oracle's."""
    rs = _many_insertions(n_distinct)
    for threshold in (8, 0):
        loci = _loci(rs, "chr1:90-130")
        got = germline_threshold_reads(gpu_ctx, rs, loci, threshold, True, True)
        want = O.germline_threshold(rs, loci, threshold, True, True)
        assert got == want and len(want) > 0


def test_rederive_gives_the_same_records(gpu_ctx):
    """gq_reads_rederive drops every derived structure and derives it again from the resident SoA
    (the bench's cold step): the germline and somatic records are those of the first derivation,
    and a second re-derivation reuses the same buffers."""
    from guacamole_amd.commands import somatic_standard_reads
    g = generate(120_000, 30, seed=11, indel_rate=3e-4)
    reads = gpu_ctx.upload(g.arrays)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([119_999], np.int64), np.array([0], np.int64))
    want = gpu_ctx.germline_threshold(reads, loci, 8).tuples(g.contig_names)
    st0 = gpu_ctx.proj_stats(reads)
    for _ in range(2):
        gpu_ctx.rederive(reads)
        st = gpu_ctx.proj_stats(reads)
        assert st["projected"] == 0
        assert gpu_ctx.germline_threshold(reads, loci, 8).tuples(g.contig_names) == want
        st = gpu_ctx.proj_stats(reads)
        assert (st["proj_bytes"], st["pev_count"], st["n_rows"]) == (st0["proj_bytes"], st0["pev_count"], st0["n_rows"])
    t = generate(100_000, 60, seed=3, somatic_rate=2e-4, tumor=True, read_seed=11)
    n = generate(100_000, 30, seed=3, somatic_rate=2e-4, tumor=False, read_seed=12)
    td, nd = gpu_ctx.upload(t.arrays), gpu_ctx.upload(n.arrays)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([99_999], np.int64), np.array([0], np.int64))
    first = gpu_ctx.somatic_standard(td, nd, loci).rows
    assert first
    gpu_ctx.rederive(td)
    gpu_ctx.rederive(nd)
    assert gpu_ctx.somatic_standard(td, nd, loci).rows == first
