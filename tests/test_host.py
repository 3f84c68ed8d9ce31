"""CPU tests of the host side of the path: LociSet / partitioning (DistributedUtilSuite,
LociSetSuite strings), the product's MD-event parser against the oracle's MD
reconstruction, the SoA packing invariants, and the multi-rank gather (gloo, world 2)."""
import os

import numpy as np
import pytest

from guacamole_amd import soa
from guacamole_amd.loci import (LociMapBuilder, LociSet, partition_loci_by_approximate_depth,
                                partition_loci_uniformly)
from guacamole_amd.reads import load_reads, make_read, make_read_set, parse_cigar
from tests.conftest import fixture


# ---- DistributedUtilSuite.scala:35-64 ---------------------------------------------------
def test_partition_uniformly_strings():
    s = LociSet.parse("chr21:100-200,chr20:0-10,chr20:8-15,chr20:100-121,empty:10-10").result()
    assert partition_loci_uniformly(1, s).as_inverse_map()[0] == s
    r2 = partition_loci_uniformly(2, s).as_inverse_map()
    assert r2[0].count == s.count // 2 and r2[1].count == s.count // 2
    assert r2[0] != r2[1] and r2[0].union(r2[1]) == s
    assert str(partition_loci_uniformly(4, LociSet.parse("chrM:0-16571").result())) == \
        "chrM:0-4143=0,chrM:4143-8286=1,chrM:8286-12428=2,chrM:12428-16571=3"
    b = LociMapBuilder()
    for i in range(100):
        b.put("chrM", i + 1000, i + 1001, i)
    assert partition_loci_uniformly(100, LociSet.parse("chrM:1000-1100").result()) == b.result()
    assert str(partition_loci_uniformly(3, LociSet.parse("chrM:0-10").result())) == "chrM:0-3=0,chrM:3-7=1,chrM:7-10=2"
    assert str(partition_loci_uniformly(4, LociSet.parse("chrM:0-3").result())) == "chrM:0-1=0,chrM:1-2=1,chrM:2-3=2"
    assert str(partition_loci_uniformly(4, LociSet.parse("empty:10-10").result())) == ""


def test_partition_uniformly_large():  # :66-75 ("should not take a noticeable amount of time")
    s = LociSet.parse("chr21:0-3000000000").result()
    inv = partition_loci_uniformly(2000, s).as_inverse_map()
    assert len(inv) == 2000 and sum(v.count for v in inv.values()) == 3000000000


def test_partition_by_depth():  # :77-94
    reads = make_read_set([make_read("A", "1M", "1", st) for st in (5, 6, 7, 8)])
    loci = LociSet.parse("chr1:0-100").result()
    assert str(partition_loci_by_approximate_depth(2, loci, 100, reads.regions())) == "chr1:0-7=0,chr1:7-100=1"


def test_partition_one_task_shortcut():
    """commands.partition takes the uniform map for one task: the approximate-depth map of a
    single task is the same map (every locus on task 0), so the region counts are skipped."""
    from guacamole_amd.commands import partition
    reads = make_read_set([make_read("A", "1M", "1", st) for st in (5, 6, 7, 8, 50)] +
                          [make_read("AC", "2M", "2", st) for st in (3, 90)])
    for spec in ("chr1:0-100,chr2:0-40,chr2:60-100", "chr1:5-6", "all"):
        loci = LociSet.parse(spec).result({"chr1": 100, "chr2": 100})
        for acc in (0, 1, 250):
            want = partition_loci_by_approximate_depth(1, loci, max(acc, 1), reads.regions())
            assert partition(loci, 1, acc, reads) == want
            assert partition(loci, 0, acc, reads, world=1) == want


# ---- LociSetSuite.scala:155-167 -----------------------------------------------------------
def test_loci_set_strings():
    assert str(LociSet.parse("chr1:40-43").result().union(LociSet.parse("chr1:40-42").result())) == "chr1:40-43"
    got = LociSet.parse("chr1,chr2,17,chr2:3-5,chr20:10-20").result(
        {"chr1": 10, "chr2": 20, "17": 12, "chr20": 5000})
    assert str(got) == "17:0-12,chr1:0-10,chr2:0-20,chr20:10-20"


def test_loci_all_excludes_last_base():  # LociSet.scala:205-207
    got = LociSet.parse("all").result({"chrM": 16571, "1": 100})
    assert str(got) == "1:0-99,chrM:0-16570"


# ---- MD events (product parser, guacamole_amd/soa.py) vs the oracle's MD reconstruction ---
@pytest.mark.parametrize("seq,cigar,md", [
    ("GATGATTCGA", "10M", "10"), ("GATGATTCGA", "10M", "0CC8"), ("GATGACCCTTCGA", "5M3I5M", "10"),
    ("GATA", "3M6D1M", "3^GATTCG1"), ("GCGGGTACTCGAA", "2M3I8M", "1A5G2"), ("ACTCGA", "5M4D1M", "5^AACG1"),
    ("CCCCAGCCTAGGCCTTCGACACTGGGGGGCTGAGGGAAGGGGCACCTGCC", "7M191084N43M", "9T24T7G7"),
    ("TCATCTCAAAAGAGATCGA", "2M2D1M2I2M4I2M2D6M", "2^GA5^TC6"),
])
def test_md_events_match_oracle(seq, cigar, md):
    from oracle import oracle as O
    cig = parse_cigar(cigar)
    ops = [(c & 15, c >> 4) for c in cig]
    events, n_mm = soa.md_events(md.encode(), 0, ops)
    ev = {e >> 8: chr(e & 0xFF) for e in events}
    rs = make_read_set([make_read(seq, cigar, md, 0)])
    span = sum(ln for op, ln in ops if op in (0, 2, 3, 7, 8))
    for off in range(span):
        ref = O.elements_at(rs, "chr1", off, own_ref=True)[0]
        kind = O.elements_at(rs, "chr1", off, own_ref=True)[1][0]["kind"]
        if off in ev:
            assert ev[off] == ref, (off, ev[off], ref)
        elif kind != "Clipped":
            # no event: reference = sequenced base (M) — checked by the oracle's own element
            assert kind in ("Match", "Insertion", "Deletion"), (off, kind)
    assert n_mm == sum(1 for c in md if c in "ACGTN") - sum(
        len(x) for x in __import__("re").findall(r"\^([A-Z]+)", md))


def test_pack_invariants_chrM():
    rs = load_reads(fixture("chrM.sorted.bam"))
    a = soa.pack(rs)
    assert a["start"].dtype == np.int32 and a["pmax_end"].dtype == np.int32
    assert np.all(np.diff(a["start"]) >= 0)
    assert np.all(np.diff(a["pmax_end"]) >= 0) and np.all(a["pmax_end"] >= a["end"])
    assert a["contig_read_begin"][-1] == rs.n


# ---- distributed: rank split + variable-size gather over gloo (world size 2) --------------
def _gather_worker(rank, world, port, q):
    import torch.distributed as dist
    from guacamole_amd.distributed import gather_to_rank0
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = np.arange(rank * 7 + 3, dtype=np.uint8)
    out = gather_to_rank0(buf)
    if rank == 0:
        q.put([o.tolist() for o in out])
    dist.barrier()
    dist.destroy_process_group()


def test_gather_gloo_world2():
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == [list(range(3)), list(range(10))]


def test_split_loci_covers_set():
    from guacamole_amd.distributed import split_loci
    s = LociSet.parse("chr20:0-63025519,chr21:0-100").result()
    parts = split_loci(s, 8)
    assert len(parts) == 8
    u = parts[0]
    for p in parts[1:]:
        u = u.union(p)
    assert u == s and sum(p.count for p in parts) == s.count
