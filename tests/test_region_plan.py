"""The region plan of the multi-GPU ingest (gqpileup.h gq_bam_dev_plan), on the host: for a rank's
loci the plan must name every BGZF record that can overlap them (DistributedUtil.scala:584-597 ships
each read to every task it overlaps), start each segment on a true record boundary, and read only
a fraction of the file for a small region.  Checked against the records' known places in written
BAMs, with the BAI linear index (exact for any read span) and without one (host probes, `halo`
loci of margin)."""
import random
import struct

import pytest

from guacamole_amd import bamdev
from guacamole_amd.loci import LociSet
from tests import bam_writer as bw

CONTIGS = [("c1", 400_000), ("c2", 300_000), ("c10", 200_000)]
HEADER = "@HD\tVN:1.6\tSO:coordinate\n"


def _records(rng, per_contig, long_every=0):
    """Sorted records: 60 bp reads at random steps; every `long_every`-th spans 3 kb (an N skip)."""
    recs = []
    for ref, (_, ln) in enumerate(CONTIGS):
        pos = 0
        for i in range(per_contig):
            pos += rng.randrange(0, 2 * ln // per_contig)
            if pos >= ln - 4000:
                break
            cig = "30M3000N30M" if long_every and i % long_every == 7 else "60M"
            seq = "".join(rng.choice("ACGT") for _ in range(60))
            recs.append(bw.record(ref, pos, "r%d_%d" % (ref, i), cig, seq, [30] * 60, tags=bw.tag_z("MD", "60")))
    return recs


def _table(path_records, block):
    """(ref, pos, end, block index, offset in block) per record, from the writer's layout."""
    hdr = bw.header(HEADER, CONTIGS)
    x, out = len(hdr), []
    for r in path_records:
        ref, pos = struct.unpack_from("<ii", r, 4)
        l_name, = struct.unpack_from("<B", r, 12)
        n_cig, = struct.unpack_from("<H", r, 16)
        span = sum(op >> 4 for op in struct.unpack_from("<%dI" % n_cig, r, 36 + l_name) if (op & 15) in (0, 2, 3, 7, 8))
        out.append((ref, pos, pos + span, x // block, x % block))
        x += len(r)
    return out


def _check(plan, table, region, names):
    segs = plan["segments"]
    starts = {(b, o) for _, _, _, b, o in table}
    for b0, first, b1, eof in segs:
        assert (b0, first) in starts, "segment starts off a record boundary"
    need = 0
    for ref, pos, end, b, o in table:
        hit = any(s < end and pos < e for s, e in region.on_contig(names[ref]).ranges)
        if not hit:
            continue
        need += 1
        assert any((b0, first) <= (b, o) and b < (b1 if eof else b1 - 1) for b0, first, b1, eof in segs), \
            "record at %s:%d not in the plan" % (names[ref], pos)
    return need


@pytest.mark.parametrize("index", [False, True])
@pytest.mark.parametrize("block", [65280, 4000])
def test_plan_names_every_overlapping_record(tmp_path, index, block):
    rng = random.Random(block + index)
    recs = _records(rng, 3000, long_every=50)
    p = str(tmp_path / "x.bam")
    bw.write_bam(p, HEADER, CONTIGS, recs, block=block, index=index)
    table = _table(recs, block)
    names = [c for c, _ in CONTIGS]
    lengths = dict(CONTIGS)
    regions = ["c2:100000-100500", "c1:0-50000,c10:150000-200000", "c1:200000-210000,c1:230000-240000",
               "c2", "c1,c2,c10", "c10:190000-196000"]
    for expr in regions:
        region = LociSet.parse(expr).result(lengths)
        m = bamdev.MappedBam(p, populate=False)
        plan = m.plan(region, halo=4000, bai=bamdev.bai_path(p))
        assert plan["used_index"] == int(index)
        need = _check(plan, table, region, names)
        assert need > 0
        if expr == "c2:100000-100500" and block == 4000:
            assert plan["n_blocks"] < 10  # a few blocks of a ~300-block file
        m.close()


def test_index_is_exact_past_the_halo(tmp_path):
    """With the BAI a read reaching further back than the halo is still found; without it the
    halo decides (the device load then re-plans from the longest span it saw)."""
    rng = random.Random(5)
    recs = _records(rng, 3000, long_every=20)
    p = str(tmp_path / "y.bam")
    bw.write_bam(p, HEADER, CONTIGS, recs, block=3000, index=True)
    table = _table(recs, 3000)
    names = [c for c, _ in CONTIGS]
    region = LociSet.parse("c1:100000-100100").result(dict(CONTIGS))
    m = bamdev.MappedBam(p, populate=False)
    _check(m.plan(region, halo=0, bai=p + ".bai"), table, region, names)  # halo ignored: the index is exact
    m2 = bamdev.MappedBam(p, populate=False)
    plan = m2.plan(region, halo=4000, bai=None)
    _check(plan, table, region, names)
    assert not plan["used_index"] and plan["probes"] > 0


def test_plan_refused_without_sort_order(tmp_path):
    rng = random.Random(1)
    p = str(tmp_path / "u.bam")
    bw.write_bam(p, "@HD\tVN:1.6\n", CONTIGS, _records(rng, 200))
    m = bamdev.MappedBam(p, populate=False)
    assert m.plan(LociSet.parse("c1").result(dict(CONTIGS))) is None


def test_stale_or_foreign_index_is_ignored(tmp_path):
    import os
    rng = random.Random(2)
    recs = _records(rng, 500)
    p = str(tmp_path / "s.bam")
    bw.write_bam(p, HEADER, CONTIGS, recs, block=2000, index=True)
    os.utime(p + ".bai", (1, 1))  # older than the BAM
    region = LociSet.parse("c2:1000-5000").result(dict(CONTIGS))
    plan = bamdev.MappedBam(p, populate=False).plan(region, halo=4000, bai=p + ".bai")
    assert not plan["used_index"]
    _check(plan, _table(recs, 2000), region, [c for c, _ in CONTIGS])
    q = str(tmp_path / "f.bai")
    with open(q, "wb") as fh:
        fh.write(b"BAI\1" + struct.pack("<i", 7))  # another dictionary
    plan = bamdev.MappedBam(p, populate=False).plan(region, halo=4000, bai=q)
    assert not plan["used_index"]


def test_parallel_block_walk_equals_the_sequential_one(tmp_path, monkeypatch):
    """A file past 128 MB is walked in chunks on several host threads (gq_bam_dev_map_ex) and
    stitched along the true chain: the block table must be the sequential walk's.  Compared through
    the plan of the whole dictionary (every block, its stream bytes) and of a few ranges."""
    from guacamole_amd import synthetic
    g = synthetic.generate(5_000_000, 30.0, seed=3)
    path = str(tmp_path / "big.bam")
    g.write_bam(path, level=1)
    import os
    assert os.path.getsize(path) > (128 << 20)
    names = g.contig_names
    regions = [LociSet.parse("all").result(dict(zip(names, [5_000_000]))),
               LociSet.parse("%s:1000000-1200000,%s:4000000-4100000" % (names[0], names[0])).result(
                   dict(zip(names, [5_000_000])))]
    out = {}
    for nt in ("1", "16"):
        monkeypatch.setenv("GQ_MAP_THREADS", nt)
        got = []
        for reg in regions:
            m = bamdev.MappedBam(path, populate=False)
            got.append(m.plan(reg, 1 << 20, None))
            m.close()
        out[nt] = got
    assert out["1"] == out["16"]
    assert out["1"][0]["n_blocks"] > 2000


def test_early_map_is_adopted(tmp_path):
    """The CLI's early host map (guacamole_amd._early: gq_bam_dev_map_ex on a thread while the
    interpreter imports) is taken by the command's MappedBam for the same path, once, with the
    same header; a second MappedBam of the path maps it again.  Without a GPU the early context
    open fails quietly and take() gives None (the ordinary open reports the error)."""
    from guacamole_amd import _early
    from tests.conftest import fixture
    bam = fixture("chrM.sorted.bam")
    _early._maps.clear()
    _early._map_threads.clear()
    _early.start(["germline-threshold", "--reads", bam, "--device", "0"])
    assert bam in _early._map_threads
    m = bamdev.MappedBam(bam)
    assert m.ok and bam not in _early._map_threads and bam not in _early._maps
    names, lengths = m.contigs()
    m2 = bamdev.MappedBam(bam)
    assert m2.contigs() == (names, lengths) and "chrM" in names
    m.close()
    m2.close()
    h = _early.take(0)
    assert h is None or h.value  # (a GPU box: the opened context's handle)
