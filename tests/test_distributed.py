"""Multi-GPU driver pieces on the CPU: the task-to-rank split, the reads each rank receives
(halo duplication, DistributedUtil.scala:584-597), the record buffers' packing and the
world-size-2 gather over gloo."""
import multiprocessing as mp
import os
import socket

import numpy as np

from conftest import fixture
from guacamole_amd import native
from guacamole_amd.distributed import assign_tasks_to_ranks, rank_share, reads_overlapping
from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
from guacamole_amd.reads import InputFilters, load_reads


def _chrm():
    return load_reads(fixture("chrM.sorted.bam"),
                      InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True))


def test_tasks_to_ranks_contiguous_and_balanced():
    rs = _chrm()
    flat = flatten_partitions(partition_loci_uniformly(16, LociSet.parse("all").result(rs.contig_lengths_map)),
                              rs.contig_index())
    for world in (2, 3, 4, 8):
        rr = assign_tasks_to_ranks(flat, world, [rs], len(rs.contig_names))
        assert np.all(np.diff(rr) >= 0) and rr[0] == 0 and rr[-1] == world - 1
        # ranks own whole tasks
        for t in np.unique(flat[3]):
            assert len(set(rr[flat[3] == t].tolist())) == 1
        # read starts per rank within a factor 2 of the mean (16 tasks of chrM over <= 8 ranks)
        counts = [len(rank_share(rs, flat, rr, r)[0].start) for r in range(world)]
        assert max(counts) <= 2.2 * (sum(counts) / world), counts


def test_reads_overlapping_is_the_halo():
    rs = _chrm()
    cut = 8000
    left = reads_overlapping(rs, np.array([0]), np.array([0]), np.array([cut]))
    right = reads_overlapping(rs, np.array([0]), np.array([cut]), np.array([16570]))
    brute_l = np.nonzero(rs.start < cut)[0]
    brute_r = np.nonzero(rs.end > cut)[0]
    assert np.array_equal(left, brute_l) and np.array_equal(right, brute_r)
    straddle = np.intersect1d(left, right)
    assert len(straddle) > 50  # reads crossing the cut go to both sides
    assert np.array_equal(np.union1d(left, right), np.arange(rs.n))


def _somatic_calls(n, seed):
    rng = np.random.default_rng(seed)
    ev = np.zeros(n, native._EVIDENCE_DTYPE)
    for k in native.EVIDENCE_FIELDS:
        ev[k] = rng.integers(0, 100, n) if "depth" in k else rng.random(n)
    cols = dict(contig=rng.integers(0, 5, n).astype(np.int32), pos=rng.integers(0, 10 ** 9, n).astype(np.int64),
                sample=np.zeros(n, np.uint8), ref_off=(2 * np.arange(n)).astype(np.int64), ref_len=np.ones(n, np.int32),
                alt_off=(2 * np.arange(n) + 1).astype(np.int64), alt_len=np.ones(n, np.int32),
                log_odds=rng.random(n), gq=rng.integers(0, 99, n).astype(np.int32), tumor=ev, normal=ev.copy(),
                flags=np.zeros(n, np.uint8))
    return native.SomaticCalls(cols, bytes(rng.choice(list(b"ACGT"), 2 * n).tolist()), 1000 + n, 7 * n)


def test_somatic_pack_roundtrip():
    for n in (0, 1, 17):
        c = _somatic_calls(n, n)
        d = native.SomaticCalls.unpack(c.pack())
        assert len(d) == n and d.pool == c.pool and d.visited_loci == c.visited_loci
        assert d.rows == c.rows


def test_germline_image_decoder():
    """GermlineCalls.from_image reads the image layout gqpileup.h documents."""
    n = 5
    al = lambda x: (x + 63) & ~63
    vals = {"contig": np.arange(n, dtype=np.int32), "pos": np.arange(n, dtype=np.int64) * 10,
            "ref_off": np.arange(n, dtype=np.int64) * 2, "alt_off": np.arange(n, dtype=np.int64) * 2 + 1,
            "ref_len": np.ones(n, np.int32), "alt_len": np.ones(n, np.int32), "sample": np.zeros(n, np.uint8),
            "gt0": np.zeros(n, np.uint8), "gt1": np.ones(n, np.uint8), "flags": np.zeros(n, np.uint8)}
    pool = b"ACGTACGTAC"
    img = bytearray(4096)
    img[:8] = np.array([len(pool)], np.int64).tobytes()
    off = 64
    for k, dt in native.GermlineCalls.IMAGE_FIELDS:
        b = vals[k].astype(dt).tobytes()
        img[off:off + len(b)] = b
        off = al(off + len(b))
    img[off:off + len(pool)] = pool
    g = native.GermlineCalls.from_image(np.frombuffer(bytes(img), np.uint8), n)
    rows = g.tuples(["c%d" % i for i in range(n)])
    assert rows[3] == ("c3", 30, 0, ("Ref", "Alt"), "G", "T", 0)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from guacamole_amd.distributed import gather_somatic
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = gather_somatic(_somatic_calls(3 + 4 * rank, rank), None)
    if rank == 0:
        q.put([c.rows for c in out])
    dist.barrier()
    dist.destroy_process_group()


def test_gather_somatic_gloo_world2():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == [_somatic_calls(3, 0).rows, _somatic_calls(7, 1).rows]


def _gatherv_worker(rank, world, port, q):
    import torch.distributed as dist
    from guacamole_amd.distributed import gather_to_rank0
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = [5, 0, 17][rank]  # an empty rank sends nothing
    out = gather_to_rank0(np.arange(n, dtype=np.uint8) + rank, None)
    if rank == 0:
        q.put([o.tolist() for o in out])
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


def test_gatherv_gloo_world3_exact_sizes():
    """Sizes all-gathered, then one grouped send/recv per non-empty rank (no padding)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gatherv_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == [list(range(5)), [], [2 + i for i in range(17)]]


def _plan_worker(rank, world, port, q, parallelism, accuracy):
    """rank_loci_and_reads with the host loader standing in for the device one: each load
    returns only the reads overlapping the region, as a region-restricted BAM load does."""
    import torch.distributed as dist
    from guacamole_amd.distributed import rank_loci_and_reads
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = _chrm()
    loads = []

    def load(region):
        loads.append([(s, e) for _, s, e in region.ranges()])
        idx = reads_overlapping(full, *[np.asarray(a) for a in zip(*[(0, s, e) for _, s, e in region.ranges()])])
        return [full.subset(idx)]
    sets, mine = rank_loci_and_reads(load, full.contig_names, full.contig_lengths, LociSet.parse("all"), parallelism,
                                     accuracy, rank, world, "cpu")
    q.put((rank, [a.tolist() for a in mine], int(sets[0].n), loads))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_loci_world2_equal_one_process_partition():
    """The ranks' task split is the one-process partition (uniform, and by approximate depth with
    the micro-partition counts summed over ranks), every task on exactly one rank, and each rank
    holds exactly the reads overlapping its tasks' loci."""
    from guacamole_amd.commands import partition
    full = _chrm()
    loci = LociSet.parse("all").result(full.contig_lengths_map)
    for parallelism, accuracy in ((5, 0), (2, 250), (7, 250)):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=_plan_worker, args=(r, 2, port, q, parallelism, accuracy)) for r in range(2)]
        for p in ps:
            p.start()
        got = sorted(q.get(timeout=120) for _ in range(2))
        for p in ps:
            p.join(timeout=60)
            assert p.exitcode == 0
        want = flatten_partitions(partition(loci, parallelism, accuracy, full), full.contig_index())
        joined = [np.concatenate([np.asarray(g[1][k]) for g in got]) for k in range(4)]
        for a, b in zip(joined, want):
            assert np.array_equal(a, b), (parallelism, accuracy)
        for rank, mine, n, loads in got:
            assert len(mine[0]) > 0
            # the rank holds the reads overlapping what it loaded: exactly its tasks' loci, or (by
            # depth, when the micro-partition share + slack already covers its tasks) a superset
            need = len(reads_overlapping(full, *[np.asarray(x) for x in mine[:3]]))
            last = np.asarray(loads[-1])
            assert n == len(reads_overlapping(full, np.zeros(len(last), np.int32), last[:, 0], last[:, 1]))
            assert n >= need
            if loads[-1] == [(int(s), int(e)) for s, e in zip(mine[1], mine[2])]:
                assert n == need
            # uniform: one load of the tasks' loci; by depth: the micro-partition share (+ slack),
            # then the tasks' loci again where the depth-balanced cut lies outside it (chrM's depth
            # varies 2x along the contig)
            assert len(loads) <= (1 if accuracy == 0 else 2), loads
            if accuracy == 0:
                assert n == need


class _Loaded:
    def __init__(self, n, span, halo):
        self.n = n
        self.timings = {"max_span": span, "plan": {"used_index": 0, "halo": halo}}


def _span_worker(rank, world, port, q):
    """Rank 0's segments hold a read spanning 5000 loci; rank 1 planned with a 1000-locus halo and
    saw none that long: rank 1 must load again with a halo covering it, rank 0 must not."""
    import torch.distributed as dist
    from guacamole_amd.distributed import rank_loci_and_reads
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def load(region, halos=None):
        calls.append(halos)
        h = 1000 if halos is None else halos[0]
        return [_Loaded(1, 5000 if rank == 0 else 150, h)]
    sets, _ = rank_loci_and_reads(load, ["c"], [100_000], LociSet.parse("all"), 4, 0, rank, world, "cpu")
    q.put((rank, calls, sets[0].timings["plan"]["halo"]))
    dist.barrier()
    dist.destroy_process_group()


def test_probe_halo_is_widened_by_another_ranks_span():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_span_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == (0, [None, [10000]], 10000)  # (this stand-in load does not re-plan itself)
    assert got[1] == (1, [None, [10000]], 10000)


def _fail_worker(rank, world, port, q):
    """Rank 1's load raises (a malformed record in its segments only): both ranks must raise, rank
    1 its own error and rank 0 a PeerLoadError naming it, instead of rank 0 blocking."""
    import torch.distributed as dist
    from guacamole_amd.distributed import PeerLoadError, rank_loci_and_reads
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def load(region, halos=None):
        if rank == 1:
            raise ValueError("bad record 7 in rank 1's segments")
        return [_Loaded(1, 150, 1000)]
    try:
        rank_loci_and_reads(load, ["c"], [100_000], LociSet.parse("all"), 4, 0, rank, world, "cpu")
        q.put((rank, "returned"))
    except PeerLoadError as e:
        q.put((rank, "peer: " + str(e)))
    except ValueError as e:
        q.put((rank, "own: " + str(e)))
    dist.barrier()
    dist.destroy_process_group()


def test_load_error_on_one_rank_raises_on_every_rank():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_fail_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == (0, "peer: rank 1 failed to load its reads (ValueError: bad record 7 in rank 1's segments)")
    assert got[1] == (1, "own: bad record 7 in rank 1's segments")


def test_depth_bounds_balance_reads_not_loci():
    """Rank bounds by cumulative read counts: a deep first half puts the cut inside it."""
    from guacamole_amd.distributed import depth_bounds
    sizes = np.full(8, 1000, np.int64)
    counts = np.array([300, 300, 300, 300, 50, 50, 50, 50], np.int64)
    assert depth_bounds(sizes, counts, 2) == [0, 2000, 8000]
    assert depth_bounds(sizes, np.zeros(8, np.int64), 4) == [0, 2000, 4000, 6000, 8000]
    assert depth_bounds(sizes, counts, 1) == [0, 8000]


def test_depth_bounds_stay_inside_the_probe_windows():
    """With slack, each cut stays within `slack` micro partitions of the loci-uniform cut, so both
    neighbouring ranks decoded it for the counts (a cut far outside the window made
    most ranks decode their region a second time)."""
    from guacamole_amd.distributed import depth_bounds
    sizes = np.full(100, 1000, np.int64)
    counts = np.array([1000] * 10 + [1] * 90, np.int64)  # all the depth in the first tenth
    free = depth_bounds(sizes, counts, 4)
    assert free[1] < 10_000 and free[2] < 10_000  # read-balanced: cuts deep inside the first tenth
    clamped = depth_bounds(sizes, counts, 4, slack=5)
    for r in range(1, 4):
        u = 25 * r * 1000
        assert u - 5000 <= clamped[r] <= u + 5000
    assert clamped[0] == 0 and clamped[-1] == 100_000
    assert clamped == sorted(clamped)
    # even depth: the clamp changes nothing
    even = np.full(100, 7, np.int64)
    assert depth_bounds(sizes, even, 4, slack=5) == depth_bounds(sizes, even, 4)


def test_bench_refuses_a_world_size_other_than_gpus():
    """bench.py --gpus N under a launcher with WORLD_SIZE != N exits non-zero before any GPU work."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=root, env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr
