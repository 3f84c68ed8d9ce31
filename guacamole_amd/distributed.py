"""Multi-GPU driver: one process per GPU, a static split of the loci tasks, one terminal gather.

Loci shard embarrassingly: each locus depends only on the reads overlapping it
(DistributedUtil.scala:584-597 with halfWindowSize = 0), and the reference already runs its
tasks independently (:621-633).  The multi-GPU driver therefore keeps the reference's own task
partition (``--parallelism`` tasks from partitionLociUniformly / ByApproximateDepth,
DistributedUtil.scala:55-251) and hands each rank a contiguous block of tasks, balanced by read
count.  Every task keeps its own SlidingWindow on its rank, so a run on N GPUs gives exactly the
records of the same task partition on one GPU.  Each rank uploads only the reads overlapping its
tasks' loci, reads straddling a cut going to both sides (the reference's "expanded regions",
:584-597).  There is no data-path collective: the single exchange is the end-of-job gather of
the per-rank result buffers to rank 0 over RCCL (backend "nccl" on ROCm) — or gloo in tests —
where they are concatenated in rank order, which is task order.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .loci import LociSet, partition_loci_uniformly


OWN_GROUP = False  # init_from_env created the process group (and _finish_rank ends it)
SECOND_LOADS = 0  # rank_loci_and_reads calls whose ranks decoded their region again (a cut outside the probe)


def rank_info() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def hip_runtimes() -> List[str]:
    """The HIP runtime libraries (libamdhip64) mapped into this process."""
    try:
        with open("/proc/self/maps") as fh:
            return sorted({line.split()[-1] for line in fh if "libamdhip64" in line})
    except OSError:
        return []


def check_hip_runtimes() -> None:
    """torch ships its own HIP runtime (torch/lib/libamdhip64.so); libgqpileup.so links the
    system's (/opt/rocm).  When torch is imported first, the library binds to torch's runtime (the
    same SONAME) and both share one device context.  When libgqpileup.so is loaded first (a
    native.Context opened before `import torch`), torch brings its own copy and the process holds
    two HIP runtimes: torch then reports "No HIP GPUs are available" at its first device call.
    Raise a clear error for that order instead (init_from_env / bench.py import torch before the
    library at world > 1)."""
    libs = hip_runtimes()
    if len(libs) > 1:
        raise RuntimeError("two HIP runtimes in this process (%s): libgqpileup.so was loaded before torch; import "
                           "torch (or call guacamole_amd.distributed.init_from_env) before opening a native.Context"
                           % ", ".join(libs))


def init_from_env():
    """Join the process group torch.distributed.run set up (one rank per GPU).  Returns
    (rank, world, local GPU, gather device): the gather device is "cuda:<local>" for RCCL, or
    "cpu" when GQ_DIST_BACKEND=gloo (ranks may then share GPUs: a rehearsal of the flow)."""
    rank, world, local = rank_info()
    if world == 1:
        return rank, world, local, None
    import torch
    import torch.distributed as dist
    check_hip_runtimes()
    backend = os.environ.get("GQ_DIST_BACKEND", "nccl")
    if dist.is_initialized():  # a caller's group (bench.py runs the commands in its ranks): joined, not owned
        if dist.get_backend() == "nccl":  # (the group's own backend, not the environment's)
            return rank, world, local, "cuda:%d" % local
        return rank, world, local % max(1, torch.cuda.device_count()), "cpu"
    global OWN_GROUP
    OWN_GROUP = True
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return rank, world, local, "cuda:%d" % local
    local = local % max(1, torch.cuda.device_count())
    dist.init_process_group(backend)
    return rank, world, local, "cpu"


def split_loci(loci: LociSet, world: int) -> List[LociSet]:
    """Static contiguous split of a LociSet into `world` parts in partition order
    (partitionLociUniformly with tasks = world, DistributedUtil.scala:83-108)."""
    inv = partition_loci_uniformly(world, loci).as_inverse_map()
    return [inv.get(r, LociSet()) for r in range(world)]


def _starts_by_contig(read_sets, n_contigs: int):
    out = [[] for _ in range(n_contigs)]
    for rs in read_sets:
        for c in range(n_contigs):
            m = rs.contig == c
            if m.any():
                out[c].append(np.asarray(rs.start[m], np.int64))
    return [np.sort(np.concatenate(x)) if x else np.zeros(0, np.int64) for x in out]


def assign_tasks_to_ranks(flat_loci, world: int, read_sets: Sequence, n_contigs: int) -> np.ndarray:
    """Rank of each flattened loci range (flatten_partitions order: task, contig, start): tasks in
    contiguous blocks, cut where the running weight crosses k / world of the total.  Weight of a
    range = reads starting in it (all read sets) + 1e-3 per locus (so empty stretches still spread)."""
    contig, start, end, task = (np.asarray(a) for a in flat_loci)
    n = len(task)
    if n == 0 or world == 1:
        return np.zeros(n, np.int64)
    starts = _starts_by_contig(read_sets, n_contigs)
    w = np.empty(n, np.float64)
    for i in range(n):
        s = starts[int(contig[i])]
        w[i] = (np.searchsorted(s, end[i], "left") - np.searchsorted(s, start[i], "left")) + 1e-3 * (end[i] - start[i])
    tasks = np.unique(task)
    tw = np.zeros(len(tasks))
    np.add.at(tw, np.searchsorted(tasks, task), w)
    cum = np.cumsum(tw)
    total = cum[-1] if cum[-1] > 0 else 1.0
    rank_of_task = np.minimum(world - 1, np.floor((cum - tw / 2) * world / total)).astype(np.int64)
    rank_of_task = np.maximum.accumulate(rank_of_task)  # contiguous blocks, rank order = task order
    return rank_of_task[np.searchsorted(tasks, task)]


def reads_overlapping(rs, contig, start, end) -> np.ndarray:
    """Indices (ascending) of the reads overlapping any of the ranges (contig, [start, end)):
    the reads the reference shuffles to those loci's tasks (DistributedUtil.scala:585-597)."""
    contig = np.asarray(contig)
    keep = []
    for c in np.unique(contig):
        m = contig == c
        s, e = np.asarray(start, np.int64)[m], np.asarray(end, np.int64)[m]
        o = np.argsort(s, kind="stable")
        s, e = s[o], e[o]
        idx = np.nonzero(rs.contig == c)[0]
        if len(idx) == 0:
            continue
        rst, ren = np.asarray(rs.start[idx], np.int64), np.asarray(rs.end[idx], np.int64)
        k = np.searchsorted(e, rst, "right")  # first range ending after the read's start
        hit = k < len(e)
        hit[hit] = s[k[hit]] < ren[hit]
        keep.append(idx[hit])
    return np.sort(np.concatenate(keep)) if keep else np.zeros(0, np.int64)


def rank_share(rs, flat_loci, rank_of_range: np.ndarray, rank: int):
    """(this rank's reads, its flattened loci ranges with their original task ids)."""
    sel = rank_of_range == rank
    loci = tuple(np.ascontiguousarray(np.asarray(a)[sel]) for a in flat_loci)
    return rs.subset(reads_overlapping(rs, loci[0], loci[1], loci[2])), loci


def _positions(flat_loci):
    """Each flattened range's first locus as a position in loci order (flatten order: task,
    contig, start — tasks take consecutive loci, so this is LociSet order) and each task's
    (first position, loci)."""
    contig, start, end, task = (np.asarray(a) for a in flat_loci)
    n = np.asarray(end, np.int64) - np.asarray(start, np.int64)
    pos = np.concatenate([[0], np.cumsum(n)])[:-1] if len(n) else np.zeros(0, np.int64)
    return pos, n


def ranks_by_position(flat_loci, bounds: Sequence[int]) -> np.ndarray:
    """Rank of each flattened range: every task goes whole to the rank whose loci-position
    interval [bounds[r], bounds[r + 1]) holds the task's middle locus (contiguous blocks of
    tasks, rank order = task order)."""
    contig, start, end, task = (np.asarray(a) for a in flat_loci)
    if len(task) == 0:
        return np.zeros(0, np.int64)
    pos, n = _positions(flat_loci)
    tasks, first = np.unique(task, return_index=True)
    tot = np.zeros(len(tasks), np.int64)
    np.add.at(tot, np.searchsorted(tasks, task), n)
    mid = pos[first] + tot // 2
    rot = np.clip(np.searchsorted(np.asarray(bounds[1:-1], np.int64), mid, "right"), 0, len(bounds) - 2)
    rot = np.maximum.accumulate(rot)
    return rot[np.searchsorted(tasks, task)]


def loci_of(flat_loci, names: Sequence[str]) -> LociSet:
    """The LociSet of some flattened ranges (contig ids index `names`)."""
    from .loci import LociMapBuilder
    b = LociMapBuilder()
    for c, s, e in zip(*(np.asarray(a) for a in flat_loci[:3])):
        b.put(names[int(c)], int(s), int(e), 0)
    return LociSet(b.result())


def covers(outer: LociSet, inner: LociSet) -> bool:
    """Every locus of `inner` is in `outer`."""
    for c in inner.contigs:
        o = outer.on_contig(c).ranges
        starts = [s for s, _ in o]
        import bisect
        for s, e in inner.on_contig(c).ranges:
            i = bisect.bisect_right(starts, s) - 1
            if i < 0 or o[i][1] < e:
                return False
    return True


def _all_true(ok: bool, device) -> bool:
    """Logical AND of a flag over the ranks (so every rank takes the same branch)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int64, device=torch.device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def _any_true(flag: bool, device) -> bool:
    return not _all_true(not flag, device)


def _all_max(vals: Sequence[int], device) -> List[int]:
    """Element-wise maximum of an int list over the ranks."""
    import torch
    import torch.distributed as dist
    if not vals:
        return []
    t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=torch.device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [int(v) for v in t.cpu().tolist()]


def all_gather_objects(obj) -> list:
    import torch.distributed as dist
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


class PeerLoadError(RuntimeError):
    """Raised on every rank whose own load succeeded when another rank's load failed: the ranks
    load different parts of the input, so an error in one rank's segments must end all of them
    together instead of leaving the others blocked in the next collective."""


def _together(fn, device):
    """Run fn() on every rank; if it raised on any rank, raise on every rank.  The failing rank
    re-raises its own exception (type and message unchanged: the CLI reports it as the
    one-process run does); the others raise PeerLoadError naming the first failing rank and its
    message."""
    err, out = None, None
    try:
        out = fn()
    except Exception as e:  # re-raised below, on every rank
        err = e
    if _all_true(err is None, device):
        return out
    msgs = all_gather_objects(None if err is None else "%s: %s" % (type(err).__name__, err))
    if err is not None:
        raise err
    r = next(i for i, m in enumerate(msgs) if m is not None)
    raise PeerLoadError("rank %d failed to load its reads (%s)" % (r, msgs[r]))


def device_ingest_ranks(ctx, paths: Sequence[str], filters, builder, parallelism: int, accuracy: int, rank: int,
                        world: int, device):
    """The multi-GPU ingest: each rank decodes on its own GPU only the BGZF blocks whose records
    can overlap its tasks' loci (bamdev.load_reads_device with a region; the reference ships a
    read to exactly the tasks it overlaps, DistributedUtil.scala:584-597), with no host copy of
    the whole input on any rank.  Returns ([DeviceReadSet per path], this rank's flattened loci
    ranges with their task ids, the contig names) or None when some rank cannot take the device
    path (plain gzip, an unsorted file, device memory): every rank then takes the host loader."""
    from .bamdev import MappedBam, load_reads_device
    maps = _together(lambda: [MappedBam(p, populate=False) for p in paths], device)
    if not _all_true(all(m.ok for m in maps), device):
        return None
    dicts = [m.contigs() for m in maps]
    names, lengths = dicts[0]
    if any(d != dicts[0] for d in dicts[1:]):
        raise ValueError("Tumor and normal samples have different sequence dictionaries.")
    first = {"maps": maps}

    def load(region, halos=None):
        ms = first.pop("maps", [None] * len(paths))  # the host mappings serve the first load
        if halos is None:
            return [load_reads_device(ctx, p, filters, m, region=region) for p, m in zip(paths, ms)]
        return [load_reads_device(ctx, p, filters, m, region=region, halo=h) for p, m, h in zip(paths, ms, halos)]
    got = rank_loci_and_reads(load, names, lengths, builder, parallelism, accuracy, rank, world, device)
    return None if got is None else (got[0], got[1], names)


def rank_loci_and_reads(load, names, lengths, builder, parallelism: int, accuracy: int, rank: int, world: int,
                        device):
    """This rank's share of the single-process task partition and its reads, with reads loaded
    by region only: load(LociSet) -> [read set per input] (None entries: that input cannot be
    loaded so; every rank then gives up, None).

    partitionLociUniformly (DistributedUtil.scala:83-108) needs no reads.  For
    partitionLociByApproximateDepth (:162-251) the micro partitions are split across the ranks;
    each rank loads its share (+ 5 % slack each side), counts the reads overlapping its own micro
    partitions (:181-189), and an all-reduce of the counts gives every rank the counts one
    process computes — so the same tasks.  Tasks go whole to ranks in contiguous blocks
    (ranks_by_position); a rank whose tasks reach past what it loaded loads its tasks' loci."""
    from .loci import (LociMapBuilder, flatten_partitions, micro_partition_count, partition_loci_by_counts,
                       partition_loci_uniformly, _region_counts)
    loci = builder.result(dict(zip(names, lengths)))
    tasks = parallelism if parallelism > 0 else max(1, world)
    cidx = {c: i for i, c in enumerate(names)}
    sets = None
    decoded = None
    if accuracy == 0 or (tasks == 1 and loci.count > 0):
        parts = partition_loci_uniformly(tasks, loci)
        flat = flatten_partitions(parts, cidx)
        total = int(loci.count)
        bounds = [total * r // world for r in range(world + 1)]
    else:
        n_micro = micro_partition_count(tasks, loci, accuracy)
        micro = partition_loci_uniformly(n_micro, loci)
        inv = micro.as_inverse_map()
        m0, m1 = rank * n_micro // world, (rank + 1) * n_micro // world
        slack = max(1, (m1 - m0) // 20)
        b = LociMapBuilder()
        for m in range(max(0, m0 - slack), min(n_micro, m1 + slack)):
            b.put_set(inv[m], 0)
        decoded = LociSet(b.result())
        sets = _together(lambda: load(decoded), device)
        if not _all_true(all(x is not None for x in sets), device):
            return None
        # the counts must see every read overlapping the micro partitions: widen the halo first
        sets = _widen_halos(sets, lambda halos: load(decoded, halos), device)
        if sets is None:
            return None
        counts = np.zeros(n_micro, np.int64)
        for x in sets:
            counts += _region_counts(micro, x.regions(), n_micro)
        counts[:m0] = 0
        counts[m1:] = 0
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(counts).to(torch.device(device))
        dist.all_reduce(t)
        counts = t.cpu().numpy()
        parts = partition_loci_by_counts(tasks, loci, micro, counts)
        flat = flatten_partitions(parts, cidx)
        sizes = np.array([inv[m].count for m in range(n_micro)], np.int64)
        bounds = depth_bounds(sizes, counts, world, slack=max(1, n_micro // world // 20))
    rr = ranks_by_position(flat, bounds)
    sel = rr == rank
    mine = tuple(np.ascontiguousarray(np.asarray(a)[sel]) for a in flat)
    region = loci_of(mine, names)
    if _any_true(sets is None or not covers(decoded, region), device):
        global SECOND_LOADS
        SECOND_LOADS += 1  # (every rank counts it: the branch is taken together)
        if sets is None or not covers(decoded, region):
            sets = None  # (the first load's memory goes before the second)
        sets = _together(lambda: load(region) if sets is None else sets, device)
    if not _all_true(all(x is not None for x in sets), device):
        return None
    sets = _widen_halos(sets, lambda halos: load(region, halos), device)
    return None if sets is None else (sets, mine)


def depth_bounds(sizes: np.ndarray, counts: np.ndarray, world: int, slack: Optional[int] = None) -> List[int]:
    """Rank bounds in loci positions from the all-reduced micro-partition read counts: rank r's
    block starts at the micro-partition edge nearest to where the cumulative count (+ 1e-3 per
    locus, so empty stretches still spread) crosses r / world of the total — balanced by read weight as
    assign_tasks_to_ranks balances the host path, not by loci.

    slack (micro partitions): each cut stays within `slack` partitions of the loci-uniform cut
    r * n / world, so it lies inside what both neighbouring ranks decoded for the counts
    ([m0 - slack, m1 + slack)); on uneven depth the balance is then approximate, but no rank has to
    decode its region a second time because a cut moved out of its probe window."""
    sizes = np.asarray(sizes, np.int64)
    n = len(sizes)
    w = np.asarray(counts, np.float64) + 1e-3 * sizes
    cum = np.concatenate([[0.0], np.cumsum(w)])
    edge = np.concatenate([[0], np.cumsum(sizes)])
    total = cum[-1] if cum[-1] > 0 else 1.0
    out = [0]
    for r in range(1, world):
        want = total * r / world
        m = int(np.searchsorted(cum, want, "left"))  # the nearer of the two micro-partition edges
        if m > 0 and (m >= len(cum) or want - cum[m - 1] < cum[m] - want):
            m -= 1
        if slack is not None:
            u = r * n // world
            m = min(max(m, u - slack), u + slack)
        out.append(max(out[-1], int(edge[min(m, len(sizes))])))
    out.append(int(edge[-1]))
    return out


def _widen_halos(sets, reload, device):
    """Without an index a rank plans `halo` loci back from each of its ranges: a read reaching
    further back is found only by the rank whose segments hold its start.  The longest span any
    rank saw (per input) is shared, and a rank whose probe plan's halo is shorter loads again
    with twice that span (reload(halos) -> sets).  Every rank takes the branch together."""
    spans = _all_max([int(getattr(x, "timings", {}).get("max_span", 0)) for x in sets], device)
    plans = [getattr(x, "timings", {}).get("plan") for x in sets]
    short = [p is not None and not p["used_index"] and g > p["halo"] for p, g in zip(plans, spans)]
    if _any_true(any(short), device):  # (collectives inside)
        halos = [max(2 * g, p["halo"]) if p is not None else 0 for p, g in zip(plans, spans)]
        if any(short):
            sets = None
        sets = _together(lambda: reload(halos) if sets is None else sets, device)
        if not _all_true(all(x is not None for x in sets), device):
            return None
    return sets


def _gatherv_to_rank0(mine, sizes: List[int], device):
    """Variable-size gather of one uint8 tensor per rank (``mine``: exactly ``sizes[rank]``
    bytes, on ``device``) to rank 0, rank order.  Every rank's bytes travel once, at their own
    size: rank 0 posts one receive per non-empty rank and the others one send, batched into a
    single group (``batch_isend_irecv``: one RCCL group call, so the transfers run concurrently,
    each over its own xGMI link into rank 0 — no ring, no padding to the largest rank)."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    if rank == 0:
        parts = [mine] + [torch.empty(max(0, sizes[r]), dtype=torch.uint8, device=device) for r in range(1, world)]
        ops = [dist.P2POp(dist.irecv, parts[r], r) for r in range(1, world) if sizes[r] > 0]
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return parts
    if sizes[rank] > 0:
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, mine, 0)]):
            w.wait()
    return None


def _all_sizes(n: int, device) -> List[int]:
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(n)], dtype=torch.int64, device=device)
    out = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [int(x.item()) for x in out]


def gather_images_to_rank0(calls, device: str):
    """Every rank's germline result image (left in HBM by gq_germline_threshold_device) to rank 0:
    sizes all-gathered, then the images gathered at their own sizes (_gatherv_to_rank0) over
    RCCL / xGMI (device "cuda:k"), or through host memory with gloo (device "cpu").  Returns
    rank 0's list of per-rank uint8 tensors (rank order), None elsewhere."""
    import ctypes as C

    import torch

    calls.check_current()
    dev = torch.device(device)
    sizes = _all_sizes(int(calls.image_bytes), dev)
    mine = torch.empty(int(calls.image_bytes), dtype=torch.uint8, device=dev)
    if calls.image_bytes:
        on_gpu = dev.type == "cuda"
        if on_gpu:
            torch.cuda.synchronize(dev)
        hip = C.CDLL("libamdhip64.so.7")  # by SONAME: the HIP runtime already loaded in this process
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        # device to device (RCCL) or device to host (gloo)
        rc = hip.hipMemcpy(C.c_void_p(mine.data_ptr()), C.c_void_p(calls.image), int(calls.image_bytes),
                           3 if on_gpu else 2)
        if rc != 0:
            raise RuntimeError("hipMemcpy of the result image failed (%d)" % rc)
    return _gatherv_to_rank0(mine, sizes, dev)


def gather_germline(calls, device: str):
    """gather_images_to_rank0 plus each rank's record count and run counters; rank 0 gets one
    GermlineCalls per rank (rank order), other ranks None."""
    import torch
    import torch.distributed as dist

    from .native import GermlineCalls
    world = dist.get_world_size()
    meta = torch.tensor([len(calls), calls.visited_loci, calls.complex_loci, calls.ambiguous_loci, calls.tie_loci],
                        dtype=torch.int64, device=torch.device(device))
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta)
    images = gather_images_to_rank0(calls, device)
    if images is None:
        return None
    out = []
    for img, m in zip(images, metas):
        m = [int(x) for x in m.cpu().tolist()]
        out.append(GermlineCalls.from_image(img.cpu().numpy(), m[0], *m[1:]))
    return out


def gather_to_rank0(buf: np.ndarray, device: Optional[str] = None) -> Optional[List[np.ndarray]]:
    """Variable-size gather of one uint8 buffer per rank to rank 0 (_gatherv_to_rank0).

    device: torch device for the collective ("cuda:k" => RCCL over xGMI; None => CPU/gloo)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [buf]
    dev = torch.device(device) if device else torch.device("cpu")
    sizes = _all_sizes(int(buf.size), dev)
    mine = torch.from_numpy(np.ascontiguousarray(buf, np.uint8)).to(dev)
    parts = _gatherv_to_rank0(mine, sizes, dev)
    return None if parts is None else [p.cpu().numpy() for p in parts]


def gather_somatic(calls, device: Optional[str]):
    """Each rank's SomaticCalls (host arrays) to rank 0 (rank order), packed as raw columns."""
    from .native import SomaticCalls
    parts = gather_to_rank0(calls.pack(), device)
    return None if parts is None else [SomaticCalls.unpack(p) for p in parts]
