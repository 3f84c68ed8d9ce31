"""BAM reads decoded on the GPU (gqpileup.h: gq_bam_dev_*), for the callers' single pass.

The host loader (``ingest.load_bam``: libgqingest, 16 host threads) inflates and decodes the
BAM on the CPU, then ``soa.pack`` + ``Context.upload`` parse MD tags and copy the SoA to HBM.
Here the compressed file is copied to HBM once, and the BGZF inflate, record parse, the
loader's filters (Read.InputFilters, reads/Read.scala:95-122, :411-428), MD events and the SoA
layout all run on the device.  The same rules give the same arrays, read for read
(tests/test_gpu_bamdev.py compares every array with the host loader's).

``load_reads_device`` returns a ``DeviceReadSet``: the host-side facts the commands use
(contig dictionary, sample names, read count, read regions on demand) plus the resident
read set, already in the ``commands.device_reads`` cache of its context.  It returns None
where the host loader must run instead: a gzip stream without BGZF block sizes, or kept reads
out of (contig, start) order (the host loader sorts them).
"""
from __future__ import annotations

import ctypes as C
import os
import time
import weakref
from typing import Dict, List, Optional

import numpy as np

from . import native, soa
from .reads import InputFilters, ReadLoadError, _header_read_groups

GQ_E_UNSORTED = 6
GQ_E_HIP = 8
GQ_E_BAM_IO = 11
GQ_E_BAM_FORMAT = 12
GQ_E_BAM_RECORD = 13
GQ_E_MD_PARSE = 14
GQ_E_NOT_BGZF = 15


class gq_bam_dev_filters(C.Structure):
    _fields_ = [("non_duplicate", C.c_int32), ("passed_vendor_quality_checks", C.c_int32),
                ("is_paired", C.c_int32), ("has_md_tag", C.c_int32), ("use_loci", C.c_int32),
                ("loci_begin", C.c_void_p), ("loci_start", C.c_void_p), ("loci_end", C.c_void_p),
                ("n_rg", C.c_int32), ("rg_ids", C.c_char_p)]


class gq_bam_dev_sizes(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("n_records", "n_reads", "seq_bytes", "cigar_len", "md_events", "comp_bytes",
                                         "bam_bytes", "n_blocks")] + [
        (k, C.c_float) for k in ("map_ms", "h2d_ms", "inflate_ms", "records_ms", "parse_ms")] + [
        ("max_span", C.c_int64)]


class gq_bam_dev_plan_info(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("n_segments", "n_blocks", "comp_bytes", "bam_bytes", "probes")] + [
        ("used_index", C.c_int32), ("pad", C.c_int32)]


GQ_E_PLAN = 16
# Loci of margin before each planned range when the BAM has no index: a read that starts further
# back and still overlaps the range is missed unless some rank sees one that long (the load then
# re-plans with a wider halo, see load_reads_device).  1 Mb at 30x is ~0.2 M extra records
# decoded per range boundary.  GQ_INGEST_HALO overrides it (tests use a small one).
DEFAULT_HALO = int(os.environ.get("GQ_INGEST_HALO", 1 << 20))


class DeviceReadSet:
    """A read set loaded straight into HBM: what the commands read on the host, and the
    resident gq_dev_reads (``reads``)."""

    def __init__(self, ctx: native.Context, reads: native.DeviceReads, contig_names: List[str],
                 contig_lengths: List[int], sample_names: List[str], n: int, timings: Dict[str, float]):
        self.contig_names = contig_names
        self.contig_lengths = contig_lengths
        self.sample_names = sample_names
        self._n = n
        self.reads = reads
        self.timings = timings
        self._pos = None
        # commands.device_reads finds the resident set here (no host SoA to upload)
        self._device = {id(ctx): (weakref.ref(ctx), reads)}

    @property
    def n(self) -> int:
        return self._n

    @property
    def contig_lengths_map(self) -> Dict[str, int]:
        return dict(zip(self.contig_names, self.contig_lengths))

    def contig_index(self) -> Dict[str, int]:
        return {c: i for i, c in enumerate(self.contig_names)}

    def positions(self):
        """(contig_read_begin, start, end) copied from HBM (once)."""
        if self._pos is None:
            L = native.lib()
            begin = np.zeros(len(self.contig_names) + 1, np.int64)
            start = np.empty(self._n, np.int32)
            end = np.empty(self._n, np.int32)
            native._check(L.gq_reads_contig_begin(self.reads.h, begin.ctypes.data))
            if self._n:
                native._check(L.gq_reads_positions(self.reads.h, start.ctypes.data, end.ctypes.data))
            self._pos = (begin, start.astype(np.int64), end.astype(np.int64))
        return self._pos

    def regions(self):
        """(contig name, starts, ends) per contig, for partitionLociByApproximateDepth."""
        begin, start, end = self.positions()
        return [(name, start[begin[i]:begin[i + 1]], end[begin[i]:begin[i + 1]])
                for i, name in enumerate(self.contig_names) if begin[i + 1] > begin[i]]


def download(reads: native.DeviceReads) -> Dict[str, np.ndarray]:
    """Every SoA array of a resident read set, copied to the host (gq_reads_download)."""
    L = native.lib()
    info = native.gq_reads_info()
    native._check(L.gq_reads_get_info(reads.h, C.byref(info)))
    n, nc = int(info.n_reads), int(info.n_contigs)
    arrs = dict(contig_read_begin=np.empty(nc + 1, np.int64), start=np.empty(n, np.int32),
                end=np.empty(n, np.int32), pmax_end=np.empty(n, np.int32), mapq=np.empty(n, np.uint8),
                flags=np.empty(n, np.uint8), sample=np.empty(n, np.uint8), seq_off=np.empty(n, np.int64),
                seq_len=np.empty(n, np.int32), cigar_off=np.empty(n, np.int64), n_cigar=np.empty(n, np.int32),
                md_off=np.empty(n, np.int64), n_md=np.empty(n, np.int32), n_mismatch=np.empty(n, np.uint16),
                seq=np.empty(int(info.seq_bytes), np.uint8), qual=np.empty(int(info.seq_bytes), np.uint8),
                cigar=np.empty(int(info.cigar_len), np.uint32), md_ev=np.empty(int(info.md_len), np.uint32),
                sample_hash=np.zeros(int(info.n_samples), np.uint32),
                n_contigs=np.int64(nc), n_samples=np.int64(info.n_samples))
    s, _ = native.make_gq_reads(arrs)
    native._check(L.gq_reads_download(reads.h, C.byref(s)))
    return arrs


class MappedBam:
    """A BAM file mapped on the host with its BGZF block table and header (gq_bam_dev_map): the
    part of the device load that needs no GPU, so it can run while the context starts.  None-like
    (``ok`` False) for a plain gzip stream.  populate=False: the file's pages are not faulted in
    up front (a region-restricted load reads only its segments)."""

    def __init__(self, path: str, populate: bool = True):
        self.path = path
        self.h = C.c_void_p()
        from . import _early
        got = _early.take_map(path) if populate else None  # (the CLI's map, made while it imported)
        if got is not None and got[0] == 0:  # (a failed early map is redone here: its message is that thread's)
            rc, self.h, self.t, self.t_mapped = got
            native.lib()
        else:
            self.t = time.perf_counter()
            rc = native.lib().gq_bam_dev_map_ex(path.encode(), int(populate), C.byref(self.h))
            self.t_mapped = time.perf_counter()
        self.ok = rc != GQ_E_NOT_BGZF
        if self.ok:
            _raise(rc)

    def contigs(self):
        """(names, lengths) of the header's reference dictionary."""
        L = native.lib()
        n = L.gq_bam_dev_n_contigs(self.h)
        return ([L.gq_bam_dev_contig_name(self.h, i).decode() for i in range(n)],
                [int(L.gq_bam_dev_contig_length(self.h, i)) for i in range(n)])

    def plan(self, region, halo: int = DEFAULT_HALO, bai: Optional[str] = None):
        """gq_bam_dev_plan over a LociSet (the ranges of the header's contigs it names): the next
        load reads only the records that can overlap it.  Returns the plan info as a dict with
        its segments, or None when the file does not allow a plan (GQ_E_PLAN: not declared
        coordinate-sorted) — the load then reads the whole file."""
        names, _ = self.contigs()
        begin, starts, ends = _loci_arrays(region, names)
        info = gq_bam_dev_plan_info()
        L = native.lib()
        rc = L.gq_bam_dev_plan(self.h, begin.ctypes.data, starts.ctypes.data, ends.ctypes.data, int(halo),
                               (bai or "").encode(), C.byref(info))
        if rc == GQ_E_PLAN:
            return None
        _raise(rc)
        n = int(info.n_segments)
        b0, off, b1 = (np.zeros(max(n, 1), np.int64) for _ in range(3))
        eof = np.zeros(max(n, 1), np.int32)
        _raise(L.gq_bam_dev_plan_segments(self.h, b0.ctypes.data, off.ctypes.data, b1.ctypes.data, eof.ctypes.data))
        out = {k: int(getattr(info, k)) for k in ("n_segments", "n_blocks", "comp_bytes", "bam_bytes", "probes",
                                                  "used_index")}
        out["segments"] = [(int(b0[i]), int(off[i]), int(b1[i]), bool(eof[i])) for i in range(n)]
        out["halo"] = int(halo)
        return out

    def close(self) -> None:
        if self.h:
            native.lib().gq_bam_dev_close(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def map_bams(paths) -> Dict[str, object]:
    """MappedBam per path, on a host thread (ctypes releases the GIL in the native calls):
    start it, create the GPU context, then join().  join() returns {path: MappedBam} or raises
    what the mapping raised."""
    import threading
    box: Dict[str, object] = {}

    def run():
        try:
            box["maps"] = {p: MappedBam(p) for p in paths}
        except BaseException as e:  # re-raised by join
            box["err"] = e

    th = threading.Thread(target=run, daemon=True)
    th.start()

    def join():
        th.join()
        if "err" in box:
            raise box["err"]
        return box["maps"]
    return {"join": join}


def _loci_arrays(loci, names):
    """A LociSet as gq_bam_dev loci arrays over the header's contigs: (begin[n + 1], starts, ends)."""
    begin, starts, ends = [0], [], []
    for name in names:
        for s, e in loci.on_contig(name).ranges:
            starts.append(s)
            ends.append(e)
        begin.append(len(starts))
    return np.asarray(begin, np.int64), np.asarray(starts or [0], np.int64), np.asarray(ends or [0], np.int64)


def bai_path(path: str) -> Optional[str]:
    """The BAM's index by samtools' names (X.bam.bai, then X.bai), if present."""
    import os
    for p in (path + ".bai", path[:-4] + ".bai" if path.endswith(".bam") else None):
        if p and os.path.exists(p):
            return p
    return None


def load_reads_device(ctx: native.Context, path: str, filters: InputFilters = InputFilters(),
                      mapped: Optional[MappedBam] = None, region=None,
                      halo: int = DEFAULT_HALO) -> Optional[DeviceReadSet]:
    """BAM -> resident read set on ctx's GPU (None: the host loader must run, see the module
    docstring).  Raises ReadLoadError / soa.MdParseError as the host loader does.  `mapped`:
    the file already mapped (map_bams), else it is mapped here.

    region (a LociSet, the multi-GPU ingest): keep only the reads overlapping it, reading only
    the BGZF blocks whose records can overlap it (gq_bam_dev_plan: from the BAI's linear index
    when the file has one, else by host probes with `halo` loci of margin).  The reads kept are
    those of the filters within the region (the region lies inside the filters' loci).  Without
    an index the load checks the longest reference span it saw against the halo and, if a read
    could reach further back, plans again with twice that span (timings["replans"])."""
    replans = 0
    while True:
        rs = _load_reads_device(ctx, path, filters, mapped, region, halo)
        if rs is None or region is None or rs.timings.get("plan") is None:
            break
        plan = rs.timings["plan"]
        if plan["used_index"] or rs.timings["max_span"] <= halo:
            break
        halo = 2 * rs.timings["max_span"]
        mapped = None
        replans += 1
    if rs is not None:
        rs.timings["replans"] = replans
    return rs


def _load_reads_device(ctx, path, filters, mapped, region, halo, use_plan=True):
    L = native.lib()
    planned = region is not None and use_plan
    m = mapped if mapped is not None and (mapped.h or not mapped.ok) else MappedBam(path, populate=not planned)
    if not m.ok:
        return None
    t0 = m.t
    tp = time.perf_counter()
    plan = m.plan(region, halo, bai_path(path)) if planned else None
    tl = time.perf_counter()
    h, m.h = m.h, C.c_void_p()  # the handle now belongs to this load
    try:
        rc = L.gq_bam_dev_load(ctx.h, h)
        tl1 = time.perf_counter()
        if rc == GQ_E_HIP:  # out of device memory for the loader's buffers: the host loader's footprint is smaller
            L.gq_bam_dev_close(h)
            return None
        _raise(rc)
        t1 = time.perf_counter()
        n_ref = L.gq_bam_dev_n_contigs(h)
        names = [L.gq_bam_dev_contig_name(h, i).decode() for i in range(n_ref)]
        lengths = [int(L.gq_bam_dev_contig_length(h, i)) for i in range(n_ref)]
        text = L.gq_bam_dev_header_text(h).decode("utf-8", "replace")
        rg_samples = _header_read_groups(text)  # ID -> SM (None: no SM), header order
        rg_ids = list(rg_samples)
        if len(rg_ids) > 254:  # the device classes read groups in a byte: the host loader takes such headers
            L.gq_bam_dev_close(h)
            return None
        f = gq_bam_dev_filters(int(filters.non_duplicate), int(filters.passed_vendor_quality_checks),
                               int(filters.is_paired), int(filters.has_md_tag), 0, None, None, None, len(rg_ids),
                               b"".join(x.encode() + b"\0" for x in rg_ids) or None)
        keep = []
        loci = region
        if loci is None and filters.overlaps_loci is not None:
            loci = filters.overlaps_loci.result(dict(zip(names, lengths)))
        if loci is not None:
            keep = list(_loci_arrays(loci, names))
            f.use_loci = 1
            f.loci_begin, f.loci_start, f.loci_end = (a.ctypes.data for a in keep)
        first = np.full(len(rg_ids) + 1, -1, np.int64)
        z = gq_bam_dev_sizes()
        rc = L.gq_bam_dev_scan(h, C.byref(f), first.ctypes.data, C.byref(z))
        if rc == GQ_E_PLAN:  # a record runs past a planned segment: read the whole file
            L.gq_bam_dev_close(h)
            return _load_reads_device(ctx, path, filters, None, region, halo, use_plan=False)
        if rc == GQ_E_HIP:
            L.gq_bam_dev_close(h)
            return None
        _raise(rc)
        t2 = time.perf_counter()
        # samples: RG -> SM (else "default"), numbered by first appearance in file order
        samples: List[str] = []
        class_sample = np.zeros(256, np.uint8)
        for k in sorted(range(len(first)), key=lambda k: first[k]):
            if first[k] < 0:
                continue
            name = (rg_samples[rg_ids[k]] if k < len(rg_ids) else None) or "default"
            if name not in samples:
                samples.append(name)
            class_sample[k] = samples.index(name)
        n_samples = max(1, len(samples))
        sh = soa.sample_hashes(samples, n_samples)
        out = C.c_void_p()
        fill_ms = C.c_float()
        t3 = time.perf_counter()
        rc = L.gq_bam_dev_reads(h, class_sample.ctypes.data, n_samples, sh.ctypes.data, C.byref(out), C.byref(fill_ms))
        if rc in (GQ_E_UNSORTED, GQ_E_HIP):
            L.gq_bam_dev_close(h)
            return None
        _raise(rc)
    except BaseException:
        L.gq_bam_dev_close(h)
        raise
    t4 = time.perf_counter()
    dr = native.DeviceReads(ctx, out, None)
    timings = {k: float(getattr(z, k)) for k in ("map_ms", "h2d_ms", "inflate_ms", "records_ms", "parse_ms")}
    info = ctx.proj_stats(dr)
    timings.update(fill_ms=float(fill_ms.value), derive_ms=float(info.get("derive_ms", 0.0)),
                   open_s=t1 - t0, scan_s=t2 - t1, total_s=time.perf_counter() - t0,
                   # open_s's parts: the host map (and the wait for it when mapped on a thread), the
                   # plan (host probes or the BAI), gq_bam_dev_load (map_ms + h2d_ms + inflate_ms
                   # and their allocations), the header; then the scan, the sample table, the reads
                   wall_s={"map": (getattr(m, "t_mapped", tp) - t0), "to_plan": tp - getattr(m, "t_mapped", tp),
                           "plan": tl - tp, "dev_load": tl1 - tl, "header": t1 - tl1, "scan": t2 - t1,
                           "samples": t3 - t2, "dev_reads": t4 - t3, "stats": time.perf_counter() - t4},
                   records=int(z.n_records), comp_bytes=int(z.comp_bytes), bam_bytes=int(z.bam_bytes),
                   blocks=int(z.n_blocks), max_span=int(z.max_span), plan=plan)
    rs = DeviceReadSet(ctx, dr, names, lengths, samples, int(z.n_reads), timings)
    # the loader's buffers (compressed file, inflated stream, record tables: ~2.5x the file's
    # inflated size) are released now, so the callers have the HBM; on a host thread, off the
    # load's critical path (their hipFree calls take ~45 ms at chr20 30x)
    if DEFER_RELEASE and 3 * int(z.bam_bytes) < _free_device_bytes() // 4:  # (see DEFER_RELEASE)
        _deferred.append(h)
        return rs
    import threading
    th = threading.Thread(target=L.gq_bam_dev_close, args=(h,), name="gq_bam_dev_close")
    th.start()
    _release_threads.append(th)
    return rs


_release_threads: List[object] = []
# DEFER_RELEASE (set by `python -m guacamole_amd`, a process that exits after one command): the
# loaders' buffers are not released after the load.  hipFree synchronises the device and holds
# the HIP runtime while it runs (~45 ms for a chr20 30x BAM's buffers), so a release on a host
# thread beside the call made the CLI's first call wait for it (call stage 40-60 ms against a
# 3 ms cold call in-process).  The process ends with os._exit, which returns the memory; a
# load whose buffers would not leave room for the call (over a quarter of the device's free
# memory after the load) is released as before.
DEFER_RELEASE = False
_deferred: List[object] = []


def _free_device_bytes() -> int:
    """hipMemGetInfo's free bytes on the current device (0 if it cannot be read)."""
    try:
        hip = C.CDLL("libamdhip64.so.7")  # the HIP runtime libgqpileup.so already loaded
        free, total = C.c_size_t(), C.c_size_t()
        if hip.hipMemGetInfo(C.byref(free), C.byref(total)) != 0:
            return 0
        return int(free.value)
    except OSError:
        return 0


def join_release_threads() -> None:
    """Wait for the device loaders' buffer releases (before a hard process exit)."""
    while _release_threads:
        _release_threads.pop().join()


def _raise(rc: int) -> None:
    if rc == 0:
        return
    msg = native.lib().gq_last_error().decode()
    if rc == GQ_E_MD_PARSE:
        raise soa.MdParseError(msg)
    if rc in (GQ_E_BAM_IO, GQ_E_BAM_FORMAT, GQ_E_BAM_RECORD):
        raise ReadLoadError(msg)
    raise native.GQError(rc, msg)
