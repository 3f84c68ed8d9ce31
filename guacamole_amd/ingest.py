"""ctypes binding of libgqingest (include/gqingest.h): native BAM ingest and MD events.

``load_bam(path, filters)`` is what ``reads.load_reads`` runs for BAM input; ``md_events``
is what ``soa.pack`` runs for every read set.  Both raise if the library is missing: the
Python statements of the same rules (``reads._load_bam_py``, ``soa.md_events``) are the
checkers in tests/test_ingest.py, not fallbacks.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional

import numpy as np

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libgqingest.so")
_lib = None

GQI_E_RECORD = 3
GQI_E_MD = 4


class _Filters(C.Structure):
    _fields_ = [("non_duplicate", C.c_int32), ("passed_vendor_quality_checks", C.c_int32),
                ("is_paired", C.c_int32), ("has_md_tag", C.c_int32), ("use_loci", C.c_int32),
                ("loci_begin", C.c_void_p), ("loci_start", C.c_void_p), ("loci_end", C.c_void_p)]


class _Sizes(C.Structure):
    _fields_ = [("n_reads", C.c_int64), ("seq_bytes", C.c_int64), ("cigar_len", C.c_int64),
                ("md_bytes", C.c_int64), ("name_bytes", C.c_int64), ("n_rg", C.c_int32), ("sorted", C.c_int32)]


_READ_FIELDS = [("contig", np.int32, "n"), ("start", np.int64, "n"), ("end", np.int64, "n"),
                ("mapq", np.uint8, "n"), ("flags", np.uint8, "n"), ("rg", np.int32, "n"),
                ("seq_off", np.int64, "n"), ("seq_len", np.int32, "n"), ("seq", np.uint8, "seq"),
                ("qual", np.uint8, "seq"), ("cigar_off", np.int64, "n"), ("n_cigar", np.int32, "n"),
                ("cigar", np.uint32, "cigar"), ("md_off", np.int64, "n"), ("md_len", np.int32, "n"),
                ("md", np.uint8, "md"), ("name_off", np.int64, "n"), ("name_len", np.int32, "n"),
                ("names", np.uint8, "name")]


class _Reads(C.Structure):
    _fields_ = [(name, C.c_void_p) for name, _, _ in _READ_FIELDS]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError("libgqingest.so is not built (%s): run __graft_entry__.build()" % _LIB_PATH)
        L = C.CDLL(_LIB_PATH)
        L.gq_ingest_last_error.restype = C.c_char_p
        L.gq_bam_open.argtypes = [C.c_char_p, C.c_int32, C.POINTER(C.c_void_p)]
        L.gq_bam_close.argtypes = [C.c_void_p]
        L.gq_bam_header_text.argtypes = [C.c_void_p]
        L.gq_bam_header_text.restype = C.c_char_p
        L.gq_bam_n_contigs.argtypes = [C.c_void_p]
        L.gq_bam_contig_name.argtypes = [C.c_void_p, C.c_int32]
        L.gq_bam_contig_name.restype = C.c_char_p
        L.gq_bam_contig_length.argtypes = [C.c_void_p, C.c_int32]
        L.gq_bam_contig_length.restype = C.c_int64
        L.gq_bam_scan.argtypes = [C.c_void_p, C.POINTER(_Filters), C.c_int32, C.POINTER(_Sizes)]
        L.gq_bam_rg.argtypes = [C.c_void_p, C.c_int32]
        L.gq_bam_rg.restype = C.c_char_p
        L.gq_bam_rg_first.argtypes = [C.c_void_p, C.c_int32]
        L.gq_bam_rg_first.restype = C.c_int64
        L.gq_bam_fill.argtypes = [C.c_void_p, C.c_int32, C.POINTER(_Reads)]
        vp = C.c_void_p
        L.gq_md_count.argtypes = [C.c_int64, vp, vp, vp, vp, vp, vp, C.c_int32, vp, vp]
        L.gq_md_fill.argtypes = [C.c_int64, vp, vp, vp, vp, vp, vp, vp, C.c_int32, vp]
        _lib = L
    return _lib


def n_threads() -> int:
    """Host threads for ingest: OMP_NUM_THREADS when set (16 on the GPU box), else <= 16."""
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    return max(1, min(16, os.cpu_count() or 1))


def _err(L) -> str:
    return (L.gq_ingest_last_error() or b"").decode("utf-8", "replace")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


class NamePool:
    """Read names as one byte pool + offsets; list-like (len, [i], index, iteration)."""

    def __init__(self, pool: np.ndarray, off: np.ndarray, ln: np.ndarray):
        self.pool, self.off, self.len = pool, off, ln

    def __len__(self) -> int:
        return int(self.off.shape[0])

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        o = int(self.off[i])
        return self.pool[o:o + int(self.len[i])].tobytes().decode("utf-8", "replace")

    def __iter__(self):
        return (self[i] for i in range(len(self)))

    def index(self, name: str) -> int:
        for i, x in enumerate(self):
            if x == name:
                return i
        raise ValueError("%r is not in the read names" % name)


def load_bam(path: str, filters, timings: Optional[Dict[str, float]] = None) -> "ReadSet":
    """BAM -> ReadSet through libgqingest (reads._load_bam_py states the same rules).
    ``timings`` (optional) receives the seconds of open+inflate, scan and fill."""
    import time
    from .reads import ReadLoadError, ReadSet, _header_read_groups, _sample_of
    L = lib()
    nt = n_threads()
    h = C.c_void_p()
    t0 = time.perf_counter()
    st = L.gq_bam_open(os.fsencode(path), nt, C.byref(h))
    t1 = time.perf_counter()
    if st:
        raise ReadLoadError(_err(L))
    try:
        n_ref = L.gq_bam_n_contigs(h)
        contig_names = [L.gq_bam_contig_name(h, i).decode() for i in range(n_ref)]
        contig_lengths = [int(L.gq_bam_contig_length(h, i)) for i in range(n_ref)]
        text = L.gq_bam_header_text(h).decode("utf-8", "replace")
        f = _Filters(int(filters.non_duplicate), int(filters.passed_vendor_quality_checks), int(filters.is_paired),
                     int(filters.has_md_tag), 0, None, None, None)
        keep = []
        if filters.overlaps_loci is not None:
            loci = filters.overlaps_loci.result(dict(zip(contig_names, contig_lengths)))
            begin, starts, ends = [0], [], []
            for name in contig_names:
                for s, e in loci.on_contig(name).ranges:
                    starts.append(s)
                    ends.append(e)
                begin.append(len(starts))
            keep = [np.asarray(begin, np.int64), np.asarray(starts, np.int64), np.asarray(ends, np.int64)]
            f.use_loci = 1
            f.loci_begin, f.loci_start, f.loci_end = (_ptr(a) if a.size else None for a in keep)
            if not starts:
                f.loci_start = f.loci_end = None
        z = _Sizes()
        t2 = time.perf_counter()
        st = L.gq_bam_scan(h, C.byref(f), nt, C.byref(z))
        if st:
            raise ReadLoadError(_err(L))
        t3 = time.perf_counter()
        sizes = {"n": z.n_reads, "seq": z.seq_bytes, "cigar": z.cigar_len, "md": z.md_bytes, "name": z.name_bytes}
        arrs = {name: np.empty(sizes[kind], dt) for name, dt, kind in _READ_FIELDS}
        R = _Reads(*[_ptr(arrs[name]) for name, _, _ in _READ_FIELDS])
        st = L.gq_bam_fill(h, nt, C.byref(R))
        if st:
            raise ReadLoadError(_err(L))
        if timings is not None:
            timings.update(open_inflate_s=t1 - t0, scan_s=t3 - t2, fill_s=time.perf_counter() - t3, threads=nt)
        # samples: RG -> SM (else "default"), numbered by first appearance in file order
        rg_samples = _header_read_groups(text)
        rg_vals = [L.gq_bam_rg(h, k).decode("utf-8", "replace") for k in range(z.n_rg)]
        firsts = [(int(L.gq_bam_rg_first(h, k)), k) for k in range(-1, z.n_rg)]
        samples: List[str] = []
        sample_of_rg = np.zeros(z.n_rg + 1, np.int32)  # index k + 1
        for first, k in sorted(firsts):
            if first < 0:
                continue
            name = _sample_of(rg_vals[k] if k >= 0 else None, rg_samples)
            if name not in samples:
                samples.append(name)
            sample_of_rg[k + 1] = samples.index(name)
    finally:
        L.gq_bam_close(h)
    sample = sample_of_rg[arrs["rg"] + 1]
    return ReadSet(contig_names=contig_names, contig_lengths=contig_lengths, sample_names=samples,
                   contig=arrs["contig"], start=arrs["start"], end=arrs["end"], mapq=arrs["mapq"],
                   flags=arrs["flags"], sample=sample, seq_off=arrs["seq_off"], seq_len=arrs["seq_len"],
                   seq=arrs["seq"], qual=arrs["qual"], cigar_off=arrs["cigar_off"], n_cigar=arrs["n_cigar"],
                   cigar=arrs["cigar"], md_off=arrs["md_off"], md_len=arrs["md_len"], md=arrs["md"],
                   names=NamePool(arrs["names"], arrs["name_off"], arrs["name_len"]))


def md_events(cigar_off, n_cigar, cigar, md_off, md_len, md):
    """-> (n_md int32 (-1: no MD), n_mismatch uint16, md_ev uint32) for every read."""
    from .soa import MdParseError
    L = lib()
    n = int(np.asarray(md_len).shape[0])
    a = [np.ascontiguousarray(cigar_off, np.int64), np.ascontiguousarray(n_cigar, np.int32),
         np.ascontiguousarray(cigar, np.uint32), np.ascontiguousarray(md_off, np.int64),
         np.ascontiguousarray(md_len, np.int32), np.ascontiguousarray(md, np.uint8)]
    if a[5].size == 0:
        a[5] = np.zeros(1, np.uint8)
    if a[2].size == 0:
        a[2] = np.zeros(1, np.uint32)
    n_md = np.empty(n, np.int32)
    n_mm = np.empty(n, np.uint16)
    nt = n_threads()
    st = L.gq_md_count(n, *[_ptr(x) for x in a], nt, _ptr(n_md), _ptr(n_mm))
    if st:
        raise MdParseError(_err(L))
    lens = np.maximum(n_md, 0).astype(np.int64)
    off = np.zeros(n, np.int64)
    if n:
        off[1:] = np.cumsum(lens)[:-1]
    ev = np.empty(int(lens.sum()), np.uint32)
    st = L.gq_md_fill(n, *[_ptr(x) for x in a], _ptr(off), nt, _ptr(ev) if ev.size else 0)
    if st:
        raise MdParseError(_err(L))
    return n_md, n_mm, off, ev
