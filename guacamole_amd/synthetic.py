"""Synthetic coordinate-sorted reads with consistent CIGAR / MD.

The generator itself is native (csrc/gq_synth.cpp: counter-based RNG, threads,
deterministic for a seed whatever the thread count) and emits the device SoA of
soa.assemble with MD already as events, so whole-chromosome configurations never
materialise MD strings.  `SyntheticReads.to_read_set(sel)` builds the raw
ReadSet (MD strings) for any subset — the CPU oracle's input.

Model: reference i.i.d. GC 0.41; germline het SNVs 1e-3 (VAF 0.5), hom-alt 5e-4,
indels 1e-4 (1-10 bp); optional somatic SNVs at VAF U(0.1, 0.5) (tumor draw);
L = 150, Poisson starts, 50 % reverse, mapq 60 (2 % uniform 0..59), qualities on
2..41 (mean ~33.5), substitution errors with p = 10^(-q/10).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from .reads import OP_D, ReadSet
from .soa import assemble

SEED = 20261015
_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libgqsynth.so")
_lib = None


class _Params(C.Structure):
    _fields_ = [("length", C.c_int64), ("depth", C.c_double), ("read_len", C.c_int32), ("seed", C.c_uint64),
                ("read_seed", C.c_uint64), ("het", C.c_double), ("hom", C.c_double), ("indel", C.c_double),
                ("somatic", C.c_double), ("with_somatic", C.c_int32)]


class _Out(C.Structure):
    _fields_ = [("n_reads", C.c_int64)] + [(n, C.c_void_p) for n in (
        "start", "end", "pmax_end", "mapq", "flags", "sample", "seq_off", "seq_len", "cigar_off", "n_cigar", "md_off",
        "n_md", "n_mismatch")] + [("seq_bytes", C.c_int64), ("cigar_len", C.c_int64), ("md_len", C.c_int64)] + [
        (n, C.c_void_p) for n in ("seq", "qual", "cigar", "md_ev", "ref")] + [
        ("n_snv", C.c_int64), ("n_indel", C.c_int64), ("n_somatic", C.c_int64)]


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            from .build import build_synth
            build_synth()
        _lib = C.CDLL(_LIB)
        _lib.gq_synth_generate.restype = C.c_int
    return _lib


class _Owner:
    """Frees the native buffers when the last numpy view goes away."""

    def __init__(self, out: _Out):
        self.out = out

    def __del__(self):
        try:
            _load().gq_synth_free(C.byref(self.out))
        except Exception:
            pass


@dataclass
class SyntheticReads:
    contig_names: List[str]
    contig_lengths: List[int]
    arrays: Dict[str, np.ndarray]   # soa.assemble layout (views over native buffers)
    ref: np.ndarray                 # reference of contig 0
    stats: dict
    _owner: object = field(default=None, repr=False)

    @property
    def n(self) -> int:
        return int(self.arrays["start"].shape[0])

    def window(self, start: int, end: int) -> np.ndarray:
        """Indices of the reads overlapping [start, end)."""
        a = self.arrays
        hi = int(np.searchsorted(a["start"], end, side="left"))
        lo = int(np.searchsorted(a["pmax_end"], start, side="right"))
        idx = np.arange(lo, hi)
        return idx[a["end"][idx] > start]

    def write_bam(self, path: str, level: int = 6, dictionary=None, flags: int = 3, name_base: int = 0) -> None:
        """Coordinate-sorted BAM of every read (native streaming writer; read names
        r<name_base + index>, no RG).  dictionary: the header's [(contig, length)] (default: this
        set's contigs), every local contig named in it.  flags: 1 header, 2 EOF block, 4 append
        (a piece without header or EOF is whole BGZF blocks: pieces of one genome written by
        several processes concatenate into one BAM)."""
        L = _load()
        vp = C.c_void_p
        L.gq_synth_write_bam_ex.argtypes = [vp, C.c_char_p, C.c_int32, vp, vp, C.c_int32, vp, vp, C.c_int32,
                                            C.c_int32, C.c_int64]
        L.gq_synth_write_bam_ex.restype = C.c_int
        dictionary = list(dictionary) if dictionary is not None else list(zip(self.contig_names, self.contig_lengths))
        index = {c: i for i, (c, _) in enumerate(dictionary)}
        names = (C.c_char_p * max(1, len(dictionary)))(*[c.encode() for c, _ in dictionary])
        lens = np.array([int(n) for _, n in dictionary] or [0], np.int64)
        ids = np.array([index[c] for c in self.contig_names] or [0], np.int32)
        crb = np.ascontiguousarray(self.arrays["contig_read_begin"], np.int64)
        out, keep = self._out()
        rc = L.gq_synth_write_bam_ex(C.byref(out), os.fsencode(path), len(dictionary), C.cast(names, vp),
                                     lens.ctypes.data, len(self.contig_names), crb.ctypes.data, ids.ctypes.data,
                                     int(level), int(flags), int(name_base))
        del keep
        if rc != 0:
            raise OSError("gq_synth_write_bam_ex failed (%d) for %s" % (rc, path))

    def _out(self):
        """The native generator's output struct over this set's arrays (and what keeps them)."""
        if self._owner is not None:
            return self._owner.out, None
        a = self.arrays
        dt = dict(start=np.int32, end=np.int32, pmax_end=np.int32, mapq=np.uint8, flags=np.uint8, sample=np.uint8,
                  seq_off=np.int64, seq_len=np.int32, cigar_off=np.int64, n_cigar=np.int32, md_off=np.int64,
                  n_md=np.int32, n_mismatch=np.uint16, seq=np.uint8, qual=np.uint8, cigar=np.uint32, md_ev=np.uint32)
        keep = {k: np.ascontiguousarray(a[k], t) for k, t in dt.items()}
        ptr = {k: (v.ctypes.data if v.size else None) for k, v in keep.items()}
        out = _Out(self.n, *[ptr[k] for k in ("start", "end", "pmax_end", "mapq", "flags", "sample", "seq_off",
                                              "seq_len", "cigar_off", "n_cigar", "md_off", "n_md", "n_mismatch")],
                   int(keep["seq"].size), int(keep["cigar"].size), int(keep["md_ev"].size),
                   *[ptr[k] for k in ("seq", "qual", "cigar", "md_ev")], None, 0, 0, 0)
        return out, keep

    def to_read_set(self, sel: Optional[np.ndarray] = None) -> ReadSet:
        """Raw ReadSet (MD strings) for the reads `sel` (default: all) — oracle input."""
        a = self.arrays
        idx = np.arange(self.n) if sel is None else np.asarray(sel)
        seqs, quals, cigs, mds = [], [], [], []
        for i in idx:
            so, sl = int(a["seq_off"][i]), int(a["seq_len"][i])
            seqs.append(a["seq"][so:so + sl])
            quals.append(a["qual"][so:so + sl])
            co, nc = int(a["cigar_off"][i]), int(a["n_cigar"][i])
            cig = a["cigar"][co:co + nc]
            cigs.append(cig)
            mo, nm = int(a["md_off"][i]), int(a["n_md"][i])
            mds.append(md_string(cig, a["md_ev"][mo:mo + nm]))
        n = len(idx)
        seq_len = np.array([len(s) for s in seqs], dtype=np.int32)
        seq_off = np.zeros(n, np.int64)
        if n:
            seq_off[1:] = np.cumsum(seq_len)[:-1]
        n_cigar = np.array([len(c) for c in cigs], dtype=np.int32)
        cigar_off = np.zeros(n, np.int64)
        if n:
            cigar_off[1:] = np.cumsum(n_cigar)[:-1]
        md_b = [m.encode() for m in mds]
        md_len = np.array([len(m) for m in md_b], dtype=np.int32)
        md_off = np.zeros(n, np.int64)
        if n:
            md_off[1:] = np.cumsum(md_len)[:-1]
        cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
        return ReadSet(contig_names=list(self.contig_names), contig_lengths=list(self.contig_lengths),
                       sample_names=["synthetic"], contig=np.zeros(n, np.int32),
                       start=a["start"][idx].astype(np.int64), end=a["end"][idx].astype(np.int64),
                       mapq=a["mapq"][idx].copy(), flags=a["flags"][idx].copy(),
                       sample=a["sample"][idx].astype(np.int32), seq_off=seq_off, seq_len=seq_len,
                       seq=cat(seqs, np.uint8), qual=cat(quals, np.uint8), cigar_off=cigar_off, n_cigar=n_cigar,
                       cigar=cat(cigs, np.uint32), md_off=md_off, md_len=md_len,
                       md=np.frombuffer(b"".join(md_b), dtype=np.uint8).copy())


def md_string(cigar: np.ndarray, events: np.ndarray) -> str:
    """MD string for a read from its CIGAR and MD events (offset << 8 | ref base),
    walking events rather than bases."""
    ev = [(int(e) >> 8, chr(int(e) & 0xFF)) for e in events]
    out, run, ref, k = [], 0, 0, 0
    for c in cigar:
        op, ln = int(c) & 15, int(c) >> 4
        if op in (0, 7, 8):
            end = ref + ln
            while k < len(ev) and ev[k][0] < end:
                off, b = ev[k]
                run += off - ref
                out.append(str(run))
                out.append(b)
                run = 0
                ref = off + 1
                k += 1
            run += end - ref
            ref = end
        elif op == OP_D:
            out.append(str(run))
            dels = []
            for j in range(ln):
                if k < len(ev) and ev[k][0] == ref + j:
                    dels.append(ev[k][1])
                    k += 1
                else:
                    dels.append("N")
            out.append("^" + "".join(dels))
            run = 0
            ref += ln
        elif op == 3:
            ref += ln
    out.append(str(run))
    return "".join(out)


def generate_pieces(pieces, depth: float, seed: int = SEED, L: int = 150) -> SyntheticReads:
    """Reads for loci ranges of several contigs: pieces = [(contig, contig_length, start, end)],
    one range per contig, in the caller's contig order (local contig ids 0, 1, ...).  Each piece
    is generated as its own stretch [start - L, end) (seed + piece index) and shifted into place,
    so the reads straddling a piece's start are present (the halo of DistributedUtil.scala:
    584-597); the arrays are concatenated in contig order."""
    parts, names, lengths = [], [], []
    for k, (contig, clen, s, e) in enumerate(pieces):
        s0 = max(0, int(s) - L)
        g = generate(int(e) - s0, depth, seed=seed + 7919 * k, L=L, contig=contig)
        parts.append((g, s0))
        names.append(contig)
        lengths.append(int(clen))
    keys_pos = ("start", "end", "pmax_end")
    out: Dict[str, np.ndarray] = {}
    n_tot, seq_tot, cig_tot, md_tot = 0, 0, 0, 0
    begin = [0]
    cols = {k: [] for k in ("start", "end", "pmax_end", "mapq", "flags", "sample", "seq_off", "seq_len", "cigar_off",
                            "n_cigar", "md_off", "n_md", "n_mismatch", "seq", "qual", "cigar", "md_ev")}
    for g, s0 in parts:
        a = g.arrays
        for k in cols:
            v = a[k]
            if k in keys_pos:
                v = v + np.int32(s0)
            elif k == "seq_off":
                v = v + seq_tot
            elif k == "cigar_off":
                v = v + cig_tot
            elif k == "md_off":
                v = v + md_tot
            cols[k].append(np.asarray(v))
        n_tot += g.n
        seq_tot += int(a["seq"].shape[0])
        cig_tot += int(a["cigar"].shape[0])
        md_tot += int(a["md_ev"].shape[0])
        begin.append(n_tot)
    for k, v in cols.items():
        out[k] = np.concatenate(v) if v else np.zeros(0)
    out["contig_read_begin"] = np.array(begin, np.int64)
    out["n_contigs"] = np.int64(len(parts))
    out["n_samples"] = np.int64(1)
    stats = {k: sum(g.stats[k] for g, _ in parts) for k in ("n_snv", "n_indel", "n_somatic")}
    return SyntheticReads(names, lengths, out, np.zeros(0, np.uint8), stats, None)


def _gather_pool(pool: np.ndarray, off: np.ndarray, ln: np.ndarray):
    """(new pool, new offsets): the slices pool[off[i] : off[i] + ln[i]] packed in order."""
    ln = np.asarray(ln, np.int64)
    new_off = np.zeros(len(ln), np.int64)
    if len(ln) > 1:
        np.cumsum(ln[:-1], out=new_off[1:])
    tot = int(ln.sum())
    if tot == 0:
        return pool[:0].copy(), new_off
    src = np.repeat(np.asarray(off, np.int64) - new_off, ln) + np.arange(tot, dtype=np.int64)
    return pool[src], new_off


def write_bam_header(path: str, dictionary) -> None:
    """A BAM holding only the header (no BGZF EOF block): the first piece of a file whose reads
    other processes append (SyntheticReads.write_bam with flags 4)."""
    L = _load()
    out = _Out(0, *([None] * 13), 0, 0, 0, *([None] * 5), 0, 0, 0)
    vp = C.c_void_p
    L.gq_synth_write_bam_ex.argtypes = [vp, C.c_char_p, C.c_int32, vp, vp, C.c_int32, vp, vp, C.c_int32, C.c_int32,
                                        C.c_int64]
    L.gq_synth_write_bam_ex.restype = C.c_int
    names = (C.c_char_p * max(1, len(dictionary)))(*[c.encode() for c, _ in dictionary])
    lens = np.array([int(n) for _, n in dictionary] or [0], np.int64)
    crb = np.zeros(2, np.int64)
    ids = np.zeros(1, np.int32)
    rc = L.gq_synth_write_bam_ex(C.byref(out), os.fsencode(path), len(dictionary), C.cast(names, vp), lens.ctypes.data,
                                 1, crb.ctypes.data, ids.ctypes.data, 6, 1, 0)
    if rc != 0:
        raise OSError("gq_synth_write_bam_ex failed (%d) for %s" % (rc, path))


def subset_pieces(g: "SyntheticReads", pieces, mine, starts_in: bool = False) -> "SyntheticReads":
    """The reads of `g` (generate_pieces over `pieces`) overlapping the ranges `mine` (a sub-list
    of (contig, contig_length, start, end), one per contig, in `pieces`' contig order): what a
    task over those loci receives (DistributedUtil.scala:584-597), with local contig ids in
    `mine`'s order.  Reads straddling a cut are in both sides' subsets; with starts_in, only the
    reads starting inside the ranges are kept (each read in exactly one side's subset)."""
    a = g.arrays
    crb = np.asarray(a["contig_read_begin"], np.int64)
    names = [p[0] for p in pieces]
    sel, begin = [], [0]
    for contig, clen, s0, e0 in mine:
        k = names.index(contig)
        idx = np.arange(crb[k], crb[k + 1])
        keep = idx[(a["start"][idx] < e0) & ((a["start"][idx] >= s0) if starts_in else (a["end"][idx] > s0))]
        sel.append(keep)
        begin.append(begin[-1] + len(keep))
    idx = np.concatenate(sel) if sel else np.zeros(0, np.int64)
    out: Dict[str, np.ndarray] = {}
    for k in ("start", "end", "mapq", "flags", "sample", "seq_len", "n_cigar", "n_md", "n_mismatch"):
        out[k] = np.ascontiguousarray(a[k][idx])
    # prefix max of end within each contig block (SoA invariant)
    pm = out["end"].copy()
    for b0, b1 in zip(begin[:-1], begin[1:]):
        if b1 > b0:
            pm[b0:b1] = np.maximum.accumulate(pm[b0:b1])
    out["pmax_end"] = pm
    out["seq"], out["seq_off"] = _gather_pool(a["seq"], a["seq_off"][idx], a["seq_len"][idx])
    out["qual"], _ = _gather_pool(a["qual"], a["seq_off"][idx], a["seq_len"][idx])
    out["cigar"], out["cigar_off"] = _gather_pool(a["cigar"], a["cigar_off"][idx], a["n_cigar"][idx])
    out["md_ev"], out["md_off"] = _gather_pool(a["md_ev"], a["md_off"][idx], a["n_md"][idx])
    out["contig_read_begin"] = np.array(begin, np.int64)
    out["n_contigs"] = np.int64(len(mine))
    out["n_samples"] = np.int64(1)
    return SyntheticReads([m[0] for m in mine], [int(m[1]) for m in mine], out, np.zeros(0, np.uint8),
                          dict(g.stats), None)


def generate(length: int, depth: float, seed: int = SEED, L: int = 150, contig: str = "20",
             het: float = 1e-3, hom: float = 5e-4, indel_rate: float = 1e-4, somatic_rate: float = 0.0,
             tumor: bool = False, read_seed: Optional[int] = None) -> SyntheticReads:
    """Reads for one contig of `length` loci at mean `depth` (native generator)."""
    out = _Out()
    prm = _Params(int(length), float(depth), int(L), int(seed), int(seed if read_seed is None else read_seed),
                  float(het), float(hom), float(indel_rate), float(somatic_rate), int(bool(tumor)))
    rc = _load().gq_synth_generate(C.byref(prm), C.byref(out))
    if rc != 0:
        raise ValueError("synthetic generator rejected length=%d L=%d" % (length, L))
    owner = _Owner(out)
    n = out.n_reads

    def view(name, dt, count):
        if count == 0:
            return np.zeros(0, dt)
        ptr = C.cast(getattr(out, name), C.POINTER(np.ctypeslib.as_ctypes_type(dt)))
        return np.ctypeslib.as_array(ptr, shape=(count,))

    arrays = dict(contig_read_begin=np.array([0, n], np.int64), start=view("start", np.int32, n),
                  end=view("end", np.int32, n), pmax_end=view("pmax_end", np.int32, n),
                  mapq=view("mapq", np.uint8, n), flags=view("flags", np.uint8, n), sample=view("sample", np.uint8, n),
                  seq_off=view("seq_off", np.int64, n), seq_len=view("seq_len", np.int32, n),
                  cigar_off=view("cigar_off", np.int64, n), n_cigar=view("n_cigar", np.int32, n),
                  md_off=view("md_off", np.int64, n), n_md=view("n_md", np.int32, n),
                  n_mismatch=view("n_mismatch", np.uint16, n), seq=view("seq", np.uint8, out.seq_bytes),
                  qual=view("qual", np.uint8, out.seq_bytes), cigar=view("cigar", np.uint32, out.cigar_len),
                  md_ev=view("md_ev", np.uint32, out.md_len), n_contigs=np.int64(1), n_samples=np.int64(1))
    return SyntheticReads([contig], [int(length)], arrays, view("ref", np.uint8, int(length)),
                          dict(n_snv=out.n_snv, n_indel=out.n_indel, n_somatic=out.n_somatic), owner)
