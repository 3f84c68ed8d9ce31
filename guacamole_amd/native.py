"""ctypes binding of libgqpileup.so (include/gqpileup.h).

The HIP library is the only compute path: if it is missing or the GPU cannot be
opened, every entry point raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libgqpileup.so")
_lib = None

GT_NAMES = {0: "Ref", 1: "Alt", 2: "OtherAlt", 3: "NoCall"}
FLAG_AMBIGUOUS_REF = 1
FLAG_TIE = 2
FLAG_KNIFE_EDGE = 4


class GQError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__("gqpileup error %d: %s" % (code, msg))
        self.code = code


class gq_reads(C.Structure):
    _fields_ = [("n_reads", C.c_int64), ("n_contigs", C.c_int32), ("n_samples", C.c_int32)] + [
        (n, C.c_void_p) for n in ("contig_read_begin", "start", "end", "pmax_end", "mapq", "flags", "sample",
                                  "seq_off", "seq_len", "cigar_off", "n_cigar", "md_off", "n_md", "n_mismatch")] + [
        ("seq_bytes", C.c_int64), ("cigar_len", C.c_int64), ("md_len", C.c_int64)] + [
        (n, C.c_void_p) for n in ("seq", "qual", "cigar", "md_ev", "sample_hash")]


class gq_loci(C.Structure):
    _fields_ = [("n_ranges", C.c_int64), ("contig", C.c_void_p), ("start", C.c_void_p), ("end", C.c_void_p),
                ("task", C.c_void_p)]


class gq_germline_params(C.Structure):
    _fields_ = [("threshold", C.c_int32), ("emit_ref", C.c_int32), ("emit_no_call", C.c_int32)]


class gq_calls(C.Structure):
    _fields_ = [("n", C.c_int64), ("contig", C.POINTER(C.c_int32)), ("pos", C.POINTER(C.c_int64)),
                ("sample", C.POINTER(C.c_uint8)), ("gt0", C.POINTER(C.c_uint8)), ("gt1", C.POINTER(C.c_uint8)),
                ("flags", C.POINTER(C.c_uint8)), ("ref_off", C.POINTER(C.c_int64)), ("ref_len", C.POINTER(C.c_int32)),
                ("alt_off", C.POINTER(C.c_int64)), ("alt_len", C.POINTER(C.c_int32)),
                ("allele_pool", C.POINTER(C.c_uint8)), ("pool_len", C.c_int64), ("visited_loci", C.c_int64),
                ("complex_loci", C.c_int64), ("ambiguous_loci", C.c_int64), ("tie_loci", C.c_int64),
                ("block_", C.c_void_p)]


class gq_calls_device(C.Structure):
    _fields_ = [("calls", gq_calls), ("image", C.c_void_p), ("image_bytes", C.c_int64)]


class gq_allele_counts(C.Structure):
    _fields_ = [("n", C.c_int64), ("contig", C.POINTER(C.c_int32)), ("pos", C.POINTER(C.c_int64)),
                ("sample", C.POINTER(C.c_int32)), ("count", C.POINTER(C.c_int32)),
                ("ref_off", C.POINTER(C.c_int64)), ("ref_len", C.POINTER(C.c_int32)),
                ("alt_off", C.POINTER(C.c_int64)), ("alt_len", C.POINTER(C.c_int32)),
                ("allele_pool", C.c_void_p), ("pool_len", C.c_int64), ("flags", C.POINTER(C.c_uint8))]


class gq_germline_std_params(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("min_mapq", "min_read_depth", "max_read_depth", "min_alternate_read_depth",
                                         "min_likelihood", "apply_filters")]


GERMLINE_STD_DEFAULTS = dict(min_mapq=1, min_read_depth=0, max_read_depth=2 ** 31 - 1, min_alternate_read_depth=0,
                             min_likelihood=0, apply_filters=1)


class gq_vaf_params(C.Structure):
    _fields_ = [("bins", C.c_int32), ("min_read_depth", C.c_int32), ("min_vaf", C.c_int32)]


class gq_vaf_hist(C.Structure):
    _fields_ = [("counts", C.c_int64 * 101), ("variant_loci", C.c_int64), ("visited_loci", C.c_int64)]


class gq_counts(C.Structure):
    _fields_ = [("n_loci", C.c_int64), ("depth", C.POINTER(C.c_int32)), ("pos_depth", C.POINTER(C.c_int32)),
                ("base_counts", C.POINTER(C.c_int32)), ("indel_counts", C.POINTER(C.c_int32)),
                ("ref_depth", C.POINTER(C.c_int32)), ("ref_base", C.POINTER(C.c_uint8)),
                ("ambiguous", C.POINTER(C.c_uint8))]


class gq_timings(C.Structure):
    _fields_ = [("plan_ms", C.c_float), ("pileup_ms", C.c_float), ("complex_ms", C.c_float),
                ("finalize_ms", C.c_float), ("total_ms", C.c_float), ("pileup_launches", C.c_int64),
                ("tiles", C.c_int64), ("host_ms", C.c_float), ("marshal_ms", C.c_float),
                ("walk_ms", C.c_float), ("walk_tiles", C.c_int64), ("order_loci", C.c_int64),
                ("deep_loci", C.c_int64), ("deep_max", C.c_int64), ("call_ms", C.c_float), ("deep_ms", C.c_float),
                ("front_ms", C.c_float)]


class gq_reads_info(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("n_reads", "seq_bytes", "proj_bytes", "pev_count", "proj_reads", "n_rows")] + [
        ("h2d_ms", C.c_float), ("derive_ms", C.c_float), ("cigar_len", C.c_int64), ("md_len", C.c_int64),
        ("n_contigs", C.c_int32), ("n_samples", C.c_int32), ("proj_ms", C.c_float), ("projected", C.c_int32),
        ("fill_ms", C.c_float), ("proj_dev_ms", C.c_float), ("derive_dev_ms", C.c_float)]


class gq_somatic_params(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "odds", "min_mapq", "filter_multi_allelic", "max_read_depth", "min_tumor_read_depth",
        "max_tumor_read_depth", "min_normal_read_depth", "min_tumor_alternate_read_depth", "min_lod",
        "min_likelihood", "min_vaf", "min_average_mapping_quality", "min_average_base_quality",
        "max_median_mismatches", "apply_filters")]


class gq_evidence(C.Structure):
    _fields_ = [("likelihood", C.c_double), ("read_depth", C.c_int32), ("allele_read_depth", C.c_int32),
                ("forward_depth", C.c_int32), ("allele_forward_depth", C.c_int32), ("mean_mq", C.c_double),
                ("median_mq", C.c_double), ("mean_bq", C.c_double), ("median_bq", C.c_double),
                ("median_mismatches", C.c_double)]


# SomaticStandard.Arguments defaults (commands/SomaticStandardCaller.scala:40-64 and
# filters/SomaticGenotypeFilter.scala:31-56); apply_filters 1 = the driver's filter chain.
SOMATIC_DEFAULTS = dict(odds=20, min_mapq=1, filter_multi_allelic=0, max_read_depth=2 ** 31 - 1,
                        min_tumor_read_depth=0, max_tumor_read_depth=2 ** 31 - 1, min_normal_read_depth=0,
                        min_tumor_alternate_read_depth=0, min_lod=0, min_likelihood=0, min_vaf=0,
                        min_average_mapping_quality=0, min_average_base_quality=0,
                        max_median_mismatches=2 ** 31 - 1, apply_filters=1)

_EVIDENCE_DTYPE = np.dtype([("likelihood", np.float64), ("read_depth", np.int32), ("allele_read_depth", np.int32),
                            ("forward_depth", np.int32), ("allele_forward_depth", np.int32), ("mean_mq", np.float64),
                            ("median_mq", np.float64), ("mean_bq", np.float64), ("median_bq", np.float64),
                            ("median_mismatches", np.float64)])

EVIDENCE_FIELDS = ("likelihood", "read_depth", "allele_read_depth", "forward_depth", "allele_forward_depth",
                   "mean_mq", "median_mq", "mean_bq", "median_bq", "median_mismatches")


class gq_somatic_calls(C.Structure):
    _fields_ = [("n", C.c_int64), ("contig", C.POINTER(C.c_int32)), ("pos", C.POINTER(C.c_int64)),
                ("sample", C.POINTER(C.c_uint8)), ("ref_off", C.POINTER(C.c_int64)), ("ref_len", C.POINTER(C.c_int32)),
                ("alt_off", C.POINTER(C.c_int64)), ("alt_len", C.POINTER(C.c_int32)),
                ("allele_pool", C.POINTER(C.c_uint8)), ("pool_len", C.c_int64), ("log_odds", C.POINTER(C.c_double)),
                ("gq", C.POINTER(C.c_int32)), ("tumor", C.POINTER(gq_evidence)), ("normal", C.POINTER(gq_evidence)),
                ("flags", C.POINTER(C.c_uint8)), ("visited_loci", C.c_int64), ("candidate_loci", C.c_int64),
                ("block_", C.c_void_p)]


EXPORTED = ("gq_version", "gq_last_error", "gq_open", "gq_close", "gq_get_timings", "gq_set_tile", "gq_reads_upload",
            "gq_reads_wrap_device", "gq_reads_free", "gq_reads_rederive", "gq_germline_threshold", "gq_germline_threshold_device",
            "gq_free_calls", "gq_pileup_counts",
            "gq_free_counts", "gq_somatic_standard", "gq_free_somatic", "gq_reads_get_info", "gq_reference_upload",
            "gq_reference_free", "gq_somatic_standard_ref", "gq_variant_support", "gq_free_allele_counts",
            "gq_vaf_histogram", "gq_germline_standard", "gq_bam_dev_open", "gq_bam_dev_close", "gq_bam_dev_header_text",
            "gq_bam_dev_n_contigs", "gq_bam_dev_contig_name", "gq_bam_dev_contig_length", "gq_bam_dev_scan",
            "gq_bam_dev_reads", "gq_reads_positions", "gq_reads_contig_begin", "gq_reads_download", "gq_bam_dev_map",
            "gq_bam_dev_load", "gq_bam_dev_map_ex", "gq_bam_dev_plan", "gq_bam_dev_plan_segments",
            "gq_write_vcf_germline")


def lib():
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # GQ_LIB: an alternative in-tree build of the same library (kernel A/B experiments)
        path = os.environ.get("GQ_LIB", LIB_PATH)
        if not os.path.exists(path):
            raise RuntimeError("libgqpileup.so not built (%s); run __graft_entry__.build()" % path)
        L = C.CDLL(path)
        L.gq_version.restype = C.c_char_p
        L.gq_last_error.restype = C.c_char_p
        for f in ("gq_open", "gq_get_timings", "gq_set_tile", "gq_reads_upload", "gq_reads_wrap_device", "gq_reads_get_info",
                  "gq_reads_rederive",
                  "gq_germline_threshold", "gq_germline_threshold_device", "gq_pileup_counts", "gq_somatic_standard",
                  "gq_reference_upload", "gq_somatic_standard_ref", "gq_variant_support", "gq_vaf_histogram",
                  "gq_germline_standard"):
            getattr(L, f).restype = C.c_int
        L.gq_germline_threshold.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(gq_loci), C.POINTER(gq_germline_params),
                                            C.POINTER(C.POINTER(gq_calls))]
        L.gq_germline_threshold_device.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(gq_loci),
                                                   C.POINTER(gq_germline_params), C.POINTER(gq_calls_device)]
        L.gq_pileup_counts.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(gq_loci), C.POINTER(C.POINTER(gq_counts))]
        L.gq_somatic_standard.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(gq_loci),
                                          C.POINTER(gq_somatic_params), C.POINTER(C.POINTER(gq_somatic_calls))]
        L.gq_somatic_standard_ref.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(gq_loci), C.c_void_p,
                                              C.POINTER(gq_somatic_params), C.POINTER(C.POINTER(gq_somatic_calls))]
        L.gq_reference_upload.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p), C.c_void_p,
                                          C.POINTER(C.c_void_p)]
        L.gq_reference_free.argtypes = [C.c_void_p]
        L.gq_variant_support.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(gq_loci),
                                         C.POINTER(C.POINTER(gq_allele_counts))]
        L.gq_free_allele_counts.argtypes = [C.POINTER(gq_allele_counts)]
        L.gq_germline_standard.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(gq_loci), C.POINTER(gq_germline_std_params),
                                           C.POINTER(C.POINTER(gq_somatic_calls))]
        L.gq_vaf_histogram.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(gq_loci), C.POINTER(gq_vaf_params),
                                       C.POINTER(gq_vaf_hist)]
        L.gq_free_calls.argtypes = [C.POINTER(gq_calls)]
        L.gq_free_counts.argtypes = [C.POINTER(gq_counts)]
        L.gq_free_somatic.argtypes = [C.POINTER(gq_somatic_calls)]
        L.gq_reads_free.argtypes = [C.c_void_p]
        L.gq_reads_rederive.argtypes = [C.c_void_p, C.c_void_p]
        L.gq_close.argtypes = [C.c_void_p]
        vp = C.c_void_p
        for f in ("gq_bam_dev_open", "gq_bam_dev_scan", "gq_bam_dev_reads", "gq_reads_positions", "gq_reads_contig_begin",
                  "gq_reads_download"):
            getattr(L, f).restype = C.c_int
        L.gq_bam_dev_open.argtypes = [vp, C.c_char_p, C.POINTER(vp)]
        L.gq_bam_dev_map.argtypes = [C.c_char_p, C.POINTER(vp)]
        L.gq_bam_dev_map.restype = C.c_int
        L.gq_bam_dev_map_ex.argtypes = [C.c_char_p, C.c_int32, C.POINTER(vp)]
        L.gq_bam_dev_map_ex.restype = C.c_int
        L.gq_bam_dev_plan.argtypes = [vp, vp, vp, vp, C.c_int64, C.c_char_p, vp]
        L.gq_bam_dev_plan.restype = C.c_int
        L.gq_bam_dev_plan_segments.argtypes = [vp, vp, vp, vp, vp]
        L.gq_bam_dev_plan_segments.restype = C.c_int
        L.gq_write_vcf_germline.argtypes = [C.c_char_p, C.c_char_p, C.c_int64] + [vp] * 9 + [C.c_int32,
                                                                                           C.POINTER(C.c_char_p)]
        L.gq_write_vcf_germline.restype = C.c_int
        L.gq_bam_dev_load.argtypes = [vp, vp]
        L.gq_bam_dev_load.restype = C.c_int
        L.gq_bam_dev_close.argtypes = [vp]
        L.gq_bam_dev_close.restype = None
        L.gq_bam_dev_header_text.argtypes = [vp]
        L.gq_bam_dev_header_text.restype = C.c_char_p
        L.gq_bam_dev_n_contigs.argtypes = [vp]
        L.gq_bam_dev_n_contigs.restype = C.c_int32
        L.gq_bam_dev_contig_name.argtypes = [vp, C.c_int32]
        L.gq_bam_dev_contig_name.restype = C.c_char_p
        L.gq_bam_dev_contig_length.argtypes = [vp, C.c_int32]
        L.gq_bam_dev_contig_length.restype = C.c_int64
        L.gq_bam_dev_scan.argtypes = [vp, vp, vp, vp]
        L.gq_bam_dev_reads.argtypes = [vp, vp, C.c_int32, vp, C.POINTER(vp), C.POINTER(C.c_float)]
        L.gq_reads_positions.argtypes = [vp, vp, vp]
        L.gq_reads_contig_begin.argtypes = [vp, vp]
        L.gq_reads_download.argtypes = [vp, C.POINTER(gq_reads)]
        _lib = L
    return _lib


def write_vcf_germline(path: str, header: str, calls: "GermlineCalls", contig_names: Sequence[str]) -> None:
    """gq_write_vcf_germline: the header, then one line per record of `calls` (one sample)."""
    a = calls.a
    n = len(calls)
    cols = {k: np.ascontiguousarray(a[k]) for k in ("contig", "pos", "gt0", "gt1", "ref_off", "ref_len", "alt_off",
                                                   "alt_len")}
    names = (C.c_char_p * max(1, len(contig_names)))(*[x.encode() for x in contig_names])
    pool = np.frombuffer(calls.pool, np.uint8) if calls.pool else np.zeros(1, np.uint8)
    _check(lib().gq_write_vcf_germline(path.encode(), header.encode(), n, *[_ptr(cols[k]) or None for k in cols],
                                       pool.ctypes.data, len(contig_names), names))


def _check(rc: int) -> None:
    if rc != 0:
        raise GQError(rc, lib().gq_last_error().decode())


def _ptr(a) -> int:
    if isinstance(a, np.ndarray):
        return a.ctypes.data if a.size else 0
    return int(a.data_ptr())  # torch tensor already in device memory


def make_gq_reads(arrs: Dict[str, object]) -> Tuple[gq_reads, list]:
    """gq_reads over numpy (host) or torch (device) arrays from soa.pack/assemble."""
    keep = [arrs[k] for k in arrs]
    n = int(arrs["start"].shape[0])
    s = gq_reads(n, int(arrs["n_contigs"]), int(arrs["n_samples"]),
                 *[_ptr(arrs[k]) for k in ("contig_read_begin", "start", "end", "pmax_end", "mapq", "flags",
                                           "sample", "seq_off", "seq_len", "cigar_off", "n_cigar", "md_off", "n_md",
                                           "n_mismatch")],
                 int(arrs["seq"].shape[0]), int(arrs["cigar"].shape[0]), int(arrs["md_ev"].shape[0]),
                 *[_ptr(arrs[k]) for k in ("seq", "qual", "cigar", "md_ev")],
                 _ptr(arrs["sample_hash"]) if "sample_hash" in arrs else None)
    return s, keep


def make_gq_loci(contig, start, end, task) -> Tuple[gq_loci, list]:
    keep = [np.ascontiguousarray(contig, np.int32), np.ascontiguousarray(start, np.int64),
            np.ascontiguousarray(end, np.int64), np.ascontiguousarray(task, np.int64)]
    return gq_loci(len(keep[0]), *[_ptr(a) for a in keep]), keep


class Context:
    """One gq_ctx per GPU (gq_open / gq_close)."""

    def __init__(self, device: int = 0):
        from . import _early
        h = _early.take(device)  # the CLI's context, opened while the interpreter imported
        self.h = C.c_void_p()
        if h is not None and h.value:
            lib()
            self.h = h
        else:
            _check(lib().gq_open(int(device), C.byref(self.h)))
        self.device = device
        # germline calls reuse the context's result image: a DeviceCalls is valid until the
        # next germline call on this context (gqpileup.h, gq_calls_device)
        self.image_epoch = 0

    def close(self) -> None:
        if self.h:
            lib().gq_close(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_tile(self, t: int) -> None:
        _check(lib().gq_set_tile(self.h, int(t)))

    def timings(self) -> Dict[str, float]:
        t = gq_timings()
        _check(lib().gq_get_timings(self.h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in gq_timings._fields_}

    def proj_stats(self, reads: "DeviceReads") -> Dict[str, int]:
        """Sizes of a resident read set and of its upload-time projection (gq_reads_get_info)."""
        info = gq_reads_info()
        _check(lib().gq_reads_get_info(reads.h, C.byref(info)))
        return {k: (float if t is C.c_float else int)(getattr(info, k)) for k, t in gq_reads_info._fields_}

    def upload(self, arrs: Dict[str, object]) -> "DeviceReads":
        s, keep = make_gq_reads(arrs)
        h = C.c_void_p()
        _check(lib().gq_reads_upload(self.h, C.byref(s), C.byref(h)))
        return DeviceReads(self, h, None)

    def rederive(self, reads: "DeviceReads") -> None:
        """gq_reads_rederive: every derived structure of the resident read set dropped and the
        upload-time part derived again (the projection on the next call that reads it)."""
        _check(lib().gq_reads_rederive(self.h, reads.h))

    def wrap_device(self, arrs: Dict[str, object]) -> "DeviceReads":
        s, keep = make_gq_reads(arrs)
        h = C.c_void_p()
        _check(lib().gq_reads_wrap_device(self.h, C.byref(s), C.byref(h)))
        return DeviceReads(self, h, keep)

    def germline_threshold(self, reads: "DeviceReads", loci, threshold: int = 8, emit_ref: bool = False,
                           emit_no_call: bool = False) -> "GermlineCalls":
        L, keep = make_gq_loci(*loci)
        p = gq_germline_params(int(threshold), int(bool(emit_ref)), int(bool(emit_no_call)))
        out = C.POINTER(gq_calls)()
        self.image_epoch += 1
        _check(lib().gq_germline_threshold(self.h, reads.h, C.byref(L), C.byref(p), C.byref(out)))
        return GermlineCalls.from_result(out)

    def germline_threshold_device(self, reads: "DeviceReads", loci, threshold: int = 8, emit_ref: bool = False,
                                  emit_no_call: bool = False) -> "DeviceCalls":
        """gq_germline_threshold_device: the records stay in HBM (valid until the next call)."""
        L, keep = make_gq_loci(*loci)
        p = gq_germline_params(int(threshold), int(bool(emit_ref)), int(bool(emit_no_call)))
        out = gq_calls_device()
        self.image_epoch += 1
        _check(lib().gq_germline_threshold_device(self.h, reads.h, C.byref(L), C.byref(p), C.byref(out)))
        return DeviceCalls(out, self)

    def upload_reference(self, contigs: List[Optional[np.ndarray]]) -> "DeviceReference":
        """A reference genome in HBM (gq_reference_upload): contigs[k] = the unmasked bases of
        contig k of the read sets' contig list (None where the reference lacks it)."""
        keep = [None if a is None else np.ascontiguousarray(a, np.uint8) for a in contigs]
        n = len(keep)
        ptrs = (C.c_void_p * max(n, 1))(*[None if a is None else a.ctypes.data for a in keep])
        lens = np.array([-1 if a is None else len(a) for a in keep] or [0], np.int64)
        h = C.c_void_p()
        _check(lib().gq_reference_upload(self.h, n, C.cast(ptrs, C.POINTER(C.c_void_p)), lens.ctypes.data,
                                         C.byref(h)))
        return DeviceReference(h)

    def somatic_standard(self, tumor: "DeviceReads", normal: "DeviceReads", loci, reference=None,
                         **params) -> "SomaticCalls":
        """somatic-standard over the loci ranges (gq_somatic_standard, or gq_somatic_standard_ref
        with a DeviceReference).  params: the gq_somatic_params fields; defaults SOMATIC_DEFAULTS
        (the CLI defaults)."""
        L, keep = make_gq_loci(*loci)
        p = dict(SOMATIC_DEFAULTS)
        p.update(params)
        ps = gq_somatic_params(**{k: int(v) for k, v in p.items()})
        out = C.POINTER(gq_somatic_calls)()
        if reference is None:
            _check(lib().gq_somatic_standard(self.h, tumor.h, normal.h, C.byref(L), C.byref(ps), C.byref(out)))
        else:
            _check(lib().gq_somatic_standard_ref(self.h, tumor.h, normal.h, C.byref(L), reference.h, C.byref(ps),
                                                 C.byref(out)))
        return SomaticCalls.from_result(out)

    def variant_support(self, reads: "DeviceReads", loci) -> List[tuple]:
        """gq_variant_support: rows (sample index, contig index, locus, ref, alt, count, flags)."""
        L, keep = make_gq_loci(*loci)
        out = C.POINTER(gq_allele_counts)()
        _check(lib().gq_variant_support(self.h, reads.h, C.byref(L), C.byref(out)))
        try:
            c = out.contents
            n = c.n
            if n == 0:
                return []
            arr = lambda p: np.ctypeslib.as_array(p, shape=(n,)).copy()
            pool = C.string_at(c.allele_pool, c.pool_len) if c.pool_len else b""
            contig, pos, smp, cnt = arr(c.contig), arr(c.pos), arr(c.sample), arr(c.count)
            ro, rl, ao, al, fl = arr(c.ref_off), arr(c.ref_len), arr(c.alt_off), arr(c.alt_len), arr(c.flags)
            return [(int(smp[i]), int(contig[i]), int(pos[i]), pool[ro[i]:ro[i] + rl[i]].decode("latin-1"),
                     pool[ao[i]:ao[i] + al[i]].decode("latin-1"), int(cnt[i]), int(fl[i])) for i in range(n)]
        finally:
            lib().gq_free_allele_counts(out)

    def germline_standard(self, reads: "DeviceReads", loci, **params) -> "SomaticCalls":
        """germline-standard (gq_germline_standard): CalledAllele rows in the SomaticCalls layout
        (tumor = the allele's evidence, sample = its sample slot).  params: the
        gq_germline_std_params fields; defaults GERMLINE_STD_DEFAULTS (the CLI defaults)."""
        L, keep = make_gq_loci(*loci)
        p = dict(GERMLINE_STD_DEFAULTS)
        p.update(params)
        ps = gq_germline_std_params(**{k: int(v) for k, v in p.items()})
        out = C.POINTER(gq_somatic_calls)()
        _check(lib().gq_germline_standard(self.h, reads.h, C.byref(L), C.byref(ps), C.byref(out)))
        return SomaticCalls.from_result(out)

    def vaf_histogram(self, reads: "DeviceReads", loci, bins: int = 20, min_read_depth: int = 0,
                      min_vaf: int = 0) -> Dict[str, object]:
        """gq_vaf_histogram: {bin start: loci} (non-empty bins), plus variant / visited locus counts."""
        L, keep = make_gq_loci(*loci)
        prm = gq_vaf_params(int(bins), int(min_read_depth), int(min_vaf))
        h = gq_vaf_hist()
        _check(lib().gq_vaf_histogram(self.h, reads.h, C.byref(L), C.byref(prm), C.byref(h)))
        return dict(histogram={b: int(h.counts[b]) for b in range(101) if h.counts[b]},
                    variant_loci=int(h.variant_loci), visited_loci=int(h.visited_loci))

    def pileup_counts(self, reads: "DeviceReads", loci) -> Dict[str, np.ndarray]:
        L, keep = make_gq_loci(*loci)
        out = C.POINTER(gq_counts)()
        _check(lib().gq_pileup_counts(self.h, reads.h, C.byref(L), C.byref(out)))
        try:
            c = out.contents
            n = c.n_loci

            def arr(p, k=1):
                return np.ctypeslib.as_array(p, shape=(n * k,)).copy() if n else np.zeros(0)

            return dict(depth=arr(c.depth), pos_depth=arr(c.pos_depth), base_counts=arr(c.base_counts, 6).reshape(-1, 6),
                        indel_counts=arr(c.indel_counts, 4).reshape(-1, 4), ref_depth=arr(c.ref_depth),
                        ref_base=arr(c.ref_base), ambiguous=arr(c.ambiguous))
        finally:
            lib().gq_free_counts(out)


class DeviceReference:
    """A gq_reference handle (freed with the object)."""

    def __init__(self, h):
        self.h = h

    def free(self) -> None:
        if self.h:
            lib().gq_reference_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceReads:
    def __init__(self, ctx: Context, h, keep):
        self.ctx, self.h, self.keep = ctx, h, keep

    def free(self) -> None:
        if self.h:
            lib().gq_reads_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceCalls:
    """Germline records left in HBM by gq_germline_threshold_device: one contiguous device image
    (``image`` address, ``image_bytes``), its array offsets, and the run counters."""

    NAMES = ("contig", "pos", "sample", "gt0", "gt1", "flags", "ref_off", "ref_len", "alt_off", "alt_len")

    def __init__(self, d: gq_calls_device, ctx: Optional["Context"] = None):
        self.ctx, self.epoch = ctx, (ctx.image_epoch if ctx is not None else None)
        c = d.calls
        self.n, self.image, self.image_bytes = int(c.n), int(d.image or 0), int(d.image_bytes)
        self.pool_len = int(c.pool_len)
        self.visited_loci, self.complex_loci = int(c.visited_loci), int(c.complex_loci)
        self.ambiguous_loci, self.tie_loci = int(c.ambiguous_loci), int(c.tie_loci)
        base = self.image
        self.offsets = {k: (C.cast(getattr(c, k), C.c_void_p).value or base) - base for k in self.NAMES}
        self.offsets["pool"] = (C.cast(c.allele_pool, C.c_void_p).value or base) - base
        self._types = {k: np.dtype(getattr(c, k)._type_) for k in self.NAMES}

    def __len__(self) -> int:
        return self.n

    def check_current(self) -> None:
        """Raise if a later germline call on the context has replaced the image."""
        if self.ctx is not None and self.ctx.image_epoch != self.epoch:
            raise GQError(7, "DeviceCalls used after a later germline call on its context (the result image "
                             "is reused; copy it first with to_host())")

    def to_host(self) -> "GermlineCalls":
        """Copy the image over PCIe (hipMemcpy) and view it as GermlineCalls (test / export)."""
        self.check_current()
        host = np.zeros(max(self.image_bytes, 1), np.uint8)
        if self.image_bytes:
            hip = C.CDLL("libamdhip64.so.7")  # by SONAME: the HIP runtime already loaded in this process
            hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
            rc = hip.hipMemcpy(host.ctypes.data, C.c_void_p(self.image), self.image_bytes, 2)  # DeviceToHost
            if rc != 0:
                raise GQError(8, "hipMemcpy of the result image failed (%d)" % rc)
        a = {k: host[self.offsets[k]:self.offsets[k] + self.n * self._types[k].itemsize].view(self._types[k])
             for k in self.NAMES}
        pool = host[self.offsets["pool"]:self.offsets["pool"] + self.pool_len].tobytes()
        return GermlineCalls(a, pool, self.visited_loci, self.complex_loci, self.ambiguous_loci, self.tie_loci)


class GermlineCalls:
    """Germline genotype records in output order (numpy arrays; allele strings on demand)."""

    def __init__(self, arrays: Dict[str, np.ndarray], pool: bytes, visited, complex_loci, ambiguous, ties):
        self.a = arrays
        self.pool = pool
        self.visited_loci, self.complex_loci, self.ambiguous_loci, self.tie_loci = visited, complex_loci, ambiguous, ties

    @staticmethod
    def from_result(ptr) -> "GermlineCalls":
        """Zero-copy numpy views over the result block (gq_calls.block_).  The views keep
        a ctypes buffer object alive whose finalizer calls gq_free_calls."""
        import weakref

        c = ptr.contents
        n = c.n
        pool = C.string_at(c.allele_pool, c.pool_len) if c.pool_len else b""
        names = ("contig", "pos", "sample", "gt0", "gt1", "flags", "ref_off", "ref_len", "alt_off", "alt_len")
        if n == 0 or not c.block_:
            a = {k: np.zeros(0, np.dtype(getattr(c, k)._type_)) for k in names}
            out = GermlineCalls(a, pool, c.visited_loci, c.complex_loci, c.ambiguous_loci, c.tie_loci)
            lib().gq_free_calls(ptr)
            return out
        ends = [C.cast(getattr(c, k), C.c_void_p).value + n * C.sizeof(getattr(c, k)._type_) for k in names]
        size = max(ends) - c.block_
        buf = (C.c_uint8 * size).from_address(c.block_)
        weakref.finalize(buf, lib().gq_free_calls, ptr)
        a = {}
        for k in names:
            t = getattr(c, k)._type_
            a[k] = np.frombuffer(buf, dtype=np.dtype(t), count=n, offset=C.cast(getattr(c, k), C.c_void_p).value - c.block_)
        return GermlineCalls(a, pool, c.visited_loci, c.complex_loci, c.ambiguous_loci, c.tie_loci)

    IMAGE_FIELDS = (("contig", np.int32), ("pos", np.int64), ("ref_off", np.int64), ("alt_off", np.int64),
                    ("ref_len", np.int32), ("alt_len", np.int32), ("sample", np.uint8), ("gt0", np.uint8),
                    ("gt1", np.uint8), ("flags", np.uint8))

    @staticmethod
    def from_image(img: np.ndarray, n: int, visited=0, complex_loci=0, ambiguous=0, ties=0) -> "GermlineCalls":
        """Decode a result image of n records (gqpileup.h, gq_calls_device: int64 pool_len at byte
        0, then the arrays in IMAGE_FIELDS order and the pool, each on a 64-byte boundary from 64)."""
        img = np.asarray(img, np.uint8)
        al = lambda x: (x + 63) & ~63
        off, a = 64, {}
        for k, dt in GermlineCalls.IMAGE_FIELDS:
            nb = n * np.dtype(dt).itemsize
            a[k] = img[off:off + nb].view(dt).copy() if n else np.zeros(0, dt)
            off = al(off + nb)
        pool_len = int(img[:8].view(np.int64)[0]) if n else 0
        return GermlineCalls(a, img[off:off + pool_len].tobytes(), visited, complex_loci, ambiguous, ties)

    def __len__(self) -> int:
        return int(self.a["pos"].shape[0])

    def ref(self, i: int) -> str:
        o = int(self.a["ref_off"][i])
        return self.pool[o:o + int(self.a["ref_len"][i])].decode("latin-1")

    def alt(self, i: int) -> str:
        o = int(self.a["alt_off"][i])
        return self.pool[o:o + int(self.a["alt_len"][i])].decode("latin-1")

    def tuples(self, contig_names: Sequence[str]) -> List[tuple]:
        """(contig, locus, sample, (gt0, gt1), ref, alt, flags) — same shape as the oracle's rows."""
        a = self.a
        pool = self.pool
        cols = [a[k].tolist() for k in ("contig", "pos", "sample", "gt0", "gt1", "ref_off", "ref_len", "alt_off",
                                         "alt_len", "flags")]
        return [(contig_names[c], p, s, (GT_NAMES[g0], GT_NAMES[g1]), pool[ro:ro + rl].decode("latin-1"),
                 pool[ao:ao + al].decode("latin-1"), f) for c, p, s, g0, g1, ro, rl, ao, al, f in zip(*cols)]


class SomaticCalls:
    """CalledSomaticAllele records in output order: numpy columns copied out of the library's
    result (one copy per column), row dicts built on first use of ``rows``."""

    def __init__(self, cols: Dict[str, np.ndarray], pool: bytes, visited: int, candidates: int):
        self.cols, self.pool, self.visited_loci, self.candidate_loci = cols, pool, visited, candidates
        self._rows: Optional[List[dict]] = None

    COLUMNS = ("contig", "pos", "sample", "ref_off", "ref_len", "alt_off", "alt_len", "log_odds", "gq", "tumor",
               "normal", "flags")

    @staticmethod
    def from_result(ptr) -> "SomaticCalls":
        """Zero-copy numpy views over the result block (gq_somatic_calls.block_), kept alive by a
        ctypes buffer whose finalizer calls gq_free_somatic; results without a block are copied
        and freed at once."""
        import weakref

        c = ptr.contents
        n = int(c.n)
        pool = C.string_at(c.allele_pool, c.pool_len) if c.pool_len else b""
        if n == 0 or not c.block_:
            try:
                return SomaticCalls.from_struct(c, pool)
            finally:
                lib().gq_free_somatic(ptr)
        types = {k: getattr(c, k)._type_ for k in SomaticCalls.COLUMNS}
        ends = [C.cast(getattr(c, k), C.c_void_p).value + n * C.sizeof(types[k]) for k in SomaticCalls.COLUMNS]
        buf = (C.c_uint8 * (max(ends) - c.block_)).from_address(c.block_)
        weakref.finalize(buf, lib().gq_free_somatic, ptr)
        cols = {}
        for k in SomaticCalls.COLUMNS:
            dt = np.dtype(_EVIDENCE_DTYPE) if types[k] is gq_evidence else np.dtype(types[k])
            cols[k] = np.frombuffer(buf, dtype=dt, count=n, offset=C.cast(getattr(c, k), C.c_void_p).value - c.block_)
        return SomaticCalls(cols, pool, int(c.visited_loci), int(c.candidate_loci))

    @staticmethod
    def from_struct(c: gq_somatic_calls, pool: bytes) -> "SomaticCalls":
        n = int(c.n)

        def col(ptr):
            return np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n else np.zeros(0)
        cols = {k: col(getattr(c, k)) for k in SomaticCalls.COLUMNS}
        return SomaticCalls(cols, pool, int(c.visited_loci), int(c.candidate_loci))

    @property
    def rows(self) -> List[dict]:
        if self._rows is None:
            c, pool = self.cols, self.pool
            # columns to Python lists once (per-element numpy indexing cost ~25 us a row)
            L = {k: c[k].tolist() for k in ("contig", "pos", "sample", "ref_off", "ref_len", "alt_off", "alt_len",
                                            "log_odds", "gq", "flags")}
            ev = {s: list(zip(*[c[s][k].tolist() for k in EVIDENCE_FIELDS])) if len(self) else [] for s in ("tumor", "normal")}
            self._rows = [dict(contig=ct, locus=ps, sample=sm, ref=pool[ro:ro + rl].decode("latin-1"),
                               alt=pool[ao:ao + al].decode("latin-1"), log_odds=lo, gq=g, tumor=te, normal=ne, flags=fl)
                          for ct, ps, sm, ro, rl, ao, al, lo, g, fl, te, ne in
                          zip(L["contig"], L["pos"], L["sample"], L["ref_off"], L["ref_len"], L["alt_off"], L["alt_len"],
                              L["log_odds"], L["gq"], L["flags"], ev["tumor"], ev["normal"])]
        return self._rows

    def __len__(self) -> int:
        return int(self.cols["pos"].shape[0])

    COLS = ("contig", "pos", "sample", "ref_off", "ref_len", "alt_off", "alt_len", "log_odds", "gq", "tumor", "normal",
            "flags")

    def pack(self) -> np.ndarray:
        """One uint8 buffer (n, pool length, visited, candidates, the columns' raw bytes, the
        pool) for the multi-GPU gather."""
        head = np.array([len(self), len(self.pool), self.visited_loci, self.candidate_loci], np.int64)
        parts = [head.view(np.uint8)] + [np.ascontiguousarray(self.cols[k]).view(np.uint8).ravel() for k in self.COLS]
        parts.append(np.frombuffer(self.pool, np.uint8))
        return np.concatenate(parts)

    @staticmethod
    def unpack(buf: np.ndarray) -> "SomaticCalls":
        buf = np.asarray(buf, np.uint8)
        n, pl, visited, cands = (int(x) for x in buf[:32].view(np.int64))
        dts = dict(contig=np.int32, pos=np.int64, sample=np.uint8, ref_off=np.int64, ref_len=np.int32,
                   alt_off=np.int64, alt_len=np.int32, log_odds=np.float64, gq=np.int32, tumor=_EVIDENCE_DTYPE,
                   normal=_EVIDENCE_DTYPE, flags=np.uint8)
        off, cols = 32, {}
        for k in SomaticCalls.COLS:
            dt = np.dtype(dts[k])
            nb = n * dt.itemsize
            cols[k] = buf[off:off + nb].copy().view(dt)
            off += nb
        return SomaticCalls(cols, buf[off:off + pl].tobytes(), visited, cands)

