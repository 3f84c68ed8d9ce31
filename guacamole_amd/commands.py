"""Caller commands over the GPU engine — the host mirror of the reference's plugin surface.

Reference surface (paths relative to /root/reference/src/main/scala/org/hammerlab/guacamole/):
  * command registry + args       Guacamole.scala:37-77, Command.scala:33-62, Common.scala:48-136
  * germline-threshold            commands/GermlineThresholdCaller.scala:40-88
        --threshold (8), --emit-ref, --emit-no-call, + --reads/--loci/--out/--parallelism/...
  * somatic-standard              commands/SomaticStandardCaller.scala:40-160
        --tumor-reads, --normal-reads, --odds (20), --min-mapq (1), --filter-multi-allelic, ...
  * loci partitioning             DistributedUtil.scala:55-69 (--parallelism, --partition-accuracy)

The per-locus work (pileupFlatMap + callVariantsAtLocus / findPotentialVariantAtLocus)
runs in libgqpileup on the GPU; this module only loads reads, builds LociSets and
partitions, and formats output.

Launched under torch.distributed.run (WORLD_SIZE > 1) the commands run one rank per GPU:
the reference's task partition is split into contiguous blocks of tasks per rank, each rank
uploads the reads overlapping its tasks' loci and calls its share, and rank 0 gathers the
records (over RCCL) and writes the output (distributed.py).
"""
from __future__ import annotations

import argparse
import json
import sys
import weakref
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import native, soa
from .distributed import (all_gather_objects, assign_tasks_to_ranks, device_ingest_ranks, gather_germline,
                          gather_somatic, init_from_env, rank_share, reads_overlapping)
from .loci import (LociSet, LociSetBuilder, flatten_partitions, partition_loci_by_approximate_depth,
                   partition_loci_uniformly)
from .bamdev import DeviceReadSet, load_reads_device, map_bams
from .reads import InputFilters, ReadSet, is_bam, load_reads

def device_reads(ctx: native.Context, rs: ReadSet) -> native.DeviceReads:
    """Upload a ReadSet once per context and keep it resident for as long as the ReadSet lives
    (the HBM copy is held by the ReadSet object itself and freed with it)."""
    cache = rs.__dict__.setdefault("_device", {})
    hit = cache.get(id(ctx))
    if hit is not None and hit[0]() is ctx:
        return hit[1]
    d = ctx.upload(soa.pack(rs))
    cache[id(ctx)] = (weakref.ref(ctx), d)
    return d


LAST_TIMING: Optional[Dict[str, object]] = None  # the last command's stage report in this process


class StageClock:
    """Wall time per stage of a command (GQ_TIMING=1: one JSON line on stderr at the end)."""

    def __init__(self):
        import os
        import time
        self.on = os.environ.get("GQ_TIMING") == "1"
        self.t = time.perf_counter
        self.t0 = self.last = self.t()
        self.stages: Dict[str, float] = {}
        # GQ_T_SPAWN (the launcher's time.time() at spawn): interpreter start + imports before the
        # command, and when the report is written (the rest of the launcher's wall time is exit)
        self.spawn = float(os.environ.get("GQ_T_SPAWN", "0") or 0)
        if self.spawn:
            self.stages["startup_s"] = time.time() - self.spawn

    def note(self, name: str, seconds: float) -> None:
        """A timed sub-step (inside some stage), reported beside the stages."""
        self.stages[name] = self.stages.get(name, 0.0) + seconds

    def mark(self, name: str) -> None:
        now = self.t()
        self.stages[name] = self.stages.get(name, 0.0) + (now - self.last)
        self.last = now

    def report(self, **extra) -> None:
        global LAST_TIMING
        LAST_TIMING = dict(self.stages, total_s=self.t() - self.t0, **extra)
        if self.on:
            import time
            at = {"report_at_s": time.time() - self.spawn} if self.spawn else {}
            print("GQ_TIMING " + json.dumps(dict(self.stages, total_s=self.t() - self.t0, **at, **extra)), file=sys.stderr)


def task_count(parallelism: int, world: int = 1) -> int:
    """`--parallelism` or, at 0, Spark's sc.defaultParallelism (DistributedUtil.scala:59).  The
    default parallelism of a Spark job is the number of its workers' cores; here it is the
    number of ranks (1 for a single process, N under torch.distributed.run with N GPUs).  So, as
    between Spark local[1] and local[N], a run with the default and a different rank count
    cuts the loci into different tasks, and the records at heap-order loci (the first pileup of
    every task) may differ; identical output across rank counts needs
    the same explicit --parallelism."""
    return parallelism if parallelism > 0 else max(1, world)


def partition(loci: LociSet, parallelism: int, accuracy: int, *read_sets: ReadSet, world: int = 1):
    """DistributedUtil.partitionLociAccordingToArgs (DistributedUtil.scala:55-69)."""
    tasks = task_count(parallelism, world)
    if accuracy == 0 or (tasks == 1 and loci.count > 0):
        # one task takes every locus whatever the depths are (the map is the same; the
        # read-region counts are only needed to cut loci between tasks)
        return partition_loci_uniformly(tasks, loci)
    return partition_loci_by_approximate_depth(tasks, loci, accuracy, *[r.regions() for r in read_sets])


def germline_threshold_reads(ctx: native.Context, rs: ReadSet, loci, threshold: int = 8, emit_ref: bool = False,
                             emit_no_call: bool = False) -> List[tuple]:
    """pileupFlatMap(reads, partitions, skipEmpty=true, callVariantsAtLocus) on the GPU.
    `loci` = flatten_partitions(...) arrays.  Rows: (contig, locus, sample, (gt0, gt1), ref, alt, flags)."""
    calls = ctx.germline_threshold(device_reads(ctx, rs), loci, threshold, emit_ref, emit_no_call)
    return calls.tuples(rs.contig_names)


def somatic_standard_reads(ctx: native.Context, tumor: ReadSet, normal: ReadSet, loci, _gather=None,
                           reference=None, _stats=None, **params) -> Optional[List[dict]]:
    """pileupFlatMapTwoRDDs(tumor, normal, partitions, skipEmpty=true, findPotentialVariantAtLocus,
    referenceGenome) + the driver's filters on the GPU.  Rows as the oracle's somatic_standard
    (contig by name).  reference: a reference.ReferenceGenome (--reference-fasta) or None.
    _gather: the gather device of a multi-GPU run (rank 0 gets every rank's rows, others None)."""
    if tumor.contig_names != normal.contig_names:
        raise ValueError("tumor and normal reads must share the contig list")
    dref = None if reference is None else ctx.upload_reference(reference.for_contigs(tumor.contig_names))
    try:
        calls = ctx.somatic_standard(device_reads(ctx, tumor), device_reads(ctx, normal), loci, reference=dref,
                                     **params)
    finally:
        if dref is not None:
            dref.free()
    if _stats is not None:
        _stats["visited_loci"] = int(calls.visited_loci)
    per_rank = [calls] if _gather is None else gather_somatic(calls, _gather)
    if per_rank is None:
        return None
    rows = []
    for c in per_rank:
        for r in c.rows:
            r = dict(r)
            r["contig"] = tumor.contig_names[r["contig"]]
            rows.append(r)
    return rows


# ---------------------------------------------------------------------------------------------
# CLI
def _common_args(p: argparse.ArgumentParser) -> None:
    """Common.Arguments (Common.scala:48-136): Base, Loci, NoSequenceDictionary,
    ReadLoadingConfigArgs, GenotypeOutput, DistributedUtil.Arguments."""
    p.add_argument("--debug", action="store_true", help="If set, prints a higher level of debug output.")
    p.add_argument("--no-sequence-dictionary", action="store_true",
                   help="If set, get contigs and lengths directly from reads instead of from sequence dictionary.")
    p.add_argument("--recompute-md-tags", action="store_true",
                   help="Use the reference fasta to recompute the MD Tags on all mapped reads")
    p.add_argument("--bam-reader-api", default="best", help="(accepted; the native reader is always used)")
    p.add_argument("--out-chunks", type=int, default=1,
                   help="When writing out to json format, number of chunks to coalesce the genotypes into.")
    p.add_argument("--max-genotypes", type=int, default=0,
                   help="Maximum number of genotypes to output. 0 (default) means output all genotypes.")
    p.add_argument("--loci", default="", help="Loci at which to call variants (e.g. 'all', 'chr1:0-1000,chr2')")
    p.add_argument("--loci-from-file", default="", help="Path to file giving loci")
    p.add_argument("--out", default="",
                   help="Output path: .json (or empty: stdout) Avro-JSON, .vcf a VCF directory, else ADAM Parquet")
    p.add_argument("--parallelism", type=int, default=0, help="Num variant calling tasks (loci partitions)")
    p.add_argument("--partition-accuracy", type=int, default=250,
                   help="Num micro partitions per task in loci partitioning; 0 = uniform")
    p.add_argument("--device", type=int, default=0, help="GPU index")
    # ParquetArgs (bdg-utils cli; Common.scala:50): the options of the ADAM Parquet output
    p.add_argument("-parquet_block_size", type=int, default=128 * 1024 * 1024, help="Parquet block size (default = 128mb)")
    p.add_argument("-parquet_page_size", type=int, default=1 * 1024 * 1024, help="Parquet page size (default = 1mb)")
    p.add_argument("-parquet_compression_codec", default="GZIP", type=str.upper, help="Parquet compression codec")
    p.add_argument("-parquet_disable_dictionary", action="store_true", help="Disable dictionary encoding")
    p.add_argument("-parquet_logging_level", default="SEVERE", help="Parquet logging level (default = severe)")


def _loci_builder(args) -> LociSetBuilder:
    """Common.loci (Common.scala:223-239)."""
    if args.loci and args.loci_from_file:
        raise ValueError("Specify at most one of the 'loci' and 'loci-from-file' arguments")
    if args.loci:
        return LociSet.parse(args.loci)
    if args.loci_from_file:
        with open(args.loci_from_file) as fh:
            return LociSet.parse(fh.read())
    return LociSet.parse("all")


class OutputFormatError(ValueError):
    """An --out path the reference would write in a format this build does not produce."""


def _write_genotypes(path: str, genotypes: List[dict], contig_lengths=None, max_genotypes: int = 0,
                     parquet: Optional[dict] = None) -> None:
    """Common.writeVariantsFromArguments (Common.scala:246-304), by the path's extension
    (lower-cased, after stripMargin):
      * "" or .json: Avro-JSON, serially, to stdout or to the file (overwritten, :254-289);
      * .vcf: toVariantContext.coalesce(1).saveAsVcf (:290-293), a Hadoop output DIRECTORY
        holding one part-r-00000 and the committer's _SUCCESS marker (README.md:49-51); an
        existing path is refused, as Hadoop's checkOutputSpecs refuses it;
      * anything else: adamParquetSave (:294-302): a Hadoop output directory of Parquet part
        files, one per loci task (output.write_parquet_dir).  parquet: ParquetArgs (codec,
        page_size, block_size, dictionary) and the records' task ids (part_of, n_parts).
    --max-genotypes reaches RDD.sample(false, maxGenotypes, 0) as the sampling FRACTION
    (Common.scala:247-249): 1 keeps every genotype, larger values are refused by Spark's
    Bernoulli sampler ("must be on interval [0, 1]"), as here.  --out-chunks only coalesces
    partitions (order-preserving), so it does not change what is written."""
    from .output import write_json, write_parquet_dir, write_vcf_dir
    check_output_path(path)
    if max_genotypes > 1:
        raise ValueError("Sampling fraction (%s) must be on interval [0, 1]" % float(max_genotypes))
    kind = output_kind(path)
    if kind == "vcf":
        write_vcf_dir(path, genotypes, contig_lengths)
    elif kind == "parquet":
        write_parquet_dir(path, genotypes, **(parquet or {}))
    else:
        write_json(path, genotypes)


def output_kind(path: str) -> str:
    """"json", "vcf" or "parquet" (Common.scala:253-302)."""
    low = path.lower()
    if path == "" or low.endswith(".json"):
        return "json"
    return "vcf" if low.endswith(".vcf") else "parquet"


def check_output_path(path: str, codec: str = "GZIP") -> None:
    """Refuse, before any work, an output directory (VCF or Parquet) that already exists, as
    Hadoop's FileOutputFormat.checkOutputSpecs does (Common.scala:290, 294), and a Parquet codec
    this build cannot write."""
    import os
    from .output import PARQUET_CODECS
    kind = output_kind(path)
    if kind == "json":
        return
    if os.path.exists(path):
        raise OutputFormatError("Output directory %s already exists" % path)
    if kind == "parquet" and codec not in PARQUET_CODECS:
        raise OutputFormatError("-parquet_compression_codec %s: this build writes %s" % (codec, ", ".join(
            sorted(PARQUET_CODECS))))


def _all_flat(mine):
    """Every rank's flattened loci ranges (rank order = task order), on every rank."""
    got = all_gather_objects([np.asarray(a) for a in mine])
    return tuple(np.concatenate([g[k] for g in got]) for k in range(4))


def parquet_options(args, flat=None, contig_index=None, rows_contig=None, rows_pos=None) -> dict:
    """ParquetArgs (bdg-utils cli, mixed into Common.Arguments.Base, Common.scala:50) and the part
    file of each record: the loci task whose range holds it (flat = flatten_partitions arrays),
    since the callers' genotypes RDD has one partition per task.

    Divergence (parity unpinned, no fixture covers it): after --dbsnp-vcf the reference's
    keyBy + leftOuterJoin (SomaticStandardCaller.scala:143-144) reshuffles the records under a
    hash partitioner before adamParquetSave, so its record-to-part mapping is the join's, not
    the loci tasks'.  Here the parts stay per loci task in that case too; the records and their
    order within the whole output are the same, only which part file holds a record differs."""
    opts = dict(codec=args.parquet_compression_codec, page_size=args.parquet_page_size,
                block_size=args.parquet_block_size, dictionary=not args.parquet_disable_dictionary)
    if flat is not None and rows_pos is not None:
        contig, start, end, task = (np.asarray(a, np.int64) for a in flat)
        part = np.zeros(len(rows_pos), np.int64)
        if len(rows_pos) and len(task):
            key = contig * (1 << 40) + start  # ranges sorted by (contig, start) within the key space
            o = np.argsort(key, kind="stable")
            rk = np.asarray([contig_index[c] for c in rows_contig], np.int64) * (1 << 40) + np.asarray(rows_pos,
                                                                                                       np.int64)
            i = np.clip(np.searchsorted(key[o], rk, "right") - 1, 0, len(o) - 1)
            part = task[o][i]
        opts.update(part_of=part, n_parts=int(task.max()) + 1 if len(task) else 1)
    return opts


def device_ingest(args, *paths: str) -> bool:
    """Decode these BAMs on the GPU (bamdev.load_reads_device) rather than with the host
    loader: BAM input without MD recomputation or contig lengths from the reads (GQ_INGEST=host
    forces the host loader).  Under torch.distributed.run each rank decodes only the part of the
    file its tasks need (distributed.device_ingest_ranks)."""
    import os
    if os.environ.get("GQ_INGEST", "device") == "host":
        return False
    if getattr(args, "recompute_md_tags", False) or getattr(args, "no_sequence_dictionary", False):
        return False
    if getattr(args, "reference_fasta", ""):
        return False
    return all(is_bam(p) for p in paths)


def load_pair_device(ctx, ctx2, paths, filters, mapped):
    """Two BAMs decoded on the device at once: the second on ctx2 (its own stream) on a host
    thread while the first loads on ctx, so one's copy overlaps the other's inflate (ctypes
    releases the GIL).  The second read set is then registered with ctx (device pointers are
    valid across contexts of one device) and keeps ctx2 alive."""
    import threading
    import weakref
    box = {}

    def second():
        try:
            box["rs"] = load_reads_device(ctx2, paths[1], filters, mapped[paths[1]])
        except BaseException as e:  # re-raised below
            box["err"] = e
    th = threading.Thread(target=second)
    th.start()
    try:
        first = load_reads_device(ctx, paths[0], filters, mapped[paths[0]])
    finally:
        th.join()
    if "err" in box:
        raise box["err"]
    rs = box["rs"]
    if rs is not None:
        rs._device[id(ctx)] = (weakref.ref(ctx), rs.reads)
        rs._ctx2 = ctx2
    return [first, rs]


def germline_threshold_main(argv: Sequence[str]) -> int:
    p = argparse.ArgumentParser(prog="germline-threshold",
                                description="call variants by thresholding read counts (toy example)")
    p.add_argument("--reads", required=True)
    p.add_argument("--threshold", type=int, default=8, help="Make a call if at least X%% of reads support it")
    p.add_argument("--emit-ref", action="store_true", help="Output homozygous reference calls.")
    p.add_argument("--emit-no-call", action="store_true", help="Output no call calls.")
    _common_args(p)
    args = p.parse_args(argv)
    clock = StageClock()
    check_output_path(args.out, args.parquet_compression_codec)
    rank, world, local, gdev = init_from_env()
    warn_default_parallelism(args, world)
    builder = _loci_builder(args)
    # germline-threshold takes no reference (GermlineThresholdCaller.scala:64-70): with
    # --recompute-md-tags read loading fails (Read.scala:223-225)
    filters = InputFilters.make(overlaps_loci=builder, non_duplicate=True, has_md_tag=True)
    ctx = None
    rs = None
    mine = None  # this rank's loci ranges, when the device ingest planned them
    if device_ingest(args, args.reads):
        if world == 1:
            maps = map_bams([args.reads])  # the file mapped on a host thread while the context starts
            t = clock.t()
            ctx = native.Context(args.device)
            clock.note("ctx_open_s", clock.t() - t)
            rs = load_reads_device(ctx, args.reads, filters, maps["join"]()[args.reads])
        else:
            ctx = native.Context(local)
            got = device_ingest_ranks(ctx, [args.reads], filters, builder, args.parallelism, args.partition_accuracy,
                                      rank, world, gdev)
            if got is not None:
                (rs,), mine, _ = got
    if rs is None:
        rs = load_reads(args.reads, filters, recompute_md=args.recompute_md_tags,
                        contig_lengths_from_dictionary=not args.no_sequence_dictionary)
    clock.mark("load_reads")
    loci = builder.result(rs.contig_lengths_map)
    if mine is None:
        parts = partition(loci, args.parallelism, args.partition_accuracy, rs, world=world)
        flat = flatten_partitions(parts, rs.contig_index())
    clock.mark("partition")
    if ctx is None:
        ctx = native.Context(local if world > 1 else args.device)
    if world == 1:
        device_reads(ctx, rs)
        clock.mark("upload")
    names = rs.sample_names
    sample_name = lambda s: names[s] if s < len(names) else "default"  # noqa: E731
    if world > 1:
        if mine is None:
            rr = assign_tasks_to_ranks(flat, world, [rs], len(rs.contig_names))
            mine_rs, mine = rank_share(rs, flat, rr, rank)
        else:
            mine_rs = rs
        calls = ctx.germline_threshold_device(device_reads(ctx, mine_rs), mine, args.threshold, args.emit_ref,
                                              args.emit_no_call)
        t = clock.t()
        per_rank = gather_germline(calls, gdev)
        clock.note("gather_s", clock.t() - t)
        # each rank numbers its own samples (by first appearance in what it read): names travel
        rank_names = all_gather_objects(list(mine_rs.sample_names))
        flat = _all_flat(mine) if output_kind(args.out) == "parquet" else None
        if per_rank is None:
            clock.mark("call")
            clock.report(rank=rank, reads=int(mine_rs.n), loci=int(sum(np.asarray(mine[2]) - np.asarray(mine[1]))),
                         ingest="device" if isinstance(rs, DeviceReadSet) else "host",
                         device_ingest=getattr(rs, "timings", None))
            return _finish_rank(0)
        rows = [(c, l, nm[s] if s < len(nm) else "default", g, ref, alt, fl)
                for calls_r, nm in zip(per_rank, rank_names) for c, l, s, g, ref, alt, fl in calls_r.tuples(rs.contig_names)]
        sample_name = lambda s: s  # noqa: E731
    else:
        calls = ctx.germline_threshold(device_reads(ctx, rs), flat, args.threshold, args.emit_ref, args.emit_no_call)
        rows = None
    clock.mark("call")
    from .output import germline_genotype, write_vcf_dir_germline, write_vcf_dir_germline_calls
    if args.out.lower().endswith(".vcf") and args.max_genotypes <= 1:
        # the lines _write_genotypes writes for these records, without building the records
        if rows is None:
            write_vcf_dir_germline_calls(args.out, calls, rs.contig_names, sample_name, rs.contig_lengths_map)
        else:
            write_vcf_dir_germline(args.out, rows, sample_name, rs.contig_lengths_map)
    else:
        if rows is None:
            rows = calls.tuples(rs.contig_names)
        out = [germline_genotype(c, l, sample_name(s), gt, ref, alt) for c, l, s, gt, ref, alt, fl in rows]
        pq = None
        if output_kind(args.out) == "parquet":
            pq = parquet_options(args, flat, rs.contig_index(), [r[0] for r in rows], [r[1] for r in rows])
        _write_genotypes(args.out, out, rs.contig_lengths_map, args.max_genotypes, pq)
    clock.mark("write")
    n_out = len(rows) if rows is not None else len(calls)
    print("Called %d genotypes." % n_out, file=sys.stderr)
    clock.report(rank=rank, reads=int(mine_rs.n if world > 1 else rs.n), genotypes=n_out, loci=int(loci.count),
                 ingest="device" if isinstance(rs, DeviceReadSet) else "host",
                 device_ingest=getattr(rs, "timings", None))
    return _finish_rank(0)


def somatic_standard_main(argv: Sequence[str]) -> int:
    """SomaticStandard.Caller.run (commands/SomaticStandardCaller.scala:66-160)."""
    p = argparse.ArgumentParser(prog="somatic-standard",
                                description="call somatic variants using independent callers on tumor and normal")
    p.add_argument("--tumor-reads", required=True, help="Aligned reads: tumor")
    p.add_argument("--normal-reads", required=True, help="Aligned reads: normal")
    p.add_argument("--odds", type=int, default=20, help="Minimum log odds threshold for possible variant candidates")
    p.add_argument("--min-mapq", type=int, default=1, help="Minimum read mapping quality for a read (Phred-scaled)")
    p.add_argument("--filter-multi-allelic", action="store_true", help="Filter any pileups > 2 bases considered")
    p.add_argument("--min-edge-distance", type=int, default=0, help="(accepted and ignored, as in the reference)")
    p.add_argument("--min-likelihood", type=int, default=0)
    p.add_argument("--min-vaf", type=int, default=0)
    p.add_argument("--min-lod", type=int, default=0)
    p.add_argument("--min-average-mapping-quality", type=int, default=0)
    p.add_argument("--min-average-base-quality", type=int, default=0)
    p.add_argument("--min-tumor-read-depth", type=int, default=0)
    p.add_argument("--min-normal-read-depth", type=int, default=0)
    p.add_argument("--max-tumor-read-depth", type=int, default=2 ** 31 - 1)
    p.add_argument("--min-tumor-alternate-read-depth", type=int, default=0)
    p.add_argument("--max-median-mismatches", type=int, default=2 ** 31 - 1)
    p.add_argument("--reference-fasta", default="", help="Local path to a reference FASTA file")
    p.add_argument("--dbsnp-vcf", default="", help="VCF file to identify DBSNP variants")
    _common_args(p)
    args = p.parse_args(argv)
    clock = StageClock()
    check_output_path(args.out, args.parquet_compression_codec)
    rank, world, local, gdev = init_from_env()
    warn_default_parallelism(args, world)
    builder = _loci_builder(args)
    f = InputFilters.make(overlaps_loci=builder, non_duplicate=True, passed_vendor_quality_checks=True,
                          has_md_tag=True)
    reference = None
    if args.reference_fasta:  # SomaticStandardCaller.scala:75
        from .reference import ReferenceGenome
        reference = ReferenceGenome.load_fasta(args.reference_fasta)
    ctx = None
    sets = [None, None]
    mine = None  # this rank's loci ranges, when the device ingest planned them
    if device_ingest(args, args.tumor_reads, args.normal_reads):
        if world == 1:
            maps = map_bams([args.tumor_reads, args.normal_reads])
            t = clock.t()
            ctx = native.Context(args.device)
            ctx2 = native.Context(args.device)  # the normal's load: its own stream, alongside the tumor's
            clock.note("ctx_open_s", clock.t() - t)
            mapped = maps["join"]()
            sets = load_pair_device(ctx, ctx2, [args.tumor_reads, args.normal_reads], f, mapped)
        else:
            ctx = native.Context(local)
            got = device_ingest_ranks(ctx, [args.tumor_reads, args.normal_reads], f, builder, args.parallelism,
                                      args.partition_accuracy, rank, world, gdev)
            if got is not None:
                sets, mine, _ = got
    tumor, normal = [s if s is not None else
                     load_reads(path, f, reference=reference, recompute_md=args.recompute_md_tags,
                                contig_lengths_from_dictionary=not args.no_sequence_dictionary)
                     for s, path in zip(sets, (args.tumor_reads, args.normal_reads))]
    if tumor.contig_lengths_map != normal.contig_lengths_map:
        raise ValueError("Tumor and normal samples have different sequence dictionaries.")
    clock.mark("load_reads")
    loci = builder.result(normal.contig_lengths_map)
    if mine is None:
        parts = partition(loci, args.parallelism, args.partition_accuracy, tumor, normal, world=world)
        flat = flatten_partitions(parts, tumor.contig_index())
    else:
        flat = mine
    if ctx is None:
        ctx = native.Context(local if world > 1 else args.device)
    sample = tumor.sample_names[0] if tumor.sample_names else "default"
    if world > 1:
        if mine is None:
            rr = assign_tasks_to_ranks(flat, world, [tumor, normal], len(tumor.contig_names))
            tumor, flat = rank_share(tumor, flat, rr, rank)
            normal = normal.subset(reads_overlapping(normal, *flat[:3]))
        else:  # each rank read its own part: the first tumor sample of the lowest rank that has one
            sample = next((n[0] for n in all_gather_objects(list(tumor.sample_names)) if n), "default")
    stats: Dict[str, int] = {}
    all_flat = None
    if output_kind(args.out) == "parquet":  # every rank's tasks: the part file of each record
        all_flat = _all_flat(flat) if world > 1 else flat
    rows = somatic_standard_reads(
        ctx, tumor, normal, flat, odds=args.odds, min_mapq=args.min_mapq,
        filter_multi_allelic=int(args.filter_multi_allelic), max_read_depth=args.max_tumor_read_depth,
        min_tumor_read_depth=args.min_tumor_read_depth, max_tumor_read_depth=args.max_tumor_read_depth,
        min_normal_read_depth=args.min_normal_read_depth,
        min_tumor_alternate_read_depth=args.min_tumor_alternate_read_depth, min_lod=args.min_lod,
        min_likelihood=args.min_likelihood, min_vaf=args.min_vaf,
        min_average_mapping_quality=args.min_average_mapping_quality,
        min_average_base_quality=args.min_average_base_quality, max_median_mismatches=args.max_median_mismatches,
        apply_filters=1, _gather=gdev if world > 1 else None, reference=reference, _stats=stats)
    clock.mark("call")
    report = dict(rank=rank, reads=[int(tumor.n), int(normal.n)], ingest="device" if isinstance(tumor, DeviceReadSet)
                  else "host", device_ingest=[getattr(x, "timings", None) for x in (tumor, normal)], **stats)
    if rows is None:
        clock.report(**report)
        return _finish_rank(0)
    if args.dbsnp_vcf:  # SomaticStandardCaller.scala:139-149
        from .output import dbsnp_join, read_dbsnp_vcf
        rows = dbsnp_join(rows, read_dbsnp_vcf(args.dbsnp_vcf))
    from .output import somatic_genotype
    out = [somatic_genotype(r["contig"], r, sample) for r in rows]
    pq = None
    if all_flat is not None:
        pq = parquet_options(args, all_flat, tumor.contig_index(), [r["contig"] for r in rows],
                             [r["locus"] for r in rows])
    _write_genotypes(args.out, out, tumor.contig_lengths_map, args.max_genotypes, pq)
    clock.mark("write")
    print("Called %d somatic genotypes." % len(out), file=sys.stderr)
    clock.report(genotypes=len(out), **report)
    return _finish_rank(0)


def variant_loci(vcf_path: str) -> LociSet:
    """LociSet.union of the variants' [start, end) (VariantSupport.scala:82-87) over ADAM's VCF
    variants (loadVariants: one Variant per ALT allele, start = POS - 1, end = start + len(REF))."""
    from .output import read_dbsnp_vcf
    b = LociSetBuilder()
    for v in read_dbsnp_vcf(vcf_path):
        b.put(v["contig"], v["start"], v["end"])
    return b.result()


def variant_support_reads(ctx: native.Context, rs: ReadSet, loci) -> List[tuple]:
    """pileupFlatMap(reads, partitions, skipEmpty=true, pileupToAlleleCounts) on the GPU
    (VariantSupport.scala:93-100, 110-118).  Rows (sample name, contig, locus, ref, alt, count,
    flags), in the loci's call order, a locus's alleles by (ref, alt)."""
    rows = ctx.variant_support(device_reads(ctx, rs), loci)
    return [(rs.sample_names[s] if s < len(rs.sample_names) else "default", rs.contig_names[c], l, ref, alt, n, f)
            for s, c, l, ref, alt, n, f in rows]


def variant_support_main(argv: Sequence[str]) -> int:
    """VariantSupport.Caller.run (commands/VariantSupport.scala:62-103): allele counts at each
    variant of --input-variant in every BAM; saveAsTextFile layout (one part file per BAM and
    task, lines "sample, contig, locus, ref, alt, count", AlleleCount.toString :58-60)."""
    import os
    p = argparse.ArgumentParser(prog="variant-support",
                                description="Find number of reads that support each variant across BAMs")
    p.add_argument("-v", "--input-variant", required=True, help="VCF of the variants")
    p.add_argument("-o", "--output", required=True, help="Output path for CSV")
    p.add_argument("bams", nargs="+", help="Retrieve read data from BAMs at each variant position")
    p.add_argument("--parallelism", type=int, default=0, help="Num variant calling tasks")
    p.add_argument("--partition-accuracy", type=int, default=250, help="(accepted; partitioning is uniform)")
    p.add_argument("--bam-reader-api", default="best", help="(accepted; the native reader is always used)")
    p.add_argument("--recompute-md-tags", action="store_true")
    p.add_argument("--device", type=int, default=0, help="GPU index")
    args = p.parse_args(argv)
    single_process_only("variant-support")
    loci = variant_loci(args.input_variant)
    # partitionLociUniformly(args.parallelism, ...) takes the flag as given (VariantSupport.scala:89)
    parts = partition_loci_uniformly(args.parallelism, loci)
    ctx = native.Context(args.device)
    os.makedirs(args.output, exist_ok=False)
    tasks = args.parallelism
    for b, bam in enumerate(args.bams):
        rs = load_reads(bam, InputFilters(), recompute_md=args.recompute_md_tags, contig_lengths_from_dictionary=False)
        idx = rs.contig_index()
        contig, start, end, task = flatten_partitions(parts, {c: idx.get(c, -1) for c in loci.contigs})
        keep = contig >= 0  # contigs without reads hold no pileups
        flat = (contig[keep], start[keep], end[keep], task[keep])
        rows = variant_support_reads(ctx, rs, flat)
        # the task of each row: its loci range's
        by_task: Dict[int, List[str]] = {t: [] for t in range(tasks)}
        r = 0
        for sample, cname, locus, ref, alt, n, _ in rows:
            ci = idx[cname]
            while not (flat[0][r] == ci and flat[1][r] <= locus < flat[2][r]):
                r += 1
            by_task[int(flat[3][r])].append("%s, %s, %d, %s, %s, %d" % (sample, cname, locus, ref, alt, n))
        for t in range(tasks):
            with open(os.path.join(args.output, "part-%05d" % (b * tasks + t)), "w") as fh:
                fh.writelines(line + "\n" for line in by_task[t])
    open(os.path.join(args.output, "_SUCCESS"), "w").close()
    return 0


def germline_standard_reads(ctx: native.Context, rs: ReadSet, loci, **params) -> List[dict]:
    """pileupFlatMap(reads, partitions, skipEmpty=true, callVariantsAtLocus) + GenotypeFilter
    (commands/GermlineStandardCaller.scala:63-72) on the GPU.  Rows as somatic_standard_reads'
    (contig by name; sample = the sample slot; tumor = the allele's evidence)."""
    calls = ctx.germline_standard(device_reads(ctx, rs), loci, **params)
    rows = []
    for r in calls.rows:
        r = dict(r)
        r["contig"] = rs.contig_names[r["contig"]]
        rows.append(r)
    return rows


def germline_standard_main(argv: Sequence[str]) -> int:
    """GermlineStandard.Caller.run (commands/GermlineStandardCaller.scala:48-76).  The truth-set
    concordance report (--truth-genotypes) is outside the pileup path and refused."""
    p = argparse.ArgumentParser(prog="germline-standard",
                                description="call variants using a simple quality-based probability")
    p.add_argument("--reads", required=True)
    p.add_argument("--min-mapq", type=int, default=1, help="Minimum read mapping quality for a read (Phred-scaled)")
    p.add_argument("--min-read-depth", type=int, default=0, help="Minimum number of reads for a genotype call")
    p.add_argument("--max-read-depth", type=int, default=2 ** 31 - 1, help="Maximum number of reads for a genotype call")
    p.add_argument("--min-alternate-read-depth", type=int, default=0)
    p.add_argument("--min-likelihood", type=int, default=0, help="Minimum Phred-scaled likelihood. Default: 0 (off)")
    p.add_argument("--emit-ref", action="store_true", help="(accepted; callVariantsAtLocus is called without it)")
    p.add_argument("--filter-multi-allelic", action="store_true", help="(accepted, unused by this caller)")
    p.add_argument("--min-edge-distance", type=int, default=0, help="(accepted, unused by this caller)")
    p.add_argument("--debug-genotype-filters", action="store_true")
    p.add_argument("--truth-genotypes", default="", help="(concordance report: not supported)")
    _common_args(p)
    args = p.parse_args(argv)
    single_process_only("germline-standard")
    check_output_path(args.out, args.parquet_compression_codec)
    if args.truth_genotypes:
        raise ValueError("--truth-genotypes (concordance report) is not supported")
    builder = _loci_builder(args)
    rs = load_reads(args.reads, InputFilters.make(overlaps_loci=builder, non_duplicate=True, has_md_tag=True),
                    recompute_md=args.recompute_md_tags,
                    contig_lengths_from_dictionary=not args.no_sequence_dictionary)
    loci = builder.result(rs.contig_lengths_map)
    parts = partition(loci, args.parallelism, args.partition_accuracy, rs)
    flat = flatten_partitions(parts, rs.contig_index())
    ctx = native.Context(args.device)
    rows = germline_standard_reads(ctx, rs, flat, min_mapq=args.min_mapq, min_read_depth=args.min_read_depth,
                                   max_read_depth=args.max_read_depth,
                                   min_alternate_read_depth=args.min_alternate_read_depth,
                                   min_likelihood=args.min_likelihood, apply_filters=1)
    from .output import called_allele_genotype
    out = [called_allele_genotype(r["contig"], r, rs.sample_names[r["sample"]] if r["sample"] < len(rs.sample_names)
                                  else "default") for r in rows]
    pq = None
    if output_kind(args.out) == "parquet":
        pq = parquet_options(args, flat, rs.contig_index(), [r["contig"] for r in rows], [r["locus"] for r in rows])
    _write_genotypes(args.out, out, rs.contig_lengths_map, args.max_genotypes, pq)
    print("Called %d genotypes." % len(out), file=sys.stderr)
    return 0


def vaf_histogram_reads(ctx: native.Context, rs: ReadSet, loci, bins: int = 20, min_read_depth: int = 0,
                        min_vaf: int = 0) -> Dict[str, object]:
    """VAFHistogram.variantLociFromReads + generateVAFHistogram (commands/VAFHistogram.scala:
    188-229) on the GPU: {bin start: loci}, variant and visited locus counts."""
    return ctx.vaf_histogram(device_reads(ctx, rs), loci, bins, min_read_depth, min_vaf)


def vaf_histogram_main(argv: Sequence[str]) -> int:
    """VAFHistogram.Caller.run (commands/VAFHistogram.scala:89-184).  The Gaussian mixture fit
    (--cluster, Spark MLlib) is outside the pileup path and refused."""
    import os
    p = argparse.ArgumentParser(prog="vaf-histogram", description="Compute and cluster the variant allele frequencies")
    p.add_argument("bams", nargs="+", help="BAMs")
    p.add_argument("--loci", default="", help="Loci at which to compute VAFs")
    p.add_argument("--loci-from-file", default="", help="Path to file giving loci")
    p.add_argument("--out", default="", help="Path to save the histogram (saveAsTextFile layout)")
    p.add_argument("--local-out", default="", help="Local file path to save the histogram")
    p.add_argument("--bins", type=int, default=20, help="Number of bins (Default: 20)")
    p.add_argument("--cluster", action="store_true", help="(Gaussian mixture model: not supported)")
    p.add_argument("--num-clusters", type=int, default=3)
    p.add_argument("--min-read-depth", type=int, default=0, help="Minimum read depth to include variant allele frequency")
    p.add_argument("--min-vaf", type=int, default=0, help="Minimum variant allele frequency to include")
    p.add_argument("--print-stats", action="store_true", help="(accepted; statistics are not printed)")
    p.add_argument("--sample-percent", type=int, default=25)
    p.add_argument("--parallelism", type=int, default=0, help="Num variant calling tasks (loci partitions)")
    p.add_argument("--partition-accuracy", type=int, default=250)
    p.add_argument("--bam-reader-api", default="best", help="(accepted; the native reader is always used)")
    p.add_argument("--recompute-md-tags", action="store_true")
    p.add_argument("--device", type=int, default=0, help="GPU index")
    args = p.parse_args(argv)
    single_process_only("vaf-histogram")
    if args.out and args.local_out:
        raise ValueError("--out and --local-out are exclusive")
    if args.cluster:
        raise ValueError("--cluster (Gaussian mixture model over Spark MLlib) is not supported")
    builder = _loci_builder(args)
    # ReadSet(..., InputFilters.empty, contigLengthsFromDictionary = true) (:98-109)
    read_sets = [load_reads(b, InputFilters(), recompute_md=args.recompute_md_tags) for b in args.bams]
    rs0 = read_sets[0]
    loci = builder.result(rs0.contig_lengths_map)
    parts = partition(loci, args.parallelism, args.partition_accuracy, rs0)
    ctx = native.Context(args.device)
    bin_size = 100 // args.bins if 1 <= args.bins <= 100 else 1
    lines, plain = [], []
    for path, rs in zip(args.bams, read_sets):
        flat = flatten_partitions(parts, {c: rs.contig_index().get(c, -1) for c in loci.contigs})
        keep = flat[0] >= 0
        flat = tuple(a[keep] for a in flat)
        h = vaf_histogram_reads(ctx, rs, flat, args.bins, args.min_read_depth, args.min_vaf)["histogram"]
        sample = rs.sample_names[int(rs.sample[0])] if rs.n else "default"
        for b in sorted(h):
            row = "%d, %d, %d" % (b, min(b + bin_size, 100), h[b])
            lines.append("%s, %s, %s" % (path, sample, row))
            plain.append(row)
    if args.local_out:
        with open(args.local_out, "w") as fh:
            fh.write("Filename, SampleName, BinStart, BinEnd, Size\n")
            fh.writelines(l + "\n" for l in lines)
    elif args.out:
        os.makedirs(args.out, exist_ok=False)
        with open(os.path.join(args.out, "part-00000"), "w") as fh:
            fh.writelines(l + "\n" for l in lines)
        open(os.path.join(args.out, "_SUCCESS"), "w").close()
    else:
        for row in plain:
            print(row)
    return 0


def warn_default_parallelism(args, world: int) -> None:
    """--parallelism 0 means one task per rank (task_count): the records at heap-order loci then
    depend on the rank count, so say so when a multi-rank run takes the default."""
    if world > 1 and args.parallelism == 0:
        import os
        if int(os.environ.get("RANK", "0")) == 0:
            print("warning: --parallelism 0 makes %d tasks (one per rank); the records at heap-order loci (the first "
                  "pileup of each task) can then differ from a run with another rank count. Pass the same explicit "
                  "--parallelism to compare runs." % world, file=sys.stderr)


def single_process_only(command: str) -> None:
    """germline-standard, variant-support and vaf-histogram run as one process on --device: under
    torch.distributed.run every rank would repeat the whole job and write the same output, so a
    multi-rank launch is refused."""
    import os
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise RuntimeError("%s runs as a single process (WORLD_SIZE=%s): launch it without torch.distributed.run "
                           "and pick the GPU with --device" % (command, os.environ["WORLD_SIZE"]))


def _finish_rank(rc: int) -> int:
    """Leave the process group (multi-GPU runs) after every rank has finished."""
    import os
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        from . import distributed
        if dist.is_initialized():
            dist.barrier()
            if distributed.OWN_GROUP:
                dist.destroy_process_group()
                distributed.OWN_GROUP = False
    return rc


COMMANDS = {"germline-threshold": germline_threshold_main, "somatic-standard": somatic_standard_main,
            "variant-support": variant_support_main, "vaf-histogram": vaf_histogram_main,
            "germline-standard": germline_standard_main}


def main(argv: Optional[Sequence[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in COMMANDS:
        print("usage: python -m guacamole_amd <command> [args]\ncommands: " + ", ".join(sorted(COMMANDS)),
              file=sys.stderr)
        return 1
    return COMMANDS[argv[0]](argv[1:])
