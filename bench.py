#!/usr/bin/env python3
"""bench.py — pileup loci/s for germline-threshold on synthetic 30x reads (BASELINE.json configs[1]).

A "step" = one germline-threshold pass (gq_germline_threshold_device: tile planning, the
projection pileup kernel germline_proj, the walker and general-allele kernels, record sort,
the result image built in HBM) over every locus of the rank's loci, reads already resident in
HBM, plus (N > 1) the terminal RCCL gather of the per-rank result images to rank 0 over xGMI.
The PCIe copy of the results to the host (gq_germline_threshold) is not part of `value`; its
rate is reported beside it as host_results_loci_per_s.

Workload
  N = 1   one chr20-sized contig (63,025,520 loci, b37 length — T/DistributedUtilSuite.scala:72),
          30x, L = 150, seed 20261015 + 2 (configs[1]).
  N > 1   the b37 genome (lexicographic contig order, LociMap.scala:39-42) cut to N x 63,025,520
          loci and split into N contiguous parts by partitionLociUniformly (DistributedUtil.scala:
          83-108); each rank generates the reads of its part (halo included) and calls its loci
          (weak scaling: the same loci per GPU as N = 1).  --wgs splits the whole 3.1 G-locus
          genome instead (configs[3]: ~390 M loci per GPU at N = 8).

Also reported:
  roofline      germline_proj's algorithmic bytes / its HIP-event time vs 8 TB/s
  end_to_end    SoA upload (H2D + upload-time derivation), the step, the results' D2H, and
                BAM ingest (native libgqingest, rate measured on a sample BAM) for the shard
  cpu_baseline  the CPU oracle (restatement, not the JVM reference) on a bounded window of the
                same workload at 1 thread and at `cores` threads; its calls are compared to the
                GPU's on that window (parity_window)
  somatic       somatic-standard on tumor/normal 60x/30x at chr1 length (configs[2]), rank 0,
                N = 1 only (--somatic-length 0 skips it)
  configs4      somatic-standard on a 500x/500x panel (configs[4], 1 GPU; --panel-length 0 skips it)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

CHR20 = 63_025_520
CHR1 = 249_250_621
HBM_PEAK_GBS = 8000.0


def genome_parts(parts: int, wgs: bool, length: int = CHR20):
    """The split genome: [(contig, contig_length, start, end, part)] in partition order, and the
    genome's locus count.  The b37 genome (lexicographic contig order) cut to parts x length loci
    (whole with wgs), split into `parts` contiguous parts by partitionLociUniformly."""
    from guacamole_amd.genomes import B37
    from guacamole_amd.loci import LociSet, partition_loci_uniformly
    budget = None if wgs else parts * length
    lengths = {}
    ranges = []
    for name, ln in B37:  # already lexicographic
        lengths[name] = ln
        span = ln - 1  # "all" drops each contig's last base (LociSet.scala:205-207)
        if budget is not None:
            span = min(span, budget)
            budget -= span
        if span > 0:
            ranges.append("%s:0-%d" % (name, span))
        if budget == 0:
            break
    ls = LociSet.parse(",".join(ranges)).result(lengths)
    split = partition_loci_uniformly(parts, ls)
    return [(c, lengths[c], s, e, t) for c, s, e, t in split.entries()], ls.count


def rank_pieces(world: int, rank: int, wgs: bool, length: int = CHR20):
    """This rank's loci of the split genome: [(contig, contig_length, start, end)]."""
    parts, count = genome_parts(world, wgs, length)
    return [p[:4] for p in parts if p[4] == rank], count


def merged_pieces(parts):
    """One (contig, contig_length, start, end) per contig spanning all of its parts."""
    out = []
    for c, ln, s, e, _ in parts:
        if out and out[-1][0] == c:
            out[-1] = (c, ln, out[-1][2], e)
        else:
            out.append((c, ln, s, e))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--length", type=int, default=CHR20, help="loci of the N = 1 shard")
    ap.add_argument("--depth", type=float, default=30.0)
    ap.add_argument("--threshold", type=int, default=8)
    ap.add_argument("--wgs", action="store_true", help="N > 1: split the whole b37 genome (configs[3])")
    ap.add_argument("--cpu-window", type=int, default=2_000_000, help="loci in the CPU-oracle sample window")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--somatic-length", type=int, default=CHR1, help="somatic sub-run loci (0: skip)")
    ap.add_argument("--panel-length", type=int, default=1_000_000,
                    help="configs[4] sub-run: 500x/500x panel loci (0: skip)")
    ap.add_argument("--genome-ranks", type=int, default=0,
                    help="split the genome into this many parts (default: the world size); with one "
                         "process, one task per part (the N-rank job's task partition on one GPU)")
    ap.add_argument("--shared-reads", action="store_true",
                    help="generate the whole split genome's reads once (same seed on every rank) and give "
                         "each rank the reads overlapping its loci (DistributedUtil.scala:584-597), so N ranks "
                         "reproduce the 1-process records of the same task partition")
    ap.add_argument("--calls-out", default=None, help="rank 0 writes the gathered records (rank order) as JSON")
    ap.add_argument("--no-single-pass", dest="single_pass", action="store_false",
                    help="skip the measured single pass (the shard as a BAM through the CLI)")
    ap.add_argument("--no-configs3", dest="configs3", action="store_false",
                    help="skip the configs[3] rank share (one rank's share of the 30x b37 genome through the "
                         "multi-GPU ingest path, on this GPU)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_r06.json"),
                    help="PMC-derived HBM bytes per pileup launch (from a separate rocprofv3 --pmc pass)")
    args = ap.parse_args()

    # --gpus N: one rank per GPU.  Without a launcher (WORLD_SIZE unset) N > 1 starts the N ranks
    # itself as a child torch.distributed.run job, before anything here touches the GPU.
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%s: launch one rank per GPU (torch.distributed.run "
              "--nproc-per-node %d)" % (args.gpus, os.environ.get("WORLD_SIZE"), args.gpus), file=sys.stderr)
        return 2

    from guacamole_amd import native, synthetic
    from guacamole_amd.distributed import gather_images_to_rank0, rank_info

    rank, world, local = rank_info()
    dist = None
    # GQ_DIST_BACKEND=gloo: a rehearsal of the N > 1 flow on fewer GPUs (ranks share devices,
    # the gather goes through host memory); the driver's runs use RCCL, one GPU per rank
    backend = os.environ.get("GQ_DIST_BACKEND", "nccl")
    gather_dev = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            gather_dev = "cuda:%d" % local
        else:
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            dist.init_process_group(backend)
            gather_dev = "cpu"

    t0 = time.time()
    n_parts = args.genome_ranks or world
    if world == 1 and n_parts == 1:
        g = synthetic.generate(args.length, args.depth, seed=synthetic.SEED + 2)
        loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([args.length - 1], np.int64),
                np.array([0], np.int64))
        genome_loci = args.length - 1
        workload = "germline-threshold, synthetic 30x chr20-length shard per GPU (configs[1])"
    else:
        parts, genome_loci = genome_parts(n_parts, args.wgs, args.length)
        # this process's parts: its rank's (one task), or every part (one task each) in one process
        mine = [p for p in parts if world == 1 or p[4] == rank]
        pieces = merged_pieces(mine)
        if args.shared_reads:
            every = merged_pieces(parts)
            g = synthetic.subset_pieces(synthetic.generate_pieces(every, args.depth, seed=synthetic.SEED + 4),
                                        every, pieces)
        else:
            g = synthetic.generate_pieces(pieces, args.depth, seed=synthetic.SEED + 4 + 1000 * rank)
        names = [p[0] for p in pieces]
        loci = (np.array([names.index(p[0]) for p in mine], np.int32), np.array([p[2] for p in mine], np.int64),
                np.array([p[3] for p in mine], np.int64),
                np.array([p[4] if world == 1 else 0 for p in mine], np.int64))
        workload = ("germline-threshold, synthetic 30x b37 genome (%s) split into %d parts over %d GPUs (configs[3])"
                    % ("whole" if args.wgs else "first %d loci" % genome_loci, n_parts, world))
    gen_s = time.time() - t0
    ctx = native.Context(local)
    t = time.perf_counter()
    reads = ctx.upload(g.arrays)
    upload_ms = (time.perf_counter() - t) * 1e3
    st_upload = ctx.proj_stats(reads)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    def sync():  # the library's calls return with their stream drained; torch's too at N > 1
        if dist is not None:
            import torch
            torch.cuda.synchronize()

    def step(resident: bool = False):
        """One pass over the shard from the resident SoA: every structure derived from the reads
        (upload-time derivation, projection) built again, then the call (inputs
        resident, pileups rebuilt per run as GermlineThresholdCaller.run does, :58-88).
        resident=True: the call alone on the already-derived read set (resident_step_ms)."""
        if not resident:
            ctx.rederive(reads)
        calls = ctx.germline_threshold_device(reads, loci, args.threshold)
        if dist is not None:
            gather_images_to_rank0(calls, gather_dev)
        return calls

    # one shot (cold): the first call on the fresh read set derives the projection it reads
    t = time.perf_counter()
    first = step(resident=True)
    cold_ms = (time.perf_counter() - t) * 1e3
    cold_tm = ctx.timings()
    first_rows = first.to_host().tuples(g.contig_names) if rank == 0 and world == 1 else None
    for _ in range(args.warmup):
        step()
    barrier()
    pileup_ms, walk_ms, step_ms, derive_ms, proj_ms, fill_ms, dev_ms, dev_parts = [], [], [], [], [], [], [], []
    stage_ms = {"plan_ms": [], "complex_ms": [], "finalize_ms": []}
    walk_frac = []
    t = time.perf_counter()
    for _ in range(args.steps):  # the timed steps: nothing else inside the bracket
        t1 = time.perf_counter()
        calls = step()
        sync()
        step_ms.append((time.perf_counter() - t1) * 1e3)
    barrier()
    elapsed = time.perf_counter() - t
    for _ in range(args.steps):  # the same steps again, untimed, for the per-stage figures
        calls = step()
        sync()
        tm = ctx.timings()
        pileup_ms.append(tm["pileup_ms"])
        walk_ms.append(tm["walk_ms"])
        for k in stage_ms:
            stage_ms[k].append(tm[k])
        walk_frac.append(tm["walk_tiles"] / max(1, tm["tiles"]))
        sti = ctx.proj_stats(reads)
        derive_ms.append(sti["derive_ms"])
        proj_ms.append(sti["proj_ms"])
        fill_ms.append(sti["fill_ms"])
        # (the call's device span starts before its projection is derived: it holds proj_dev_ms)
        dev_parts.append((sti["derive_dev_ms"], sti["proj_dev_ms"], tm["total_ms"] - sti["proj_dev_ms"]))
        dev_ms.append(sum(dev_parts[-1]))
    # the re-derived pass gives the records of the first call on the freshly uploaded set
    rederive_identical = None if first_rows is None else calls.to_host().tuples(g.contig_names) == first_rows
    res_ms = []
    for _ in range(max(5, min(args.steps, 20))):
        t1 = time.perf_counter()
        calls = step(resident=True)
        sync()
        res_ms.append((time.perf_counter() - t1) * 1e3)
    barrier()
    if dist is not None:
        import torch
        dev = "cuda:%d" % local if backend == "nccl" else "cpu"
        x = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        elapsed = float(x.item())
        v = torch.tensor([int(calls.visited_loci)], dtype=torch.int64, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        loci_total = int(v.item())
    else:
        loci_total = int(calls.visited_loci)
    visited = int(calls.visited_loci)
    if args.calls_out:  # (before the next germline call on the context reuses the result image)
        write_calls(args, calls, g, gather_dev, world, rank)
    # the same pass with the records copied to the host (PCIe-inclusive), a few steps, rank-local
    hc = ctx.germline_threshold(reads, loci, args.threshold)  # warm-up of the host-block path
    n_host = 5
    t = time.perf_counter()
    for _ in range(n_host):
        hc = ctx.germline_threshold(reads, loci, args.threshold)
    host_ms_step = (time.perf_counter() - t) / n_host * 1e3
    assert len(hc) == len(calls)

    # ---- roofline for the pileup kernel (germline_proj): algorithmic bytes per launch,
    #      SURVEY §8(d) without qualities (germline-threshold never reads them): 1 B per read
    #      base, 16 B of metadata per read, 4 B per CIGAR op and per MD event, 32 B per record
    #      and 12 B per queued locus written.  Its share is the tiles it kept (walk_tiles go to
    #      the walker).  The bytes it actually reads are reported beside it (`read_bytes`: the
    #      projection rows of 4-bit codes, 8-B sparse entries).
    st = ctx.proj_stats(reads)
    a = g.arrays
    n_reads = int(a["start"].shape[0])
    bytes_seq = int(a["seq"].shape[0])
    bytes_meta = 16 * n_reads
    bytes_cigar = 4 * int(a["cigar"].shape[0])
    bytes_md = 4 * int(a["md_ev"].shape[0])
    bytes_out = 32 * len(calls) + 12 * int(calls.complex_loci)
    b_all = bytes_seq + bytes_meta + bytes_cigar + bytes_md + bytes_out
    read_bytes = int(st["proj_bytes"]) + 8 * int(st["pev_count"])
    kept = 1.0 - float(np.mean(walk_frac))
    b_alg = int(b_all * kept)
    k_ms = float(np.mean(pileup_ms))
    achieved = b_alg / (k_ms * 1e-3) / 1e9
    def pmc_traffic(kernel: str):
        """HBM bytes per launch of `kernel` from the PMC file (its own --pmc passes), or None."""
        try:
            with open(args.traffic) as fh:
                tr = json.load(fh)
        except (OSError, ValueError):
            return None
        if tr.get("length") != args.length or tr.get("depth") != args.depth or world != 1:
            return None
        ks = tr.get("kernels", {})  # (named with template arguments: "proj_fill_cells<4>")
        k = next((k for k in sorted(ks) if k == kernel or k.startswith(kernel + "<")), None)
        return ks[k].get("hbm_bytes_per_launch") if k else None
    direct = os.environ.get("GQ_GERM", "direct") != "proj"
    call_kernel = "germline_direct" if direct else "germline_proj"
    traffic = pmc_traffic(call_kernel)
    # the projection fill (GQ_GERM=proj only: the direct call derives no projection).  Its
    # algorithmic bytes: each projected read's bases over its span read once (sum of end - start)
    # + the pool it writes (every word of every row: the layout the call reads).
    elements = int((a["end"].astype(np.int64) - a["start"].astype(np.int64)).sum())
    f_ms = float(np.median(fill_ms))
    b_fill = elements + int(st["proj_bytes"])
    f_traffic = pmc_traffic("proj_fill_cells")
    if direct:  # the step's dominant kernel is the call's own pileup kernel
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "dram_frac": None if traffic is None else traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "kernel": call_kernel, "kernel_ms": k_ms, "algorithmic_bytes_per_launch": b_alg,
                "basis": "SURVEY 8(d) without qualities (germline-threshold never reads them): the sequence pool "
                         "(%d B), 16 B per read, 4 B per CIGAR op and per MD event, 32 B per record and 12 B per "
                         "queued locus written, times the share of tiles the kernel kept (%.4f); kernel_ms: mean "
                         "of the steps' HIP-event times on the context's stream" % (bytes_seq, kept)}
    else:
        roof = {"bound": "hbm", "achieved": b_fill / (f_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": b_fill / (f_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": f_traffic,
                "dram_frac": None if f_traffic is None else f_traffic / (f_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "kernel": os.environ.get("GQ_FILL", "cells") == "cells" and "proj_fill_cells" or
                          "projection fill (GQ_FILL=%s)" % os.environ.get("GQ_FILL"),
                "kernel_ms": f_ms, "algorithmic_bytes_per_launch": b_fill,
                "basis": "bases over the projected reads' spans (sum end - start: %d) + the projection pool "
                         "written (%d B); kernel_ms: median of the steps' HIP-event times on the context's "
                         "stream" % (elements, int(st["proj_bytes"]))}

    line = {
        "metric": "pileup loci/sec at 30x WGS; achieved HBM GB/s vs roofline",
        "value": loci_total * args.steps / elapsed,
        "unit": "loci/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (native generator: 30x, L=150, GC 0.41, het/hom SNV + indels + Phred errors)",
        "config": {"workload": workload, "genome_loci": genome_loci, "visited_loci_per_gpu": visited,
                   "reads_per_gpu": n_reads, "contigs_per_gpu": len(g.contig_names), "depth": args.depth,
                   "read_len": 150, "threshold": args.threshold, "parallelism": "loci-sharded x%d" % world},
        "roofline": roof,
        # the resident call's pileup kernel (the round-4 headline kernel)
        "call_roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                          # the bus rate: measured HBM bytes (PMC) / the kernel's time / peak
                          "dram_frac": None if traffic is None else traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                          "kernel": call_kernel, "kernel_ms": k_ms, "algorithmic_bytes_per_launch": b_alg,
                          "read_bytes_per_launch": read_bytes, "tiles_kept": kept, "walker_ms": float(np.mean(walk_ms))},
        # the whole step on SURVEY §8(d)'s basis (bases, 16 B per read, CIGAR ops, MD events, output)
        "step_roofline": {"algorithmic_bytes": b_all, "step_ms": float(np.median(step_ms)),
                          "device_ms": float(np.median(dev_ms)),
                          "achieved": b_all / (float(np.median(step_ms)) * 1e-3) / 1e9, "unit": "GB/s",
                          "frac": b_all / (float(np.median(step_ms)) * 1e-3) / 1e9 / HBM_PEAK_GBS},
        "step_ms_median": float(np.median(step_ms)),
        # wall times of the step's parts (host-side, each ending in a synchronisation) and their
        # device spans (HIP events on the context's stream: first kernel to last)
        "step_stages_ms": {"upload_derive_ms": float(np.median(derive_ms)), "projection_ms": float(np.median(proj_ms)),
                           "upload_derive_device_ms": float(np.median([x[0] for x in dev_parts])),
                           "projection_device_ms": float(np.median([x[1] for x in dev_parts])),
                           "call_device_ms": float(np.median([x[2] for x in dev_parts])), "fill_ms": f_ms},
        "rederive_identical": rederive_identical,
        "resident_step_ms": float(np.median(res_ms)),
        "resident_step_loci_per_s": visited / (float(np.median(res_ms)) * 1e-3),
        "kernel_only_loci_per_s": visited / ((k_ms + float(np.mean(walk_ms))) * 1e-3),
        "device_stages_ms": {k: float(np.mean(v)) for k, v in stage_ms.items()},
        "host_results_loci_per_s": visited / (host_ms_step * 1e-3),
        "host_results_ms_per_step": host_ms_step,
        "calls": len(calls),
        "complex_loci": int(calls.complex_loci),
        "ambiguous_loci": int(calls.ambiguous_loci),
        # loci with a count tie among passing alleles (their order is the restated Scala map
        # order), and loci whose order also depends on first occurrences (redone in element order)
        "tie_loci": int(calls.tie_loci),
        "order_loci": int(ctx.timings()["order_loci"]),
        "gen_s": gen_s,
    }
    # one shot: a cold device call on resident reads = the upload-time derivation + the first
    # call (which derives the projection: slice windows, rows, 4-bit codes, sparse entries)
    one = float(st_upload["derive_ms"]) + cold_ms
    line["one_shot"] = {"upload_derive_ms": float(st_upload["derive_ms"]), "first_call_ms": cold_ms,
                        "projection_ms": float(st["proj_ms"]), "first_call_device_ms": float(cold_tm["total_ms"]),
                        "total_ms": one, "loci_per_s": visited / (one * 1e-3),
                        "derivation_kernels": "read_prep, block_index (upload); with GQ_GERM=proj also the "
                                              "projection (proj_prep, slice_windows, row_count, proj_fill_cells, "
                                              "pev_fill) on the first call"}
    if rank == 0:
        e2e = {"upload_ms": upload_ms, "upload_h2d_ms": st["h2d_ms"], "upload_derive_ms": st["derive_ms"],
               "step_ms": line["ms_per_step"], "step_with_d2h_ms": host_ms_step, "reads": n_reads}
        e2e.update(ingest_rate(args.depth))
        e2e["ingest_s_est"] = n_reads / e2e["ingest_reads_per_s"]
        e2e["single_pass_s_est"] = e2e["ingest_s_est"] + (upload_ms + host_ms_step) / 1e3
        e2e["single_pass_loci_per_s_est"] = visited / e2e["single_pass_s_est"]
        line["end_to_end"] = e2e
    if rank == 0 and world == 1 and n_parts == 1 and args.single_pass:
        line["end_to_end"]["single_pass"] = single_pass(g, visited)
    if rank == 0 and world == 1 and n_parts == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"], line["parity_window"] = cpu_baseline(g, ctx, reads, args)
    if dist is not None and args.single_pass and n_parts == world:
        sp = multi_rank_single_pass(args, g, pieces, rank, world, dist, barrier)
        if rank == 0:
            sp["loci_per_s"] = loci_total / sp["wall_s"]
            line.setdefault("end_to_end", {})["single_pass"] = sp
    if dist is not None:
        dist.destroy_process_group()
    del reads, g
    if rank == 0 and world == 1 and args.somatic_length > 0:
        line["somatic"] = somatic_run(ctx, args)
    if rank == 0 and world == 1 and args.somatic_length > 0 and args.single_pass:
        line["somatic"]["single_pass"] = somatic_single_pass(args)
    if rank == 0 and world == 1 and args.panel_length > 0:
        line["configs4"] = somatic_run(ctx, args, steps=5, warmup=2, L=args.panel_length, tdepth=500.0, ndepth=500.0,
                                       rate=1e-3, workload="%d-locus targeted panel (configs[4], 1 GPU)"
                                       % args.panel_length)
    if rank == 0 and world == 1 and args.configs3:
        line["configs3_rank_share"] = configs3_rank_share(ctx, args)
    if rank == 0:
        print(json.dumps(line))
    return 0


def launch_ranks(n: int) -> int:
    """python bench.py --gpus N without a launcher: the same command as N ranks under
    torch.distributed.run (127.0.0.1, a free port), as a child process; its exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def write_calls(args, calls, g, gather_dev, world: int, rank: int):
    """Rank 0 writes every rank's records (rank order = task order) as JSON rows."""
    if world > 1:
        from guacamole_amd.distributed import gather_germline
        per_rank = gather_germline(calls, gather_dev)
        if rank != 0:
            return
        parts, _ = genome_parts(args.genome_ranks or world, args.wgs, args.length)
        rows = []
        for r, c in enumerate(per_rank):
            names = [p[0] for p in merged_pieces([p for p in parts if p[4] == r])]
            rows += c.tuples(names)
    else:
        rows = calls.to_host().tuples(g.contig_names)
    with open(args.calls_out, "w") as fh:
        json.dump([list(x) for x in rows], fh)


def single_pass(g, visited: int):
    """Measured single pass on configs[1]: the shard's reads written as a BGZF level-6 BAM
    (native writer), then `python -m guacamole_amd germline-threshold --reads X.bam --out Y.vcf`
    timed in a fresh process: BAM ingest with the command's filters, loci partitioning (the CLI
    defaults), upload + derivation, the call, the VCF writer (stage wall times from GQ_TIMING)."""
    import shutil
    import subprocess
    tmp = os.environ.get("TMPDIR", "/tmp")
    bam = os.path.join(tmp, "gq_single_pass_%d.bam" % os.getpid())
    out = os.path.join(tmp, "gq_single_pass_%d.vcf" % os.getpid())
    try:
        t = time.perf_counter()
        g.write_bam(bam)
        write_s = time.perf_counter() - t
        cmd = [sys.executable, "-m", "guacamole_amd", "germline-threshold", "--reads", bam, "--out", out]
        env = dict(os.environ, GQ_TIMING="1", PYTHONPATH=ROOT, GQ_T_SPAWN=repr(time.time()))
        t = time.perf_counter()
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
        wall = time.perf_counter() - t
        if r.returncode != 0:
            return {"error": r.stderr[-2000:]}
        stages = {}
        for ln in r.stderr.splitlines():
            if ln.startswith("GQ_TIMING "):
                stages = json.loads(ln[len("GQ_TIMING "):])
        if "report_at_s" in stages:  # after the report: closing the output, releasing HBM, exit
            stages["exit_s"] = wall - stages["report_at_s"]
        return {"wall_s": wall, "loci_per_s": visited / wall, "bam_bytes": os.path.getsize(bam),
                "bam_write_s": write_s, "stages_s": stages,
                "command": "python -m guacamole_amd germline-threshold --reads <shard>.bam --out <out>.vcf"}
    finally:
        if os.path.exists(bam):
            os.remove(bam)
        shutil.rmtree(out, ignore_errors=True)


def somatic_single_pass(args, L: int = CHR20):
    """Measured somatic single pass: tumor 60x / normal 30x over a chr20-length contig written as
    two BGZF level-6 BAMs, then `python -m guacamole_amd somatic-standard --tumor-reads T.bam
    --normal-reads N.bam --out Y.vcf` in a fresh process (both BAMs decoded on the device, loci
    partitioning, the call, the VCF writer; stage wall times from GQ_TIMING).  chr20 length
    rather than configs[2]'s chr1 keeps the two files (~5 GB) and the run within minutes."""
    import shutil
    import subprocess
    from guacamole_amd import synthetic
    tmp = os.environ.get("TMPDIR", "/tmp")
    paths = [os.path.join(tmp, "gq_sp_%s_%d.bam" % (k, os.getpid())) for k in ("tumor", "normal")]
    out = os.path.join(tmp, "gq_sp_somatic_%d.vcf" % os.getpid())
    seed = synthetic.SEED + 3
    try:
        t = time.perf_counter()
        for path, depth, tumor, rseed in ((paths[0], 60.0, True, 11), (paths[1], 30.0, False, 12)):
            synthetic.generate(L, depth, seed=seed, somatic_rate=2e-4, tumor=tumor, read_seed=rseed).write_bam(path)
        write_s = time.perf_counter() - t
        cmd = [sys.executable, "-m", "guacamole_amd", "somatic-standard", "--tumor-reads", paths[0], "--normal-reads",
               paths[1], "--out", out]
        env = dict(os.environ, GQ_TIMING="1", PYTHONPATH=ROOT, GQ_T_SPAWN=repr(time.time()))
        t = time.perf_counter()
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
        wall = time.perf_counter() - t
        if r.returncode != 0:
            return {"error": r.stderr[-2000:]}
        stages = {}
        for ln in r.stderr.splitlines():
            if ln.startswith("GQ_TIMING "):
                stages = json.loads(ln[len("GQ_TIMING "):])
        if "report_at_s" in stages:
            stages["exit_s"] = wall - stages["report_at_s"]
        visited = int(stages.get("visited_loci", 0))
        return {"wall_s": wall, "loci_per_s": visited / wall if visited else None, "visited_loci": visited,
                "bam_bytes": [os.path.getsize(p) for p in paths], "bam_write_s": write_s, "stages_s": stages,
                "workload": "somatic-standard, synthetic tumor/normal 60x/30x, chr20-length contig, two BAMs",
                "command": "python -m guacamole_amd somatic-standard --tumor-reads T.bam --normal-reads N.bam "
                           "--out <out>.vcf"}
    finally:
        for p in paths:
            if os.path.exists(p):
                os.remove(p)
        shutil.rmtree(out, ignore_errors=True)


def ingest_rate(depth: float):
    """BAM -> SoA (native libgqingest: parallel BGZF inflate, decode, the germline filters, MD
    events) on a synthetic sample BAM of the same model, best of 3."""
    from guacamole_amd import ingest, soa, synthetic
    from guacamole_amd.loci import LociSet
    from guacamole_amd.reads import InputFilters
    gs = synthetic.generate(4_000_000, depth, seed=synthetic.SEED + 9)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gq_bench_ingest_%d.bam" % os.getpid())
    gs.write_bam(path)
    filters = InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True)
    best = None
    try:
        for _ in range(3):
            t = time.perf_counter()
            rs = ingest.load_bam(path, filters)
            soa.pack(rs)
            s = time.perf_counter() - t
            best = s if best is None else min(best, s)
        size = os.path.getsize(path)
    finally:
        os.remove(path)
    return {"ingest_reads_per_s": rs.n / best, "ingest_threads": ingest.n_threads(),
            "ingest_sample": "BGZF level-6 BAM of %d synthetic reads (%.0f MB), best of 3" % (rs.n, size / 1e6)}


def _oracle_threads() -> int:
    env = os.environ.get("OMP_NUM_THREADS")
    n = int(env) if env and env.isdigit() else (os.cpu_count() or 1)
    return max(1, min(n, 16, os.cpu_count() or 1))


def cpu_baseline(g, ctx, reads, args):
    """The CPU oracle on a window of the same workload, timed at 1 thread and at `cores`
    threads (the window cut into `cores` contiguous parts, one oracle call per thread, as
    Spark local[*] runs one task per core; ctypes releases the GIL); its calls are compared
    with the GPU's calls over the same loci window."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O

    w0 = args.length // 3
    w1 = min(args.length - 1, w0 + args.cpu_window)
    idx = g.window(w0, w1)
    rs = g.to_read_set(idx)
    loci = (np.array([0], np.int32), np.array([w0], np.int64), np.array([w1], np.int64), np.array([0], np.int64))
    t = time.perf_counter()
    want = O.germline_threshold(rs, loci, args.threshold)
    cpu_s = time.perf_counter() - t
    gpu = ctx.germline_threshold(reads, loci, args.threshold)
    parity = gpu.tuples(g.contig_names) == want
    visited = int(gpu.visited_loci)  # loci with depth > 0 in the window (same set the oracle visits)
    # the window split over `cores` threads, each with its own reads
    cores = _oracle_threads()
    cuts = np.linspace(w0, w1, cores + 1).astype(np.int64)
    jobs = []
    for k in range(cores):
        a, b = int(cuts[k]), int(cuts[k + 1])
        jobs.append((g.to_read_set(g.window(a, b)),
                     (np.array([0], np.int32), np.array([a], np.int64), np.array([b], np.int64),
                      np.array([0], np.int64))))
    t = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        parts = list(ex.map(lambda j: O.germline_threshold(j[0], j[1], args.threshold), jobs))
    par_s = time.perf_counter() - t
    par_same = [r for p in parts for r in p] == want
    return ({"value": visited / par_s, "unit": "loci/s", "cores": cores, "kind": "port",
             "value_1_thread": visited / cpu_s,
             "sample": "CPU oracle (oracle/oracle.cpp, not the JVM reference) on loci [%d, %d) of the same synthetic "
                       "shard: %d visited loci, %d reads; 1 thread %.1f s, %d threads %.1f s (calls identical: %s)"
                       % (w0, w1, visited, len(idx), cpu_s, cores, par_s, par_same)},
            {"loci": [w0, w1], "calls": len(want), "identical": bool(parity)})


def somatic_run(ctx, args, steps: int = 3, warmup: int = 1, L: int = 0, tdepth: float = 60.0, ndepth: float = 30.0,
                rate: float = 2e-4, workload: str = "chr1-length contig (configs[2])"):
    """somatic-standard on synthetic tumor 60x / normal 30x over one chr1-length contig
    (configs[2]; the panel sub-run: 500x / 500x over a short contig, configs[4]), reads resident
    in HBM; a step = one gq_somatic_standard call (CLI defaults, driver filters on).  Roofline of
    the candidate kernel somatic_proj from its algorithmic bytes: tumor bases + qualities, 16 B
    per tumor read, 4 B per tumor CIGAR op and MD event, 8 B per normal read (the normal's depth
    needs its reads' intervals only); the bytes it reads (projection rows, 16-bit margin terms,
    sparse entries, normal intervals) beside it."""
    from guacamole_amd import synthetic
    L = L or args.somatic_length
    t0 = time.time()
    seed = synthetic.SEED + 3
    tg = synthetic.generate(L, tdepth, seed=seed, somatic_rate=rate, tumor=True, read_seed=11)
    ng = synthetic.generate(L, ndepth, seed=seed, somatic_rate=rate, tumor=False, read_seed=12)
    gen_s = time.time() - t0
    t = ctx.upload(tg.arrays)
    n = ctx.upload(ng.arrays)
    derive_ms = float(ctx.proj_stats(t)["derive_ms"]) + float(ctx.proj_stats(n)["derive_ms"])
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([L - 1], np.int64), np.array([0], np.int64))
    c0 = time.perf_counter()
    ctx.somatic_standard(t, n, loci)  # cold: the tumor's projection and margin projection are derived
    cold_ms = (time.perf_counter() - c0) * 1e3
    cold_tm = ctx.timings()
    def step(resident: bool = False):
        """One somatic-standard pass (SomaticStandardCaller.scala:66-160): both read sets'
        derived structures built again (gq_reads_rederive: the upload-time derivation; the
        tumor's projection and margin projection on the call that reads them), then the call.
        resident=True: the call alone over the already-derived sets (resident_step_ms)."""
        if not resident:
            ctx.rederive(t)
            ctx.rederive(n)
        return ctx.somatic_standard(t, n, loci)
    for _ in range(warmup):
        step()
    stages = {"pileup_ms": [], "complex_ms": [], "call_ms": [], "deep_ms": [], "finalize_ms": [], "total_ms": [],
              "host_ms": [], "marshal_ms": []}
    t1 = time.perf_counter()
    for _ in range(steps):  # the timed steps: derivation-inclusive
        calls = step()
    el = time.perf_counter() - t1
    derive_step = {"tumor_derive_ms": [], "normal_derive_ms": [], "tumor_projection_ms": []}
    for _ in range(steps):  # the same steps again, untimed, for the per-stage figures
        calls = step()
        tm = ctx.timings()
        for k in stages:
            stages[k].append(tm[k])
        st_t, st_n = ctx.proj_stats(t), ctx.proj_stats(n)
        derive_step["tumor_derive_ms"].append(float(st_t["derive_ms"]))
        derive_step["normal_derive_ms"].append(float(st_n["derive_ms"]))
        derive_step["tumor_projection_ms"].append(float(st_t["proj_ms"]))
    res_ms = []
    for _ in range(max(3, steps)):  # resident: the call alone, projections kept
        r0 = time.perf_counter()
        calls = step(resident=True)
        res_ms.append((time.perf_counter() - r0) * 1e3)
    tm = ctx.timings()
    parity = somatic_parity_window(ctx, t, n, tg, ng, L, 1_000_000 if tdepth < 500 else 100_000)
    ta = tg.arrays
    b_alg = (2 * int(ta["seq"].shape[0]) + 16 * tg.n + 4 * int(ta["cigar"].shape[0]) + 4 * int(ta["md_ev"].shape[0])
             + 8 * ng.n)
    st = ctx.proj_stats(t)
    # tumor rows: 4-bit codes (proj_bytes) + 8-bit margin terms (2 x proj_bytes)
    read_bytes = 3 * int(st["proj_bytes"]) + 8 * int(st["pev_count"]) + 8 * ng.n
    k_ms = float(np.mean(stages["pileup_ms"]))
    ach = b_alg / (k_ms * 1e-3) / 1e9
    visited = int(calls.visited_loci)
    pmc = somatic_pmc("panel" if tdepth >= 500 else "chr1", L, tdepth, ndepth)
    som_kernel = "somatic_proj" if os.environ.get("GQ_SOM") == "proj" else "somatic_direct"
    traffic = None if pmc is None else next(
        (v.get("hbm_bytes_per_launch") for k, v in sorted(pmc["kernels"].items()) if k.startswith(som_kernel)), None)
    return {"metric": "somatic-standard loci/sec, tumor %gx / normal %gx" % (tdepth, ndepth),
            "value": visited * steps / el, "unit": "loci/s", "ms_per_step": 1e3 * el / steps, "steps": steps,
            "warmup": warmup, "step": "re-derivation of both read sets (upload-time derivation, tumor projection and "
                                     "margin projection) + the call",
            "step_stages_ms": {k: float(np.median(v)) for k, v in derive_step.items()},
            "resident_step_ms": float(np.median(res_ms)),
            "resident_step_loci_per_s": visited / (float(np.median(res_ms)) * 1e-3),
            "config": {"workload": "somatic-standard, synthetic tumor/normal %gx/%gx, %s" % (tdepth, ndepth, workload),
                       "loci": L - 1, "visited_loci": visited, "tumor_reads": tg.n, "normal_reads": ng.n,
                       "somatic_rate": rate},
            "walker_tiles_frac": float(tm["walk_tiles"]) / max(1, int(tm["tiles"])),
            "device_stages_ms": {k: float(np.mean(v)) for k, v in stages.items() if k not in ("host_ms", "marshal_ms")},
            # the step's wall time beyond the device span: the C-ABI call's own host time (launch
            # gaps at its capacity checks, the results' D2H, sort and marshalling) and the ctypes
            # wrapping of the arrays
            "host_ms": {"call_wall_ms": float(np.mean(stages["host_ms"])),
                        "beyond_device_ms": float(np.mean(stages["host_ms"]) - np.mean(stages["total_ms"])),
                        "marshal_ms": float(np.mean(stages["marshal_ms"])),
                        "python_ms": float(np.median(res_ms)) - float(np.mean(stages["host_ms"]))},
            "caller": {"kernel": "somatic_call", "fast_ms": float(np.mean(stages["call_ms"])),
                       "deep_ms": float(np.mean(stages["deep_ms"])), "candidates": int(calls.candidate_loci),
                       "deep_candidates": int(tm["deep_loci"]), "deep_max_depth": int(tm["deep_max"]),
                       "ns_per_candidate": 1e6 * float(np.mean(stages["call_ms"])) / max(1, int(calls.candidate_loci))},
            "roofline": {"bound": "hbm", "kernel": som_kernel, "kernel_ms": k_ms, "achieved": ach,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "dram_frac": None if traffic is None else traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_launch": b_alg, "read_bytes_per_launch": read_bytes,
                         "traffic_source": None if traffic is None else pmc["source"]},
            "caller_roofline": caller_roofline(float(np.mean(stages["call_ms"])), pmc, "somatic_call_k<false,false"),
            "deep_caller_roofline": caller_roofline(float(np.mean(stages["deep_ms"])), pmc, "somatic_call_k<true,"),
            "candidate_loci": int(calls.candidate_loci), "calls": len(calls), "gen_s": gen_s,
            "parity_window": parity,
            # a cold call on resident reads: both sets' upload-time derivation + the first call
            # (the tumor's projection and margin projection; the normal needs neither)
            "one_shot": {"upload_derive_ms": derive_ms, "first_call_ms": cold_ms,
                         "first_call_device_ms": float(cold_tm["total_ms"]),
                         "tumor_projection_ms": float(st["proj_ms"]), "total_ms": derive_ms + cold_ms,
                         "loci_per_s": visited / ((derive_ms + cold_ms) * 1e-3)}}


class HbmPeak:
    """Device memory in use (hipMemGetInfo: total - free, every process's allocations on the
    GPU), sampled every 2 ms on a host thread between start() and stop(): the peak and the
    level at start."""

    def __init__(self, device: int = 0):
        import ctypes as C
        self.C = C
        self.hip = C.CDLL("libamdhip64.so.7")  # the HIP runtime the library already loaded
        self.hip.hipMemGetInfo.argtypes = [C.c_void_p, C.c_void_p]
        self.device = device
        self.peak = self.base = 0
        self._run = False
        self._th = None

    def used(self) -> int:
        C = self.C
        free, total = C.c_size_t(), C.c_size_t()
        if self.hip.hipMemGetInfo(C.byref(free), C.byref(total)) != 0:
            return 0
        return int(total.value - free.value)

    def start(self) -> "HbmPeak":
        import threading
        self.base = self.peak = self.used()
        self._run = True

        def poll():
            self.hip.hipSetDevice(self.device)
            while self._run:
                self.peak = max(self.peak, self.used())
                time.sleep(0.002)
        self._th = threading.Thread(target=poll, daemon=True)
        self._th.start()
        return self

    def stop(self) -> dict:
        self._run = False
        self._th.join()
        self.peak = max(self.peak, self.used())
        return {"peak_gb": self.peak / 1e9, "at_start_gb": self.base / 1e9, "peak_above_start_gb": (self.peak - self.base) / 1e9}


def configs3_rank_share(ctx, args, share_rank: int = 7, world: int = 8, margin: int = 5_000_000):
    """configs[3]'s per-GPU workload on this GPU, through the multi-GPU product path: rank
    `share_rank` of 8 in the 30x b37 genome split (genome_parts(8, wgs): ~392 M loci, ~78 M reads;
    rank 7 holds 65 contigs: 9's tail, the GL contigs, MT, X, Y, hs37d5).  Its reads, with `margin`
    loci of rank 6's share before them (so the plan must skip blocks), are written as one BGZF
    BAM (level 1) with the whole b37 dictionary; the rank's loci are planned through
    gq_bam_dev_plan (host probes: the file has no BAI) and decoded on the device with
    load_reads_device(region=...) as device_ingest_ranks does at world 8 (DistributedUtil.scala:
    584-597), then called over the rank's task of the 8-task partition; the result image is
    copied out as the gather would send it.  Peak device memory is sampled across ingest + call.
    A 2 Mb oracle window on contig X checks the records."""
    import shutil
    from guacamole_amd import synthetic
    from guacamole_amd.bamdev import load_reads_device
    from guacamole_amd.genomes import B37
    from guacamole_amd.loci import LociMapBuilder, LociSet
    from guacamole_amd.reads import InputFilters
    from oracle import oracle as O
    parts, genome_loci = genome_parts(world, True)
    mine = [p for p in parts if p[4] == share_rank]
    first = mine[0]
    pieces = merged_pieces(mine)
    gen_pieces = [(c, ln, max(0, s - margin) if c == first[0] else s, e) for c, ln, s, e in pieces]
    tmp = os.environ.get("TMPDIR", "/tmp")
    path = os.path.join(tmp, "gq_c3_%d.bam" % os.getpid())
    out = {"workload": "germline-threshold, rank %d of %d in the 30x b37 genome split (configs[3] per-GPU share)"
                       % (share_rank, world)}
    try:
        t = time.perf_counter()
        g = synthetic.generate_pieces(gen_pieces, args.depth, seed=synthetic.SEED + 4 + 1000 * share_rank)
        out["gen_s"] = time.perf_counter() - t
        x = next(p for p in pieces if p[0] == "X")
        w0 = x[2] + 50_000_000
        w1 = w0 + args.cpu_window
        win = synthetic.subset_pieces(g, gen_pieces, [("X", x[1], w0, w1)]).to_read_set()
        t = time.perf_counter()
        g.write_bam(path, level=1, dictionary=list(B37))
        out["bam_write_s"] = time.perf_counter() - t
        out["file_reads"] = g.n
        del g
        out["bam_bytes"] = os.path.getsize(path)
        b = LociMapBuilder()
        for c, _, s, e in pieces:
            b.put(c, int(s), int(e), 0)
        region = LociSet(b.result())
        filters = InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True)
        hbm = HbmPeak(ctx.device).start()
        t = time.perf_counter()
        rs = load_reads_device(ctx, path, filters, region=region)
        ingest_s = time.perf_counter() - t
        # the loader's buffers (~2.5x the share's inflated BAM) are released on a host thread;
        # their hipFree calls hold the HIP runtime, so the first call would wait for them: joined
        # here and reported as their own stage
        from guacamole_amd.bamdev import join_release_threads
        t = time.perf_counter()
        join_release_threads()
        release_s = time.perf_counter() - t
        cidx = rs.contig_index()
        loci = (np.array([cidx[p[0]] for p in mine], np.int32), np.array([p[2] for p in mine], np.int64),
                np.array([p[3] for p in mine], np.int64), np.array([p[4] for p in mine], np.int64))
        t = time.perf_counter()
        calls = ctx.germline_threshold_device(rs.reads, loci, args.threshold)
        call_ms = (time.perf_counter() - t) * 1e3
        call_tm = {k: v for k, v in ctx.timings().items() if isinstance(v, (int, float))}
        t = time.perf_counter()
        img = calls.to_host()
        image_ms = (time.perf_counter() - t) * 1e3
        mem = hbm.stop()
        warm = []  # the same call again (its buffers and code objects in place): the cold call's overhead
        for _ in range(3):
            t = time.perf_counter()
            ctx.germline_threshold_device(rs.reads, loci, args.threshold)
            warm.append((time.perf_counter() - t) * 1e3)
        st = ctx.proj_stats(rs.reads)
        tm = rs.timings
        wl = (np.array([cidx["X"]], np.int32), np.array([w0], np.int64), np.array([w1], np.int64),
              np.array([0], np.int64))
        gpu_win = ctx.germline_threshold(rs.reads, wl, args.threshold).tuples(rs.contig_names)
        want = O.germline_threshold(win, (np.array([0], np.int32),) + wl[1:], args.threshold)
        visited = int(calls.visited_loci)
        out.update({
            "loci": int(sum(p[3] - p[2] for p in mine)), "visited_loci": visited, "contigs": len(pieces),
            "reads": int(rs.n), "genome_loci": genome_loci,
            "stages_s": {"ingest": ingest_s, "loader_release": release_s, "call": call_ms / 1e3,
                         "result_image_d2h": image_ms / 1e3},
            "ingest": {k: tm.get(k) for k in ("map_ms", "h2d_ms", "inflate_ms", "records_ms", "parse_ms", "fill_ms",
                                              "derive_ms", "comp_bytes", "bam_bytes", "blocks", "max_span", "replans",
                                              "open_s", "scan_s", "total_s", "wall_s")},
            # the ingest stage against the loader's own clock: what lies outside load_reads_device's
            # last attempt (a replan's earlier loads, the DeviceReadSet wrapping)
            "ingest_unattributed_s": ingest_s - float(tm.get("total_s") or 0.0),
            "plan": {k: v for k, v in (tm.get("plan") or {}).items() if k != "segments"},
            "call_loci_per_s": visited / (call_ms * 1e-3),
            "call_device_ms": call_tm, "warm_call_ms": float(np.median(warm)),
            "warm_call_loci_per_s": visited / (float(np.median(warm)) * 1e-3),
            "projection_ms": float(st["proj_ms"]), "calls": len(img),
            "hbm": dict(mem, design_budget_gb={"load": 68, "calls": 47}),
            "parity_window": {"contig": "X", "loci": [w0, w1], "calls": len(want), "identical": gpu_win == want},
        })
        del rs, calls
    finally:
        if os.path.exists(path):
            os.remove(path)
    return out


def multi_rank_single_pass(args, g, pieces, rank: int, world: int, dist, barrier):
    """The N-rank CLI single pass over one BAM of the whole split genome: every rank writes the
    reads starting in its pieces as whole BGZF blocks, rank 0 joins the header, the pieces and
    the EOF block into one file, then every rank runs `germline-threshold --reads X.bam --out
    Y.vcf --parallelism N` in-process (commands.main over this job's process group):
    region-restricted device ingest of its share, the call, the gather of the result images to
    rank 0 over RCCL, rank 0's VCF.  Timed between barriers, the max over ranks; per-rank stage
    times from the command's stage clock."""
    import shutil
    from guacamole_amd import commands, synthetic
    from guacamole_amd.distributed import all_gather_objects
    from guacamole_amd.genomes import B37
    tmp = os.environ.get("TMPDIR", "/tmp")
    job = os.environ.get("TORCHELASTIC_RUN_ID", "job") + "_" + os.environ.get("MASTER_PORT", "0")
    seg = os.path.join(tmp, "gq_mp_%s_%d.bgzf" % (job, rank))
    bam = os.path.join(tmp, "gq_mp_%s.bam" % job)
    out = os.path.join(tmp, "gq_mp_%s.vcf" % job)
    try:
        t = time.perf_counter()
        synthetic.subset_pieces(g, pieces, pieces, starts_in=True).write_bam(seg, level=1, dictionary=list(B37),
                                                                                flags=0, name_base=rank * 10 ** 10)
        barrier()
        if rank == 0:
            synthetic.write_bam_header(bam, list(B37))
            with open(bam, "ab") as fo:
                for r in range(world):
                    with open(os.path.join(tmp, "gq_mp_%s_%d.bgzf" % (job, r)), "rb") as fi:
                        shutil.copyfileobj(fi, fo, 64 << 20)
                fo.write(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
        barrier()
        write_s = time.perf_counter() - t
        os.remove(seg)
        t = time.perf_counter()
        rc = commands.main(["germline-threshold", "--reads", bam, "--out", out, "--parallelism", str(world)])
        barrier()
        wall = time.perf_counter() - t
        import torch
        x = torch.tensor([wall], dtype=torch.float64, device="cuda" if os.environ.get("GQ_DIST_BACKEND", "nccl") ==
                         "nccl" else "cpu")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        stages = all_gather_objects(commands.LAST_TIMING)
        if rank != 0:
            return None
        genotypes = stages[0].get("genotypes") if stages[0] else None
        return {"wall_s": float(x.item()), "rc": rc, "bam_bytes": os.path.getsize(bam), "bam_write_s": write_s,
                "genotypes": genotypes, "per_rank_stages_s": stages,
                "command": "torch.distributed.run --nproc-per-node %d: germline-threshold --reads <genome>.bam "
                           "--out <out>.vcf --parallelism %d (in the bench's ranks)" % (world, world)}
    finally:
        if os.path.exists(seg):
            os.remove(seg)
        if rank == 0:
            if os.path.exists(bam):
                os.remove(bam)
            shutil.rmtree(out, ignore_errors=True)



def somatic_parity_window(ctx, t, n, tg, ng, L: int, width: int):
    """The CPU oracle's somatic-standard records (CLI defaults) on loci [L / 3, L / 3 + width) of
    the same shard against the GPU's over the same loci: every field, FP64 likelihoods, log-odds
    and evidence included, bit for bit (NaN = NaN)."""
    import math
    from oracle import oracle as O
    w0 = L // 3
    w1 = min(L - 1, w0 + width)
    loci = (np.array([0], np.int32), np.array([w0], np.int64), np.array([w1], np.int64), np.array([0], np.int64))
    got = ctx.somatic_standard(t, n, loci).rows
    ts, ns = tg.to_read_set(tg.window(w0, w1)), ng.to_read_set(ng.window(w0, w1))
    c0 = time.perf_counter()
    want = O.somatic_standard(ts, ns, loci)
    cpu_s = time.perf_counter() - c0

    def same(a, b):
        if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
            return True
        if isinstance(a, tuple):
            return len(a) == len(b) and all(same(x, y) for x, y in zip(a, b))
        return a == b
    names = tg.contig_names
    ok = len(got) == len(want) and all(
        all(same(g[k] if k != "contig" else names[g[k]], w[k]) for k in w) for g, w in zip(got, want))
    return {"loci": [w0, w1], "calls": len(want), "identical": bool(ok), "oracle_s": cpu_s}


SOMATIC_PMC = os.path.join(ROOT, "profiles", "somatic_pmc_r06.json")


def somatic_pmc(workload: str, L: int, tdepth: float, ndepth: float):
    """The PMC summary of the same somatic workload (scripts/profile_somatic.sh +
    scripts/pmc_somatic.py), or None when none was taken at this size."""
    try:
        with open(SOMATIC_PMC) as fh:
            w = json.load(fh).get(workload)
    except (OSError, ValueError):
        return None
    if not w or w.get("length") != L or w.get("tumor_depth") != tdepth or w.get("normal_depth") != ndepth:
        return None
    return w


def caller_roofline(call_ms: float, pmc, kernel: str):
    """An exact somatic caller (somatic_call_k<false>, or <true> over the deep list) is FP64 VALU
    work behind dependent loads.  Its issue roofline: VALU wave-instructions per launch (PMC of the
    same workload, SOMATIC_PMC) over this run's kernel time, against the chip's VALU issue rate
    (1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction, the convention of DESIGN.md's PMC
    readings); the wait share says what bounds it instead."""
    if pmc is None or call_ms <= 0:
        return None
    # the PMC file names kernels with their template arguments: "somatic_call_k<false, false, 3>"
    kernel, pm = next(((k, v) for k, v in sorted(pmc["kernels"].items())
                       if k.replace(" ", "").startswith(kernel.rstrip(">"))), (kernel, {}))
    insts = pm.get("SQ_INSTS_VALU")
    if not insts:
        return None
    peak = 1024 * 2.4e9 / 2
    ach = insts / (call_ms * 1e-3)
    return {"bound": "issue/latency", "kernel": kernel, "kernel_ms": call_ms,
            "valu_wave_insts_per_launch": insts, "achieved": ach, "peak": peak, "unit": "wave-instr/s",
            "frac": ach / peak,
            "wait_frac": pm.get("SQ_WAIT_ANY", 0.0) / max(1.0, pm.get("SQ_WAVE_CYCLES", 1.0)),
            "hbm_bytes_per_launch": pm.get("hbm_bytes_per_launch"),
            "source": pmc["source"]}


if __name__ == "__main__":
    sys.exit(main())
