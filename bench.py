#!/usr/bin/env python3
"""bench.py — pileup loci/s for germline-threshold on synthetic 30x reads (BASELINE.json configs[1]).

A "step" = one germline-threshold pass (gq_germline_threshold_device: tile planning, the
column pileup kernel, the walker and general-allele kernels, record sort, the result image
built in HBM) over every locus of the rank's shard, reads already resident in HBM, plus
(N > 1) the terminal RCCL gather of the per-rank result images to rank 0 over xGMI.  The
PCIe copy of the results to the host (gq_germline_threshold) is not part of `value`; its
rate is reported beside it as host_results_loci_per_s.

Workload per GPU: one chr20-sized contig (63,025,520 loci, b37 length —
T/DistributedUtilSuite.scala:72), 30x, L = 150, seed 20261015 + 2 (+ rank).
`--gpus N` under torch.distributed.run gives each rank its own chr20-sized
shard (weak scaling; the static LociSet split of a WGS run).

Also reported:
  roofline     the pileup (column) kernel's algorithmic bytes / its HIP-event time vs 8 TB/s
  cpu_baseline the CPU oracle (single-threaded restatement) on a bounded window of
               the same workload; its calls are also compared to the GPU's on that
               window (parity_window).
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
HBM_PEAK_GBS = 8000.0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--length", type=int, default=CHR20, help="loci per GPU shard")
    ap.add_argument("--depth", type=float, default=30.0)
    ap.add_argument("--threshold", type=int, default=8)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--cpu-window", type=int, default=4_000_000, help="loci in the CPU-oracle sample window")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_r01.json"),
                    help="PMC-derived HBM bytes per pileup launch (from a separate rocprofv3 --pmc pass)")
    args = ap.parse_args()

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
    g = synthetic.generate(args.length, args.depth, seed=synthetic.SEED + 2 + rank)
    gen_s = time.time() - t0
    ctx = native.Context(local)
    if args.tile:
        ctx.set_tile(args.tile)
    reads = ctx.upload(g.arrays)
    # loci "all" on the shard's contig: [0, length - 1) (LociSet.scala:205-207)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([args.length - 1], np.int64),
            np.array([0], np.int64))

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    def step():
        calls = ctx.germline_threshold_device(reads, loci, args.threshold)
        if dist is not None:
            gather_images_to_rank0(calls, gather_dev)
        return calls

    for _ in range(args.warmup):
        step()
    barrier()
    pileup_ms, walk_ms, total_ms, host_ms, marshal_ms = [], [], [], [], []
    stage_ms = {"plan_ms": [], "complex_ms": [], "finalize_ms": []}
    walk_frac = []
    t = time.perf_counter()
    for _ in range(args.steps):
        calls = step()
        tm = ctx.timings()
        pileup_ms.append(tm["pileup_ms"])
        walk_ms.append(tm["walk_ms"])
        for k in stage_ms:
            stage_ms[k].append(tm[k])
        walk_frac.append(tm["walk_tiles"] / max(1, tm["tiles"]))
        total_ms.append(tm["total_ms"])
        host_ms.append(tm["host_ms"])
        marshal_ms.append(tm["marshal_ms"])
    barrier()
    elapsed = time.perf_counter() - t
    if dist is not None:
        import torch
        x = torch.tensor([elapsed], dtype=torch.float64, device="cuda:%d" % local)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        elapsed = float(x.item())
    visited = int(calls.visited_loci)
    loci_total = visited * world
    # the same pass with the records copied to the host (PCIe-inclusive), a few steps, rank-local
    hc = ctx.germline_threshold(reads, loci, args.threshold)  # warm-up of the host-block path
    n_host = 5
    t = time.perf_counter()
    for _ in range(n_host):
        hc = ctx.germline_threshold(reads, loci, args.threshold)
    host_ms_step = (time.perf_counter() - t) / n_host * 1e3
    assert len(hc) == len(calls)

    # ---- roofline for the pileup kernel (germline_cols): algorithmic bytes per launch.  The
    #      column kernel counts every tile except the few it hands to the walker kernel
    #      (walk_tiles: reads it cannot stage or count), so its share of the bytes is the
    #      tiles it kept.
    a = g.arrays
    n_reads = int(a["start"].shape[0])
    bytes_seq = int(a["seq"].shape[0])            # 1 B per aligned/inserted base (no qualities: not read by this caller)
    bytes_meta = 16 * n_reads                     # start/end/offsets/counts/flags minimum per read
    bytes_cigar = 4 * int(a["cigar"].shape[0])
    bytes_md = 4 * int(a["md_ev"].shape[0])
    bytes_out = 32 * len(calls) + 8 * int(calls.complex_loci)
    b_all = bytes_seq + bytes_meta + bytes_cigar + bytes_md + bytes_out
    kept = 1.0 - float(np.mean(walk_frac))
    b_alg = int(b_all * kept)
    k_ms = float(np.mean(pileup_ms))
    achieved = b_alg / (k_ms * 1e-3) / 1e9
    traffic = None
    try:
        with open(args.traffic) as fh:
            tr = json.load(fh)
        if tr.get("length") == args.length and tr.get("depth") == args.depth:
            traffic = tr.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

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
        "config": {"workload": "germline-threshold, synthetic 30x chr20-length shard per GPU (configs[1])",
                   "loci_per_gpu": args.length - 1, "visited_loci_per_gpu": visited, "reads_per_gpu": n_reads,
                   "depth": args.depth, "read_len": 150, "threshold": args.threshold,
                   "parallelism": "loci-sharded x%d" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "germline_cols", "kernel_ms": k_ms, "algorithmic_bytes_per_launch": b_alg,
                     "tiles_kept": kept, "walker_ms": float(np.mean(walk_ms))},
        "kernel_only_loci_per_s": visited / ((k_ms + float(np.mean(walk_ms))) * 1e-3),
        "device_total_ms": float(np.mean(total_ms)),
        "device_stages_ms": {k: float(np.mean(v)) for k, v in stage_ms.items()},
        "host_results_loci_per_s": visited / (host_ms_step * 1e-3),
        "host_results_ms_per_step": host_ms_step,
        "host_call_ms": float(np.mean(host_ms)),
        "host_marshal_ms": float(np.mean(marshal_ms)),
        "calls": len(calls),
        "complex_loci": int(calls.complex_loci),
        "ambiguous_loci": int(calls.ambiguous_loci),
        "gen_s": gen_s,
    }

    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"], line["parity_window"] = cpu_baseline(g, ctx, reads, args)
    if rank == 0:
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()
    return 0


def cpu_baseline(g, ctx, reads, args):
    """Single-threaded CPU oracle on a window of the same workload, timed; its calls
    are compared with the GPU's calls over the same loci window."""
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
    return ({"value": visited / cpu_s, "unit": "loci/s", "cores": 1, "kind": "port",
             "sample": "CPU oracle (oracle/oracle.cpp, 1 thread, not the JVM reference) on loci [%d, %d) of the "
                       "same synthetic shard: %d visited loci, %d reads, %.1f s" % (w0, w1, visited, len(idx), cpu_s)},
            {"loci": [w0, w1], "calls": len(want), "identical": bool(parity)})


if __name__ == "__main__":
    sys.exit(main())
