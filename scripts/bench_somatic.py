#!/usr/bin/env python3
"""somatic-standard throughput on synthetic tumor/normal reads (BASELINE.json configs[2] shape).

  python scripts/bench_somatic.py [--length L] [--steps K] [--warmup W] [--out FILE]

Tumor 60x with somatic SNVs (rate 2e-4, VAF U(0.1, 0.5)) and normal 30x from the bench's
generator over one contig of L loci (default: a chr20-length shard; configs[2] names chr1,
249,250,621 loci, which --length 249250621 runs when the host has the memory), reads resident
in HBM.  A step is one gq_somatic_standard call with the CLI defaults (driver filters on).
Reports loci/s (visited loci), the per-stage device times (candidate pileup kernel, the
per-candidate FP64 caller, finalize), the candidate count, and the calls' identity with
the CPU oracle on a bounded window (--cpu-window loci).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHR20 = 63_025_520


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--length", type=int, default=CHR20)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--tumor-depth", type=float, default=60.0)
    ap.add_argument("--normal-depth", type=float, default=30.0)
    ap.add_argument("--somatic-rate", type=float, default=2e-4)
    ap.add_argument("--cpu-window", type=int, default=200_000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--rederive", action="store_true", help="re-derive both read sets every step")
    args = ap.parse_args()

    from guacamole_amd import native, synthetic
    t0 = time.time()
    seed = synthetic.SEED + 3
    tg = synthetic.generate(args.length, args.tumor_depth, seed=seed, somatic_rate=args.somatic_rate, tumor=True,
                            read_seed=11)
    ng = synthetic.generate(args.length, args.normal_depth, seed=seed, somatic_rate=args.somatic_rate, tumor=False,
                            read_seed=12)
    gen_s = time.time() - t0
    ctx = native.Context(0)
    t = ctx.upload(tg.arrays)
    n = ctx.upload(ng.arrays)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([args.length - 1], np.int64),
            np.array([0], np.int64))
    def step():
        if args.rederive:
            ctx.rederive(t)
            ctx.rederive(n)
        return ctx.somatic_standard(t, n, loci)
    for _ in range(args.warmup):
        step()
    stages = {"pileup_ms": [], "complex_ms": [], "finalize_ms": [], "total_ms": []}
    t1 = time.perf_counter()
    for _ in range(args.steps):
        calls = step()
        tm = ctx.timings()
        for k in stages:
            stages[k].append(tm[k])
    el = time.perf_counter() - t1
    visited = int(calls.visited_loci)
    line = {
        "metric": "somatic-standard loci/sec, tumor %gx / normal %gx" % (args.tumor_depth, args.normal_depth),
        "value": visited * args.steps / el,
        "unit": "loci/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * el / args.steps,
        "dtype": "u8 counts + f64 likelihoods",
        "data": "synthetic (native generator, somatic SNV rate %g)" % args.somatic_rate,
        "config": {"workload": "somatic-standard, synthetic tumor/normal %gx/%gx, %d loci" % (
                       args.tumor_depth, args.normal_depth, args.length),
                   "tumor_reads": tg.n, "normal_reads": ng.n, "visited_loci": visited},
        "device_stages_ms": {k: float(np.mean(v)) for k, v in stages.items()},
        "candidate_loci": int(calls.candidate_loci),
        "calls": len(calls), "gen_s": gen_s,
    }
    # the CPU oracle on a bounded window, and identity of the calls there
    if args.cpu_window > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from guacamole_amd.commands import somatic_standard_reads
        from guacamole_amd.loci import LociSet, flatten_partitions, partition_loci_uniformly
        from oracle import oracle as O
        from test_gpu_somatic import assert_rows_match
        w0 = args.length // 3 if args.length > 3 * args.cpu_window else 0
        w1 = min(args.length - 1, w0 + args.cpu_window)
        sel_t, sel_n = tg.window(w0, w1), ng.window(w0, w1)
        rt, rn = tg.to_read_set(sel_t), ng.to_read_set(sel_n)
        ls = LociSet.parse("%s:%d-%d" % (rt.contig_names[0], w0, w1)).result(rt.contig_lengths_map)
        wl = flatten_partitions(partition_loci_uniformly(1, ls), rt.contig_index())
        c0 = time.perf_counter()
        want = O.somatic_standard(rt, rn, wl, apply_filters=1)
        cpu_s = time.perf_counter() - c0
        got = somatic_standard_reads(ctx, rt, rn, wl, apply_filters=1)
        assert_rows_match(got, want)
        line["cpu_baseline"] = {"value": (w1 - w0) / cpu_s, "unit": "loci/s", "cores": 1, "kind": "port",
                                "sample": "CPU oracle on loci [%d, %d): %d calls, %.1f s" % (w0, w1, len(want), cpu_s)}
        line["parity_window"] = {"loci": [w0, w1], "calls": len(want), "identical": True}
    s = json.dumps(line)
    print(s)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
