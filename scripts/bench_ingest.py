#!/usr/bin/env python3
"""Host ingest measurement: BAM -> the gq_reads SoA through libgqingest.

  python scripts/bench_ingest.py [--length L] [--depth D] [--reps R] [--out profiles/r01_ingest.json]

1. Synthetic reads (native generator, the bench's model) for one contig of L loci at depth D,
   written as a coordinate-sorted BGZF BAM (level 6, libgqsynth's writer).
2. Native load (reads.load_reads -> ingest.load_bam: open + parallel inflate, parallel
   decode + filters, fill) and the MD-event parse (soa.pack -> gq_md_count / gq_md_fill),
   best of R runs, with the germline caller's filters (overlapsLoci all, nonDuplicate, hasMdTag).
3. Round trip at full size: the loaded arrays and MD events equal the generator's (start,
   end, mapq, strand, bases, qualities, CIGAR, MD events) — a size-independent parity check.
4. The Python statement of the same loader (reads._load_bam_py, the test checker) on a
   bounded sample BAM, for the per-read rate beside the native one.
Prints one JSON line (and writes it to --out).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from guacamole_amd import ingest, soa, synthetic  # noqa: E402
from guacamole_amd.loci import LociSet  # noqa: E402
from guacamole_amd.reads import InputFilters, _load_bam_py, load_reads  # noqa: E402


def gather(off, ln, pool):
    ln = np.asarray(ln, np.int64)
    tot = int(ln.sum())
    if tot == 0:
        return pool[:0]
    base = np.concatenate([[0], np.cumsum(ln)[:-1]])
    return pool[np.repeat(np.asarray(off, np.int64) - base, ln) + np.arange(tot)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--length", type=int, default=20_000_000)
    ap.add_argument("--depth", type=float, default=30.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sample-length", type=int, default=100_000)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    g = synthetic.generate(args.length, args.depth)
    path = os.path.join(args.dir, "gq_ingest_%d_%g.bam" % (args.length, args.depth))
    t = time.perf_counter()
    g.write_bam(path)
    write_s = time.perf_counter() - t
    bam_bytes = os.path.getsize(path)
    filters = InputFilters.make(overlaps_loci=LociSet.parse("all"), non_duplicate=True, has_md_tag=True)

    best = None
    for _ in range(args.reps):
        tm = {}
        t0 = time.perf_counter()
        rs = ingest.load_bam(path, filters, tm)
        t1 = time.perf_counter()
        rs._gq = None
        p = soa.pack(rs)
        t2 = time.perf_counter()
        run = dict(load_s=t1 - t0, md_events_s=t2 - t1, total_s=t2 - t0, **tm)
        if best is None or run["total_s"] < best["total_s"]:
            best = run
    raw = int(rs.seq.size * 2 + rs.cigar.size * 4 + rs.md.size + rs.n * 36)

    # round trip against the generator (reads with an end inside the contig's "all" loci)
    a = g.arrays
    keep = np.nonzero(a["end"] > 0)[0]
    if args.length - 1 < int(a["start"].max(initial=0)) + 1:  # "all" drops the contig's last base
        keep = keep[a["start"][keep] < args.length - 1]
    ok = (rs.n == len(keep)
          and np.array_equal(rs.start, a["start"][keep].astype(np.int64))
          and np.array_equal(rs.end, a["end"][keep].astype(np.int64))
          and np.array_equal(rs.mapq, a["mapq"][keep]) and np.array_equal(rs.flags, a["flags"][keep] & 1)
          and np.array_equal(rs.seq, gather(a["seq_off"][keep], a["seq_len"][keep], a["seq"]))
          and np.array_equal(rs.qual, gather(a["seq_off"][keep], a["seq_len"][keep], a["qual"]))
          and np.array_equal(rs.cigar, gather(a["cigar_off"][keep], a["n_cigar"][keep], a["cigar"]))
          and np.array_equal(p["n_md"], a["n_md"][keep])
          and np.array_equal(p["md_ev"], gather(a["md_off"][keep], np.maximum(a["n_md"][keep], 0), a["md_ev"])))

    # the Python statement on a bounded sample
    gs = synthetic.generate(args.sample_length, args.depth)
    spath = os.path.join(args.dir, "gq_ingest_sample_%d.bam" % args.sample_length)
    gs.write_bam(spath)
    t = time.perf_counter()
    py = _load_bam_py(spath, filters)
    py_s = time.perf_counter() - t
    t = time.perf_counter()
    nat = load_reads(spath, filters)
    nat_s = time.perf_counter() - t
    assert nat.n == py.n
    line = {
        "metric": "BAM ingest reads/s (BGZF inflate + decode + filters + MD events)",
        "value": rs.n / best["total_s"], "unit": "reads/s",
        "bam_MB_per_s": bam_bytes / best["load_s"] / 1e6, "record_MB_per_s": raw / best["load_s"] / 1e6,
        "threads": best["threads"], "reads": rs.n, "bam_bytes": bam_bytes, "best_of": args.reps,
        "stages_s": {k: round(v, 4) for k, v in best.items() if k.endswith("_s")},
        "config": {"length": args.length, "depth": args.depth, "read_len": 150, "bgzf_level": 6,
                   "filters": "overlapsLoci(all) + nonDuplicate + hasMdTag (germline-threshold)"},
        "roundtrip_identical": bool(ok),
        "python_statement": {"reads": py.n, "s": py_s, "reads_per_s": py.n / py_s, "native_s": nat_s,
                             "sample": "synthetic %d loci at %gx" % (args.sample_length, args.depth)},
        "write_s": write_s,
    }
    s = json.dumps(line)
    print(s)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(s + "\n")
    os.remove(path)
    os.remove(spath)
    if not ok:
        sys.exit("round trip differs")


if __name__ == "__main__":
    main()
