#!/usr/bin/env python3
"""Load one synthetic BAM through the device loader (for rocprof passes on bgzf_inflate).
  python scripts/inflate_probe.py [--length L]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from guacamole_amd import bamdev, native, synthetic
    from guacamole_amd.reads import InputFilters
    ap = argparse.ArgumentParser()
    ap.add_argument("--length", type=int, default=10_000_000)
    a = ap.parse_args()
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "gq_probe_%d.bam" % os.getpid())
    synthetic.generate(a.length, 30.0).write_bam(path)
    try:
        ctx = native.Context(0)
        t = time.perf_counter()
        d = bamdev.load_reads_device(ctx, path, InputFilters())
        print("load_s", time.perf_counter() - t, d.timings, flush=True)
    finally:
        os.remove(path)


if __name__ == "__main__":
    main()
