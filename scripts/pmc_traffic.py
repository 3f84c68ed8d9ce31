#!/usr/bin/env python3
"""Turn a scripts/profile_germline.sh output directory into the committed profile files.

  python scripts/pmc_traffic.py <profdir> <tag> --length L --depth D

writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary of the trace pass
  profiles/<tag>_pmc.csv            per-kernel averages of every PMC counter collected
  profiles/traffic_<round>.json     HBM bytes per pileup-kernel launch (read by bench.py)

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
come from separate --pmc passes (they cannot share one on gfx950), both in KiB; on gfx950
FETCH_SIZE counts half the bytes of 16-byte-per-lane reads, so it is doubled; WRITE_SIZE
is taken as is.
"""
import argparse
import csv
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter_means(path, kernel_sub):
    vals = defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if kernel_sub in row["Kernel_Name"]:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("profdir")
    ap.add_argument("tag")
    ap.add_argument("--length", type=int, required=True)
    ap.add_argument("--depth", type=float, required=True)
    ap.add_argument("--kernel", default="germline_proj")
    ap.add_argument("--round", required=True)
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(a.profdir, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, "%s_kernel_stats.csv" % a.tag))
    pm = {}
    for sub in ("fetch", "write", "sq1", "sq2"):
        p = os.path.join(a.profdir, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            pm.update(counter_means(p, a.kernel))
    with open(os.path.join(prof, "%s_pmc.csv" % a.tag), "w") as fh:
        fh.write("kernel,counter,mean_per_launch\n")
        for k in sorted(pm):
            fh.write("%s,%s,%.1f\n" % (a.kernel.rstrip("<"), k, pm[k]))
    if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm:
        fetch = pm["FETCH_SIZE"] * 1024 * 2
        write = pm["WRITE_SIZE"] * 1024
        out = {"kernel": a.kernel.rstrip("<"), "length": a.length, "depth": a.depth,
               "hbm_bytes_per_launch": fetch + write, "fetch_bytes_corrected": fetch, "write_bytes": write,
               "raw_FETCH_SIZE_KiB": pm["FETCH_SIZE"], "raw_WRITE_SIZE_KiB": pm["WRITE_SIZE"],
               "correction": ("FETCH_SIZE x2 (gfx950 tallies the kernel's 128-B coalesced requests at 64 B: raw "
                              "FETCH_SIZE is below the launch's compulsory read bytes), KiB->bytes; WRITE_SIZE as is"),
               "source": "profiles/%s_pmc.csv" % a.tag}
        with open(os.path.join(prof, "traffic_%s.json" % a.round), "w") as fh:
            json.dump(out, fh, indent=1)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
