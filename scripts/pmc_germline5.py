#!/usr/bin/env python3
"""Turn a scripts/profile_germline5.sh output directory into committed profile files.

  python scripts/pmc_germline5.py <profdir> <tag> --length L --depth D --round r05

writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary of the trace pass
  profiles/<tag>_kernel_trace_medians.txt   per-kernel median / min / max of the trace pass
  profiles/<tag>_pmc.csv            per-kernel means of every PMC counter collected
  profiles/traffic_<round>.json     per kernel: HBM bytes per launch (read by bench.py)

HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE from
separate --pmc passes, both in KiB; FETCH_SIZE doubled (the guide's gfx950 correction, calibrated
there for 16-byte-per-lane reads; these kernels load 8 bytes per lane, so the absolute is
uncalibrated: ratios between variants hold), WRITE_SIZE as is.
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import statistics
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_key(name: str) -> str:
    m = re.search(r"([A-Za-z_][A-Za-z0-9_]*(<[^>(]*>)?)\(", name)
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("profdir")
    ap.add_argument("tag")
    ap.add_argument("--length", type=int, required=True)
    ap.add_argument("--depth", type=float, required=True)
    ap.add_argument("--round", required=True)
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(glob.glob(os.path.join(a.profdir, "trace", "**", "run_kernel_stats.csv"), recursive=True)[0],
                os.path.join(prof, "%s_kernel_stats.csv" % a.tag))
    trace = glob.glob(os.path.join(a.profdir, "trace", "**", "run_kernel_trace.csv"), recursive=True)[0]
    d = defaultdict(list)
    for row in csv.DictReader(open(trace)):
        d[kernel_key(row["Kernel_Name"])].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    with open(os.path.join(prof, "%s_kernel_trace_medians.txt" % a.tag), "w") as fh:
        for k, v in sorted(d.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
            fh.write("%-44s n %4d med_us %10.1f min_us %10.1f max_us %10.1f\n" % (k[:44], len(v), statistics.median(v),
                                                                                 min(v), max(v)))
    vals = defaultdict(lambda: defaultdict(list))
    for p in glob.glob(os.path.join(a.profdir, "pmc*", "**", "run_counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(p)):
            vals[kernel_key(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    pm = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    with open(os.path.join(prof, "%s_pmc.csv" % a.tag), "w") as fh:
        fh.write("kernel,counter,mean_per_launch\n")
        for k in sorted(pm):
            for c in sorted(pm[k]):
                fh.write("%s,%s,%.1f\n" % (k, c, pm[k][c]))
    kern = {}
    for k, cs in pm.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            kern[k] = {"hbm_bytes_per_launch": cs["FETCH_SIZE"] * 1024 * 2 + cs["WRITE_SIZE"] * 1024,
                       "fetch_bytes_corrected": cs["FETCH_SIZE"] * 1024 * 2, "write_bytes": cs["WRITE_SIZE"] * 1024,
                       "raw_FETCH_SIZE_KiB": cs["FETCH_SIZE"], "raw_WRITE_SIZE_KiB": cs["WRITE_SIZE"]}
    out = {"length": a.length, "depth": a.depth, "kernels": kern, "source": "profiles/%s_pmc.csv" % a.tag,
           "correction": "FETCH_SIZE x2 (gfx950, calibrated for 16-B-per-lane reads), KiB->bytes; WRITE_SIZE as is"}
    with open(os.path.join(prof, "traffic_%s.json" % a.round), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, sort_keys=True)[:3000])


if __name__ == "__main__":
    main()
