#!/usr/bin/env python3
"""Median duration per kernel from a rocprofv3 kernel-trace CSV (robust to one outsized call)."""
import csv
import glob
import statistics
import sys
f = sys.argv[1]
if not f.endswith(".csv"):
    f = glob.glob(f + "/**/run_kernel_trace.csv", recursive=True)[0]
d = {}
for row in csv.DictReader(open(f)):
    d.setdefault(row["Kernel_Name"], []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
    print("%-60s n %4d med_us %9.1f min_us %9.1f max_us %9.1f" % (k[:60], len(v), statistics.median(v), min(v), max(v)))
