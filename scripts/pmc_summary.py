#!/usr/bin/env python3
"""Per-kernel means of every PMC counter in a profile directory's passes.

  python scripts/pmc_summary.py <profdir> [kernel-regex] [--csv out.csv]
"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    d = sys.argv[1]
    kre = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "."
    out = sys.argv[sys.argv.index("--csv") + 1] if "--csv" in sys.argv else None
    v = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(p)):
            k = row["Kernel_Name"]
            if re.search(kre, k):
                k = k.replace("(anonymous namespace)::", "")
                v[k.split("(")[0][-60:]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    rows = []
    for k, cs in v.items():
        for c, x in sorted(cs.items()):
            rows.append((k, c, sum(x) / len(x), len(x)))
            print("%-60s %-22s %14.4g  (%d)" % (k, c, sum(x) / len(x), len(x)))
    if out:
        with open(out, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["kernel", "counter", "mean_per_launch", "launches"])
            w.writerows(rows)


if __name__ == "__main__":
    main()
