#!/usr/bin/env python3
"""Turn a scripts/profile_somatic.sh output directory into committed profile files.

  python scripts/pmc_somatic.py <profdir> <tag> --workload chr1|panel --length L \
      --tumor-depth T --normal-depth N --round r04

writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary of the trace pass
  profiles/<tag>_pmc.csv            per-kernel averages of every PMC counter collected
  profiles/somatic_pmc_<round>.json  per workload and kernel: the counters, and for each kernel
                                    with FETCH_SIZE and WRITE_SIZE its HBM bytes per launch
                                    (read by bench.py for somatic.roofline.traffic and the
                                    caller rooflines)

HBM bytes as scripts/pmc_traffic.py: FETCH_SIZE (KiB) doubled per the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md, WRITE_SIZE (KiB) as is, separate passes.
"""
import argparse
import csv
import json
import os
import re
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_key(name: str) -> str:
    """'void (anonymous namespace)::somatic_call_k<false>(...)' -> 'somatic_call_k<false>'."""
    m = re.search(r"([A-Za-z_][A-Za-z0-9_]*(<[^>(]*>)?)\(", name)
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("profdir")
    ap.add_argument("tag")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--length", type=int, required=True)
    ap.add_argument("--tumor-depth", type=float, required=True)
    ap.add_argument("--normal-depth", type=float, required=True)
    ap.add_argument("--round", required=True)
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(a.profdir, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, "%s_kernel_stats.csv" % a.tag))
    vals = defaultdict(lambda: defaultdict(list))
    for sub in sorted(os.listdir(a.profdir)):
        p = os.path.join(a.profdir, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        with open(p) as fh:
            for row in csv.DictReader(fh):
                vals[kernel_key(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    pm = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
    with open(os.path.join(prof, "%s_pmc.csv" % a.tag), "w") as fh:
        fh.write("kernel,counter,mean_per_launch\n")
        for k in sorted(pm):
            for c in sorted(pm[k]):
                fh.write("%s,%s,%.1f\n" % (k, c, pm[k][c]))
    for k, cs in pm.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            cs["hbm_bytes_per_launch"] = cs["FETCH_SIZE"] * 1024 * 2 + cs["WRITE_SIZE"] * 1024
    out_p = os.path.join(prof, "somatic_pmc_%s.json" % a.round)
    doc = {}
    if os.path.exists(out_p):
        with open(out_p) as fh:
            doc = json.load(fh)
    doc[a.workload] = {"length": a.length, "tumor_depth": a.tumor_depth, "normal_depth": a.normal_depth,
                       "source": "profiles/%s_pmc.csv" % a.tag, "kernels": pm,
                       "correction": "FETCH_SIZE x2 (gfx950), KiB->bytes; WRITE_SIZE as is"}
    with open(out_p, "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=True)
    print(json.dumps(doc[a.workload], sort_keys=True)[:2000])


if __name__ == "__main__":
    main()
