#!/usr/bin/env python3
"""Per-shape FETCH_SIZE / WRITE_SIZE correction factors from scripts/calib/calib.sh's output:
known bytes (each byte of the 1 GiB buffer touched once in that shape) / counter bytes.
Writes <outdir>/calibration.json (copied to profiles/ by hand for the round)."""
import csv
import glob
import json
import os
import re
import sys


def counters(d, name):
    out = {}
    for p in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(p)):
            if row["Counter_Name"] != name:
                continue
            k = re.match(r"[A-Za-z_0-9]+", row["Kernel_Name"]).group(0)
            out.setdefault(k, []).append(float(row["Counter_Value"]) * 1024)  # KiB -> bytes
    return {k: sum(v) / len(v) for k, v in out.items()}


def main(d):
    times = {}
    for line in open(os.path.join(d, "calib_times.jsonl")):
        r = json.loads(line)
        times[r["kernel"]] = r
    f, w = counters(os.path.join(d, "fetch"), "FETCH_SIZE"), counters(os.path.join(d, "write"), "WRITE_SIZE")
    out = {}
    for k, r in times.items():
        wr = k.startswith("wr_")
        got = (w if wr else f).get(k)
        out[k] = {"known_bytes": r["bytes"], "counter": "WRITE_SIZE" if wr else "FETCH_SIZE", "counter_bytes": got,
                  "factor": None if not got else r["bytes"] / got, "best_ms": r["best_ms"], "gbs": r["gbs"],
                  "other_counter_bytes": (f if wr else w).get(k)}
    res = {"source": "scripts/calib/calib_fetch.hip (1 GiB buffer, each byte once per shape)", "shapes": out}
    with open(os.path.join(d, "calibration.json"), "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, v in out.items():
        print("%-12s factor %s  (%s %.3e of %.3e B)  %.0f GB/s" % (k, v["factor"] and round(v["factor"], 3), v["counter"],
                                                                 v["counter_bytes"] or 0, v["known_bytes"], v["gbs"]))


if __name__ == "__main__":
    main(sys.argv[1])
