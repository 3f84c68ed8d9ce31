#!/usr/bin/env python3
"""Turn a scripts/profile_germline6.sh output directory into committed profile files, with the
round-6 per-shape FETCH_SIZE calibration (profiles/r06_pmc_calibration.json).

  python scripts/pmc_germline6.py <profdir> <tag> --length L --depth D --round r06

writes
  profiles/<tag>_kernel_stats.csv          rocprofv3 --stats summary of the trace pass
  profiles/<tag>_kernel_trace_medians.txt  per-kernel median / min / max of the trace pass
  profiles/<tag>_pmc.csv                   per-kernel means of every PMC counter collected
  profiles/traffic_<round>.json            per kernel: HBM bytes per launch (read by bench.py)
                                           and the derivation-inclusive step's traffic table

HBM bytes (/opt/skills/guides/MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE from separate
--pmc passes, both in KiB.  The guide's x2 FETCH correction holds for wide coalesced reads only;
the calibration microbenchmark (scripts/calib/calib_fetch.hip: each byte of a 1 GiB buffer once
per shape) measured x2.0 for 16-B and 4-B coalesced lanes, x1.88 for 8-B unaligned coalesced
lanes, and x1.0 for lane-private 8-B streams and scattered 64-B records or 2-B fields.  Each
kernel takes the factor of its dominant load shape (KERNEL_SHAPE below), and the raw counter
and both bounds (x1: every load scattered, x2: every load coalesced) are printed beside it.
WRITE_SIZE is exact for 16-B and 8-B stores (x1.0 both).
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import statistics
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# dominant load shape per kernel (prefix match), a shape of the calibration file
KERNEL_SHAPE = [
    ("germline_direct", "u64_g4_ua"),     # groups of four lanes on one read's 32 bytes, 16 reads per load
    ("somatic_direct", "u64_coal_ua"),   # rotated schedule: the lanes a slot covers read it together
    ("germline_complex", "rec64_perm"),   # a wave per queued locus: scattered per-read records
    ("germline_walk", "rec64_perm"),
    ("germline_standard", "rec64_perm"),
    ("somatic_call", "rec64_perm"),
    ("cand_prep", "rec64_perm"),
    ("proj_fill_cells", "u64_coal_ua"),   # a lane per cell: 8-B unaligned loads along one read's run
    ("proj_fill", "u64_coal_ua"),
    ("mproj_fill", "u64_coal_ua"),
    ("germline_proj", "b32_rows"),        # 4-B lanes over 64-B projection rows
    ("somatic_proj", "b32_rows"),
]
DEFAULT_SHAPE = "stream16"  # lane = element, consecutive lanes on consecutive words (read_prep, scans, ...)
DERIVE = ("read_prep", "block_index", "pool_clean", "col_count", "col_derive", "scan_tiles", "scan_u32",
          "ev_bases", "validate")


def kernel_key(name: str) -> str:
    m = re.search(r"([A-Za-z_][A-Za-z0-9_]*(<[^>(]*>)?)\(", name)
    return m.group(1) if m else name


def shape_of(k: str) -> str:
    for pre, sh in KERNEL_SHAPE:
        if k.startswith(pre):
            return sh
    return DEFAULT_SHAPE


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("profdir")
    ap.add_argument("tag")
    ap.add_argument("--length", type=int, required=True)
    ap.add_argument("--depth", type=float, required=True)
    ap.add_argument("--round", required=True)
    ap.add_argument("--calib", default=os.path.join(ROOT, "profiles", "r06_pmc_calibration.json"))
    ap.add_argument("--call-kernel", default="germline_direct<false>")
    ap.add_argument("--somatic", default=None, help="also write somatic_pmc_<round>.json for this workload "
                    "(chr1|panel:L:tumor_depth:normal_depth)")
    a = ap.parse_args()
    cal = json.load(open(a.calib))["shapes"]
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
    launches = {k: len(cs.get("FETCH_SIZE", [])) for k, cs in vals.items()}
    with open(os.path.join(prof, "%s_pmc.csv" % a.tag), "w") as fh:
        fh.write("kernel,counter,mean_per_launch\n")
        for k in sorted(pm):
            for c in sorted(pm[k]):
                fh.write("%s,%s,%.1f\n" % (k, c, pm[k][c]))
    kern = {}
    for k, cs in pm.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        sh = shape_of(k)
        f = cal[sh]["factor"]
        raw_f, raw_w = cs["FETCH_SIZE"] * 1024, cs["WRITE_SIZE"] * 1024
        kern[k] = {"hbm_bytes_per_launch": raw_f * f + raw_w, "fetch_bytes_corrected": raw_f * f,
                   "write_bytes": raw_w, "fetch_shape": sh, "fetch_factor": f,
                   "hbm_bytes_bounds": [raw_f + raw_w, 2 * raw_f + raw_w],
                   "raw_FETCH_SIZE_KiB": cs["FETCH_SIZE"], "raw_WRITE_SIZE_KiB": cs["WRITE_SIZE"],
                   "launches": launches.get(k, 0)}
    # the derivation-inclusive step: the derivation kernels once per re-derivation, the call's
    # kernels as often per call as they launched per launch of the call's pileup kernel
    n_call = max(1, launches.get(a.call_kernel, 0))
    n_der = max(1, launches.get("read_prep", 0))
    step = {}
    for k, v in kern.items():
        if k.startswith("__amd") or k.startswith("warm_k"):
            continue
        per = v["launches"] / (n_der if k.startswith(DERIVE) else n_call)
        if per < 0.5:
            continue  # not in every step (cold-call or test-only kernels)
        step[k] = {"per_step": round(per, 2), "hbm_bytes": v["hbm_bytes_per_launch"] * round(per),
                   "bounds": [x * round(per) for x in v["hbm_bytes_bounds"]]}
    tot = sum(v["hbm_bytes"] for v in step.values())
    out = {"length": a.length, "depth": a.depth, "kernels": kern, "source": "profiles/%s_pmc.csv" % a.tag,
           "calibration": "profiles/r06_pmc_calibration.json",
           "correction": "FETCH_SIZE x the calibrated factor of the kernel's dominant load shape (fetch_shape), "
                         "KiB->bytes; WRITE_SIZE as is (calibrated x1.0); hbm_bytes_bounds = [FETCH x1, FETCH x2] + WRITE",
           "step": {"kernels": step, "hbm_bytes": tot,
                    "hbm_bytes_bounds": [sum(v["bounds"][0] for v in step.values()),
                                         sum(v["bounds"][1] for v in step.values())]}}
    if a.somatic:  # the somatic bench's PMC summary (bench.somatic_pmc reads it)
        wl, L, td, nd = a.somatic.split(":")
        out_p = os.path.join(prof, "somatic_pmc_%s.json" % a.round)
        doc = json.load(open(out_p)) if os.path.exists(out_p) else {}
        ks = {k: dict(pm[k], **kern.get(k, {})) for k in pm}
        doc[wl] = {"length": int(L), "tumor_depth": float(td), "normal_depth": float(nd),
                   "source": "profiles/%s_pmc.csv" % a.tag, "kernels": ks, "calibration": out["calibration"],
                   "correction": out["correction"]}
        with open(out_p, "w") as fh:
            json.dump(doc, fh, indent=1, sort_keys=True)
        return
    with open(os.path.join(prof, "traffic_%s.json" % a.round), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for k, v in sorted(step.items(), key=lambda kv: -kv[1]["hbm_bytes"]):
        print("%-34s x%-5s %8.3f GB  [%6.3f, %6.3f]  (%s)" % (k[:34], v["per_step"], v["hbm_bytes"] / 1e9,
                                                             v["bounds"][0] / 1e9, v["bounds"][1] / 1e9,
                                                             kern[k]["fetch_shape"]))
    print("step: %.3f GB  bounds [%.3f, %.3f]" % (tot / 1e9, out["step"]["hbm_bytes_bounds"][0] / 1e9,
                                                  out["step"]["hbm_bytes_bounds"][1] / 1e9))


if __name__ == "__main__":
    main()
