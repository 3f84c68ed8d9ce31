#!/bin/bash
# Kernel timeline of the last germline step of a short bench run (rocprofv3 kernel trace):
# each kernel's start offset, duration and the gap before it.
#   usage (GPU box, repo root): scripts/ktimeline.sh <outdir> [bench args]
set -e
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --somatic-length 0 --panel-length 0 --no-single-pass "$@" > $OUT/bench.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the last germline_proj launch and what follows it until the next germline_proj / plan
idx = [i for i, r in enumerate(rows) if "germline_proj" in r["Kernel_Name"]]
a = idx[-2] - 1 if len(idx) >= 2 else 0
b = idx[-1] - 1
t0 = int(rows[a]["Start_Timestamp"])
prev = None
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print("%9.1f us  dur %8.1f us  gap %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, r["Kernel_Name"][:90]))
    prev = e
PY
