#!/bin/bash
# Per-kernel durations of one short bench run (rocprofv3 kernel trace + stats), summarised.
#   usage (GPU box, repo root): scripts/kstats.sh <outdir> [bench args]
set -e
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/bench.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for row in csv.DictReader(open(f)):
    print("%-60s calls %4s avg_us %10.1f pct %5.1f" % (row["Name"][:60], row["Calls"], float(row["AverageNs"]) / 1e3, float(row["Percentage"])))
PY
