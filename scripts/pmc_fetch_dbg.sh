#!/bin/bash
# FETCH_SIZE (KiB, raw) of the germline kernel under GQ_DBG variants (traffic attribution; e.g. 1 =
# projection loads out of range, so the difference to 0 is the projection's share).
#   usage (GPU box, repo root): scripts/pmc_fetch_dbg.sh <outdir> <dbg values...>
set -e
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for A in "$@"; do
  GQ_DBG=$A timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "${GQ_KRE:-germline_proj}" --output-format csv -d $OUT/f$A -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --somatic-length 0 --panel-length 0 --no-single-pass > $OUT/f$A.log 2>&1
  python3 - $OUT/f$A/run_counter_collection.csv $A <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for row in csv.DictReader(open(sys.argv[1])):
    v[row["Counter_Name"]].append(float(row["Counter_Value"]))
print("DBG", sys.argv[2], " ".join("%s=%.6g" % (k, sum(x) / len(x)) for k, x in sorted(v.items())))
PY
done
