#!/bin/bash
# VALU / SALU / LDS instruction counts of germline_cols under GQ_DBG variants (phase attribution).
#   usage (GPU box, repo root): scripts/pmc_dbg.sh <outdir> <dbg values...>
set -e
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for A in "$@"; do
  GQ_DBG=$A timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM --kernel-include-regex "${GQ_KRE:-germline_proj}" --output-format csv -d $OUT/a$A -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/a$A.log 2>&1
  python3 - $OUT/a$A/run_counter_collection.csv $A <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for row in csv.DictReader(open(sys.argv[1])):
    v[row["Counter_Name"]].append(float(row["Counter_Value"]))
print("DBG", sys.argv[2], " ".join("%s=%.4g" % (k, sum(x) / len(x)) for k, x in sorted(v.items())))
PY
done
