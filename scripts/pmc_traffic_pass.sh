#!/bin/bash
# HBM traffic of one kernel (regex) of bench.py: FETCH_SIZE and WRITE_SIZE in separate passes.
#   usage (GPU box, repo root): scripts/pmc_traffic_pass.sh <outdir> <kernel-regex> [bench args]
set -e
OUT=$1; shift
KRE=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 - "$OUT" "$KRE" <<'PY'
import csv, sys, os, re, collections
out, kre = sys.argv[1], sys.argv[2]
for sub in ("fetch", "write"):
    p = os.path.join(out, sub, "run_counter_collection.csv")
    v = collections.defaultdict(list)
    for row in csv.DictReader(open(p)):
        if re.search(kre, row["Kernel_Name"]):
            v[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, x in v.items():
        print(k, "mean %.4g over %d launches" % (sum(x) / len(x), len(x)))
PY
