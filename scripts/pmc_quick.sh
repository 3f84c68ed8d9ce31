#!/bin/bash
# Quick PMC passes for one kernel (regex) of bench.py: instruction mix and stalls.
#   usage: scripts/pmc_quick.sh <outdir> <kernel-regex> [bench args...]
set -e
OUT=$1; shift
KRE=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$KRE" --output-format csv -d $OUT/sq1 -o run -- python3 bench.py $ARGS > $OUT/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --kernel-include-regex "$KRE" --output-format csv -d $OUT/sq2 -o run -- python3 bench.py $ARGS > $OUT/sq2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY --kernel-include-regex "$KRE" --output-format csv -d $OUT/sq3 -o run -- python3 bench.py $ARGS > $OUT/sq3.log 2>&1 || true
python3 - "$OUT" "$KRE" <<'PY'
import csv, sys, os, re, collections
out, kre = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(list)
for sub in ("sq1", "sq2", "sq3"):
    p = os.path.join(out, sub, "run_counter_collection.csv")
    if not os.path.exists(p): continue
    for row in csv.DictReader(open(p)):
        if re.search(kre, row["Kernel_Name"]):
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
with open(os.path.join(out, "summary.csv"), "w") as fh:
    for k in sorted(vals):
        v = sum(vals[k]) / len(vals[k])
        fh.write("%s,%.1f\n" % (k, v)); print(k, "%.4g" % v)
PY
