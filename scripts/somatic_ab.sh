#!/bin/bash
# A/B of library builds on the somatic bench (chr20 length, re-derived steps): time per step and
# somatic_direct's FETCH_SIZE.  usage (GPU box, repo root): scripts/somatic_ab.sh <outdir> <lib>...  ("-": default)
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so); if [ "$L" = "-" ]; then n=default; unset GQ_LIB; else export GQ_LIB=$L; fi
  timeout -k 10 200 python -u scripts/bench_somatic.py --rederive --steps 4 --warmup 1 --cpu-window 0 > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex somatic_direct --output-format csv -d $OUT/$n.fetch -o run -- python3 scripts/bench_somatic.py --rederive --steps 2 --warmup 0 --cpu-window 0 > $OUT/$n.fetch.log 2>&1 || { echo "$n pmc failed"; exit 1; }
  python3 - <<PY
import csv, glob, json
d = json.load(open("$OUT/$n.json"))
v = [float(r["Counter_Value"]) for p in glob.glob("$OUT/$n.fetch/**/run_counter_collection.csv", recursive=True) for r in csv.DictReader(open(p))]
print("$n", round(d["ms_per_step"], 3), round(d["device_stages_ms"]["pileup_ms"], 3), d["candidate_loci"], "FETCH_GB_raw", round(sum(v) / max(1, len(v)) * 1024 / 1e9, 2))
PY
done
