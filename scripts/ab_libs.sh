#!/bin/bash
# A/B of alternative in-tree builds of libgqpileup (GQ_LIB) on the germline bench.
#   usage (GPU box, repo root): scripts/ab_libs.sh <outdir> <lib>...   ("-" = the default build)
set -e
OUT=$1; shift
mkdir -p $OUT
for L in "$@"; do
  n=$(basename $L .so)
  if [ "$L" = "-" ]; then n=default; unset GQ_LIB; else export GQ_LIB=$L; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --somatic-length 0 --panel-length 0 --no-single-pass > $OUT/$n.json 2> $OUT/$n.err
  python3 -c "import json,sys; d=json.load(open('$OUT/$n.json')); print('$n', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['device_stages_ms'])"
done
