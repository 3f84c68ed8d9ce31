#!/bin/bash
# germline_proj time under GQ_DBG ablations (1 = no projection loads, 2 = no sparse entries,
# 4 = no decision; results are wrong under them): what each phase costs.
#   usage (GPU box, repo root): scripts/ablate_proj.sh <outdir> <dbg values...>
set -e
OUT=$1; shift
mkdir -p $OUT
for A in "$@"; do
  GQ_DBG=$A timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --somatic-length 0 --panel-length 0 --no-single-pass > $OUT/d$A.json 2> $OUT/d$A.err || true
  python3 -c "import json; d=json.load(open('$OUT/d$A.json')); print('dbg $A', round(d['roofline']['kernel_ms'],4))" || echo "dbg $A failed"
done
