#!/bin/bash
# somatic_direct ablations (GPU box, repo root): the candidate kernel's time (pileup_ms) per
# somatic_direct diagnostics setting (GQ_DBG = d << 16) on the chr20-length 60x/30x bench (re-derived steps).  usage: scripts/somatic_direct_ablate.sh <out>
OUT=$1
mkdir -p $(dirname $OUT)
for d in ${DBGS:-0 1 2 32 64 33}; do
  GQ_DBG=$((d << 16)) timeout -k 10 200 python -u scripts/bench_somatic.py --rederive --steps 4 --warmup 1 --cpu-window 0 ${SOM_ARGS} > $OUT.$d.json 2> $OUT.$d.err || { echo "dbg $d failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT.$d.json')); print('GQ_DBG=$d', round(d['ms_per_step'],3), d['device_stages_ms'])"
done
