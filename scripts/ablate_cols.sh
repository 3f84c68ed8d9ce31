#!/bin/bash
# Phase clocks and ablations of the germline column kernel (diagnostics; GQ_DBG bits in
# gq_germline_cols.h).  Run on the GPU box from the repo root:  scripts/ablate_cols.sh [bench args]
set -e
for d in ${GQ_DBG_LIST:-0 16 1 2 4 8 3 7}; do
  echo "== GQ_DBG=$d"
  GQ_DBG=$d timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" 2>&1 \
    | python3 -c "
import sys, json
for line in sys.stdin:
    if line.startswith('{'):
        j = json.loads(line); print('kernel_ms %.3f  step_ms %.3f' % (j['roofline']['kernel_ms'], j['ms_per_step']))
    elif 'gq prof' in line:
        last = line.strip()
try: print(last)
except NameError: pass
"
done
