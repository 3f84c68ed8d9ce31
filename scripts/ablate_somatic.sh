#!/bin/bash
# somatic_call phase ablations (GQ_DBG bits; results are wrong under them): the caller's device
# time (complex_ms) with the kernel cut after each phase.  GPU box, repo root.
#   usage: scripts/ablate_somatic.sh <outdir> [bench_somatic args]
set -e
OUT=$1; shift
mkdir -p $OUT
for d in 0 1024 2048 4096 8192; do
  GQ_DBG=$d timeout -k 10 200 python3 -u scripts/bench_somatic.py --steps 3 --warmup 1 --cpu-window 0 "$@" > $OUT/dbg$d.log 2>&1
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/dbg$d.log') if l.startswith('{')][0]); print('GQ_DBG=$d', 'complex_ms %.3f' % d['device_stages_ms']['complex_ms'])"
done
