#!/bin/bash
# germline_proj ablations (diagnostics only: the records are wrong when set): GQ_DBG 1 skips the
# projection loads, 2 the sparse entries, 4 the decision; the bench line's kernel_ms for each.
TAG=$1
mkdir -p gpurun_out
for D in 0 1 2 4; do
  GQ_DBG=$D timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --somatic-length 0 --panel-length 0 --no-single-pass > gpurun_out/${TAG}_dbg$D.json 2> gpurun_out/${TAG}_dbg$D.err
  rc=$?; echo "dbg$D rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
