#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (repo root): the microbenchmark's trace,
# then one --pmc pass per counter (they cannot share a pass).  usage: scripts/calib/calib.sh <outdir>
OUT=$1
mkdir -p $OUT
export TMPDIR=/tmp
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 120 ./scripts/calib/_build/calib_fetch 3 > $OUT/calib_times.jsonl
run timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- ./scripts/calib/_build/calib_fetch 1 > $OUT/fetch.log 2>&1
run timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- ./scripts/calib/_build/calib_fetch 1 > $OUT/write.log 2>&1
run python3 scripts/calib/factors.py $OUT
