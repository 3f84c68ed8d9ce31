#!/bin/bash
# Round-5: a GPU test subset, then the default bench line (every leg) with its own time limit.
#   usage: scripts/gpu_r5_full.sh <tag> [pytest paths/args...]
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread -m gpu "$@" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; stop $rc
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/${TAG}_bench.err; stop $rc
