#!/bin/bash
# round-4 step: GPU tests, the fills' A/B (1 or 4 words per lane: rocprof kernel traces of the
# somatic bench at chr20 length), the bench line, and a kernel trace of the bench.
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; stop $rc
for U in 1 2; do
  GQ_FILL_U=$U timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_fill$U -o run -- python3 scripts/bench_somatic.py --steps 1 --warmup 0 --cpu-window 0 > gpurun_out/${TAG}_fill$U.log 2>&1
  rc=$?; echo "fill$U rc=$rc"; stop $rc
done
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; stop $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --no-single-pass > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
