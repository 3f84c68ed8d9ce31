#!/bin/bash
# One GPU call: the GPU tests, then (unless a step crashed or timed out) the bench line and a
# rocprofv3 kernel-trace of the same bench command.  usage: scripts/gpu_round.sh <tag> [pytest args]
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu "$@" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; stop $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; stop $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --no-single-pass > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
