#!/bin/bash
# Round-6 iteration call: a GPU test subset (optional), the germline bench line (no sub-runs)
# and its rocprofv3 kernel stats.  usage: scripts/gpu_r6.sh <tag> [pytest paths/args...]
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu "$@" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; stop $rc
fi
B="--steps 10 --warmup 3 --somatic-length 0 --panel-length 0 --no-single-pass --no-cpu-baseline --no-configs3 ${BENCH_ARGS}"
timeout -k 10 300 python -u bench.py $B > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; stop $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py $B > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; stop $rc
f=$(find gpurun_out/${TAG}_prof -name run_kernel_stats.csv | head -1)
cp $f gpurun_out/${TAG}_kernel_stats.csv
python3 scripts/ktrace_median.py gpurun_out/${TAG}_prof | head -${KTOP:-30}
