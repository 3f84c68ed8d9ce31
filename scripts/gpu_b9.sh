#!/bin/bash
# round-4 b9: the projection and the margin projection in one read-major pass (pm_fill_rw) —
# GPU tests of its callers, rocprof kernel traces of the somatic bench at chr20 length (one pass
# vs GQ_FILL_SEP=1), then the bench line (chr1 somatic one-shot).
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_somatic.py tests/test_gpu_germline_standard.py tests/test_gpu_reference.py tests/test_gpu_scala_order.py tests/test_gpu_branches.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; stop $rc
for V in one sep; do
  E=""; [ $V = sep ] && E="GQ_FILL_SEP=1"
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$V -o run -- python3 scripts/bench_somatic.py --steps 1 --warmup 0 --cpu-window 200000 > gpurun_out/${TAG}_$V.log 2>&1
  rc=$?; echo "$V rc=$rc"; stop $rc
done
timeout -k 10 500 python -u bench.py --no-single-pass > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; exit $rc
