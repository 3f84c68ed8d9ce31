#!/bin/bash
# round-4 b8: read-major fills with 1 / 2 / 4 consecutive words of a read per lane (GQ_FILL_W):
# the variants test, then rocprof kernel traces of the somatic bench at chr20 length.
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_somatic.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; stop $rc
for W in 1 2 4; do
  GQ_FILL_W=$W timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_w$W -o run -- python3 scripts/bench_somatic.py --steps 1 --warmup 0 --cpu-window 0 > gpurun_out/${TAG}_w$W.log 2>&1
  rc=$?; echo "fill w$W rc=$rc"; stop $rc
done
exit 0
