#!/bin/bash
# round-4 b7: branch-free LDS margin terms — somatic / variant / germline-standard GPU tests, then
# a rocprof kernel trace of the somatic bench (chr20 length, oracle parity window).
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_somatic.py tests/test_gpu_germline_standard.py tests/test_gpu_variants.py tests/test_gpu_germline.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; stop $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_som -o run -- python3 scripts/bench_somatic.py --steps 1 --warmup 0 --cpu-window 200000 > gpurun_out/${TAG}_som.log 2>&1
rc=$?; echo "somatic rc=$rc"; stop $rc
exit 0
