#!/bin/bash
# round-4 b10: slice rows padded to a multiple of 4 (one bound per row batch in germline_proj):
# projection consumers' GPU tests, then the germline bench kernel time and phase clocks.
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_germline.py tests/test_gpu_somatic.py tests/test_gpu_branches.py tests/test_gpu_distributed.py tests/test_gpu_variants.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; stop $rc
bash scripts/ablate_proj.sh gpurun_out/${TAG}_abl 0 16
grep -h "gq prof" gpurun_out/${TAG}_abl/d16.err | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --somatic-length 0 --panel-length 0 --no-single-pass > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
