#!/bin/bash
# round-4 b12: germline_proj's record writing (one 64-bit LDS reservation, uniform locus mask,
# unrolled) — germline GPU tests, then the bench kernel time and the output-path ablation.
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_germline.py tests/test_gpu_scala_order.py tests/test_gpu_branches.py tests/test_gpu_distributed.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; stop $rc
bash scripts/ablate_proj.sh gpurun_out/${TAG}_abl 0 8 0
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_abl/d0.json')); print('parity', d['parity_window'] if 'parity_window' in d else None, d['calls'])"
