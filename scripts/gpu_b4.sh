#!/bin/bash
# round-4 b4: germline_proj decision rewrite (tests + bench + ablations) and the read-major
# fills' ablations (GQ_FILL_DBG 1 no word loads, 2 no word stores, 4 XCD-contiguous batches).
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_germline.py tests/test_gpu_scala_order.py tests/test_gpu_somatic.py tests/test_gpu_branches.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; stop $rc
bash scripts/ablate_proj.sh gpurun_out/${TAG}_abl 0 4 16
bash scripts/ab_libs.sh gpurun_out/${TAG}_ab - guacamole_amd/_lib/var/nogmin.so
grep -h "gq prof" gpurun_out/${TAG}_abl/d16.err | tail -1
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_abl/d0.json')); print('parity', d.get('parity_window'), 'calls', d['calls'])" || true
for D in 0 1 2 3 4; do
  W=0; [ $D = 0 ] && W=200000
  GQ_FILL_DBG=$D timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_d$D -o run -- python3 scripts/bench_somatic.py --steps 1 --warmup 0 --cpu-window $W > gpurun_out/${TAG}_d$D.log 2>&1
  rc=$?; echo "fill d$D rc=$rc"; stop $rc
done
exit 0
