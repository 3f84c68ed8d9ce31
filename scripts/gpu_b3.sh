#!/bin/bash
# round-4 b3: read-major fill ablations (GQ_FILL_DBG 1 no word loads, 2 no word stores, 4
# XCD-contiguous batches) as rocprof kernel traces of the somatic bench at chr20 length.
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
for D in 0 1 2 3 4; do
  W=0; [ $D = 0 ] && W=200000
  GQ_FILL_DBG=$D timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_d$D -o run -- python3 scripts/bench_somatic.py --steps 1 --warmup 0 --cpu-window $W > gpurun_out/${TAG}_d$D.log 2>&1
  rc=$?; echo "d$D rc=$rc"; stop $rc
done
exit 0
