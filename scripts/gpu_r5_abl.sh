#!/bin/bash
# Kernel ablations: the germline bench under rocprofv3 once per GQ_FILL_DBG value (results wrong
# under an ablation; timings only).  usage: scripts/gpu_r5_abl.sh <tag> <kernel regex> <dbg values...>
TAG=$1; KRE=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --somatic-length 0 --panel-length 0 --no-single-pass --no-cpu-baseline --no-configs3 ${BENCH_ARGS}"
for v in "$@"; do
  GQ_FILL_DBG=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_d$v -o run -- python3 bench.py $B > gpurun_out/${TAG}_d$v.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "dbg $v rc=$rc"; exit $rc; }
  echo "GQ_FILL_DBG=$v"; python3 scripts/ktrace_median.py gpurun_out/${TAG}_d$v | grep -E "$KRE"
done
