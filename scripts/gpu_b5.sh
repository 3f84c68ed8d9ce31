#!/bin/bash
# round-4 b5: germline_proj at HEAD (bench kernel time + phase clocks) and the read-major fills at
# 1, 2 and 4 words per lane and round (rocprof kernel traces of the somatic bench, chr20 length).
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
bash scripts/ablate_proj.sh gpurun_out/${TAG}_abl 0 16
grep -h "gq prof" gpurun_out/${TAG}_abl/d16.err | tail -1
for U in 1 2 4; do
  GQ_FILL_U=$U timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_u$U -o run -- python3 scripts/bench_somatic.py --steps 1 --warmup 0 --cpu-window 0 > gpurun_out/${TAG}_u$U.log 2>&1
  rc=$?; echo "fill u$U rc=$rc"; stop $rc
done
exit 0
