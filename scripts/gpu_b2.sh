#!/bin/bash
# round-4 b2: read-major fills — GPU tests of the projection consumers, the fills' A/B (rocprof
# kernel traces of the somatic bench at chr20 length: read-major at 1/2/4 words per lane and
# round, and the slice-major fill), then germline_proj's ablations.
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { case $1 in 0) ;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_germline.py tests/test_gpu_somatic.py tests/test_gpu_germline_standard.py tests/test_gpu_branches.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; stop $rc
for V in rw2 rw1 rw4 slice; do
  case $V in rw2) E="GQ_FILL_U=2";; rw1) E="GQ_FILL_U=1";; rw4) E="GQ_FILL_U=4";; slice) E="GQ_FILL=slice GQ_FILL_U=1";; esac
  W=0; [ $V = rw2 ] && W=200000
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$V -o run -- python3 scripts/bench_somatic.py --steps 1 --warmup 0 --cpu-window $W > gpurun_out/${TAG}_$V.log 2>&1
  rc=$?; echo "$V rc=$rc"; stop $rc
done
bash scripts/ablate_proj.sh gpurun_out/${TAG}_abl 0 1 2 4 7 16
grep -h "gq prof" gpurun_out/${TAG}_abl/*.err
exit 0
