#!/bin/bash
# PMC passes (one counter group per pass) for the dominant kernels at HEAD:
#   germline_proj on configs[1] (scripts/profile_germline.sh), somatic_proj + the somatic callers on
#   configs[2] at chr1 length, and the deep caller on the configs[4] panel.
# usage: scripts/gpu_pmc.sh <tag> [germline|somatic|panel ...]
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for what in "$@"; do
  case $what in
    germline)
      bash scripts/profile_germline.sh gpurun_out/${TAG}_germ; rc=$?; echo "germline rc=$rc"; stop $rc;;
    somatic)
      KRE="somatic_proj|somatic_call_k|mproj_fill|proj_fill|row_count" bash scripts/profile_somatic.sh gpurun_out/${TAG}_som --length 249250621; rc=$?; echo "somatic rc=$rc"; stop $rc;;
    panel)
      KRE="somatic_call_k|somatic_proj" bash scripts/profile_somatic.sh gpurun_out/${TAG}_panel --length 1000000 --tumor-depth 500 --normal-depth 500 --somatic-rate 1e-3; rc=$?; echo "panel rc=$rc"; stop $rc;;
  esac
done
