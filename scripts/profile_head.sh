#!/bin/bash
# HEAD profiles for the round: germline_proj PMC passes + somatic (configs[2] chr1) trace and PMC.
#   usage (GPU box, repo root): scripts/profile_head.sh <outdir>
set -e
OUT=$1
mkdir -p $OUT
KRE=germline_proj scripts/profile_germline.sh $OUT/germ
KRE=somatic_call_k scripts/profile_somatic.sh $OUT/som --length 249250621
