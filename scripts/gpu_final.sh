#!/bin/bash
# Round-end GPU call: every GPU test, the bench line, a rocprof kernel trace of the bench, then
# germline_proj's PMC passes (scripts/profile_germline.sh) for traffic_r04.json.
TAG=$1
bash scripts/gpu_round.sh $TAG
rc=$?; [ $rc = 0 ] || exit $rc
bash scripts/gpu_pmc.sh ${TAG}p germline
