#!/bin/bash
# Run one gpurun call (builder convenience); retries only when gpurun reports that nothing ran
# (transient box loss, back-off, no slot).  usage: scripts/gpu_call.sh <tag> <timeout> '<command>'  — retries only when gpurun reports that nothing ran
TAG=$1; TO=$2; CMD=$3
for attempt in 1 2 3 4 5; do
  timeout $((TO + 1500)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > /root/repo/gpurun_out/${TAG}_call.log 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|no box\|slot free" /root/repo/gpurun_out/${TAG}_call.log && ! grep -q "status=ok" /root/repo/gpurun_out/${TAG}_call.log; then
    sleep 60; continue
  fi
  if [ $rc -eq 3 ]; then sleep 60; continue; fi
  break
done
echo "rc=$rc attempts=$attempt" >> /root/repo/gpurun_out/${TAG}_call.log
