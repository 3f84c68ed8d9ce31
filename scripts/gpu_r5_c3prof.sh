#!/bin/bash
# rocprofv3 kernel stats of the configs[3] rank-share leg alone (a 1 Mb germline shard first).
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--length 1000000 --steps 3 --warmup 1 --somatic-length 0 --panel-length 0 --no-single-pass --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py $B > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${TAG}_prof -name run_kernel_stats.csv | head -1)
cp $f gpurun_out/${TAG}_kernel_stats.csv
python3 - gpurun_out/${TAG}_kernel_stats.csv <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    print("%-50s calls %4s avg_us %9.1f max_us %9.1f tot_ms %8.2f" % (row["Name"][:50], row["Calls"], float(row["AverageNs"]) / 1e3, float(row["MaxNs"]) / 1e3, float(row["TotalDurationNs"]) / 1e6))
PY
