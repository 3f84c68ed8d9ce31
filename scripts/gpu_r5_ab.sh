#!/bin/bash
# A/B of library env switches: the germline bench (plus BENCH_ARGS) under rocprofv3 once per
# "NAME=VALUE" argument ("-" = defaults), kernels matching a regex.  usage: gpu_r5_ab.sh <tag> <regex> <env...>
TAG=$1; KRE=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --somatic-length 0 --panel-length 0 --no-single-pass --no-cpu-baseline --no-configs3 ${BENCH_ARGS}"
i=0
for v in "$@"; do
  i=$((i+1))
  if [ "$v" = "-" ]; then E=""; else E="$v"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_v$i -o run -- python3 bench.py $B > gpurun_out/${TAG}_v$i.json 2> gpurun_out/${TAG}_v$i.err
  rc=$?; [ $rc -ne 0 ] && { echo "variant $v rc=$rc"; tail -3 gpurun_out/${TAG}_v$i.err; exit $rc; }
  echo "== $v: $(python3 -c "import json,sys; p=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('step_ms_median', round(p['step_ms_median'],3), 'stages', p['step_stages_ms'], 'identical', p['rederive_identical'], 'somatic_ms', p.get('somatic',{}).get('ms_per_step'), 'somatic_one_shot', p.get('somatic',{}).get('one_shot',{}).get('total_ms'))" gpurun_out/${TAG}_v$i.json)"
  python3 scripts/ktrace_median.py gpurun_out/${TAG}_v$i | grep -E "$KRE"
done
