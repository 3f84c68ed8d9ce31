#!/bin/bash
# Round-6 germline profile (GPU box, repo root): one kernel-trace + stats pass of the germline
# bench, then PMC groups over every kernel, one rocprofv3 run each (FETCH_SIZE and WRITE_SIZE
# cannot share a pass on gfx950).  usage: scripts/profile_germline6.sh <outdir>
OUT=$1
mkdir -p $OUT
export TMPDIR=/tmp
B="--steps 3 --warmup 1 --no-cpu-baseline --somatic-length 0 --panel-length 0 --no-single-pass --no-configs3 ${BENCH_ARGS}"
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $B > $OUT/trace.log 2>&1
i=0
for G in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
         ${PMC_EXTRA}; do
  i=$((i+1))
  run timeout -s KILL 200 rocprofv3 --pmc $G ${KRE:+--kernel-include-regex "$KRE"} --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $B > $OUT/pmc$i.log 2>&1
done
echo done
