#!/bin/bash
# Memory-pipeline PMC passes for one kernel of the germline bench (GPU box, repo root): TA / TD /
# TCP / UTCL1 / TCC counters, one rocprofv3 --pmc run per group (the per-block limits: 2 TA, 2 TD,
# 4 TCP, 4 TCC).  usage: scripts/pmc_fill_pipe.sh <outdir> <kernel regex>
OUT=$1; KRE=$2
mkdir -p $OUT
export TMPDIR=/tmp
B="--steps 2 --warmup 1 --no-cpu-baseline --somatic-length 0 --panel-length 0 --no-single-pass --no-configs3"
i=0
for G in "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE SQ_WAVES SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES" \
         "TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_UTCL1_TRANSLATION_MISS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
         "TCP_TCP_TA_DATA_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_UTCL1_STALL_INFLIGHT_MAX TCP_UTCL1_TRANSLATION_HIT TCC_HIT TCC_MISS TCC_EA0_RDREQ_DRAM"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $G --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $B > $OUT/pmc$i.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; exit $rc; fi
done
echo done
