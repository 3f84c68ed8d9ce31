#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the germline bench for kernels matching
# a regex.  usage: scripts/gpu_r5_pmc.sh <tag> <kernel regex>
TAG=$1; KRE=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 2 --warmup 0 --somatic-length 0 --panel-length 0 --no-single-pass --no-cpu-baseline --no-configs3 ${BENCH_ARGS}"
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $G --kernel-include-regex "$KRE" --output-format csv -d gpurun_out/${TAG}_pmc/p$i -o run -- python3 bench.py $B > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "pmc pass $i rc=$rc"; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/${TAG}_pmc "$KRE"
