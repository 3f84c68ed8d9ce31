#!/bin/bash
# Round-6 somatic profile (GPU box, repo root): the chr1-length 60x/30x somatic bench with
# re-derived steps (scripts/bench_somatic.py --rederive): a kernel-trace + stats pass, then PMC
# groups, one rocprofv3 run each.  usage: scripts/profile_somatic6.sh <outdir>
OUT=$1
mkdir -p $OUT
export TMPDIR=/tmp
B="--length ${SOM_LEN:-249250621} --rederive --steps 3 --warmup 1 --cpu-window 0"
KRE=${KRE:-"somatic_direct|somatic_call_k|cand_prep|read_prep|block_index|somatic_tile"}
run() { "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "step rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/bench_somatic.py $B > $OUT/trace.log 2>&1
i=0
for G in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  run timeout -s KILL 240 rocprofv3 --pmc $G --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc$i -o run -- python3 scripts/bench_somatic.py $B > $OUT/pmc$i.log 2>&1
done
echo done
