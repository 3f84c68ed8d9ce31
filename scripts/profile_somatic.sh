#!/bin/bash
# rocprofv3 passes for the somatic-standard kernels (GPU box, repo root).
#   usage: scripts/profile_somatic.sh <outdir> [bench_somatic args...]   (KRE = kernel regex, default somatic_call_k)
# Pass 1: kernel trace + stats.  Then PMC counters, one group per pass (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950).
set -e
OUT=$1; shift
KRE=${KRE:-somatic_call_k}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --cpu-window 0 $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 scripts/bench_somatic.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$KRE" --output-format csv -d $OUT/sq1 -o run -- python3 scripts/bench_somatic.py $ARGS > $OUT/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex "$KRE" --output-format csv -d $OUT/sq2 -o run -- python3 scripts/bench_somatic.py $ARGS > $OUT/sq2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/fetch -o run -- python3 scripts/bench_somatic.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/write -o run -- python3 scripts/bench_somatic.py $ARGS > $OUT/write.log 2>&1
