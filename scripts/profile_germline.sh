#!/bin/bash
# rocprofv3 passes for the germline pileup kernel (run on the GPU box from the repo root).
#   usage: scripts/profile_germline.sh <outdir> [bench args...]   (KRE = kernel regex, default germline_proj)
# Pass 1: kernel trace + stats.  Passes 2-5: PMC counters, one group per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -e
OUT=$1; shift
KRE=${KRE:-germline_proj}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --somatic-length 0 --panel-length 0 --no-single-pass $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $KRE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $KRE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex $KRE --output-format csv -d $OUT/sq1 -o run -- python3 bench.py $ARGS > $OUT/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex $KRE --output-format csv -d $OUT/sq2 -o run -- python3 bench.py $ARGS > $OUT/sq2.log 2>&1
