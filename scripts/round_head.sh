#!/bin/bash
# One GPU call's worth of HEAD evidence (GPU box, repo root): the GPU suite, the default bench
# line, rocprof kernel stats of the bench, and rocprof kernel stats of one germline-threshold
# CLI single pass with the BAM decoded on the device.
#   usage: scripts/round_head.sh <outdir>
set -e
OUT=$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-single-pass > $OUT/trace.log 2>&1
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0, '.')
from guacamole_amd import synthetic
synthetic.generate(63025520, 30.0).write_bam('/tmp/gq_sp.bam')" > $OUT/spbam.log 2>&1
rm -rf /tmp/gq_sp_out.vcf
GQ_TIMING=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sptrace -o run -- python3 -m guacamole_amd germline-threshold --reads /tmp/gq_sp.bam --out /tmp/gq_sp_out.vcf > $OUT/sptrace.log 2>&1
rm -rf /tmp/gq_sp.bam /tmp/gq_sp_out.vcf
