#!/bin/bash
# Build an alternative libgqpileup with extra -D flags, for scripts/ab_libs.sh (container side).
#   usage: scripts/build_variant.sh <out.so> [-DNAME=VALUE ...]
set -e
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
for s in gq_pileup gq_somatic gq_heapref gq_bamdev; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -I$ROOT/include "$@" \
    -o $TMP/$s.o $ROOT/guacamole_amd/csrc/$s.hip &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $TMP/gq_pileup.o $TMP/gq_somatic.o $TMP/gq_heapref.o $TMP/gq_bamdev.o -lz
rm -rf $TMP
